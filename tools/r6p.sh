# round-6 GPU session: per-doc LDS cells for jittered histogram-only grids (ESGPU_HDIRECT A/B), config 3 traffic after
# the hot-pass prefetch clamp, layout / rounding / hot-cold tests
set -u
R=$GRAFT_REPO_ROOT
TAG=${1:-r6p}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_layouts.py tests/test_gpu_rounding.py tests/test_gpu_hotcold.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
K="python3 $R/tools/kbench.py"
for d in 100000000 1000000000; do
  for h in 4 2 0; do
    ESGPU_HDIRECT=$h timeout -k 10 300 $K --docs $d --reps 5 --only config2_dh_ext --ts-jitter 3600000 > $O/kb_c2_${d}_jit1h_hd$h.log 2>&1 || exit 1
  done
done
timeout -k 10 300 $K --docs 1000000000 --reps 5 --only config2_dh_ext,date_hist,north_star --ts-jitter 60000 > $O/kb_1b_jit1m.log 2>&1 || exit 1
timeout -k 10 300 $K --docs 125000000 --reps 7 --only config3_url,config3_url_f > $O/kb_c3_125m.log 2>&1 || exit 1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/pmcall_config3_url_125000000_$c -o kb -- python3 $R/tools/kbench.py --docs 125000000 --reps 3 --only config3_url > $O/pmcall_config3_url_125000000_$c.log 2>&1 || exit 1
done
echo ALLOK
