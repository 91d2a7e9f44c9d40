# round-6 GPU session: the one-run integer grids' multi-key zone blocks through the window accumulators (kWinMK;
# build/variants nowmk without) -- config 2 and date_histogram{stats} sorted / ±1 min / ±1 h at 1B, then the layout,
# rounding and parity suites
set -u
R=$GRAFT_REPO_ROOT
TAG=${1:-r6aw}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
K="python3 $R/tools/kbench.py"
for J in 0 60000 3600000; do
  timeout -k 10 300 $K --docs 1000000000 --reps 5 --ts-jitter $J --only config2_dh_ext,dh_stats > $O/kb_main_j$J.log 2>&1 || exit 1
  ESGPU_LIBRARY=$R/build/variants/libesgpu_nowmk.so timeout -k 10 300 $K --docs 1000000000 --reps 5 --ts-jitter $J --only config2_dh_ext,dh_stats > $O/kb_nowmk_j$J.log 2>&1 || exit 1
done
timeout -k 10 300 $K --docs 100000000 --reps 9 --only config2_dh_ext > $O/kb_main_100m.log 2>&1 || exit 1
cd $R
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_layouts.py tests/test_gpu_rounding.py tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
echo ALLOK
