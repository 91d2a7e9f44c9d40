# round-6 GPU session: zone-keys per-workgroup words (no shared atomic), 16-byte grid fills, layouts / parity / rounding tests, NS kbench
set -u
R=$GRAFT_REPO_ROOT
TAG=${1:-r6aa}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_layouts.py tests/test_gpu_parity.py tests/test_gpu_rounding.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 $R/tools/kbench.py --docs 1000000000 --reps 5 --only north_star,config2_dh_ext,config5 > $O/kb.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o kb -- python3 $R/tools/kbench.py --docs 1000000000 --reps 3 --only north_star > $O/prof.log 2>&1 || exit 1
timeout -k 10 300 python3 $R/bench.py --cpu-docs 0 > $O/bench_ns.log 2>&1 || exit 1
echo ALLOK
