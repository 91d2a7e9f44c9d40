# round-6 GPU session: two-slot window accumulators for the one-run grids' multi-key zone blocks (build/variants mk2)
# against the main library -- config 2 / date_histogram{stats} sorted and ±1 min at 1B, then the layout / rounding /
# parity suites on the variant
set -u
R=$GRAFT_REPO_ROOT
TAG=${1:-r6ay}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
K="python3 $R/tools/kbench.py"
V=$R/build/variants/libesgpu_mk2.so
for J in 0 60000; do
  timeout -k 10 300 $K --docs 1000000000 --reps 5 --ts-jitter $J --only config2_dh_ext,dh_stats > $O/kb_main_j$J.log 2>&1 || exit 1
  ESGPU_LIBRARY=$V timeout -k 10 300 $K --docs 1000000000 --reps 5 --ts-jitter $J --only config2_dh_ext,dh_stats > $O/kb_mk2_j$J.log 2>&1 || exit 1
done
cd $R
ESGPU_LIBRARY=$V timeout -k 10 600 python3 -u -m pytest tests/test_gpu_layouts.py tests/test_gpu_rounding.py tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_mk2.log 2>&1 || exit 1
echo ALLOK
