# round-6 GPU session: 24-bit block deltas (a high-byte plane) for roughly time-ordered timestamps -- jitter tests, then
# the jitter table at 1B (sorted / ±1 min / ±1 h) with the plane and without it (ESGPU_B24=0)
set -u
R=$GRAFT_REPO_ROOT
TAG=${1:-r6ab}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_layouts.py tests/test_gpu_rounding.py tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
for J in 0 60000 3600000; do
  timeout -k 10 300 python3 $R/tools/kbench.py --docs 1000000000 --reps 5 --ts-jitter $J --only north_star,config2_dh_ext > $O/kb_j$J.log 2>&1 || exit 1
done
for J in 60000 3600000; do
  ESGPU_B24=0 timeout -k 10 300 python3 $R/tools/kbench.py --docs 1000000000 --reps 5 --ts-jitter $J --only north_star,config2_dh_ext > $O/kb_j${J}_nob24.log 2>&1 || exit 1
done
echo ALLOK
