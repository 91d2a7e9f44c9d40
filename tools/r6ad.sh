# round-6 GPU session: window accumulators for integer runs over roughly time-ordered data (histogram-only grids at ±1 h)
# -- jitter / layout / rounding tests, the jitter rows at 1B with and without them (build/variants nowin), SQ passes
set -u
R=$GRAFT_REPO_ROOT
TAG=${1:-r6ad}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_layouts.py tests/test_gpu_rounding.py tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
for J in 0 3600000; do
  timeout -k 10 300 python3 $R/tools/kbench.py --docs 1000000000 --reps 5 --ts-jitter $J --only config2_dh_ext,north_star > $O/kb_j$J.log 2>&1 || exit 1
  ESGPU_B24=2 timeout -k 10 300 python3 $R/tools/kbench.py --docs 1000000000 --reps 5 --ts-jitter $J --only config2_dh_ext,north_star > $O/kb_j${J}_b24.log 2>&1 || exit 1
  ESGPU_LIBRARY=$R/build/variants/libesgpu_nowin.so timeout -k 10 300 python3 $R/tools/kbench.py --docs 1000000000 --reps 5 --ts-jitter $J --only config2_dh_ext > $O/kb_j${J}_nowin.log 2>&1 || exit 1
done
G1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES"
G2="SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_SALU SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD"
for grp in "$G1" "$G2"; do
  tag=$(echo "$grp" | cut -d' ' -f1)
  timeout -s KILL 150 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $O/pmc_config2_dh_ext_$tag -o kb -- python3 $R/tools/kbench.py --docs 1000000000 --reps 1 --ts-jitter 3600000 --only config2_dh_ext > $O/pmc_config2_$tag.log 2>&1 || exit 1
done
echo ALLOK
