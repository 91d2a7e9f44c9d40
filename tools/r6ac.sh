# round-6 GPU session: 24-bit runs gated on the zone span (±1 min takes them, ±1 h the 32-bit deltas) -- jitter tests,
# the jitter rows at 1B, and SQ counter passes of the ±1 h north star and config 2 (where the kernel is not bytes-bound)
set -u
R=$GRAFT_REPO_ROOT
TAG=${1:-r6ac}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_layouts.py tests/test_gpu_rounding.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
for J in 60000 3600000; do
  timeout -k 10 300 python3 $R/tools/kbench.py --docs 1000000000 --reps 5 --ts-jitter $J --only north_star,config2_dh_ext > $O/kb_j$J.log 2>&1 || exit 1
done
G1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES"
G2="SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_SALU SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD"
for v in north_star config2_dh_ext; do
  for grp in "$G1" "$G2"; do
    tag=$(echo "$grp" | cut -d' ' -f1)
    timeout -s KILL 150 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $O/pmc_${v}_$tag -o kb -- python3 $R/tools/kbench.py --docs 1000000000 --reps 1 --ts-jitter 3600000 --only $v > $O/pmc_${v}_$tag.log 2>&1 || exit 1
  done
done
echo ALLOK
