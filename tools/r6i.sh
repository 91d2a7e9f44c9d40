# round-6 GPU session: kernel variants (kbench A/B on one box) and SQ counter passes (north star 1B, config 2 100M)
set -u
R=$GRAFT_REPO_ROOT
TAG=${1:-r6i}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
K="python3 $R/tools/kbench.py"
S=${KBENCH_ONLY:-north_star,ns_avg,config5}
timeout -k 10 300 $K --docs 1000000000 --reps 5 --only $S > $O/kb_main.log 2>&1 || exit 1
for so in $R/build/variants/libesgpu_*.so; do
  [ -e "$so" ] || continue
  v=$(basename $so .so)
  ESGPU_LIBRARY=$so timeout -k 10 300 $K --docs 1000000000 --reps 5 --only $S > $O/kb_$v.log 2>&1 || exit 1
done
timeout -k 10 300 $K --docs 1000000000 --reps 5 --only $S > $O/kb_main2.log 2>&1 || exit 1
G1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES"
G2="SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_SALU SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD"
for spec in north_star:1000000000 config2_dh_ext:100000000; do
  v=${spec%%:*}; d=${spec##*:}
  for grp in "$G1" "$G2"; do
    tag=$(echo "$grp" | cut -d' ' -f1)
    timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $O/pmc_${v}_$tag -o kb -- python3 $R/tools/kbench.py --docs $d --reps 1 --only $v > $O/pmc_${v}_$tag.log 2>&1 || exit 1
  done
done
echo ALLOK
