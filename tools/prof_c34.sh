set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r1f
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/profk -o kb -- python3 $R/tools/kbench.py --docs 1000000000 --reps 3 --only config4_card,config3_url > $OUT/profk.log 2>&1 || exit 1
for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD" "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  tag=$(echo "$grp" | cut -d' ' -f1)
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $OUT/pmc_$tag -o kb -- python3 $R/tools/kbench.py --docs 1000000000 --reps 1 --only config4_card,config3_url > $OUT/pmc_$tag.log 2>&1 || exit 2
done
echo done
