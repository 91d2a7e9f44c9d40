# round-6 GPU session: kernel timings (1B, 125M, jittered), GPU parity files, SQ counters of the north star, rank_sim
set -u
R=$GRAFT_REPO_ROOT
TAG=${1:-r6d}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
K="python3 $R/tools/kbench.py"
# timeout -k 10 300 $K --docs 1000000000 --reps 5 --only north_star,ns_avg,config5,terms_dh,config2_dh_ext,date_hist > $O/kb_main_1b.log 2>&1 || exit 1
for j in; do
  timeout -k 10 300 $K --docs 1000000000 --reps 5 --ts-jitter $j --only north_star,config2_dh_ext,date_hist,terms_dh,config5 > $O/kb_jitter_$j.log 2>&1 || exit 1
done
timeout -k 10 900 python3 -u -m pytest $R/tests/test_gpu_rounding.py $R/tests/test_gpu_layouts.py $R/tests/test_gpu_comm_build_reduce.py $R/tests/test_gpu_scale.py -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
for w in north_star config3 config4 config5; do
  timeout -k 10 300 python3 $R/tools/rank_sim.py --workload $w --ranks 8 --docs 125000000 --reqs 20 > $O/ranksim_$w.log 2>&1 || exit 1
done
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES" "SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_SALU SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD"; do
  tag=$(echo "$grp" | cut -d' ' -f1)
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $O/pmc_ns_$tag -o kb -- python3 $R/tools/kbench.py --docs 1000000000 --reps 1 --only north_star > $O/pmc_ns_$tag.log 2>&1 || exit 1
done
echo ALLOK
