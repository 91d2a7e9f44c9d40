# round-6 GPU session: 8 docs per thread and 6 waves per SIMD for the one-run integer grids -- full GPU suite, config 2
# and date_histogram{stats} at 1B / 100M, the jitter rows, the config 2 bench line
set -u
R=$GRAFT_REPO_ROOT
TAG=${1:-r6ah}
O=$R/gpurun_out/$TAG
mkdir -p $O
bash $R/tools/gpu_check.sh $TAG tests || exit 1
cd /tmp && export TMPDIR=/tmp
K="python3 $R/tools/kbench.py"
timeout -k 10 300 $K --docs 1000000000 --reps 5 --only config2_dh_ext,dh_stats,north_star > $O/kb.log 2>&1 || exit 1
timeout -k 10 300 $K --docs 100000000 --reps 9 --only config2_dh_ext > $O/kb_100m.log 2>&1 || exit 1
for J in 60000 3600000; do
  timeout -k 10 300 $K --docs 1000000000 --reps 5 --ts-jitter $J --only config2_dh_ext > $O/kb_j$J.log 2>&1 || exit 1
done
timeout -k 10 300 python3 $R/bench.py --workload config2 --cpu-docs 0 > $O/bench_config2.log 2>&1 || exit 1
echo ALLOK
