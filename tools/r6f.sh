# round-6 GPU session: LDS-conflict variants of the north-star kernel (lane copies, hot-term registers) and rank_sim
set -u
R=$GRAFT_REPO_ROOT
TAG=${1:-r6f}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
K="python3 $R/tools/kbench.py"
S=north_star,ns_avg,config5
timeout -k 10 300 $K --docs 1000000000 --reps 5 --only $S > $O/kb_main.log 2>&1 || exit 1
ESGPU_PI_COPIES=2 timeout -k 10 300 $K --docs 1000000000 --reps 5 --only $S > $O/kb_copies2.log 2>&1 || exit 1
ESGPU_LIBRARY=$R/build/variants/libesgpu_hotu.so timeout -k 10 300 $K --docs 1000000000 --reps 5 --only $S > $O/kb_hotu.log 2>&1 || exit 1
ESGPU_PI_COPIES=2 ESGPU_LIBRARY=$R/build/variants/libesgpu_hotu.so timeout -k 10 300 $K --docs 1000000000 --reps 5 --only $S > $O/kb_hotu_copies2.log 2>&1 || exit 1
timeout -k 10 300 $K --docs 1000000000 --reps 5 --only $S > $O/kb_main2.log 2>&1 || exit 1
for w in north_star config3 config4 config5; do
  timeout -k 10 300 python3 $R/tools/rank_sim.py --workload $w --rccl --docs 125000000 --reqs 30 > $O/ranksim_rccl_$w.log 2>&1 || exit 1
  timeout -k 10 300 python3 $R/tools/rank_sim.py --workload $w --ranks 8 --docs 125000000 --reqs 20 > $O/ranksim_$w.log 2>&1 || exit 1
done
echo ALLOK
