# round-6 GPU session: full GPU suite after the lazy count zeroing; config 3 / 4 bench lines; north star with and
# without the final window flush (timing variant build/variants/libesgpu_noflush.so)
set -u
R=$GRAFT_REPO_ROOT
TAG=${1:-r6r}
O=$R/gpurun_out/$TAG
mkdir -p $O
bash $R/tools/gpu_check.sh $TAG tests || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 $R/bench.py --workload config3 --shards 8 --docs 125000000 --cpu-docs 320000000 > $O/bench_config3.log 2>&1 || exit 1
timeout -k 10 300 python3 $R/bench.py --workload config4 --shards 8 --docs 125000000 --cpu-docs 320000000 > $O/bench_config4.log 2>&1 || exit 1
K="python3 $R/tools/kbench.py"
for d in 125000000 1000000000; do
  timeout -k 10 300 $K --docs $d --reps 7 --only north_star,ns_avg > $O/kb_ns_${d}_main.log 2>&1 || exit 1
  ESGPU_LIBRARY=$R/build/variants/libesgpu_noflush.so timeout -k 10 300 $K --docs $d --reps 7 --only north_star,ns_avg > $O/kb_ns_${d}_noflush.log 2>&1 || exit 1
done
echo ALLOK
