# round-6 final session: smoke, the full GPU suite, the bench lines (north star + every BASELINE config, CPU baselines),
# rocprof kernel stats (north star, configs 2 and 3)
set -u
R=$GRAFT_REPO_ROOT
TAG=${1:-r6x}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
bash $R/tools/gpu_check.sh $TAG tests bench configs prof || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_config3 -o bench -- python3 $R/bench.py --workload config3 --shards 8 --docs 125000000 --cpu-docs 0 --steps 10 --warmup 3 --inflight 1 > $O/prof_config3.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_config2 -o bench -- python3 $R/bench.py --workload config2 --docs 100000000 --cpu-docs 0 --steps 10 --warmup 3 --inflight 1 > $O/prof_config2.log 2>&1 || exit 1
echo ALLOK
