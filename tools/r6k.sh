# round-6 GPU session: north-star kernel A/B + SQ passes (r6i), the hot/cold deferral tests, config 3 with and without
# the deferred cold lists
set -u
R=$GRAFT_REPO_ROOT
TAG=${1:-r6k}
O=$R/gpurun_out/$TAG
mkdir -p $O
bash $R/tools/r6i.sh $TAG || exit 1
cd $R
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_hotcold.py tests/test_gpu_layouts.py tests/test_gpu_parity.py tests/test_gpu_comm_build_reduce.py -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
cd /tmp
timeout -k 10 300 python3 $R/bench.py --workload config3 --steps 20 --warmup 3 --cpu-docs 0 > $O/bench_config3.log 2>&1 || exit 1
ESGPU_HC_PRUNE=0 timeout -k 10 300 python3 $R/bench.py --workload config3 --steps 20 --warmup 3 --cpu-docs 0 > $O/bench_config3_noprune.log 2>&1 || exit 1
timeout -k 10 300 python3 $R/tools/rank_sim.py --workload config3 --rccl --docs 125000000 --reqs 30 > $O/ranksim_rccl_config3.log 2>&1 || exit 1
echo ALLOK
