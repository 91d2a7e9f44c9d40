# round-6 GPU session: one-launch build copies and no per-collect D2H copy (config 2 step), tests, bench config 2 / NS
set -u
R=$GRAFT_REPO_ROOT
TAG=${1:-r6t}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_layouts.py tests/test_gpu_parity.py tests/test_gpu_rounding.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
for i in 1 2; do
  timeout -k 10 300 python3 $R/bench.py --workload config2 --docs 100000000 --cpu-docs 0 > $O/bench_config2_$i.log 2>&1 || exit 1
done
timeout -k 10 300 python3 $R/bench.py --cpu-docs 0 > $O/bench_ns.log 2>&1 || exit 1
echo ALLOK
