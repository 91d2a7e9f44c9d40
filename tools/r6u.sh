# round-6 GPU session: packed hot-run accounting A/B (build/variants hotpk0), one-launch build copies, tests, benches
set -u
R=$GRAFT_REPO_ROOT
TAG=${1:-r6u}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_layouts.py tests/test_gpu_parity.py tests/test_gpu_rounding.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
K="python3 $R/tools/kbench.py"
S=north_star,ns_avg,config5
timeout -k 10 300 $K --docs 1000000000 --reps 5 --only $S > $O/kb_main.log 2>&1 || exit 1
ESGPU_LIBRARY=$R/build/variants/libesgpu_hotpk0.so timeout -k 10 300 $K --docs 1000000000 --reps 5 --only $S > $O/kb_hotpk0.log 2>&1 || exit 1
timeout -k 10 300 $K --docs 1000000000 --reps 5 --only $S > $O/kb_main2.log 2>&1 || exit 1
ESGPU_LIBRARY=$R/build/variants/libesgpu_hotpk0.so timeout -k 10 300 $K --docs 1000000000 --reps 5 --only $S > $O/kb_hotpk0_2.log 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 300 python3 $R/bench.py --workload config2 --docs 100000000 --cpu-docs 0 > $O/bench_config2_$i.log 2>&1 || exit 1
done
timeout -k 10 300 python3 $R/bench.py --cpu-docs 0 > $O/bench_ns.log 2>&1 || exit 1
echo ALLOK
