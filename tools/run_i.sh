#!/bin/bash
# GPU session I: wide-window parity + jitter sweep + build-cost experiments (one-off; every step time-limited)
set -u
O=gpurun_out/r2i
mkdir -p $O
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 $secs "$@" > $O/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -3 $O/$name.log; [ $rc -eq 0 ] || exit $rc; }
step tests 600 python3 -u -m pytest tests/test_gpu_rounding.py tests/test_gpu_tree_shapes.py tests/test_gpu_parity.py -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread
step memprobe 120 python3 tools/host_mem_probe.py
for j in 0 60000 3600000; do
  step kbench_j$j 300 python3 tools/kbench.py --docs 1000000000 --reps 5 --ts-jitter $j --only north_star,config2_dh_ext,date_hist,terms_dh,config5
done
step kb125_base 200 python3 tools/kbench.py --docs 125000000 --reps 5 --shards 8 --only north_star,ns_avg,config4_card
MALLOC_MMAP_THRESHOLD_=4000000000 MALLOC_TRIM_THRESHOLD_=4000000000 step kb125_malloc 200 python3 tools/kbench.py --docs 125000000 --reps 5 --shards 8 --only north_star,ns_avg
step kb125_s1 200 python3 tools/kbench.py --docs 125000000 --reps 5 --shards 1 --only north_star
step bench_config4 300 python3 bench.py --workload config4 --shards 8 --docs 125000000 --cpu-docs 0
echo "== done"
