#!/bin/bash
# GPU session N: zone-key precompute check (one-off; every step time-limited)
set -u
O=gpurun_out/${RUN_TAG:-r2n}
mkdir -p $O
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 $secs "$@" > $O/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -2 $O/$name.log; [ $rc -eq 0 ] || exit $rc; }
step tests 600 python3 -u -m pytest tests/test_gpu_rounding.py tests/test_gpu_parity.py tests/test_gpu_tree_shapes.py -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread
for j in 0 3600000; do
  step kbench_j$j 300 python3 tools/kbench.py --docs 1000000000 --reps 5 --ts-jitter $j --only north_star,config2_dh_ext,date_hist,terms_dh,config5,terms_host,config1_terms_stats,config4_card,config3_url
done
step bench 300 python3 bench.py --cpu-docs 0
echo "== done"
