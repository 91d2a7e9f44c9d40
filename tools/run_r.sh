#!/bin/bash
# GPU session R: config 3 counting chunks and config 4 2-bit snapshot A/B (one-off; time-limited steps)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${RUN_TAG:-r2r}
mkdir -p $O
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 $secs "$@" > $O/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -2 $O/$name.log; [ $rc -eq 0 ] || exit $rc; }
T="tests/test_gpu_scale.py tests/test_gpu_parity.py -k config3_or_config4"
step tests 600 python3 -u -m pytest tests/test_gpu_scale.py tests/test_gpu_parity.py -k "config3 or config4 or cardinality or partitioned" -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread
ESGPU_LIBRARY=$R/build/variants/libesgpu_hllb2.so step tests_hllb2 600 python3 -u -m pytest tests/test_gpu_scale.py tests/test_gpu_parity.py -k "config4 or cardinality" -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread
for d in 1000000000 125000000; do
  step kb_default_$d 300 python3 tools/kbench.py --docs $d --reps 5 --shards 8 --only config3_url,config4_card
  ESGPU_LIBRARY=$R/build/variants/libesgpu_cnt4.so step kb_cnt4_$d 300 python3 tools/kbench.py --docs $d --reps 5 --shards 8 --only config3_url
  ESGPU_LIBRARY=$R/build/variants/libesgpu_hllb2.so step kb_hllb2_$d 300 python3 tools/kbench.py --docs $d --reps 5 --shards 8 --only config4_card
done
echo "== done"
