#!/bin/bash
# GPU session K: full GPU suite + build-cost trace at 125M docs/shard (one-off; every step time-limited)
set -u
O=gpurun_out/r2k
mkdir -p $O
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 $secs "$@" > $O/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -3 $O/$name.log; [ $rc -eq 0 ] || exit $rc; }
step tests 1000 python3 -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread
ESGPU_TRACE_BUILD=1 step kb125_trace 300 python3 tools/kbench.py --docs 125000000 --reps 5 --shards 8
step bench_ns8 300 python3 bench.py --shards 8 --docs 125000000 --cpu-docs 0
step bench_c5 300 python3 bench.py --workload config5 --shards 8 --docs 125000000 --cpu-docs 0
for so in build/variants/libesgpu_bpw*.so; do
  v=$(basename $so .so)
  ESGPU_LIBRARY=$so step kb125_$v 300 python3 tools/kbench.py --docs 125000000 --reps 5 --shards 8
done
step kb125_default 300 python3 tools/kbench.py --docs 125000000 --reps 5 --shards 8
echo "== done"
