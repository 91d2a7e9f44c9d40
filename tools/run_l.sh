#!/bin/bash
# GPU session L: full GPU suite + bench lines after the build/reduce host work (one-off; every step time-limited)
set -u
O=gpurun_out/${RUN_TAG:-r2l}
mkdir -p $O
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 $secs "$@" > $O/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -2 $O/$name.log; [ $rc -eq 0 ] || exit $rc; }
step tests 1000 python3 -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread
step kb125 300 python3 tools/kbench.py --docs 125000000 --reps 5 --shards 8
step bench 300 python3 bench.py --cpu-docs 0
step bench_ns8 300 python3 bench.py --shards 8 --docs 125000000 --cpu-docs 0
step bench_c5 300 python3 bench.py --workload config5 --shards 8 --docs 125000000 --cpu-docs 0
step bench_c3 300 python3 bench.py --workload config3 --shards 8 --docs 125000000 --cpu-docs 0
echo "== done"
