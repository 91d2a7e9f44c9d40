#!/bin/bash
# GPU session T: threaded shard builds in the multi-shard bench (one-off; time-limited steps)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${RUN_TAG:-r2t}
mkdir -p $O
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 $secs "$@" > $O/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -2 $O/$name.log; [ $rc -eq 0 ] || exit $rc; }
step bench_ns8 300 python3 bench.py --shards 8 --docs 125000000 --cpu-docs 0
step bench_c5 300 python3 bench.py --workload config5 --shards 8 --docs 125000000 --cpu-docs 0
step bench_c3 300 python3 bench.py --workload config3 --shards 8 --docs 125000000 --cpu-docs 0
step bench_c4 300 python3 bench.py --workload config4 --shards 8 --docs 125000000 --cpu-docs 0
step bench_ns8_if2 300 python3 bench.py --shards 8 --docs 125000000 --cpu-docs 0 --inflight 2
step bench 300 python3 bench.py --cpu-docs 0
echo "== done"
