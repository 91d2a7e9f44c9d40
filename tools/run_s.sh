#!/bin/bash
# GPU session S: HIP runtime trace of the 8-shard bench (host-side stall), config 3 counting rule (one-off)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${RUN_TAG:-r2s}
mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "== $name"; (cd /tmp && timeout -k 10 $secs "$@") > $O/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -2 $O/$name.log; [ $rc -eq 0 ] || exit $rc; }
step rt_ns8 300 rocprofv3 --runtime-trace --kernel-trace --output-format csv -d $O/rt_ns8 -o t -- python3 $R/bench.py --shards 8 --docs 125000000 --cpu-docs 0 --steps 3 --warmup 1
for d in 1000000000 125000000; do
  step kb_c3_$d 300 python3 $R/tools/kbench.py --docs $d --reps 5 --shards 8 --only config3_url
done
echo "== done"
