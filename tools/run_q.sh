#!/bin/bash
# GPU session Q: kernel timelines of the 8-shard bench and the 125M config 3/4 paths (one-off; time-limited steps)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${RUN_TAG:-r2q}
mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "== $name"; (cd /tmp && timeout -k 10 $secs "$@") > $O/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -2 $O/$name.log; [ $rc -eq 0 ] || exit $rc; }
step tl_ns8 300 rocprofv3 --kernel-trace --output-format csv -d $O/tl_ns8 -o t -- python3 $R/bench.py --shards 8 --docs 125000000 --cpu-docs 0 --steps 5 --warmup 2
step tl_c34 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tl_c34 -o t -- python3 $R/tools/kbench.py --docs 125000000 --reps 3 --shards 8 --only config3_url,config4_card
step kb_realdict 400 python3 $R/tools/kbench.py --docs 125000000 --reps 5 --shards 8 --real-dict --only config3_url,north_star,config1_terms_stats
echo "== done"
