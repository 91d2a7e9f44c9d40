#!/bin/bash
# GPU session: smoke() entry point + every BASELINE config's bench line on the current build
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${RUN_TAG:-f1}
mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 $secs "$@" > $O/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -1 $O/$name.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc; }
step smoke 300 python3 -c "import sys; sys.path.insert(0, '$R'); import __graft_entry__ as g; g.smoke()"
step bench_config2 300 python3 $R/bench.py --workload config2 --docs 100000000 --cpu-docs 160000000
step bench_config4 300 python3 $R/bench.py --workload config4 --shards 8 --docs 125000000 --cpu-docs 320000000
step bench_config5 300 python3 $R/bench.py --workload config5 --shards 8 --docs 125000000 --cpu-docs 320000000
step bench_ns8 300 python3 $R/bench.py --shards 8 --docs 125000000 --cpu-docs 0
step bench 300 python3 $R/bench.py
echo "== done"
