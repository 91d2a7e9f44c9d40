#!/bin/bash
# GPU session: hot/cold postings path (config 3) -- A/B against the scatter path and 2 hot workgroups per CU, breakdown
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${RUN_TAG:-p7}
mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 $secs "$@" > $O/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -1 $O/$name.log; [ $rc -eq 0 ] || exit $rc; }
step kb 300 python3 $R/tools/kbench.py --docs 125000000 --reps 5 --only config3_url --shards 8
step kb1b 300 python3 $R/tools/kbench.py --docs 1000000000 --reps 5 --only config3_url
for v in scatter hot2; do
  ESGPU_LIBRARY=$R/build/variants/libesgpu_$v.so step kb_$v 300 python3 $R/tools/kbench.py --docs 125000000 --reps 5 --only config3_url --shards 8
done
cd /tmp
step prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o kb -- python3 $R/tools/kbench.py --docs 125000000 --reps 3 --only config3_url --shards 8
python3 - $O/prof/kb_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "hc_" in r["Name"]: print("%-50s %4s %10.1f us" % (r["Name"][:50], r["Calls"], float(r["AverageNs"]) / 1000))
PY
echo "== done"
