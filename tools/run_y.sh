#!/bin/bash
# GPU session Y: hot/cold scatter timing breakdown via variants (classify only, loads only, no hot table, NT loads)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${RUN_TAG:-r2y}
mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 $secs "$@" > $O/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
cd /tmp
for v in ${VARIANTS:-exp1 exp2 nohot nt}; do
  export ESGPU_LIBRARY=$R/build/variants/libesgpu_$v.so; step prof_$v 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$v -o kb -- python3 $R/tools/kbench.py --docs 125000000 --reps 3 --only config3_url
  python3 - $O/prof_$v/kb_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "hc_" in r["Name"]: print("%-60s %10.1f us" % (r["Name"][:60], float(r["AverageNs"]) / 1000))
PY
done
echo "== done"
