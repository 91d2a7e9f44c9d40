#!/bin/bash
# GPU session: config 4 (HLL p=18) per-kernel breakdown at 125M and 1B docs
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${RUN_TAG:-h1}
mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 $secs "$@" > $O/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
cd /tmp
for d in 125000000 1000000000; do
  step prof_$d 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$d -o kb -- python3 $R/tools/kbench.py --docs $d --reps 3 --only config4_card
  python3 - $O/prof_$d/kb_kernel_stats.csv $O/prof_$d/kb_kernel_trace.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "hll" in r["Name"]: print("%-60s %4s %10.1f us  total %10.1f" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1000, float(r["TotalDurationNs"]) / 1000))
# one request's kernel sequence (the last): name, duration, gap before
rows = sorted(csv.DictReader(open(sys.argv[2])), key=lambda r: int(r["Start_Timestamp"]))
hll = [r for r in rows if "hll" in r["Kernel_Name"] or "fill" in r["Kernel_Name"]]
seq = hll[-40:]
prev = None
for r in seq:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print("  %-44s %8.1f us  gap %7.1f" % (r["Kernel_Name"][:44], (e - s) / 1000, (s - prev) / 1000 if prev else 0))
    prev = e
PY
done
echo "== done"
