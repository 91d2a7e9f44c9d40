#!/bin/bash
# GPU session: per-launch sequence of 125M-doc shard collects (fixed costs per collect)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${RUN_TAG:-s1}
mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 $secs "$@" > $O/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
cd /tmp
for w in terms_host north_star; do
  step prof_$w 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$w -o kb -- python3 $R/tools/kbench.py --docs 125000000 --reps 3 --only $w
  grep '^{"name' $O/prof_$w.log | cut -c1-200
  python3 - $O/prof_$w/kb_kernel_trace.csv <<'PY'
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
rows = [r for r in rows if "synth" not in r["Kernel_Name"] and "zone_map" not in r["Kernel_Name"]]
prev = None
for r in rows[-14:]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print("  %-60s grid %-8s wg %-5s lds %-6s %8.1f us  gap %7.1f" % (r["Kernel_Name"][:60], r.get("Grid_Size", ""), r.get("Workgroup_Size", ""), r.get("LDS_Block_Size", r.get("Lds_Size", "")), (e - s) / 1000, (s - prev) / 1000 if prev else 0))
    prev = e
PY
done
echo "== done"
