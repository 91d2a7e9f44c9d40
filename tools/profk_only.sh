#!/bin/bash
# rocprofv3 kernel-trace stats of the kbench shapes in $1 (comma list): gpurun -- bash tools/profk_only.sh <shapes> <tag>
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${2:-profk}
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o kb -- python3 $R/tools/kbench.py --docs ${DOCS:-1000000000} --reps 3 --only $1 > $OUT/run.log 2>&1
rc=$?
grep -h '"name"' $OUT/run.log
python3 - "$OUT/kb_kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print("%-70s %6s %12.1f us" % (r["Name"][:70], r["Calls"], float(r["AverageNs"]) / 1000))
PY
exit $rc
