#!/bin/bash
# One rocprofv3 PMC pass per counter group over a kbench shape (each pass its own process, under a hard time limit):
#   gpurun -- bash tools/pmc_pass.sh <tag> <shape> "<counters>" ["<counters>" ...]
# Output: gpurun_out/<tag>/p<i>/... (counter_collection.csv per pass)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1
SHAPE=$2
shift 2
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for ctrs in "$@"; do
    i=$((i + 1))
    echo "== pass $i: $ctrs $(date +%T)"
    timeout -s KILL 150 rocprofv3 --pmc $ctrs --kernel-trace -d "$OUT/p$i" -o pass -- \
        python3 "$R/tools/kbench.py" --docs ${DOCS:-1000000000} --reps ${REPS:-3} --only "$SHAPE" > "$OUT/p$i.log" 2>&1
    rc=$?
    [ $rc -eq 0 ] || { tail -5 "$OUT/p$i.log"; exit $rc; }
done
echo "== done"
