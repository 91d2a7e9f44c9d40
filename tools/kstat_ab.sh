#!/bin/bash
# Per-kernel average durations (rocprofv3 --kernel-trace --stats) of a kbench shape for the in-tree library and each
# build/variants/libesgpu_<name>.so named:   gpurun -- bash tools/kstat_ab.sh <tag> <shape> <kernel substring> [variant...]
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; SHAPE=$2; KER=$3; shift 3
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for v in base "$@"; do
    lib=""
    [ "$v" = base ] || lib=$R/build/variants/libesgpu_$v.so
    ESGPU_LIBRARY=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/$v" -o ks --output-format csv -- \
        python3 "$R/tools/kbench.py" --docs ${DOCS:-1000000000} --reps ${REPS:-3} --only "$SHAPE" > "$OUT/$v.log" 2>&1 || { tail -5 "$OUT/$v.log"; exit 1; }
    python3 - "$OUT/$v/ks_kernel_stats.csv" "$KER" "$v" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if sys.argv[2] in r["Name"]:
        print("%-8s %-60s calls %4s avg %.4f ms" % (sys.argv[3], r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e6))
PY
done
