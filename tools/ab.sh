#!/bin/bash
# A/B of kernel builds on one box: kbench of the in-tree libesgpu.so and of every build/variants/libesgpu_<name>.so
# named on the command line, interleaved over ROUNDS rounds so box drift hits every build alike.
#   gpurun -- bash tools/ab.sh <tag> <shapes comma list> <variant> [variant...]
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1
SHAPES=$2
shift 2
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for round in $(seq 1 ${ROUNDS:-2}); do
    for v in base "$@"; do
        lib=""
        [ "$v" = base ] || lib=$R/build/variants/libesgpu_$v.so
        echo "== round $round $v $(date +%T)"
        ESGPU_LIBRARY=$lib timeout -k 10 300 python3 "$R/tools/kbench.py" --docs ${DOCS:-1000000000} --reps ${REPS:-5} \
            --only "$SHAPES" > "$OUT/kb_${v}_$round.log" 2>&1
        rc=$?
        grep -h '"name"' "$OUT/kb_${v}_$round.log" | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print('   %-22s %8.4f ms %8.1f GB/s' % (d['name'], d['kernel_ms'], d['gbs']))"
        [ $rc -eq 0 ] || { tail -20 "$OUT/kb_${v}_$round.log"; exit $rc; }
    done
done
echo "== done"
