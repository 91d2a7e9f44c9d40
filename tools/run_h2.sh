#!/bin/bash
# GPU session: HLL floor folded into the snapshot kernel; phase-0 size and phase growth A/B (config 4, 125M and 1B)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${RUN_TAG:-h2}
mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 $secs "$@" > $O/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -1 $O/$name.log | cut -c1-160; [ $rc -eq 0 ] || exit $rc; }
step pytest_hll 600 python3 -u -m pytest $R/tests -m gpu -k "card or hll or config4" -x -v -p no:cacheprovider --timeout 300 --timeout-method thread
for v in main cut1 cut2 grow8 grow16; do
  lib=$R/elasticsearch_amd/libesgpu.so; [ $v = main ] || lib=$R/build/variants/libesgpu_$v.so
  ESGPU_LIBRARY=$lib step kb125_$v 300 python3 $R/tools/kbench.py --docs 125000000 --reps 7 --only config4_card
  ESGPU_LIBRARY=$lib step kb1b_$v 300 python3 $R/tools/kbench.py --docs 1000000000 --reps 5 --only config4_card
done
echo "== done"
