#!/bin/bash
# GPU session: histogram under histogram with the inner key index derived in the collect kernel's loader, and
# combined per-thread / per-wave LDS atomics for counting ORD x histogram grids (full GPU suite, then A/B on the
# heat-map, date_histogram{terms} and terms{date_histogram} shapes)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${RUN_TAG:-hm}
mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 $secs "$@" > $O/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -1 $O/$name.log | cut -c1-160; [ $rc -eq 0 ] || exit $rc; }
step pytest_gpu 900 python3 -u -m pytest $R/tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
for v in main ${VARIANTS:-nocomb hcp4 nofuse}; do
  lib=$R/elasticsearch_amd/libesgpu.so; [ $v = main ] || lib=$R/build/variants/libesgpu_$v.so
  ESGPU_LIBRARY=$lib step kb_$v 300 python3 $R/tools/kbench.py --docs 1000000000 --reps 5 --only ${ONLY:-heatmap,dh_terms,terms_dh,north_star}
done
echo "== done"
