#!/bin/bash
# GPU session: A/B of a wider LDS key window (one 1024-thread workgroup per CU) on time-sorted data at the BASELINE
# per-shard size (fewer window flushes per workgroup) and at 1B docs
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${RUN_TAG:-wide}
mkdir -p $O
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 $secs "$@" > $O/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
for v in main wide4 wide8; do
  lib=$R/elasticsearch_amd/libesgpu.so; [ $v = main ] || lib=$R/build/variants/libesgpu_$v.so
  ESGPU_LIBRARY=$lib step kb125_$v 300 python3 $R/tools/kbench.py --docs 125000000 --reps 7 --shards 8 --only north_star,config5,terms_dh,config2_dh_ext,dh_terms
  ESGPU_LIBRARY=$lib step kb1b_$v 300 python3 $R/tools/kbench.py --docs 1000000000 --reps 5 --only north_star,config5,terms_dh
done
echo "== done"
