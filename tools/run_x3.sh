#!/bin/bash
# GPU session: hot/cold scatter bisection (full / classify only / loads only) at 125M docs, kernel stats per variant
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${RUN_TAG:-x3}
mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 $secs "$@" > $O/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
cd /tmp
for v in main exp1 exp2; do
  lib=$R/elasticsearch_amd/libesgpu.so; [ $v = main ] || lib=$R/build/variants/libesgpu_$v.so
  export ESGPU_LIBRARY=$lib
  step prof_$v 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$v -o kb -- python3 $R/tools/kbench.py --docs 125000000 --reps 3 --only config3_url --shards 8
  python3 - $O/prof_$v/kb_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "hc_" in r["Name"]: print("%-50s %10.1f us" % (r["Name"][:50], float(r["AverageNs"]) / 1000))
PY
done
unset ESGPU_LIBRARY
step pmc_a 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_INSTS_SALU --kernel-trace --output-format csv -d $O/pmc_a -o kb -- python3 $R/tools/kbench.py --docs 125000000 --reps 1 --only config3_url --shards 8
echo "== done"
