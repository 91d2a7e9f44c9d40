#!/bin/bash
# GPU session Z: LDS utilisation counters of the hot/cold scatter (full kernel and the classify-only variant)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${RUN_TAG:-r2z}
mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 $secs "$@" > $O/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
cd /tmp
for v in main exp1; do
  lib=$R/elasticsearch_amd/libesgpu.so; [ $v = main ] || lib=$R/build/variants/libesgpu_$v.so
  export ESGPU_LIBRARY=$lib; step pmc_${v}_a 120 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY --kernel-trace --output-format csv -d $O/pmc_${v}_a -o kb -- python3 $R/tools/kbench.py --docs 125000000 --reps 1 --only config3_url
  step pmc_${v}_b 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/pmc_${v}_b -o kb -- python3 $R/tools/kbench.py --docs 125000000 --reps 1 --only config3_url
  unset ESGPU_LIBRARY
done
echo "== done"
