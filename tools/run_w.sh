#!/bin/bash
# GPU session W: hot/cold counting timing + HBM traffic counters (config 3, 125M docs)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${RUN_TAG:-r2w}
mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 $secs "$@" > $O/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -3 $O/$name.log; [ $rc -eq 0 ] || exit $rc; }
step pytest_hc 600 python3 -u -m pytest $R/tests/test_gpu_hotcold.py $R/tests/test_gpu_parity.py -k "hotcold or high_card or config3 or zipf or clustered or flat or cold_ord or two_seg or multi_segment" -x -q -p no:cacheprovider --timeout 300 --timeout-method thread
cd /tmp
step profk125 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/profk125 -o kb -- python3 $R/tools/kbench.py --docs 125000000 --reps 3 --only config3_url
for grp in FETCH_SIZE WRITE_SIZE "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM"; do
  tag=$(echo "$grp" | cut -d' ' -f1)
  step "pmc_$tag" 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $O/pmc_$tag -o kb -- python3 $R/tools/kbench.py --docs 125000000 --reps 1 --only config3_url
done
echo "== done"
