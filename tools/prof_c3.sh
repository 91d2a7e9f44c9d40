#!/bin/bash
# GPU session: per-kernel breakdown + LDS/VALU counters of config 3 (10M url ordinals) at the BASELINE shard (125M docs)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${RUN_TAG:-c3}
mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 $secs "$@" > $O/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -2 $O/$name.log; [ $rc -eq 0 ] || exit $rc; }
cd /tmp
step kb 300 python3 $R/tools/kbench.py --docs 125000000 --reps 5 --only config3_url,config4_card --shards 8
step prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o kb -- python3 $R/tools/kbench.py --docs 125000000 --reps 3 --only config3_url --shards 8
step pmc_a 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_VALU --kernel-trace --output-format csv -d $O/pmc_a -o kb -- python3 $R/tools/kbench.py --docs 125000000 --reps 1 --only config3_url --shards 8
step pmc_f 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc_f -o kb -- python3 $R/tools/kbench.py --docs 125000000 --reps 1 --only config3_url --shards 8
step pmc_w 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmc_w -o kb -- python3 $R/tools/kbench.py --docs 125000000 --reps 1 --only config3_url --shards 8
echo "== done"
