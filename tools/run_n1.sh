#!/bin/bash
# GPU session: north-star collect kernel instruction mix and stall counters (1B docs, one launch per pass)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${RUN_TAG:-n1}
mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 $secs "$@" > $O/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
cd /tmp
step pmc_a 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS --kernel-trace --output-format csv -d $O/pmc_a -o kb -- python3 $R/tools/kbench.py --docs 1000000000 --reps 1 --only north_star
step pmc_b 180 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_WAVES --kernel-trace --output-format csv -d $O/pmc_b -o kb -- python3 $R/tools/kbench.py --docs 1000000000 --reps 1 --only north_star
python3 - $O <<'PY'
import csv, sys, collections
for f in ("pmc_a", "pmc_b"):
    agg = collections.defaultdict(float)
    for r in csv.DictReader(open(sys.argv[1] + "/" + f + "/kb_counter_collection.csv")):
        if "collect_kernel" in r["Kernel_Name"]:
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
    print(f, {k: int(v) for k, v in sorted(agg.items())})
PY
echo "== done"
