#!/bin/bash
# GPU session: hot/cold postings defaults (2 hot workgroups per CU, 16-row hot reduce) -- parity + timing
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${RUN_TAG:-p8}
mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 $secs "$@" > $O/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -1 $O/$name.log; [ $rc -eq 0 ] || exit $rc; }
step pytest_hc 600 python3 -u -m pytest $R/tests/test_gpu_hotcold.py $R/tests/test_gpu_scale.py -k "hotcold or config3 or zipf or clustered or flat or cold_ord or two_seg" -x -v -p no:cacheprovider --timeout 300 --timeout-method thread
step kb 300 python3 $R/tools/kbench.py --docs 125000000 --reps 5 --only config3_url --shards 8
step kb1b 300 python3 $R/tools/kbench.py --docs 1000000000 --reps 5 --only config3_url
step bench_c3 300 python3 $R/bench.py --workload config3 --shards 8 --docs 125000000 --cpu-docs 320000000
cd /tmp
step prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o kb -- python3 $R/tools/kbench.py --docs 125000000 --reps 3 --only config3_url --shards 8
python3 - $O/prof/kb_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "hc_" in r["Name"]: print("%-50s %4s %10.1f us" % (r["Name"][:50], r["Calls"], float(r["AverageNs"]) / 1000))
PY
step pmc_f 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc_f -o kb -- python3 $R/tools/kbench.py --docs 125000000 --reps 1 --only config3_url --shards 8
step pmc_w 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmc_w -o kb -- python3 $R/tools/kbench.py --docs 125000000 --reps 1 --only config3_url --shards 8
echo "== done"
