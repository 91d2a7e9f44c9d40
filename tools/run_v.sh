#!/bin/bash
# GPU session V: hot/cold partitioned counting (config 3) parity + kernel timing
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${RUN_TAG:-r2v}
mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 $secs "$@" > $O/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -4 $O/$name.log; [ $rc -eq 0 ] || exit $rc; }
step pytest_hc 600 python3 -u -m pytest $R/tests/test_gpu_hotcold.py $R/tests/test_gpu_parity.py -k "hotcold or high_card or config3 or zipf or clustered or flat or cold_ord or two_seg or multi_segment or keyword_range" -x -v -p no:cacheprovider --timeout 300 --timeout-method thread
step kb125 300 python3 $R/tools/kbench.py --docs 125000000 --reps 5 --only config3_url
step kb1b 300 python3 $R/tools/kbench.py --docs 1000000000 --reps 5 --only config3_url
cd /tmp
step profk125 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/profk125 -o kb -- python3 $R/tools/kbench.py --docs 125000000 --reps 5 --only config3_url
echo "== done"
