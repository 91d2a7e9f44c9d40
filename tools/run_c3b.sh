#!/bin/bash
# GPU session: hot/cold scatter prologue-order fix (config 3) and HLL load-buffer count (config 4): parity + timing
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${RUN_TAG:-c3b}
mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 $secs "$@" > $O/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -3 $O/$name.log; [ $rc -eq 0 ] || exit $rc; }
step pytest_hc 600 python3 -u -m pytest $R/tests/test_gpu_hotcold.py $R/tests/test_gpu_scale.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread
step kb 300 python3 $R/tools/kbench.py --docs 125000000 --reps 5 --only config3_url,config4_card --shards 8
step kb1b 300 python3 $R/tools/kbench.py --docs 1000000000 --reps 5 --only config4_card
export ESGPU_LIBRARY=$R/build/variants/libesgpu_nbuf3.so
step kb_nbuf3 300 python3 $R/tools/kbench.py --docs 125000000 --reps 5 --only config4_card --shards 8
step kb1b_nbuf3 300 python3 $R/tools/kbench.py --docs 1000000000 --reps 5 --only config4_card
unset ESGPU_LIBRARY
cd /tmp
step prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o kb -- python3 $R/tools/kbench.py --docs 125000000 --reps 3 --only config3_url --shards 8
echo "== done"
