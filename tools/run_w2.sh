#!/bin/bash
# GPU session: wire-stream parity, hot/cold merged flush (config 3) A/B, full GPU suite
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${RUN_TAG:-w2}
mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 $secs "$@" > $O/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -3 $O/$name.log; [ $rc -eq 0 ] || exit $rc; }
step pytest_wire 300 python3 -u -m pytest $R/tests/test_gpu_wire_stream.py $R/tests/test_gpu_hotcold.py -x -v -p no:cacheprovider --timeout 120 --timeout-method thread
step kb 300 python3 $R/tools/kbench.py --docs 125000000 --reps 5 --only config3_url --shards 8
ESGPU_LIBRARY=$R/build/variants/libesgpu_nomerge.so step kb_nomerge 300 python3 $R/tools/kbench.py --docs 125000000 --reps 5 --only config3_url --shards 8
cd /tmp
step prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o kb -- python3 $R/tools/kbench.py --docs 125000000 --reps 3 --only config3_url --shards 8
cd $R
step pytest_all 900 python3 -u -m pytest $R/tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread
echo "== done"
