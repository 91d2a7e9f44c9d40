#!/bin/bash
# GPU session P: terms under terms + full suite on the split-TU build, bench inflight A/B (one-off; time-limited steps)
set -u
O=gpurun_out/${RUN_TAG:-r2p}
mkdir -p $O
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 $secs "$@" > $O/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -2 $O/$name.log; [ $rc -eq 0 ] || exit $rc; }
step tut 300 python3 -u -m pytest tests/test_gpu_terms_under_terms.py tests/test_gpu_boundary_errors.py -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread
step tests 1000 python3 -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread
step bench_if2 300 python3 bench.py --cpu-docs 0
step bench_if1 300 python3 bench.py --cpu-docs 0 --inflight 1
step kb_ns 300 python3 tools/kbench.py --docs 1000000000 --reps 5 --only north_star
echo "== done"
