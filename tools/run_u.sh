#!/bin/bash
# GPU session U (round 2, re-entry): GPU parity tests on the rebuilt tree, per-kernel breakdown of config 3 / 4 at 125M
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${RUN_TAG:-r2u2}
mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 $secs "$@" > $O/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -3 $O/$name.log; [ $rc -eq 0 ] || exit $rc; }
step pytest_gpu 900 python3 -u -m pytest $R/tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread
cd /tmp
step profk125 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/profk125 -o kb -- python3 $R/tools/kbench.py --docs 125000000 --reps 5 --only config3_url,config4_card
echo "== done"
