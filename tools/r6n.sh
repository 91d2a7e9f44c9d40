# round-6 GPU session: config 3 filtered / deleted-docs requests on the deferred hot-slot path (path 9)
set -u
R=$GRAFT_REPO_ROOT
TAG=${1:-r6n}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_hotcold.py -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_hotcold.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
K="python3 $R/tools/kbench.py"
for d in 125000000 1000000000; do
  timeout -k 10 300 $K --docs $d --reps 7 --only config3_url,config3_url_f > $O/kb_${d}.log 2>&1 || exit 1
  timeout -k 10 300 $K --docs $d --reps 7 --only config3_url --deletes 0.2 > $O/kb_${d}_del20.log 2>&1 || exit 1
  ESGPU_HC_PRUNE=0 timeout -k 10 300 $K --docs $d --reps 7 --only config3_url,config3_url_f > $O/kb_${d}_noprune.log 2>&1 || exit 1
  ESGPU_HC_PRUNE=0 timeout -k 10 300 $K --docs $d --reps 7 --only config3_url --deletes 0.2 > $O/kb_${d}_del20_noprune.log 2>&1 || exit 1
done
cd $R
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_comm_build_reduce.py tests/test_gpu_fuzz.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
echo ALLOK
