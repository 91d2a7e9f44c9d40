# round-6 GPU session: the breadth-first replay over the inner field's hot terms (replay_hot), tests and hosts_urls A/B
set -u
R=$GRAFT_REPO_ROOT
TAG=${1:-r6s}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_breadth_first.py -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_bf.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
K="python3 $R/tools/kbench.py"
for d in 125000000 1000000000; do
  timeout -k 10 300 $K --docs $d --reps 5 --only hosts_urls > $O/kb_${d}_hot.log 2>&1 || exit 1
  ESGPU_REPLAY_HOT=0 timeout -k 10 300 $K --docs $d --reps 5 --only hosts_urls > $O/kb_${d}_nohot.log 2>&1 || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_replay -o kb -- python3 $R/tools/kbench.py --docs 1000000000 --reps 3 --only hosts_urls > $O/prof_replay.log 2>&1 || exit 1
cd $R
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_three_levels.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
echo ALLOK
