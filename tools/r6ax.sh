# round-6 GPU session: the final library (kWinMK off) -- smoke, kbench config 2 / date_histogram{stats} / north star at
# 1B (sorted, ±1 h), the full GPU suite
set -u
R=$GRAFT_REPO_ROOT
TAG=${1:-r6ax}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
K="python3 $R/tools/kbench.py"
timeout -k 10 300 $K --docs 1000000000 --reps 5 --only config2_dh_ext,dh_stats,north_star > $O/kb.log 2>&1 || exit 1
timeout -k 10 300 $K --docs 1000000000 --reps 5 --ts-jitter 3600000 --only config2_dh_ext > $O/kb_j1h.log 2>&1 || exit 1
bash $R/tools/gpu_check.sh $TAG tests || exit 1
echo ALLOK
