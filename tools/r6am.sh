# round-6 GPU session: the hot ordinal's register count in counting terms x histogram grids (ESGPU_ORDH_HOT; the
# build/variants nohot library without it) -- kbench A/B, then the full GPU suite
set -u
R=$GRAFT_REPO_ROOT
TAG=${1:-r6am}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
K="python3 $R/tools/kbench.py"
S=terms_dh,dh_terms,north_star
timeout -k 10 300 $K --docs 1000000000 --reps 5 --only $S > $O/kb_main.log 2>&1 || exit 1
ESGPU_LIBRARY=$R/build/variants/libesgpu_nohot.so timeout -k 10 300 $K --docs 1000000000 --reps 5 --only $S > $O/kb_nohot.log 2>&1 || exit 1
timeout -k 10 300 $K --docs 1000000000 --reps 5 --only $S > $O/kb_main2.log 2>&1 || exit 1
timeout -k 10 300 $K --docs 1000000000 --reps 5 --ts-jitter 60000 --only terms_dh > $O/kb_main_j1m.log 2>&1 || exit 1
bash $R/tools/gpu_check.sh $TAG tests || exit 1
echo ALLOK
