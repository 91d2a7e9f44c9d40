# round-6 GPU session: packed-cell extrema in one divergent region per pair of docs (build/variants mmu5) against one
# per doc -- north star, terms{stats} and config 5 at 1B, alternating
set -u
R=$GRAFT_REPO_ROOT
TAG=${1:-r6au}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
K="python3 $R/tools/kbench.py"
for i in 1 2; do
  timeout -k 10 300 $K --docs 1000000000 --reps 5 --only north_star,config1_terms_stats > $O/kb_main_$i.log 2>&1 || exit 1
  ESGPU_LIBRARY=$R/build/variants/libesgpu_mmu5.so timeout -k 10 300 $K --docs 1000000000 --reps 5 --only north_star,config1_terms_stats > $O/kb_mmu5_$i.log 2>&1 || exit 1
done
echo ALLOK
