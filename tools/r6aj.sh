# round-6 GPU session: packed-cell (min, max) updates as one divergent loop per lane (build/variants mmu4) against the
# per-doc regions -- north star, terms{stats}, config 5 (avg: no extrema, control), north star at ±1 h; twice each
set -u
R=$GRAFT_REPO_ROOT
TAG=${1:-r6aj}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
K="python3 $R/tools/kbench.py"
one() {
  local t=$1; shift
  env "$@" timeout -k 10 300 $K --docs 1000000000 --reps 5 --only north_star,config1_terms_stats,config5 > $O/kb_$t.log 2>&1 || return 1
  env "$@" timeout -k 10 300 $K --docs 1000000000 --reps 5 --ts-jitter 3600000 --only north_star > $O/kb_${t}_j1h.log 2>&1 || return 1
}
one main ESGPU_X=0 || exit 1
one mmu4 ESGPU_LIBRARY=$R/build/variants/libesgpu_mmu4.so || exit 1
one main2 ESGPU_X=0 || exit 1
one mmu4b ESGPU_LIBRARY=$R/build/variants/libesgpu_mmu4.so || exit 1
echo ALLOK
