# round-6 GPU session: histogram-only metric grids' load depth (buffers x waves per SIMD, 8 docs per thread): config 2 at
# 1B and 100M docs, date_histogram{stats}, config 2 at ±1 h -- main build, then every build/variants library
set -u
R=$GRAFT_REPO_ROOT
TAG=${1:-r6ag}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
K="python3 $R/tools/kbench.py"
one() {  # tag, then env
  local t=$1; shift
  env "$@" timeout -k 10 300 $K --docs 1000000000 --reps 5 --only config2_dh_ext,dh_stats > $O/kb_$t.log 2>&1 || return 1
  env "$@" timeout -k 10 300 $K --docs 100000000 --reps 9 --only config2_dh_ext > $O/kb_${t}_100m.log 2>&1 || return 1
  env "$@" timeout -k 10 300 $K --docs 1000000000 --reps 5 --ts-jitter 3600000 --only config2_dh_ext > $O/kb_${t}_j1h.log 2>&1 || return 1
}
one main ESGPU_X=0 || exit 1
for so in $R/build/variants/libesgpu_*.so; do
  [ -e "$so" ] || continue
  v=$(basename $so .so)
  one $v ESGPU_LIBRARY=$so || exit 1
done
one main2 ESGPU_X=0 || exit 1
echo ALLOK
