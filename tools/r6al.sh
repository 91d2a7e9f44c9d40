# round-6 GPU session: waves per SIMD of the raw-load counting grids with a terms dimension (build/variants ow6, ow6nb4,
# ow8) -- terms, terms{date_histogram}, date_histogram{terms}, terms{terms} at 1B
set -u
R=$GRAFT_REPO_ROOT
TAG=${1:-r6al}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
K="python3 $R/tools/kbench.py"
S=terms_host,terms_dh,dh_terms,hosts_urls
timeout -k 10 300 $K --docs 1000000000 --reps 5 --only $S > $O/kb_main.log 2>&1 || exit 1
for so in $R/build/variants/libesgpu_*.so; do
  [ -e "$so" ] || continue
  v=$(basename $so .so)
  ESGPU_LIBRARY=$so timeout -k 10 300 $K --docs 1000000000 --reps 5 --only $S > $O/kb_$v.log 2>&1 || exit 1
done
timeout -k 10 300 $K --docs 1000000000 --reps 5 --only $S > $O/kb_main2.log 2>&1 || exit 1
echo ALLOK
