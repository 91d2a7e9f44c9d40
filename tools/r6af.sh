# round-6 GPU session: config 2 load-depth variants (buffers, waves, 8 docs per thread) at 1B and 100M docs
set -u
R=$GRAFT_REPO_ROOT
TAG=${1:-r6af}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
K="python3 $R/tools/kbench.py"
timeout -k 10 300 $K --docs 1000000000 --reps 5 --only config2_dh_ext > $O/kb_main.log 2>&1 || exit 1
timeout -k 10 300 $K --docs 100000000 --reps 9 --only config2_dh_ext > $O/kb_main_100m.log 2>&1 || exit 1
for so in $R/build/variants/libesgpu_*.so; do
  [ -e "$so" ] || continue
  v=$(basename $so .so)
  ESGPU_LIBRARY=$so timeout -k 10 300 $K --docs 1000000000 --reps 5 --only config2_dh_ext > $O/kb_$v.log 2>&1 || exit 1
  ESGPU_LIBRARY=$so timeout -k 10 300 $K --docs 100000000 --reps 9 --only config2_dh_ext > $O/kb_${v}_100m.log 2>&1 || exit 1
done
echo ALLOK
