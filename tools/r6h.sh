# round-6 GPU session: hot-term register-run variants of the north-star kernel (kbench A/B on one box)
set -u
R=$GRAFT_REPO_ROOT
TAG=${1:-r6h}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
K="python3 $R/tools/kbench.py"
S=${KBENCH_ONLY:-north_star,ns_avg,config5}
timeout -k 10 300 $K --docs 1000000000 --reps 5 --only $S > $O/kb_main.log 2>&1 || exit 1
for so in $R/build/variants/libesgpu_*.so; do
  v=$(basename $so .so)
  ESGPU_LIBRARY=$so timeout -k 10 300 $K --docs 1000000000 --reps 5 --only $S > $O/kb_$v.log 2>&1 || exit 1
done
timeout -k 10 300 $K --docs 1000000000 --reps 5 --only $S > $O/kb_main2.log 2>&1 || exit 1
timeout -k 10 300 $K --docs 125000000 --reps 7 --only $S > $O/kb_main_125m.log 2>&1 || exit 1
echo ALLOK
