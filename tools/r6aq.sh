# round-6 GPU session: workgroup range lengths after the load-depth change -- config 2 at 100M over ESGPU_HIST_MIN_BPW,
# the north star at 125M over ESGPU_MIN_BPW_ENV (kernel only)
set -u
R=$GRAFT_REPO_ROOT
TAG=${1:-r6aq}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
K="python3 $R/tools/kbench.py"
for b in 16 8 24 32 16; do
  ESGPU_HIST_MIN_BPW=$b timeout -k 10 300 $K --docs 100000000 --reps 9 --only config2_dh_ext > $O/kb_c2_bpw$b.log 2>&1 || exit 1
done
for b in 32 16 48 64 32; do
  ESGPU_MIN_BPW_ENV=$b timeout -k 10 300 $K --docs 125000000 --reps 9 --only north_star,config5 > $O/kb_ns125_bpw$b.log 2>&1 || exit 1
done
echo ALLOK
