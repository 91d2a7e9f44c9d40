# round-6 GPU session: a small grid's counts zeroed in the reset's fill launch (ESGPU_EAGER_ZERO A/B on the north-star
# bench, alternating), then the full GPU suite
set -u
R=$GRAFT_REPO_ROOT
TAG=${1:-r6ap}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for i in 1 2; do
  timeout -k 10 300 python3 $R/bench.py --cpu-docs 0 --steps 20 > $O/bench_eager_$i.log 2>&1 || exit 1
  ESGPU_EAGER_ZERO=0 timeout -k 10 300 python3 $R/bench.py --cpu-docs 0 --steps 20 > $O/bench_lazy_$i.log 2>&1 || exit 1
done
timeout -k 10 300 python3 $R/bench.py --shards 8 --docs 125000000 --cpu-docs 0 > $O/bench_ns8_eager.log 2>&1 || exit 1
ESGPU_EAGER_ZERO=0 timeout -k 10 300 python3 $R/bench.py --shards 8 --docs 125000000 --cpu-docs 0 > $O/bench_ns8_lazy.log 2>&1 || exit 1
bash $R/tools/gpu_check.sh $TAG tests || exit 1
echo ALLOK
