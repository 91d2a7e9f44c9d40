# round-6 GPU session: PMC FETCH_SIZE / WRITE_SIZE passes (one counter per pass) of the final north-star and config 2
# collects, for tools/pmc_traffic.py -> profiles/hbm_traffic.json
set -u
R=$GRAFT_REPO_ROOT
TAG=${1:-r6at}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for spec in north_star:1000000000 config2_dh_ext:100000000 config2_dh_ext:1000000000; do
  v=${spec%%:*}; d=${spec##*:}
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 150 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/pmc_${v}_${d}_$c -o kb -- python3 $R/tools/kbench.py --docs $d --reps 3 --only $v > $O/pmc_${v}_${d}_$c.log 2>&1 || exit 1
  done
done
echo ALLOK
