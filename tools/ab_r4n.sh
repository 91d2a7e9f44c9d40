set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r4n
mkdir -p $OUT
export TMPDIR=/tmp
for v in main fsnb3 fswg512 fswg512nb3; do
  if [ $v = main ]; then L=""; else L="ESGPU_LIBRARY=$R/build/variants/libesgpu_$v.so"; fi
  env $L timeout -k 10 300 python3 $R/tools/kbench.py --docs 125000000 --reps 5 --only config4_card > $OUT/kb125_c4_$v.log 2>&1 || exit 1
done
for v in main wgw1 wgw2; do
  if [ $v = main ]; then L=""; else L="ESGPU_LIBRARY=$R/build/variants/libesgpu_$v.so"; fi
  env $L timeout -k 10 400 python3 $R/tools/kbench.py --docs 1000000000 --reps 5 --only north_star,ns_avg,config5,config2_dh_ext,terms_dh > $OUT/kb1b_$v.log 2>&1 || exit 1
  env $L timeout -k 10 300 python3 $R/tools/kbench.py --docs 125000000 --reps 5 --only north_star,config5 > $OUT/kb125_$v.log 2>&1 || exit 1
done
timeout -k 10 300 python3 $R/tools/kbench.py --docs 125000000 --reps 5 --only config3_url --deletes 0.2 > $OUT/kbench_c3_del20.log 2>&1
