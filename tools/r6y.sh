# round-6 GPU session: config 2 load buffers / waves per SIMD (build/variants nb4, nb4w8, w8) at 100M and 1B; the
# packed-cell kernel's occupancy (pw8)
set -u
R=$GRAFT_REPO_ROOT
TAG=${1:-r6y}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
K="python3 $R/tools/kbench.py"
run() {  # tag lib
  for d in 100000000 1000000000; do
    ESGPU_LIBRARY=$2 timeout -k 10 300 $K --docs $d --reps 7 --only config2_dh_ext > $O/kb_${1}_$d.log 2>&1 || return 1
  done
}
run main $R/elasticsearch_amd/libesgpu.so || exit 1
for v in nb4 nb4w8 w8; do run $v $R/build/variants/libesgpu_$v.so || exit 1; done
run main2 $R/elasticsearch_amd/libesgpu.so || exit 1
# the north star's packed-cell kernel at 8 waves per SIMD with a 40 KB window (4 workgroups per CU): build/variants pw8
for v in main pw8 main3 pw8_2; do
  lib=$R/elasticsearch_amd/libesgpu.so
  case $v in pw8*) lib=$R/build/variants/libesgpu_pw8.so ;; esac
  ESGPU_LIBRARY=$lib timeout -k 10 300 $K --docs 1000000000 --reps 5 --only north_star,ns_avg,config5 > $O/kb_ns_$v.log 2>&1 || exit 1
done
echo ALLOK
