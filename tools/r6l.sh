# round-6 GPU session: config 2's packed run updates (ESGPU_DOT16) and workgroup sizing at 100M / 1B; the 125M-doc
# north-star shape (isolated vs back-to-back launches, blocks per workgroup); layouts + rounding tests
set -u
R=$GRAFT_REPO_ROOT
TAG=${1:-r6l}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
K="python3 $R/tools/kbench.py"
for d in 100000000 1000000000; do
  timeout -k 10 300 $K --docs $d --reps 7 --only config2_dh_ext,date_hist > $O/kb_c2_${d}_dot.log 2>&1 || exit 1
  ESGPU_DOT16=0 timeout -k 10 300 $K --docs $d --reps 7 --only config2_dh_ext > $O/kb_c2_${d}_nodot.log 2>&1 || exit 1
done
for b in 4 16 32; do
  ESGPU_HIST_MIN_BPW=$b timeout -k 10 300 $K --docs 100000000 --reps 7 --only config2_dh_ext > $O/kb_c2_100m_bpw$b.log 2>&1 || exit 1
done
timeout -k 10 300 python3 $R/tools/back2back.py --docs 125000000 --launches 8 --reps 5 --only north_star,config5,config2_dh_ext > $O/b2b_125m.log 2>&1 || exit 1
for b in 8 12 40; do
  ESGPU_MIN_BPW_ENV=$b timeout -k 10 300 $K --docs 125000000 --reps 7 --only north_star,config5 > $O/kb_ns125_bpw$b.log 2>&1 || exit 1
done
timeout -k 10 300 $K --docs 125000000 --reps 7 --only north_star,config5 > $O/kb_ns125_default.log 2>&1 || exit 1
G1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES"
timeout -s KILL 120 rocprofv3 --pmc $G1 --kernel-trace --output-format csv -d $O/pmc_config2_G1 -o kb -- python3 $R/tools/kbench.py --docs 100000000 --reps 1 --only config2_dh_ext > $O/pmc_config2_G1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc $G1 --kernel-trace --output-format csv -d $O/pmc_ns125_G1 -o kb -- python3 $R/tools/kbench.py --docs 125000000 --reps 1 --only north_star > $O/pmc_ns125_G1.log 2>&1 || exit 1
cd $R
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_layouts.py tests/test_gpu_rounding.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
echo ALLOK
