# round-6 GPU session: 8 docs per thread for the histogram-only integer-run kernels (A/B against build/variants d8h0)
set -u
R=$GRAFT_REPO_ROOT
TAG=${1:-r6m}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
K="python3 $R/tools/kbench.py"
S=config2_dh_ext
for d in 100000000 1000000000; do
  timeout -k 10 300 $K --docs $d --reps 7 --only $S > $O/kb_${d}_main.log 2>&1 || exit 1
  ESGPU_LIBRARY=$R/build/variants/libesgpu_d8h0.so timeout -k 10 300 $K --docs $d --reps 7 --only $S > $O/kb_${d}_d8h0.log 2>&1 || exit 1
  timeout -k 10 300 $K --docs $d --reps 7 --only $S > $O/kb_${d}_main2.log 2>&1 || exit 1
  timeout -k 10 300 $K --docs $d --reps 5 --only $S --ts-jitter 3600000 > $O/kb_${d}_jit1h.log 2>&1 || exit 1
done
G1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES"
timeout -s KILL 120 rocprofv3 --pmc $G1 --kernel-trace --output-format csv -d $O/pmc_config2_G1 -o kb -- python3 $R/tools/kbench.py --docs 100000000 --reps 1 --only config2_dh_ext > $O/pmc_config2_G1.log 2>&1 || exit 1
cd $R
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_layouts.py tests/test_gpu_rounding.py tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
echo ALLOK
