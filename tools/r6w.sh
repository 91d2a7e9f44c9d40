# round-6 GPU session: calendar / DST inner histograms (bucket table), hist-under-hist + rounding + fuzz suites
set -u
R=$GRAFT_REPO_ROOT
TAG=${1:-r6w}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_hist_under_hist.py tests/test_gpu_rounding.py tests/test_gpu_fuzz.py tests/test_gpu_tree_shapes.py tests/test_gpu_boundary_errors.py tests/test_gpu_cardinality_buckets.py -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
echo ALLOK
