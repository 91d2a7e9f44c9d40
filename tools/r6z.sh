# round-6 GPU session: cross-rank reduce of filtered config 3 (path 9 under xr_terms), boundary / hot-cold suites
set -u
R=$GRAFT_REPO_ROOT
TAG=${1:-r6z}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_comm_build_reduce.py tests/test_gpu_boundary_errors.py tests/test_gpu_hotcold.py -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
echo ALLOK
