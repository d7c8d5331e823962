set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/optab
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_golden.py -x -q -m gpu -k "optimise or opt" --timeout 120 --timeout-method thread > gpurun_out/optab/pytest.log 2>&1 || { tail -n 30 gpurun_out/optab/pytest.log; exit 1; }
tail -n 3 gpurun_out/optab/pytest.log
for r in 1 2; do for v in libhpe_head.so libhpe.so; do echo $v; HPE_LIB_VARIANT=$v timeout -k 10 120 python tools/opt_time.py || exit 1; done; done
