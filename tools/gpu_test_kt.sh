# GPU tests on the new build, then rocprofv3 kernel-trace A/B against libhpe_head.so
# (two pairs).  Usage (on the box): bash tools/gpu_test_kt.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/tkt
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/tkt/pytest.log 2>&1 || { tail -n 40 gpurun_out/tkt/pytest.log; exit 1; }
tail -n 2 gpurun_out/tkt/pytest.log
bash tools/gpu_kt_ab.sh libhpe_head.so libhpe.so libhpe_head.so libhpe.so
