# One iteration on the box: the GPU parity suite, then an A/B of libhpe_base.so (the
# previous build) against libhpe.so over three bench configs (tools/gpu_ab3.sh).
# Usage (on the box): bash tools/gpu_iter.sh [rounds]
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/iter
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/iter/pytest_gpu.log 2>&1 && \
bash tools/gpu_ab3.sh libhpe_base.so ${1:-1} && \
python3 tools/ab_show.py > gpurun_out/iter/ab.txt
