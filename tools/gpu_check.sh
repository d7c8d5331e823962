# GPU check of the current tree (usage on the box: bash tools/gpu_check.sh NAME [pytest -k expr]):
# the GPU tests, then the default bench line.  Each step has its own time limit; the chain
# stops at the first failure.
set -o pipefail
R=${1:-check}
K=${2:-}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/$R
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu ${K:+-k "$K"} --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1
