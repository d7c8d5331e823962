# session check: GPU tests, default bench, resident bench (refine without fused prep), stamps
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/s2
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline --resident > $O/bench_resident.log 2>&1 && \
timeout -k 10 200 python tools/stamps.py 4 > $O/stamps.log 2>&1
