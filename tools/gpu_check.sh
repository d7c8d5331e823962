# quick GPU check: parity tests, bench with graphs, bench without graphs
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/chk
timeout -k 10 400 python -m pytest tests -x -q -m gpu > gpurun_out/chk/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/chk/bench_graph.log 2>&1 && \
HPE_NO_GRAPH=1 timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/chk/bench_nograph.log 2>&1
