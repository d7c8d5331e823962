set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r01
timeout -k 10 400 python -m pytest tests -x -q -m gpu > gpurun_out/r01/pytest_gpu.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r01/kt -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r01/bench_kt.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/r01/pmc_fetch -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/r01/pmc_fetch.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/r01/pmc_write -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/r01/pmc_write.log 2>&1
