# Round-1 GPU evidence: GPU tests, bench (default config, CPU baseline), rocprofv3
# kernel-trace stats of the same bench command, the two PMC passes (FETCH_SIZE,
# WRITE_SIZE) and the BASELINE configs (tools/gpu_configs.sh).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r01
rm -rf $O; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py --no-cpu-baseline > $O/bench_kt.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc_fetch -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/pmc_fetch.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmc_write -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/pmc_write.log 2>&1 && \
bash tools/gpu_configs.sh
