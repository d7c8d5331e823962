# One round's GPU evidence (usage on the box: bash tools/gpu_round.sh r02): box facts,
# GPU tests, bench (default config + CPU baseline), rocprofv3 kernel-trace stats of the
# same bench command, the two PMC passes (FETCH_SIZE, WRITE_SIZE; one counter group per
# run), and the BASELINE configs.  Every GPU step has its own time limit; the chain stops
# at the first failure.
set -o pipefail
R=${1:-r02}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/$R
mkdir -p $O
{ nproc; python3 -c 'import os; print(len(os.sched_getaffinity(0)))'; cat /sys/fs/cgroup/cpu.max 2>&1; echo "OMP_NUM_THREADS=$OMP_NUM_THREADS"; grep -m1 "model name" /proc/cpuinfo; } > $O/box.txt 2>&1
{ [ -n "$SKIP_TESTS" ] || timeout -k 10 900 python -u -m pytest tests -x -v -s -m gpu --timeout 600 --timeout-method thread > $O/pytest_gpu.log 2>&1; } && \
{ [ -n "$SKIP_TESTS" ] || HPE_REFINE_EXACT=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py -x -v -s -k config3 --timeout 280 --timeout-method thread > $O/pytest_exact_seq.log 2>&1; } && \
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py --no-cpu-baseline > $O/bench_kt.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc_fetch -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/pmc_fetch.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmc_write -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/pmc_write.log 2>&1 && \
python3 tools/prof_summary.py stats $O/kt $O/kernel_stats.csv > $O/kernel_stats.txt && \
python3 tools/prof_summary.py pmc $O/pmc_fetch $O/pmc_write k_pso_gen 256 250 $O/pmc_k_pso_gen.json > /dev/null && \
python3 tools/prof_summary.py pmc $O/pmc_fetch $O/pmc_write k_refine 256 250 $O/pmc_k_refine.json > /dev/null && \
bash tools/gpu_configs.sh $R
