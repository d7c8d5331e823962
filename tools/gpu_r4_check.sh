# Round-4 check on the box: the bench line in both refine forms, rocprofv3 kernel stats of
# the default bench, then the GPU tests (hand-frame refine, the default).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r04_check}
mkdir -p $O
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_rigid.log 2>&1 && \
HPE_REFINE_EXACT=1 timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_exact.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py --no-cpu-baseline > $O/bench_kt.log 2>&1 && \
python3 tools/prof_summary.py stats $O/kt $O/kernel_stats.csv > $O/kernel_stats.txt && \
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
echo "rc=$?"
