# GPU: the exchange / multi-rank tests, then the refine timeline (timelines build).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r04_rts}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_bench_ranks.py tests/test_gpu_mw_fail.py -x -v -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 && \
timeout -k 10 300 python tools/ref_ts.py 20 > $O/ref_ts.txt 2>&1
echo "rc=$?"
