# pipelined loop: GPU tests, bench (zero copy vs SDMA upload), loop without events, trace gaps
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/zc; rm -rf $O; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 && \
for r in 1 2; do
  HPE_PIPE_UPLOAD=1 timeout -k 10 200 python bench.py --no-cpu-baseline > $O/upload_$r.log 2>&1 || exit 1
  timeout -k 10 200 python bench.py --no-cpu-baseline > $O/zc_$r.log 2>&1 || exit 1
done && \
timeout -k 10 120 python3 tools/loop_time.py 40 > $O/loop.log 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o run -- python3 tools/loop_time.py 40 > $O/kt.log 2>&1
