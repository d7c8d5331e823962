# quick GPU iteration: PSO/track parity subset, stamps, bench (no CPU baseline)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/q
mkdir -p $O
timeout -k 10 400 python -m pytest tests -x -q -m gpu > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 200 python tools/stamps.py 4 > $O/stamps.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.log 2>&1
timeout -k 10 60 ./tools/ubench > $O/ubench.log 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline --resident > $O/bench_resident.log 2>&1
timeout -k 10 300 python tools/stamps.py 4 > $O/stamps_prep.log 2>&1
