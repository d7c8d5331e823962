# Resident raw sequences (hpe_track_raw_sequence_dev) on the box: the new parity test,
# then the bench with K = 8 frames per graph (the N = 1 default) and K = 0 (one pipelined
# graph per frame, raw frames from host memory) alternated on the same box, and the
# rocprofv3 kernel trace of the default.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r04_raw}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_prep.py -x -v -m gpu -k "raw_sequence or pipelined or sequence" --timeout 240 --timeout-method thread > $O/pytest_raw.log 2>&1 || { echo "rc=$?"; exit 1; }
for r in 1 2 3; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 40 > $O/bench_k8_$r.log 2>&1 || { echo "rc=$?"; exit 1; }
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 40 --frames-per-graph 0 > $O/bench_k0_$r.log 2>&1 || { echo "rc=$?"; exit 1; }
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py --no-cpu-baseline > $O/bench_kt.log 2>&1 && \
python3 tools/prof_summary.py stats $O/kt $O/kernel_stats.csv > $O/kernel_stats.txt
echo "rc=$?"
