# kernel + memory-copy timeline of the end-to-end bench (no PMC)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/kt2
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d gpurun_out/kt2 -o run -- python3 bench.py --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/kt2/bench.log 2>&1
