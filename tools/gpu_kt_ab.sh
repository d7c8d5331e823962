# rocprofv3 kernel-trace stats of the default bench for two in-tree builds (graph replay
# included), summary per kernel.  Usage (on the box): bash tools/gpu_kt_ab.sh libA.so libB.so
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ktab
for v in "$@"; do
  n=$(basename $v .so)
  HPE_LIB_VARIANT=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ktab/$n -o run -- python3 bench.py --steps 40 --no-cpu-baseline > gpurun_out/ktab/$n.log 2>&1 || exit 1
  python3 tools/prof_summary.py stats gpurun_out/ktab/$n gpurun_out/ktab/$n.csv > gpurun_out/ktab/$n.txt || exit 1
  echo "== $n"; head -n 5 gpurun_out/ktab/$n.txt
done
