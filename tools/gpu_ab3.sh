# A/B two in-tree builds over three bench configs: default (N = 250), full cloud, 4096 x 40.
# Usage (on the box): bash tools/gpu_ab3.sh [libA.so] [rounds]
set -o pipefail
A=${1:-libhpe_base.so}
R=${2:-2}
rm -rf gpurun_out/ab; mkdir -p gpurun_out/ab
for r in $(seq 1 $R); do
  for v in "$A" libhpe.so; do
    tag=$(basename $v .so)_$r
    HPE_LIB_VARIANT=$v timeout -k 10 200 python bench.py --steps 40 --no-cpu-baseline > gpurun_out/ab/bench_$tag.log 2>&1 || exit 1
    HPE_LIB_VARIANT=$v timeout -k 10 200 python bench.py --steps 10 --full-cloud --no-cpu-baseline > gpurun_out/ab/full_$tag.log 2>&1 || exit 1
    HPE_LIB_VARIANT=$v timeout -k 10 200 python bench.py --steps 10 --particles 4096 --generations 40 --no-cpu-baseline > gpurun_out/ab/p4096_$tag.log 2>&1 || exit 1
  done
done
