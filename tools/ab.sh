#!/bin/bash
# A/B two in-tree builds on the GPU box: libhpe.so (B) vs $1 (A, default libhpe_base.so).
# Usage (on the box): bash tools/ab.sh [libA.so] [rounds] [extra bench args]
set -o pipefail
A=${1:-libhpe_base.so}
R=${2:-2}
EXTRA=${3:-}
rm -rf gpurun_out/ab; mkdir -p gpurun_out/ab
for r in $(seq 1 $R); do
  for v in "$A" libhpe.so; do
    tag=$(basename $v .so)_$r
    HPE_LIB_VARIANT=$v timeout -k 10 200 python bench.py --steps 40 --no-cpu-baseline > gpurun_out/ab/bench_$tag.log 2>&1 || exit 1
    if [ -n "$EXTRA" ]; then
      HPE_LIB_VARIANT=$v timeout -k 10 200 python bench.py --steps 20 --no-cpu-baseline $EXTRA > gpurun_out/ab/benchx_$tag.log 2>&1 || exit 1
    fi
    HPE_LIB_VARIANT=$v timeout -k 10 200 python tools/opt_time.py ${OPT_P:-32} 100 1 > gpurun_out/ab/opt_$tag.log 2>&1 || exit 1
  done
done
