#!/bin/bash
# Copy a round's GPU evidence (tools/gpu_round.sh output under gpurun_out/<round>/) into
# the tracked profiles/ directory: bench lines, rocprofv3 kernel stats, PMC traffic per
# launch (stamped with the libhpe.so sha256 the bench compares), GPU test log, configs.
set -e -o pipefail
cd "$(dirname "$0")/.."
R=${1:-r02}
S=gpurun_out/$R
grep '^{' $S/bench.log | tail -1 | python3 -m json.tool > profiles/${R}_bench.json
grep '^{' $S/bench_kt.log | tail -1 | python3 -m json.tool > profiles/${R}_bench_under_rocprof.json
cp $S/kernel_stats.csv profiles/${R}_kernel_stats.csv
cp $S/pmc_k_pso_gen.json profiles/pmc_k_pso_gen.json
[ -f $S/pmc_k_refine.json ] && cp $S/pmc_k_refine.json profiles/pmc_k_refine.json
[ -f $S/pytest_gpu.log ] && cp $S/pytest_gpu.log profiles/${R}_pytest_gpu.log
cp $S/box.txt profiles/${R}_box.txt
mkdir -p profiles/${R}_configs
for f in $S/configs/*.log; do
  grep '^{' $f | tail -1 | python3 -m json.tool > profiles/${R}_configs/$(basename $f .log).json
done
echo "profiles updated ($R)"
