#!/bin/bash
# Copy the round's GPU evidence (tools/gpu_round1.sh output under gpurun_out/) into the
# tracked profiles/ directory: bench lines, rocprofv3 kernel stats, PMC traffic, test log.
set -e -o pipefail
cd "$(dirname "$0")/.."
R=${1:-r01}
S=gpurun_out/r01
grep '^{' $S/bench.log | tail -1 | python3 -m json.tool > profiles/${R}_bench.json
grep '^{' $S/bench_kt.log | tail -1 | python3 -m json.tool > profiles/${R}_bench_under_rocprof.json
python3 tools/prof_summary.py stats $S/kt profiles/${R}_kernel_stats.csv > /dev/null
python3 tools/prof_summary.py pmc $S/pmc_fetch $S/pmc_write k_pso_gen 256 250 profiles/pmc_k_pso_gen.json > /dev/null
cp $S/pytest_gpu.log profiles/${R}_pytest_gpu.log
mkdir -p profiles/${R}_configs
for f in gpurun_out/configs/*.log; do
  grep '^{' $f | tail -1 | python3 -m json.tool > profiles/${R}_configs/$(basename $f .log).json
done
echo "profiles updated ($R)"
