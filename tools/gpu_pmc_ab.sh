# HBM traffic of k_pso_gen per launch for two in-tree builds (A/B): separate FETCH_SIZE and
# WRITE_SIZE passes (MI355X_MICROARCH.md: one counter group per --pmc run).
# Usage (on the box): bash tools/gpu_pmc_ab.sh [libA.so] [libB.so]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/pmc_ab
rm -rf $O; mkdir -p $O
for v in ${1:-libhpe_base.so} ${2:-libhpe.so}; do
  tag=$(basename $v .so)
  for c in FETCH_SIZE WRITE_SIZE; do
    HPE_LIB_VARIANT=$v timeout -k 10 120 rocprofv3 --pmc $c --kernel-trace --output-format csv \
      -d $O/${tag}_$c -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline \
      > $O/${tag}_$c.log 2>&1 || exit 1
  done
  python3 tools/prof_summary.py pmc $O/${tag}_FETCH_SIZE $O/${tag}_WRITE_SIZE k_pso_gen 256 250 $O/$tag.json > /dev/null || exit 1
done
