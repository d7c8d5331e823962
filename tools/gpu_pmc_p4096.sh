# PMC traffic of one generation kernel at a BASELINE config for libhpe_base.so and
# libhpe.so (one counter group per rocprofv3 run).  Usage (on the box):
#   bash tools/gpu_pmc_p4096.sh [config] [kernel] [P] [N]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
CFG=${1:-p4096}; KER=${2:-k_pso_gen_w}; P=${3:-4096}; N=${4:-250}
O=gpurun_out/pmc_$CFG
rm -rf $O; mkdir -p $O
for v in libhpe_base.so libhpe.so; do
  t=$(basename $v .so)
  HPE_LIB_VARIANT=$v timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/f_$t -o run -- python3 bench.py --config $CFG --steps 3 --warmup 1 --no-cpu-baseline > $O/f_$t.log 2>&1 || exit 1
  HPE_LIB_VARIANT=$v timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/w_$t -o run -- python3 bench.py --config $CFG --steps 3 --warmup 1 --no-cpu-baseline > $O/w_$t.log 2>&1 || exit 1
  HPE_LIB_VARIANT=$v python3 tools/prof_summary.py pmc $O/f_$t $O/w_$t $KER $P $N $O/pmc_$t.json > /dev/null || exit 1
done
grep -h bytes_per_launch $O/pmc_*.json
