# The MFMA-filtered search (HPE_MFMA_SEARCH=1 build, libhpe_mf.so) on the box: the random /
# adversarial match check against bf_search, the whole GPU suite on that build, then
# alternated bench pairs (default build vs it) at N = 250 and at N = full.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r04_mf}
V=${2:-libhpe_mf.so}
mkdir -p $O
timeout -k 5 120 tools/mfma_check > $O/mfma_check.txt 2>&1 || { echo "check rc=$?"; cat $O/mfma_check.txt; exit 1; }
HPE_LIB_VARIANT=$V timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/pytest_mf.log 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest_mf.log; exit 1; }
for r in 1 2 3; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 40 > $O/bench_base_$r.log 2>&1 || exit 1
  HPE_LIB_VARIANT=$V timeout -k 10 300 python bench.py --no-cpu-baseline --steps 40 > $O/bench_mf_$r.log 2>&1 || exit 1
done
for r in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --full-cloud --steps 10 --warmup 2 > $O/full_base_$r.log 2>&1 || exit 1
  HPE_LIB_VARIANT=$V timeout -k 10 300 python bench.py --no-cpu-baseline --full-cloud --steps 10 --warmup 2 > $O/full_mf_$r.log 2>&1 || exit 1
done
echo rc=0
