# GPU: PMC of k_pso_gen for in-tree builds (FETCH_SIZE, WRITE_SIZE, TCC hit / miss; one
# counter group per pass) and rocprofv3 kernel-time pairs.  usage: O lib1.so lib2.so ...
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; shift
mkdir -p $O
B="python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline ${BENCH_EXTRA}"
for v in "$@"; do
  n=$(basename $v .so)
  for grp in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum"; do
    tag=$(echo $grp | tr ' ' '_')
    HPE_LIB_VARIANT=$v timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $O/${n}_$tag -o run -- $B > $O/${n}_$tag.log 2>&1 || exit 1
    python3 tools/prof_summary.py counters $O/${n}_$tag k_pso_gen $grp >> $O/${n}_counters.jsonl || exit 1
  done
done
for r in 1 2; do
  for v in "$@"; do
    n=$(basename $v .so)
    HPE_LIB_VARIANT=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${n}_kt$r -o run -- python3 bench.py --steps 40 --no-cpu-baseline ${BENCH_EXTRA} > $O/${n}_kt$r.log 2>&1 || exit 1
    python3 tools/prof_summary.py stats $O/${n}_kt$r $O/${n}_kt$r.csv > $O/${n}_kt$r.txt || exit 1
  done
done
echo ok
