# The default bench line N times on one box (run-to-run spread of the headline).
# Usage (on the box): bash tools/gpu_bench_repeat.sh [N]
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/rep; rm -rf $O; mkdir -p $O
for r in $(seq 1 ${1:-5}); do
  timeout -k 10 200 python bench.py --no-cpu-baseline > $O/b_$r.log 2>&1 || exit 1
done
cat $O/b_*.log | grep '^{' | python3 -c "
import sys, json, statistics as st
d=[json.loads(l) for l in sys.stdin]
v=[x['ms_per_step'] for x in d]
print('default bench x%d: ms/frame mean %.4f min %.4f max %.4f stdev %.4f' % (len(v), st.mean(v), min(v), max(v), st.pstdev(v)))
print([round(x, 4) for x in v])"
