# A/B one build under two environments (default bench, R rounds): ENV_B is exported for
# the B runs.  Usage (on the box): ENV_B="X=1" bash tools/gpu_env_ab2.sh R
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/envab2; rm -rf $O; mkdir -p $O
for r in $(seq 1 ${1:-3}); do
  timeout -k 10 200 python bench.py --steps 40 --no-cpu-baseline > $O/a_$r.log 2>&1 || exit 1
  env $ENV_B timeout -k 10 200 python bench.py --steps 40 --no-cpu-baseline > $O/b_$r.log 2>&1 || exit 1
done
for v in a b; do
  cat $O/${v}_*.log | grep '^{' | python3 -c "
import sys, json, statistics as st
d=[json.loads(l) for l in sys.stdin]
print('$v', 'ms/frame', round(st.mean(x['ms_per_step'] for x in d), 4), [round(x['ms_per_step'], 4) for x in d])"
done
