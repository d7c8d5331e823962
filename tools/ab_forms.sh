# A/B of refine forms on one box (usage on the box: bash tools/ab_forms.sh NAME "form1 form2 ..." [rounds] [steps]):
# bench.py (40 timed frames, no CPU baseline) under HPE_REFINE_TEAM=<form>, alternated; each
# line: form, ms/frame, k_refine avg us (events), k_pso_gen avg us.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
R=${1:-ab}; FORMS=${2:-"0 1"}; N=${3:-3}; S=${4:-40}
O=gpurun_out/$R; mkdir -p $O
for r in $(seq 1 $N); do
  for f in $FORMS; do
    HPE_REFINE_TEAM=$f timeout -k 10 200 python bench.py --steps $S --warmup 3 --no-cpu-baseline > $O/b_${f}_$r.json 2> $O/b_${f}_$r.err || exit 1
    python3 -c "
import json,sys; d=json.loads(open('$O/b_${f}_$r.json').read().strip().splitlines()[-1]); k=d['kernels']
print('$f', '%.4f' % d['ms_per_step'], 'refine %.1f' % k['k_refine']['avg_us'], 'gen %.3f' % k['k_pso_gen']['avg_us'], 'evals/frame %.1f' % d['refine_evals_per_frame'], 'cost %.10f' % d['final_cost'])" | tee -a $O/summary.txt
  done
done
