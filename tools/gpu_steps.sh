# frame time vs the timed frame count on one box (default config)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/steps
rm -rf $O; mkdir -p $O
for s in 20 40 20 40; do
  timeout -k 10 200 python bench.py --steps $s --no-cpu-baseline > $O/s$s.log 2>&1 || exit 1
  grep '^{' $O/s$s.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); k=d['kernels']
ks=k['k_refine']['avg_us']+30*k['k_pso_gen']['avg_us']+k['k_pso_init']['avg_us']+k['k_pso_final']['avg_us']
print($s, round(d['ms_per_step']*1e3,1), 'kernels', round(ks,1), 'graph', round(k['frame_graph']['avg_us'],1), 'host', round(d['host_us_per_step'],1), k['frame_graph']['per_frame_us'])
print('  refine per launch?', k['k_refine'])"
done
