# Offline sequence API (hpe_track_sequence_dev) against one graph per frame, resident
# frames, same box: ms per frame for frames_per_graph 0 (per-frame graphs) / 4 / 8 / 16,
# twice each, then the 400-frame sequence both ways.  Usage (on the box): bash tools/gpu_seq_ab.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/seq; rm -rf $O; mkdir -p $O
for r in 1 2; do
  for k in 0 4 8 16; do
    timeout -k 10 200 python bench.py --resident --frames-per-graph $k --steps 40 --no-cpu-baseline > $O/k${k}_$r.log 2>&1 || exit 1
  done
done
timeout -k 10 300 python bench.py --resident --steps 400 --warmup 1 --no-cpu-baseline > $O/seq400_k0.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --resident --frames-per-graph 8 --steps 400 --warmup 1 --no-cpu-baseline > $O/seq400_k8.log 2>&1 || exit 1
for f in $O/*.log; do
  grep '^{' $f | tail -1 | python3 -c "
import sys, json; b=json.loads(sys.stdin.read())
print('%-16s ms/frame %.4f  fps %.0f  cold %s  final_cost %.6f' % ('$(basename $f .log)', b['ms_per_step'], b['tracked_fps'], b.get('cold_graphs_ms_per_step'), b['final_cost']))"
done
