# A/B one environment variable of the same build over the default bench config.
# Usage (on the box): bash tools/gpu_env_ab.sh VAR VALUE [rounds]
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/envab
rm -rf $O; mkdir -p $O
for r in $(seq 1 ${3:-3}); do
  timeout -k 10 200 python bench.py --steps 60 --no-cpu-baseline > $O/bench_default_$r.log 2>&1 || exit 1
  env $1=$2 timeout -k 10 200 python bench.py --steps 60 --no-cpu-baseline > $O/bench_$1_$r.log 2>&1 || exit 1
done
python3 - <<'PY'
import glob, json
for f in sorted(glob.glob("gpurun_out/envab/*.log")):
    for line in open(f):
        if line.startswith("{"):
            d = json.loads(line); k = d["kernels"]
            print(f"{f.split('/')[-1]:28s} {d['ms_per_step']:.4f} ms/frame  graph {k['frame_graph']['avg_us']:6.1f}  refine {k['k_refine']['avg_us']:6.1f}  gen {k['k_pso_gen']['avg_us']:5.2f}  host {d['host_us_per_step']:6.1f}")
PY
