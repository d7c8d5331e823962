# A/B of the grid-resident PSO form (k_pso_loop) against one launch per generation, same
# build: GPU parity suite first (default = persistent), then bench.py pairs.
# Usage (on the box): bash tools/gpu_persist_ab.sh [rounds]
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/pab
rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
for r in $(seq 1 ${1:-2}); do
  for p in 0 1; do
    HPE_PSO_PERSIST=$p timeout -k 10 200 python bench.py --steps 40 --no-cpu-baseline > $O/bench_p${p}_$r.log 2>&1 || exit 1
    HPE_PSO_PERSIST=$p timeout -k 10 200 python bench.py --steps 10 --full-cloud --no-cpu-baseline > $O/full_p${p}_$r.log 2>&1 || exit 1
  done
done
python3 - <<'PY'
import glob, json
for f in sorted(glob.glob("gpurun_out/pab/*.log")):
    if "pytest" in f: continue
    for line in open(f):
        if line.startswith("{"):
            d = json.loads(line); k = d["kernels"]
            print(f"{f.split('/')[-1]:22s} {d['ms_per_step']:.4f} ms/frame  {d['value']/1e6:6.2f} M evals/s  refine {k['k_refine']['avg_us']:6.1f}  gen {k['k_pso_gen']['avg_us']:5.2f} x{k['k_pso_gen']['launches']}  loop {k.get('k_pso_loop',{}).get('avg_us',0):7.1f}  init {k['k_pso_init']['avg_us']:5.2f} final {k['k_pso_final']['avg_us']:5.2f}")
PY
