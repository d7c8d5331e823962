# A/B several in-tree builds (HPE_LIB_VARIANT files) on the default bench config.
# Usage (on the box): [BENCH_ARGS="--config p4096"] bash tools/gpu_ab_multi.sh rounds lib1.so lib2.so ...
set -o pipefail
cd $GRAFT_REPO_ROOT
R=$1; shift
O=gpurun_out/abm
rm -rf $O; mkdir -p $O
for r in $(seq 1 $R); do
  for v in "$@"; do
    HPE_LIB_VARIANT=$v timeout -k 10 200 python bench.py --steps 40 --no-cpu-baseline $BENCH_ARGS > $O/bench_$(basename $v .so)_$r.log 2>&1 || exit 1
  done
done
python3 - <<'PY'
import glob, json, collections
agg = collections.defaultdict(list)
for f in sorted(glob.glob("gpurun_out/abm/*.log")):
    for line in open(f):
        if line.startswith("{"):
            d = json.loads(line); k = d["kernels"]
            name = f.split('/')[-1].rsplit('_', 1)[0]
            agg[name].append((d['ms_per_step'], k['k_refine']['avg_us'], k['k_pso_gen']['avg_us']))
for n, v in agg.items():
    import statistics as st
    print(f"{n:24s} ms/frame {st.mean(x[0] for x in v):.4f} (min {min(x[0] for x in v):.4f})  refine {st.mean(x[1] for x in v):6.1f}  gen {st.mean(x[2] for x in v):5.3f}")
PY
