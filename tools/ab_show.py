"""Summarise tools/ab.sh logs."""
import ast
import glob
import json
import sys

for f in sorted(glob.glob("gpurun_out/ab/bench*.log")):
    for line in open(f):
        if line.startswith("{"):
            d = json.loads(line)
            k = d["kernels"]
            print(f"{f.split('/')[-1]:32s} {d['ms_per_step']:.4f} ms/frame  refine {k['k_refine']['avg_us']:7.1f} us  "
                  f"gen {k['k_pso_gen']['avg_us']:5.2f} us  graph {k['frame_graph']['avg_us']:7.1f} us")
for f in sorted(glob.glob("gpurun_out/ab/opt_*.log")):
    for line in open(f):
        if line.startswith("{"):
            d = ast.literal_eval(line)
            print(f"{f.split('/')[-1]:32s} wall {d['wall_ms']:7.2f} ms  descent {d['k_opt_descent']['avg_us']:7.1f} us  "
                  f"move {d['k_opt_move']['avg_us']:5.2f} us  cost {d['cost']:.6g}")
