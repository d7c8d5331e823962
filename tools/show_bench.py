import json, sys
for f in sys.argv[1:]:
    for line in open(f):
        if line.startswith("{"):
            d = json.loads(line)
            k = {n: (v["launches"], round(v["avg_us"], 2)) for n, v in d["kernels"].items()}
            print(f"{d['value']:.4g} evals/s  {d['ms_per_step']:.4f} ms/step  {d['tracked_fps']:.1f} fps  "
                  f"cost {d['final_cost']:.12g}  frac {d['roofline']['frac']:.4f}  {k}")
