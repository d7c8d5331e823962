"""Average rocprofv3 --pmc counters per dispatch, per kernel (csv output directories).
usage: pmc_avg.py DIR [DIR ...]"""
import csv
import glob
import os
import sys
from collections import defaultdict

acc = defaultdict(lambda: defaultdict(list))
for d in sys.argv[1:]:
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            name = row.get("Kernel_Name", "")
            short = name.split("(")[0].replace("void ", "")
            acc[short][row["Counter_Name"]].append(float(row["Counter_Value"]))
for k in sorted(acc):
    if not any(s in k for s in ("k_pso_gen", "k_refine", "k_pso_init", "k_opt")):
        continue
    print(k)
    for c, v in sorted(acc[k].items()):
        print(f"   {c:24s} {sum(v) / len(v):14.1f}   ({len(v)} samples)")
