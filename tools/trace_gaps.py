import csv, sys, glob
f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
gaps = []
for a, b in zip(rows, rows[1:]):
    if 'k_pso_final' in a['Kernel_Name'] and 'k_refine' in b['Kernel_Name']:
        gaps.append((int(b['Start_Timestamp']) - int(a['End_Timestamp'])) / 1000)
print(sys.argv[1], "final->refine gaps (us):", len(gaps), "median %.1f" % sorted(gaps)[len(gaps)//2] if gaps else "", [round(g, 1) for g in gaps[:30]])
