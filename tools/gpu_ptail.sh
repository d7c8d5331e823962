set -o pipefail
cd $GRAFT_REPO_ROOT
for p in 1024 2048 3072 3584 4096 5120 6144; do
  timeout -k 10 120 python bench.py --config p4096 --particles $p --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/pt_$p.log 2>&1 || exit 1
  grep '^{' gpurun_out/pt_$p.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']; g=[v for n,v in k.items() if n.startswith('k_pso_gen')][0]; print($p, round(g['avg_us'],2))"
done
