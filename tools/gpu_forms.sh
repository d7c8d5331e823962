# PSO kernel forms: parity tests, then bench 1 frame-equivalent per (P, form)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/forms
mkdir -p $O
timeout -k 10 400 python -m pytest tests -x -q -m gpu > $O/pytest_gpu.log 2>&1 || exit 1
for P in 256 1024 4096; do
  for F in block wave; do
    G=30; [ $P = 4096 ] && G=40
    HPE_PSO_FORM=$F timeout -k 10 300 python bench.py --no-cpu-baseline --no-refine --particles $P --generations $G --steps 10 --warmup 2 > $O/bench_${P}_${F}.log 2>&1 || exit 1
  done
done
