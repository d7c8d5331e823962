# GPU tests on the new build, then A/B against libhpe_head.so: default bench (R rounds),
# pso_optimise timing.  Usage (on the box): bash tools/gpu_ab_full.sh [rounds]
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/abf
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/abf/pytest.log 2>&1 || { tail -n 40 gpurun_out/abf/pytest.log; exit 1; }
tail -n 2 gpurun_out/abf/pytest.log
bash tools/gpu_ab_multi.sh ${1:-3} libhpe_head.so libhpe.so || exit 1
for v in libhpe_head.so libhpe.so; do echo $v; HPE_LIB_VARIANT=$v timeout -k 10 120 python tools/opt_time.py | python3 -c "import sys,ast; d=ast.literal_eval(sys.stdin.read().strip().splitlines()[-1]); print(round(d['wall_ms'],2), round(d['k_opt_descent']['avg_us'],1), d['cost'])" || exit 1; done
