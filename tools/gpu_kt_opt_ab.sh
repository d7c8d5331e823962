# rocprofv3 kernel-trace A/B of two builds (default bench) plus pso_optimise timing.
# Usage (on the box): bash tools/gpu_kt_opt_ab.sh libA.so libB.so
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_kt_ab.sh "$1" "$2" "$1" "$2" || exit 1
for v in "$1" "$2" "$1" "$2"; do echo $v; HPE_LIB_VARIANT=$v timeout -k 10 120 python tools/opt_time.py | python3 -c "import sys,ast; d=ast.literal_eval(sys.stdin.read().strip().splitlines()[-1]); print(round(d['wall_ms'],2), round(d['k_opt_descent']['avg_us'],1), d['cost'])" || exit 1; done
