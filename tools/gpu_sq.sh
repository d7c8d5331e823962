# SQ counter passes (one rocprofv3 --pmc run per group) over a short bench of the given
# config; per-dispatch averages per kernel into gpurun_out/sq/summary.txt.
# Usage (on the box): bash tools/gpu_sq.sh [bench args]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/sq; rm -rf $O; mkdir -p $O
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_BUSY_CYCLES"
P2="SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INST_LEVEL_LDS SQ_LDS_ADDR_CONFLICT SQ_THREAD_CYCLES_VALU"
i=0
for grp in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $O/p$i -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline "$@" > $O/p$i.log 2>&1 || exit 1
done
python3 tools/pmc_avg.py $O/p1 $O/p2 > $O/summary.txt && cat $O/summary.txt
