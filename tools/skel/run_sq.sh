# On the box: SQ instruction counts per k_pso_gen_w dispatch for each skeleton build
# (bench.py --config CONFIG, refine off), one rocprofv3 --pmc pass per build.
# usage: bash tools/skel/run_sq.sh NAME CONFIG "variant ..."
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
R=${1:-skel}; CFG=${2:-p4096}; VS=${3:-"base nofk nosearch noalign nophilox"}
O=gpurun_out/$R; mkdir -p $O
for v in $VS; do
  L=libhpe_skel_$v.so; [ "$v" = prod ] && L=libhpe.so
  HPE_LIB_VARIANT=$L timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES --kernel-trace --output-format csv -d $O/pmc_$v -o run -- python3 bench.py --config $CFG --no-refine --steps 2 --warmup 1 --no-cpu-baseline > $O/pmc_$v.log 2>&1 || exit 1
  HPE_LIB_VARIANT=$L timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$v -o run -- python3 bench.py --config $CFG --no-refine --steps 5 --warmup 1 --no-cpu-baseline > $O/kt_$v.log 2>&1 || exit 1
  echo "== $v" >> $O/sq.txt
  python3 tools/prof_summary.py counters $O/pmc_$v k_pso_gen_w SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES >> $O/sq.txt
  python3 tools/prof_summary.py stats $O/kt_$v $O/kt_$v.csv > $O/kt_$v.txt; grep k_pso_gen_w $O/kt_$v.csv >> $O/sq.txt || true
done
