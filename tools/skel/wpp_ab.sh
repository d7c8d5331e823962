# On the box: k_pso_gen_w time per launch, one vs two waves per particle (HPE_PSO_WPP), for
# bench configs given as arguments (refine off); kernel-trace stats under gpurun_out/$1.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
R=$1; shift; O=gpurun_out/$R; mkdir -p $O
for cfg in "$@"; do for w in 1 2; do
  HPE_PSO_WPP=$w timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_${cfg}_$w -o run -- python3 bench.py --config $cfg --no-refine --steps 5 --warmup 1 --no-cpu-baseline > $O/kt_${cfg}_$w.log 2>&1 || exit 1
  python3 tools/prof_summary.py stats $O/kt_${cfg}_$w $O/kt_${cfg}_$w.csv > /dev/null
  echo "$cfg wpp=$w $(grep -h 'k_pso_gen_w\|k_pso_init_w' $O/kt_${cfg}_$w.csv | tr '\n' ' ')" >> $O/ab.txt
done; done
