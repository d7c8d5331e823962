# On the box: k_pso_gen_w time per launch for each waves-per-particle setting (HPE_PSO_WPP),
# ABAB over the settings, for one bench config (refine off); kernel-trace stats under
# gpurun_out/$1.  usage: bash tools/skel/wpp_ab.sh NAME CONFIG "1 2 4"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
R=$1; CFG=$2; WS=${3:-"1 2"}; O=gpurun_out/$R; mkdir -p $O
for rep in 1 2; do for w in $WS; do
  HPE_PSO_WPP=$w timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_${CFG}_${w}_$rep -o run -- python3 bench.py --config $CFG --no-refine --steps 5 --warmup 1 --no-cpu-baseline > $O/kt_${CFG}_${w}_$rep.log 2>&1 || exit 1
  python3 tools/prof_summary.py stats $O/kt_${CFG}_${w}_$rep $O/kt_${CFG}_${w}_$rep.csv > /dev/null
  echo "$CFG wpp=$w rep=$rep $(grep -h 'k_pso_gen_w' $O/kt_${CFG}_${w}_$rep.csv | tr '\n' ' ')" >> $O/ab.txt
done; done
