# On the box: k_pso_gen_w per launch with and without the cooperative FK (HPE_FK_COOP), ABAB
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
R=$1; O=gpurun_out/$R; mkdir -p $O; for CFG in p4096 subswarm8; do
for rep in 1 2; do for c in 1 0; do
  HPE_FK_COOP=$c timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_${CFG}_${c}_$rep -o run -- python3 bench.py --config $CFG --no-refine --steps 5 --warmup 1 --no-cpu-baseline > $O/kt_${CFG}_${c}_$rep.log 2>&1 || exit 1
  python3 tools/prof_summary.py stats $O/kt_${CFG}_${c}_$rep $O/kt_${CFG}_${c}_$rep.csv > /dev/null
  echo "$CFG coop=$c rep=$rep $(grep -h 'k_pso_gen_w' $O/kt_${CFG}_${c}_$rep.csv | tr '\n' ' ')" >> $O/ab.txt
done; done; done
