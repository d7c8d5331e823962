# On the box: k_pso_gen_w per launch for skeleton builds (HPE_LIB_VARIANT=libhpe_skel_<v>.so),
# ABAB, one bench config (refine off).  usage: bash tools/skel/var_ab.sh NAME CONFIG "v1 v2"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
R=$1; CFG=$2; VS=$3; O=gpurun_out/$R; mkdir -p $O
for rep in 1 2; do for v in $VS; do
  L=libhpe_skel_$v.so; [ "$v" = prod ] && L=libhpe.so
  HPE_LIB_VARIANT=$L timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_${CFG}_${v}_$rep -o run -- python3 bench.py --config $CFG --no-refine --steps 5 --warmup 1 --no-cpu-baseline > $O/kt_${CFG}_${v}_$rep.log 2>&1 || exit 1
  python3 tools/prof_summary.py stats $O/kt_${CFG}_${v}_$rep $O/kt_${CFG}_${v}_$rep.csv > /dev/null
  echo "$CFG $v rep=$rep $(grep -h 'k_pso_gen_w' $O/kt_${CFG}_${v}_$rep.csv | tr '\n' ' ')" >> $O/ab.txt
done; done
