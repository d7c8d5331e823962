# On the box: per-launch kernel times of several settings, ABAB, for one bench command.
# A setting is a build (HPE_LIB_VARIANT=libhpe_skel_<v>.so; "prod" = libhpe.so) or an
# environment assignment "VAR=value" run on the product build (e.g. HPE_FK_COOP=0,
# HPE_PSO_WPP=4).
# usage: bash tools/skel/var_ab.sh NAME LABEL "bench args" "s1 s2 ..." [kernel-regex]
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
R=$1; LB=$2; ARGS=$3; VS=$4; KR=${5:-k_pso_gen}; O=gpurun_out/$R; mkdir -p $O
for rep in 1 2; do for v in $VS; do
  case "$v" in
    *=*) L=libhpe.so; EV="$v"; TAG=$(echo "$v" | tr '=' '_') ;;
    prod) L=libhpe.so; EV=""; TAG=prod ;;
    *) L=libhpe_skel_$v.so; EV=""; TAG=$v ;;
  esac
  env $EV HPE_LIB_VARIANT=$L timeout -s KILL 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_${LB}_${TAG}_$rep -o run -- python3 bench.py $ARGS --steps 5 --warmup 1 --no-cpu-baseline > $O/kt_${LB}_${TAG}_$rep.log 2>&1 || exit 1
  python3 tools/prof_summary.py stats $O/kt_${LB}_${TAG}_$rep $O/kt_${LB}_${TAG}_$rep.csv > /dev/null
  echo "$LB $v rep=$rep $(grep -hE "$KR" $O/kt_${LB}_${TAG}_$rep.csv | tr '\n' ' ')" >> $O/ab.txt
done; done
