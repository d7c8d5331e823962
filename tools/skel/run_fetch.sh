# On the box: FETCH_SIZE / WRITE_SIZE per k_pso_gen launch (bench.py default config, refine
# on) for each build, one rocprofv3 --pmc pass per counter per build.
# usage: bash tools/skel/run_fetch.sh NAME "variant ..."   (prod = libhpe.so)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
R=${1:-fetch}; VS=${2:-"prod"}
O=gpurun_out/$R; mkdir -p $O
for v in $VS; do
  L=libhpe_skel_$v.so; [ "$v" = prod ] && L=libhpe.so
  for c in FETCH_SIZE WRITE_SIZE; do
    HPE_LIB_VARIANT=$L timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/${c}_$v -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/${c}_$v.log 2>&1 || exit 1
  done
  python3 tools/prof_summary.py pmc $O/FETCH_SIZE_$v $O/WRITE_SIZE_$v k_pso_gen 256 250 $O/pmc_$v.json > /dev/null || exit 1
  echo "$v $(python3 -c "import json; d=json.load(open('$O/pmc_$v.json')); print(d['fetch_size_kb_raw'], d['write_size_kb'], d['bytes_per_launch'])")" >> $O/fetch.txt
done
