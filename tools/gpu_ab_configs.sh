# A/B in-tree builds on several bench configs: tools/gpu_ab_multi.sh per config, each
# summary into gpurun_out/abc/<config>.txt.
# Usage (on the box): bash tools/gpu_ab_configs.sh rounds "cfg1|cfg2|..." lib1.so lib2.so ...
#   a config is a quoted bench.py argument string ("" = the default sequence)
set -o pipefail
cd $GRAFT_REPO_ROOT
R=$1; CFGS=$2; shift 2
mkdir -p gpurun_out/abc
IFS='|' read -ra CA <<< "$CFGS"
for cfg in "${CA[@]}"; do
  tag=$(echo "default $cfg" | tr -c 'a-zA-Z0-9\n' '_')
  BENCH_ARGS="$cfg" bash tools/gpu_ab_multi.sh $R "$@" > gpurun_out/abc/$tag.txt 2>&1 || exit 1
  echo "== $cfg"; cat gpurun_out/abc/$tag.txt
done
