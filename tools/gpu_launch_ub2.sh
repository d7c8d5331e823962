# Launch-boundary microbenchmark: kernel-argument pointers (mode 0) against link-time
# constant addresses (mode 3, no kernarg load), 1 and 256 workgroups, three repeats.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r04_launch2}
mkdir -p $O
U=tools/ubench_launch
{
for r in 1 2 3; do
  for d in 0 3; do
    for B in 1 256; do
      timeout -k 5 60 $U $B 30 $d || exit 1
    done
  done
done
} > $O/launch.txt 2>&1
echo rc=$?
