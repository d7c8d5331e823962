# Launch-boundary microbenchmark (tools/ubench_launch.hip) under runtime settings.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r04_launch}
mkdir -p $O
U=tools/ubench_launch
{
for d in 0 1 2; do
  for B in 1 256; do
    echo "== default"; timeout -k 5 60 $U $B 30 $d || exit 1
    echo "== DEBUG_CLR_GRAPH_PACKET_CAPTURE=0"; DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 5 60 $U $B 30 $d || exit 1
    echo "== DEBUG_CLR_GRAPH_PACKET_CAPTURE=1"; DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 timeout -k 5 60 $U $B 30 $d || exit 1
    echo "== HIP_FORCE_DEV_KERNARG=1"; HIP_FORCE_DEV_KERNARG=1 timeout -k 5 60 $U $B 30 $d || exit 1
    echo "== HIP_FORCE_DEV_KERNARG=0"; HIP_FORCE_DEV_KERNARG=0 timeout -k 5 60 $U $B 30 $d || exit 1
  done
done
} > $O/launch.txt 2>&1
echo rc=$?
