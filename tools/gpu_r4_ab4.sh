# GPU: the hand-frame node microbenchmark (1 and 8 waves) and a frame A/B of compile-time
# refine knobs (inline trig, fused node, no static priority) against the default build.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r04_ab4}
mkdir -p $O
timeout -k 10 60 tools/ubench_rigid 1 > $O/ubench_rigid_1.txt 2>&1 && \
timeout -k 10 60 tools/ubench_rigid 8 > $O/ubench_rigid_8.txt 2>&1 && \
bash tools/gpu_ab_multi.sh 3 libhpe.so libhpe_ti.so libhpe_fu.so libhpe_np.so > $O/ab.txt 2>&1
rc=$?
cp -r gpurun_out/abm $O/ 2>/dev/null
echo "rc=$rc"
