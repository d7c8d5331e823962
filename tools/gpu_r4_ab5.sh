# GPU: Goldstein speculation policy A/B on the hand-frame refine (GOLD_MIX default against
# GOLD_8 everywhere and GOLD_MIX2), 4 alternated rounds of 40 frames.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r04_ab5}
mkdir -p $O
bash tools/gpu_ab_multi.sh 4 libhpe.so libhpe_g8.so libhpe_m2.so > $O/ab.txt 2>&1
rc=$?
cp -r gpurun_out/abm $O/ 2>/dev/null
echo "rc=$rc"
