# GPU: the refine's correspondence search spread one item per wave (HPE_RF_SPREAD=1) against
# the default, 4 alternated rounds of 40 frames, then the GPU suite on the variant.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r04_ab6}
mkdir -p $O
bash tools/gpu_ab_multi.sh 4 libhpe.so libhpe_sp.so > $O/ab.txt 2>&1 && \
HPE_LIB_VARIANT=libhpe_sp.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_sp.log 2>&1
rc=$?
cp -r gpurun_out/abm $O/ 2>/dev/null
echo "rc=$rc"
