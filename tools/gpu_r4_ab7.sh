# GPU: the refine gradient heads before the correspondence search (HPE_RF_HEAD_FIRST=1, and the previous default HPE_RF_SPREAD=0) against
# the default, 4 alternated rounds of 40 frames, then the GPU suite on the variant.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r04_ab7}
mkdir -p $O
bash tools/gpu_ab_multi.sh 4 libhpe.so libhpe_hf.so libhpe_ns.so > $O/ab.txt 2>&1 && \
HPE_LIB_VARIANT=libhpe_hf.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_hf.log 2>&1
rc=$?
cp -r gpurun_out/abm $O/ 2>/dev/null
echo "rc=$rc"
