# GPU: N = full parity (split generation kernel), refine A/B of in-tree builds, and the
# N = full bench with and without the split generation.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r04_ab2}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_host.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 && \
bash tools/gpu_ab_multi.sh 3 libhpe_r1.so libhpe_cw.so libhpe_fn.so libhpe_fnit.so > $O/ab.txt 2>&1 && \
timeout -k 10 300 python bench.py --full-cloud --no-cpu-baseline --steps 10 > $O/full_split.log 2>&1 && \
HPE_PSO_SPLIT=1 timeout -k 10 300 python bench.py --full-cloud --no-cpu-baseline --steps 10 > $O/full_nosplit.log 2>&1
echo "rc=$?"
