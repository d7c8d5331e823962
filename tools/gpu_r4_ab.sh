# GPU: refine parity tests on the current build, then an A/B of in-tree builds.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r04_ab}
mkdir -p $O
shift
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_golden.py -x -v -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 && \
bash tools/gpu_ab_multi.sh 3 "$@" > $O/ab.txt 2>&1
echo "rc=$?"
