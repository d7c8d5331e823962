# parity tests on the new build, then A/B against libhpe_base.so (default + resident bench,
# pso_optimise, standalone preprocessing)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/ab_pytest.log 2>&1 && \
bash tools/ab.sh libhpe_base.so ${AB_ROUNDS:-2} "--resident" && python tools/ab_show.py > gpurun_out/ab/summary.txt && \
for v in libhpe_base.so libhpe.so; do HPE_LIB_VARIANT=$v timeout -k 10 120 python tools/prep_time.py 16 >> gpurun_out/ab/summary.txt 2>&1 || exit 1; done
