# Fast-sincos variants (HPE_FAST_TRIG): GPU suite per variant, then the bench A/B.
# Usage (on the box): bash tools/gpu_ft.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/ft; rm -rf $O; mkdir -p $O
for v in libhpe_ft.so libhpe_ft2.so; do
  HPE_LIB_VARIANT=$v timeout -k 10 300 python -u -m pytest tests -q -m gpu --timeout 200 --timeout-method thread > $O/pytest_$v.log 2>&1
  rc=$?; echo "$v tests rc=$rc" >> $O/summary.txt
  [ $rc -le 1 ] || exit 1
done
bash tools/gpu_ab_multi.sh 3 libhpe.so libhpe_ft.so libhpe_ft2.so > $O/ab.txt 2>&1
