set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/e2e; mkdir -p $O
HPE_PREP_SERIAL=1 timeout -k 10 300 python bench.py --no-cpu-baseline > $O/serial.log 2>&1 && \
HPE_PREP_SERIAL=1 HPE_NO_GRAPH=1 timeout -k 10 300 python bench.py --no-cpu-baseline > $O/serial_nograph.log 2>&1
