# GPU: default-config A/B (rigid v1 vs head vs head with the inbox rows line-aligned), the
# N = full A/B (r1, head) and head in the exact refine form at N = full.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r04_ab6}
mkdir -p $O
bash tools/gpu_ab_multi.sh 3 libhpe_r1.so libhpe_head.so libhpe_ib.so > $O/ab.txt 2>&1 && \
BENCH_ARGS="--full-cloud --steps 10" bash tools/gpu_ab_multi.sh 1 libhpe_r1.so libhpe_head.so > $O/ab_full.txt 2>&1 && \
HPE_REFINE_EXACT=1 timeout -k 10 300 python bench.py --full-cloud --no-cpu-baseline --steps 10 > $O/full_exact.log 2>&1 && \
HPE_REFINE_MW=0 timeout -k 10 300 python bench.py --full-cloud --no-cpu-baseline --steps 10 > $O/full_nomw.log 2>&1
echo "rc=$?"
