# BASELINE configs on one GPU: default e2e bench (with CPU baseline),
# N = full cloud, the 400-frame sequence (config 3), 4096 x 40 (config 4).
set -o pipefail
O=gpurun_out/configs
rm -rf $O; mkdir -p $O
timeout -k 10 300 python bench.py > $O/default.log 2>&1 && \
timeout -k 10 300 python bench.py --full-cloud --no-cpu-baseline > $O/full_cloud.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 400 --warmup 1 --no-cpu-baseline > $O/seq400.log 2>&1 && \
timeout -k 10 300 python bench.py --particles 4096 --generations 40 --no-cpu-baseline > $O/p4096.log 2>&1 && \
timeout -k 10 300 python bench.py --particles 32 --generations 10 --no-cpu-baseline > $O/p32.log 2>&1
