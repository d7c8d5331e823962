# BASELINE configs on one GPU, each its own bench.py run: N = full
# cloud, the 400-frame sequence (config 3), 4096 x 40 (config 4), 32 x 10 (config 1's
# shape), one 1024-particle subswarm of config 5, the per-frame pipelined loop (raw frames
# from host memory), prepared frames resident per frame / 8 per graph, and configs 2 and 5's
# loops with the library's subswarm exchange on a one-rank RCCL communicator (the N > 1 loop).
set -o pipefail
O=gpurun_out/${1:-r02}/configs
rm -rf $O; mkdir -p $O
timeout -k 10 300 python bench.py --full-cloud --no-cpu-baseline > $O/full_cloud.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 400 --warmup 1 --no-cpu-baseline > $O/seq400.log 2>&1 && \
timeout -k 10 300 python bench.py --config p4096 --no-cpu-baseline > $O/p4096.log 2>&1 && \
timeout -k 10 300 python bench.py --config p32 --no-cpu-baseline > $O/p32.log 2>&1 && \
timeout -k 10 300 python bench.py --config subswarm8 --no-cpu-baseline > $O/subswarm1.log 2>&1 && \
timeout -k 10 300 python bench.py --frames-per-graph 0 --no-cpu-baseline > $O/pipelined.log 2>&1 && \
timeout -k 10 300 python bench.py --resident --frames-per-graph 0 --no-cpu-baseline > $O/resident.log 2>&1 && \
timeout -k 10 300 python bench.py --resident --frames-per-graph 8 --no-cpu-baseline > $O/resident_seq8.log 2>&1 && \
timeout -k 10 300 python bench.py --subswarm-world1 --no-cpu-baseline > $O/seq_subswarm_world1.log 2>&1 && \
timeout -k 10 300 python bench.py --config subswarm8 --subswarm-world1 --no-cpu-baseline > $O/subswarm1_world1.log 2>&1 && \
timeout -k 10 300 python bench.py --config p32 --full-cloud --no-cpu-baseline > $O/p32_full.log 2>&1 && \
timeout -k 10 300 python bench.py --config p4096 --full-cloud --steps 10 --warmup 2 --no-cpu-baseline > $O/p4096_full.log 2>&1 && \
timeout -k 10 300 python bench.py --config subswarm8 --full-cloud --steps 10 --warmup 2 --no-cpu-baseline > $O/subswarm1_full.log 2>&1 && \
timeout -k 10 300 python bench.py --full-cloud --steps 100 --warmup 1 --no-cpu-baseline > $O/seq100_full.log 2>&1
