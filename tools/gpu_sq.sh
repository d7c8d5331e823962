# SQ counter pass over the default bench (one rocprofv3 --pmc pass, kernel-trace only):
# issue vs wait breakdown of k_pso_gen / k_refine.  Summary: tools/pmc_avg.py.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/sq
rm -rf $O; mkdir -p $O
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU --kernel-trace --output-format csv -d $O/p1 -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/p1.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA --kernel-trace --output-format csv -d $O/p2 -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/p2.log 2>&1
