# Latency / cache counters of one bench step per scene, each counter group in its own pass.
# Usage: tools/pmc_latency.sh scene [bench args]
set -o pipefail
export TMPDIR=/tmp
S=${1:-biplane}; shift
A="--scene $S --steps 1 --warmup 0 --no-cpu --no-roofline $@"
O=gpurun_out/pmclat_$S
mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM SQ_INSTS_LDS SQ_INST_LEVEL_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_BRANCH --output-format csv -d $O/p1 -o run -- python3 bench.py $A > $O/p1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TOTAL_CACHE_ACCESSES_sum SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC --output-format csv -d $O/p2 -o run -- python3 bench.py $A > $O/p2.log 2>&1 || exit 2
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F32 --output-format csv -d $O/p3 -o run -- python3 bench.py $A > $O/p3.log 2>&1 || exit 3
python3 tools/pmc_sum.py $O/p1 queue_kernel; python3 tools/pmc_sum.py $O/p2 queue_kernel; python3 tools/pmc_sum.py $O/p3 queue_kernel
