# Instruction mix of the queue kernel for one bench step (own pass): vector-memory reads and
# writes (scratch spills included), scalar and LDS instructions.  Usage: tools/pmc_mix.sh scene [bench args]
set -o pipefail
export TMPDIR=/tmp
S=${1:-biplane}; shift
O=gpurun_out/pmcmix_$S
mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_FLAT SQ_WAVES --output-format csv -d $O/p1 -o run -- python3 bench.py --scene $S --steps 1 --warmup 0 --no-cpu --no-roofline --sync $@ > $O/p1.log 2>&1 || exit 1
python3 tools/pmc_sum.py $O/p1 queue_kernel
