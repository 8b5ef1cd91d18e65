# Texture-address / L1 pressure counters of one bench step (own pass): is the kernel bound by
# the vector-memory path (TA/TD/TCP busy and stalls) rather than by latency?
set -o pipefail
export TMPDIR=/tmp
S=${1:-biplane}; shift
O=gpurun_out/pmcta_$S
mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum GRBM_GUI_ACTIVE --output-format csv -d $O/p1 -o run -- python3 bench.py --scene $S --steps 1 --warmup 0 --no-cpu --no-roofline $@ > $O/p1.log 2>&1 || exit 1
python3 tools/pmc_sum.py $O/p1 queue_kernel
