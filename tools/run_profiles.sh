#!/bin/bash
# Collects the rocprofv3 evidence for one workload on the GPU box (run through gpurun):
#   1) kernel trace + --stats of bench.py (the committed summary),
#   2) FETCH_SIZE (HBM read bytes; x2 on gfx950 per MI355X_MICROARCH.md §HBM) in its own pass,
#   3) SQ occupancy / stall / VALU counters and lane utilisation in their own passes,
#   4) L2 (TCC) hits and misses in its own pass,
#   5) the vector-memory units' busy cycles (TA address, TD data return) in its own pass,
# plus the device-code build id the counters belong to (rt_amd.abi.kernel_build_id).
# Counter passes run the bench synchronously (--sync): one trace dispatch at a time.
# Usage: tools/run_profiles.sh <tag> [bench args...]; then python tools/prof_summary.py <tag>
set -o pipefail
TAG=${1:-r2}; shift
ARGS=${@:---steps 2 --warmup 1 --no-configs}
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
python3 -c "import sys; sys.path.insert(0, 'gpu-ray_trace-rust_amd'); from rt_amd import abi; print(abi.kernel_build_id())" > $OUT/build_id || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
    python3 bench.py $ARGS --no-cpu > $OUT/bench_trace.log 2>&1 || exit 2
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- \
    python3 bench.py $ARGS --sync --no-cpu --no-roofline > $OUT/bench_fetch.log 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD --output-format csv -d $OUT/sq -o run -- \
    python3 bench.py $ARGS --sync --no-cpu --no-roofline > $OUT/bench_sq.log 2>&1 || exit 4
timeout -k 10 300 rocprofv3 --pmc SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_SALU --output-format csv -d $OUT/sq2 -o run -- \
    python3 bench.py $ARGS --sync --no-cpu --no-roofline > $OUT/bench_sq2.log 2>&1 || exit 5
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $OUT/tcc -o run -- \
    python3 bench.py $ARGS --sync --no-cpu --no-roofline > $OUT/bench_tcc.log 2>&1 || exit 6
timeout -k 10 300 rocprofv3 --pmc TA_TA_BUSY_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE --output-format csv -d $OUT/tatd -o run -- \
    python3 bench.py $ARGS --sync --no-cpu --no-roofline > $OUT/bench_tatd.log 2>&1 || exit 7
echo profiles_ok $TAG
