# Small overlapped launches (a380 at its batch of 1 spp): pipeline slots (RT_DEBUG_LAUNCH slots) x
# HIP hardware queues x the share of the resident grid each launch takes (RT_DEBUG_LAUNCH grid_div),
# one warmed-up process per setting (tools/gpu_a380_calib.py)
set -o pipefail
mkdir -p gpurun_out/grid
for cfg in ${CFGS:-"12 8 1" "16 8 1" "24 8 1" "24 12 1" "24 16 1" "32 16 1" "24 8 2" "24 8 4" "24 16 4"}; do
  set -- $cfg
  TAG="q$1_s$2_d$3" GPU_MAX_HW_QUEUES=$1 RT_DEBUG_LAUNCH=slots=$2,grid_div=$3 timeout -k 10 200 python -u tools/gpu_a380_calib.py ${ARGS:-a380 1 200} > gpurun_out/grid/q$1_s$2_d$3.log 2>&1 || exit 1
  grep RES gpurun_out/grid/q$1_s$2_d$3.log
done
