# Mid-size overlapped launches (biplane at 10 spp, spaceship_r1 at 25 spp, triangles at 10 spp):
# treated as "small" launches (RT_DEBUG_LAUNCH small_items) with more slots and a share of the grid
set -o pipefail
mkdir -p gpurun_out/mid
for sc in ${SCENES:-"biplane 10 20" "spaceship_r1 25 8" "triangles 10 60"}; do
  set -- $sc
  for cfg in ${CFGS:-"2 1" "4 1" "4 2" "6 2" "6 3" "8 4" "12 8"}; do
    set -- $sc $cfg
    TAG="$1_s$4_d$5" RT_DEBUG_LAUNCH=small_items=100000000,slots=$4,grid_div=$5 timeout -k 10 250 python -u tools/gpu_a380_calib.py $1 $2 $3 > gpurun_out/mid/$1_s$4_d$5.log 2>&1 || exit 1
    grep RES gpurun_out/mid/$1_s$4_d$5.log
  done
done
