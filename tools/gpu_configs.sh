# Every BASELINE.json config on one MI355X with the current kernels (bench lines, no CPU leg).
set -o pipefail
mkdir -p gpurun_out/configs_r1s
run() {  # name, bench args
  local n=$1; shift
  timeout -k 10 240 python -u bench.py --steps 2 --warmup 1 --no-cpu "$@" > gpurun_out/configs_r1s/$n.log 2>&1 || { tail -20 gpurun_out/configs_r1s/$n.log; exit 1; }
  echo "$n $(tail -1 gpurun_out/configs_r1s/$n.log | cut -c1-110)"
}
run triangles --scene triangles
run a380 --scene a380
run biplane_200 --scene biplane --spp-per-step 200
run walled --scene walled
run spaceship_4096 --scene spaceship_r1 --width 4096 --height 4096 --spp-per-step 25
