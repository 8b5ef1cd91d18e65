# Every BASELINE.json config on one MI355X at the schemes' own batch sizes (gpu_render_batch),
# async (default) and synchronous dispatch: bench lines, no CPU leg.  Usage: tools/gpu_configs.sh [extra bench args]
set -o pipefail
mkdir -p gpurun_out/configs
run() {  # name, bench args
  local n=$1; shift
  timeout -k 10 240 python -u bench.py --no-cpu --no-roofline "$@" > gpurun_out/configs/$n.log 2>&1 || { tail -20 gpurun_out/configs/$n.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/configs/$n.log').read().strip().splitlines()[-1]); print('%-22s %10.1f Msamples/s  %8.2f ms/step  launches/step %.1f' % ('$n', d['value'], d['ms_per_step'], d['launch']['trace_launches_per_step']))"
}
for mode in "" "--sync"; do
  tag=${mode:+_sync}
  run triangles$tag --scene triangles --steps 10 --warmup 2 $mode "$@"
  run a380_b1$tag --scene a380 --steps 60 --warmup 3 $mode "$@"
  run a380_b10$tag --scene a380 --spp-per-step 10 --steps 15 --warmup 2 $mode "$@"
  run biplane_b10$tag --scene biplane --steps 20 --warmup 3 $mode "$@"
  run spaceship_b25$tag --scene spaceship_r1 --steps 8 --warmup 2 $mode "$@"
  run spaceship4096_b25$tag --scene spaceship_r1 --width 4096 --height 4096 --steps 3 --warmup 1 $mode "$@"
  run walled$tag --scene walled --steps 5 --warmup 1 $mode "$@"
done
