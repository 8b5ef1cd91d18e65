# Stripe height A/B for one rank's share (bench.py --as-rank --stripe): 1-row stripes against
# the default (rt_amd.shard.stripe_rows).
set -o pipefail
mkdir -p gpurun_out
run() {  # tag, bench args...
  timeout -k 10 200 python -u bench.py --no-cpu --no-roofline "${@:2}" > gpurun_out/stripe_$1.log 2>&1 || exit 1
  echo "$1: $(tail -1 gpurun_out/stripe_$1.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["config"]["stripes"])')"
}
C5="--scene spaceship_r1 --width 4096 --height 4096 --strong --as-rank 0/8 --steps 12 --warmup 2"
for i in 1 2; do
  run c5_s1 $C5 --stripe 1
  run c5_auto $C5
  run biplane_s1 --scene biplane --as-rank 0/8 --steps 4 --warmup 1 --stripe 1
  run biplane_auto --scene biplane --as-rank 0/8 --steps 4 --warmup 1
  run walled_s1 --as-rank 0/8 --steps 3 --warmup 1 --stripe 1
  run walled_auto --as-rank 0/8 --steps 3 --warmup 1
done
