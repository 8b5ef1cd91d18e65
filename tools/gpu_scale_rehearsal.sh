# 1-GPU rehearsal of the N-GPU runs: one rank's share of N ranks, timed alone (bench.py --as-rank).
#  - walled strong scaling (bench.py's N > 1 headline, the driver's SCALE run): the whole frame,
#    rank 0 of N = 2, 4, 8 and rank 7 of 8
#  - BASELINE config 5 (strong): spaceship_r1 at 4096^2, batch 25, the full frame on one GPU
#    and ranks 0 and 7 of 8
set -o pipefail
mkdir -p gpurun_out
run() {  # tag, bench args...
  timeout -k 10 300 python -u bench.py --no-cpu --no-roofline "${@:2}" > gpurun_out/rehearsal_$1.log 2>&1 || exit 1
  echo "$1: $(tail -1 gpurun_out/rehearsal_$1.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["unit"], "ms_per_step", d["ms_per_step"], d["config"].get("rehearsal", "full frame"))')"
}
run walled_full --steps 3 --warmup 1
for n in 2 4 8; do
  run walled_0of$n --as-rank 0/$n --steps 8 --warmup 2
done
run walled_7of8 --as-rank 7/8 --steps 8 --warmup 2
C5="--scene spaceship_r1 --width 4096 --height 4096"
run c5_full $C5 --steps 6 --warmup 2
run c5_0of8 $C5 --as-rank 0/8 --steps 12 --warmup 2
run c5_7of8 $C5 --as-rank 7/8 --steps 12 --warmup 2
