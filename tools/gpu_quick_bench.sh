# quick perf check of the three main scenes (no roofline / CPU legs)
set -o pipefail
mkdir -p gpurun_out
for s in walled biplane spaceship_r1; do timeout -k 10 200 python -u bench.py --scene $s --steps 3 --warmup 1 --no-cpu --no-roofline > gpurun_out/bench_$s.log 2>&1 || exit 2; tail -1 gpurun_out/bench_$s.log | cut -c1-120; done
