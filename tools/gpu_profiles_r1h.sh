set -o pipefail
bash tools/run_profiles.sh r1h --steps 3 --warmup 1 || exit 1
bash tools/run_profiles.sh r1h_biplane --scene biplane --steps 2 --warmup 1 || exit 1
for s in spaceship_r1 a380 biplane; do timeout -k 10 200 python -u bench.py --scene $s --steps 3 --warmup 1 --no-cpu > gpurun_out/bench_$s.log 2>&1 || exit 2; tail -1 gpurun_out/bench_$s.log | cut -c1-300; done
