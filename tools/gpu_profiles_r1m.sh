set -o pipefail
bash tools/run_profiles.sh r1m --steps 3 --warmup 1 || exit 1
bash tools/run_profiles.sh r1m_biplane --scene biplane --steps 2 --warmup 1 || exit 1
timeout -k 10 300 python -u bench.py --scene spaceship_r1 --width 4096 --height 4096 --steps 2 --warmup 1 --no-cpu > gpurun_out/bench_spaceship_4096.log 2>&1 || exit 2
tail -1 gpurun_out/bench_spaceship_4096.log | cut -c1-400
timeout -k 10 300 python -u bench.py --scene a380 --spp-per-step 10 --steps 3 --warmup 1 --no-cpu > gpurun_out/bench_a380.log 2>&1 || exit 3
tail -1 gpurun_out/bench_a380.log | cut -c1-300
