# Round-1 evidence with the sphere-only kernel's 256-item minimum grab: GPU parity tests, the default bench line, then
# the rocprofv3 passes for walled (the bench workload) and biplane.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 300 python -u bench.py > gpurun_out/bench_default.log 2> gpurun_out/bench_default.err || exit 2
tail -1 gpurun_out/bench_default.log | cut -c1-300
bash tools/run_profiles.sh r1s --steps 3 --warmup 1 || exit 3
bash tools/run_profiles.sh r1s_biplane --scene biplane --steps 2 --warmup 1 || exit 4
