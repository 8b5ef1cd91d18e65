set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 gpu-ray_trace-rust_amd/lib/check_libm_gpu > gpurun_out/check_libm_gpu.json 2>&1 || { cat gpurun_out/check_libm_gpu.json; exit 1; }
cat gpurun_out/check_libm_gpu.json
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
for s in walled biplane spaceship_r1; do timeout -k 10 200 python -u bench.py --scene $s --steps 3 --warmup 1 --no-cpu --no-roofline > gpurun_out/bench_$s.log 2>&1 || exit 2; tail -1 gpurun_out/bench_$s.log | cut -c1-200; done
timeout -k 10 200 python -u bench.py --scene a380 --spp-per-step 10 --steps 3 --warmup 1 --no-cpu --no-roofline > gpurun_out/bench_a380.log 2>&1 && tail -1 gpurun_out/bench_a380.log | cut -c1-200
