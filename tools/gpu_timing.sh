# Wave-clock split of the queue kernels (diagnostic build: make -C gpu-ray_trace-rust_amd diag -> lib/variants/librt_diag_timing.so);
set -o pipefail
# the diag counters are global and reset by a launch's last wave: overlapped launches would mix
export RT_DEBUG_LAUNCH=overlap=0
mkdir -p gpurun_out
for s in biplane spaceship_r1 a380; do
  timeout -k 10 200 python -u tools/variant_bench.py --scene $s --spp 40 --rounds 1 diag_timing > gpurun_out/tm_$s.log 2>&1 || exit 1
  echo "== $s"; grep RT_TIMING gpurun_out/tm_$s.log | tail -1
done
