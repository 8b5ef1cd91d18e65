# Wave-clock split of the queue kernels (diagnostic build -DRT_TIMING=1 as lib/variants/librt_tm.so);
# walled: python tools/variant_bench.py --scene walled --spp 200 --rounds 1 tm (path starts,
# normalize, closest hit, shading, segments in the packet..pk_refs columns)
set -o pipefail
mkdir -p gpurun_out
for s in biplane spaceship_r1 a380; do
  timeout -k 10 200 python -u tools/variant_bench.py --scene $s --spp 40 --rounds 1 tm > gpurun_out/tm_$s.log 2>&1 || exit 1
  echo "== $s"; grep RT_TIMING gpurun_out/tm_$s.log | tail -1
done
