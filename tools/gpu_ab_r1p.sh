# A/B: sqrt of uniform draws without the tiny-input guard (RT_DRAW_SQRT), and one 1000-spp
# queue launch per step (RT_QUEUE_RADIANCE_GIB=12) against three 334-spp launches.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/variant_bench.py --scene walled --spp 334 --rounds 4 base dsq > gpurun_out/ab_dsq_walled.log 2>&1 || { tail -20 gpurun_out/ab_dsq_walled.log; exit 1; }
cat gpurun_out/ab_dsq_walled.log
timeout -k 10 200 python -u tools/variant_bench.py --scene biplane --spp 10 --rounds 4 base dsq > gpurun_out/ab_dsq_biplane.log 2>&1 || { tail -20 gpurun_out/ab_dsq_biplane.log; exit 2; }
cat gpurun_out/ab_dsq_biplane.log
for g in 4 12 4 12; do
  RT_QUEUE_RADIANCE_GIB=$g timeout -k 10 200 python -u bench.py --steps 6 --warmup 1 --no-cpu --no-roofline > gpurun_out/ab_rad_$g.log 2>&1 || { tail -20 gpurun_out/ab_rad_$g.log; exit 3; }
  echo "GIB=$g $(tail -1 gpurun_out/ab_rad_$g.log | cut -c1-140)"
done
