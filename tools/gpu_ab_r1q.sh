# A/B of the queue's grab sizes at the end of a launch: minimum grab (RT_QMIN) and the divisor
# of the adaptive grab (RT_QDIV), walled at one 1000-spp launch and biplane at 10 spp.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/variant_bench.py --scene walled --spp 1000 --rounds 4 base qmin128 qmin256 qdiv8 qdiv32 > gpurun_out/ab_grab_walled.log 2>&1 || { tail -20 gpurun_out/ab_grab_walled.log; exit 1; }
cat gpurun_out/ab_grab_walled.log
timeout -k 10 300 python -u tools/variant_bench.py --scene biplane --spp 10 --rounds 4 base qmin128 qmin256 qdiv8 qdiv32 > gpurun_out/ab_grab_biplane.log 2>&1 || { tail -20 gpurun_out/ab_grab_biplane.log; exit 2; }
cat gpurun_out/ab_grab_biplane.log
