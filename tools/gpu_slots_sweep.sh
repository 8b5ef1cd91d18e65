# Mesh configs at their scheme batches by HIP hardware queues (GPU_MAX_HW_QUEUES) and pipeline
# slots (RT_DEBUG_LAUNCH slots)
set -o pipefail
mkdir -p gpurun_out/slots
run() {  # tag scene extra
  local t=$1 sc=$2; shift 2
  timeout -k 10 200 python -u bench.py --no-cpu --no-roofline --scene $sc "$@" > gpurun_out/slots/$t.log 2>&1 || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/slots/$t.log').read().strip().splitlines()[-1]); print('$t', d['value'], d['ms_per_step'], d['launch']['trace_ms_per_launch'])"
}
for q in 4 8 12; do for n in 4 8; do
  GPU_MAX_HW_QUEUES=$q RT_DEBUG_LAUNCH=slots=$n run a380b1_q${q}_s$n a380 --steps 20 --warmup 3
  GPU_MAX_HW_QUEUES=$q RT_DEBUG_LAUNCH=slots=$n run a380b1L_q${q}_s$n a380 --steps 60 --warmup 3
done
GPU_MAX_HW_QUEUES=$q run a380b10_q${q} a380 --spp-per-step 10 --steps 5 --warmup 1
GPU_MAX_HW_QUEUES=$q run a380b10L_q${q} a380 --spp-per-step 10 --steps 15 --warmup 2
done
