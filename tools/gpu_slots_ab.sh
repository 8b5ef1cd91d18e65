set -o pipefail
mkdir -p gpurun_out/slots
for n in 2 3 4; do for sc in "a380 --steps 20 --warmup 3" "biplane --steps 20 --warmup 3" "spaceship_r1 --steps 8 --warmup 2" "a380 --spp-per-step 10 --steps 5 --warmup 1"; do
  set -- $sc; name=$1
  RT_PIPELINE_SLOTS=$n timeout -k 10 200 python -u bench.py --no-cpu --no-roofline --scene $sc > gpurun_out/slots/$name_$n.log 2>&1 || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/slots/$name_$n.log').read().strip().splitlines()[-1]); print('slots $n', d['config']['workload'][:40], round(d['value'],1))"
done; done
