set -o pipefail
mkdir -p gpurun_out
for env in "" RT_PIPELINE_SLOTS=3 RT_PIPELINE_SLOTS=4 RT_PIPELINE=0; do
env $env timeout -k 10 300 python bench.py --scene spaceship_r1 --width 4096 --height 4096 --spp-per-step 25 --as-rank 0/8 --steps 10 --warmup 2 --no-cpu --no-roofline --no-configs > gpurun_out/reh_$$.json 2>/dev/null || exit 4
python -c "import json; d=json.load(open('gpurun_out/reh_$$.json')); print('c5 0/8 $env', d['value'], d['ms_per_step'], d['launch']['trace_ms_per_launch'])"
done
