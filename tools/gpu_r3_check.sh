set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/b_default.json 2>gpurun_out/b_default.err || { tail -5 gpurun_out/b_default.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/b_default.json'))
print(d['value'], d['roofline']['bound'], d['roofline']['frac'], d['roofline'].get('valu',{}).get('min_insts_frac'))
for k,v in d['configs'].items(): print(k, v['value'], v['roofline']['bound'], v['roofline']['frac'], v['cpu_baseline']['value'], v['speedup_vs_cpu'])
"
