set -o pipefail
mkdir -p gpurun_out
RT_CREATE_TIMING=1 timeout -k 10 300 python -c "
import sys, time; sys.path[:0]=['gpu-ray_trace-rust_amd','tests']
import torch
from conftest import load_scene
from rt_amd import render
for n in ['a380','a380','biplane','spaceship_r1']:
    sc=load_scene(n); t=time.perf_counter()
    with render.Context(sc): pass
    print(n, 'ctx', round(time.perf_counter()-t,3), flush=True)
" 2>&1 | grep -v Warn
timeout -k 10 300 python tools/host_rates.py > gpurun_out/host_rates.jsonl 2>gpurun_out/host_rates.err || { tail -5 gpurun_out/host_rates.err; exit 1; }
cat gpurun_out/host_rates.jsonl
timeout -k 10 600 python -u -m pytest tests/test_gpu_scenes.py tests/test_gpu_production.py tests/test_gpu_edges.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t5.log 2>&1 || { tail -30 gpurun_out/t5.log; exit 1; }
tail -1 gpurun_out/t5.log
