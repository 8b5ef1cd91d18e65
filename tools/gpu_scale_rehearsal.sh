# 1-GPU rehearsal of the N-GPU weak-scaling bench: rank 0's share of N ranks, timed alone.
set -o pipefail
mkdir -p gpurun_out
for n in 2 8; do timeout -k 10 200 python -u bench.py --as-rank 0/$n --steps 3 --warmup 1 --no-cpu --no-roofline > gpurun_out/rehearsal_$n.log 2>&1 || exit 1; tail -1 gpurun_out/rehearsal_$n.log | cut -c1-160; done
