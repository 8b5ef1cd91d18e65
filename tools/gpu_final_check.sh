# Round-end rehearsal: smoke(), the default bench line (as the driver runs it), profiles.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAILED; tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log | cut -c1-200
SECONDS=0; timeout -k 10 600 python -u bench.py > gpurun_out/bench_default.log 2> gpurun_out/bench_default.err || { tail -20 gpurun_out/bench_default.err; exit 2; }
echo "bench wall ${SECONDS} s"
tail -1 gpurun_out/bench_default.log
