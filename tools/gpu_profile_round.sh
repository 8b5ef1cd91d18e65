# Round evidence on one MI355X (run through gpurun): the default bench line (as the driver runs
# it), then the rocprofv3 passes of the bench workload (walled) and of biplane at its scheme batch.
# Usage: tools/gpu_profile_round.sh <tag>; afterwards python tools/prof_summary.py <tag> and <tag>_biplane
set -o pipefail
TAG=${1:-r2}
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py > gpurun_out/bench_default.log 2> gpurun_out/bench_default.err || { tail -20 gpurun_out/bench_default.err; exit 1; }
tail -1 gpurun_out/bench_default.log | cut -c1-400
bash tools/run_profiles.sh $TAG --steps 3 --warmup 1 || exit 2
bash tools/run_profiles.sh ${TAG}_biplane --scene biplane --steps 6 --warmup 2 || exit 3
