set -o pipefail
mkdir -p gpurun_out
C5="--scene spaceship_r1 --width 4096 --height 4096 --strong --as-rank 0/8 --steps 12 --warmup 2 --no-cpu --no-roofline"
for cfg in "RT_DEBUG_LAUNCH=slots=2" "RT_DEBUG_LAUNCH=slots=3" "RT_DEBUG_LAUNCH=slots=4" "RT_DEBUG_LAUNCH=slots=8" "RT_DEBUG_LAUNCH=overlap=0"; do
  env $cfg timeout -k 10 120 python -u bench.py $C5 > gpurun_out/c5s.log 2>&1 || exit 1
  echo "$cfg $(tail -1 gpurun_out/c5s.log | cut -c1-110)"
done
