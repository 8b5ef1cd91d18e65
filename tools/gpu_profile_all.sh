# The round's rocprofv3 evidence on one MI355X (run through gpurun): for the bench workload and
# every BASELINE config bench.py times beside it, tools/run_profiles.sh's kernel trace and counter
# passes at the config's own launch shape (round 4: the batch group's launch, bench.py GROUP_ITEMS); then python tools/prof_summary.py <tag>_<config> for
# each (profiles/<tag>_<config>_*, counters keyed on the kernel build).
# Usage: tools/gpu_profile_all.sh <tag> [config ...]
set -o pipefail
TAG=${1:-r3}; shift
CONFIGS=${@:-walled biplane a380 spaceship4096 triangles}
for c in $CONFIGS; do
  case $c in
    walled) A="--scene walled --steps 2 --warmup 1";;
    biplane) A="--scene biplane --spp-per-step 20 --steps 2 --warmup 1";;   # config 3's batch group: 2 x 10 spp
    a380) A="--scene a380 --spp-per-step 10 --steps 2 --warmup 1";;         # config 2's batch group: 10 x 1 spp
    spaceship4096) A="--scene spaceship_r1 --width 4096 --height 4096 --spp-per-step 25 --steps 2 --warmup 1";;
    triangles) A="--scene triangles --spp-per-step 10 --steps 2 --warmup 1";;
    *) echo "unknown config $c"; exit 9;;
  esac
  bash tools/run_profiles.sh ${TAG}_$c $A --no-configs || exit $?
done
echo profile_all_ok
