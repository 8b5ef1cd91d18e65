# A/B of kernel variants on the mesh scenes only (tools/gpu_ab.sh without walled).
# Usage: tools/gpu_ab_mesh.sh name1 name2 ...   (run through gpurun)
set -o pipefail
mkdir -p gpurun_out
for s in biplane spaceship_r1 a380; do
  timeout -k 10 300 python -u tools/variant_bench.py --scene $s --spp 40 --rounds 3 "$@" 2>&1 | grep --line-buffered -v Warning | tee -a gpurun_out/ab.log || exit 1
done
