# A/B of kernel variants (lib/variants/librt_<name>.so, tools/build_variants.sh) on every
# benchmark scene, interleaved in one process per scene (tools/variant_bench.py).  The mesh
# scenes run 40 spp per launch so that the ~10 ms drain tail of a launch stays small.
# Usage: tools/gpu_ab.sh name1 name2 ...   (run through gpurun)
set -o pipefail
mkdir -p gpurun_out
run() {  # scene spp
  timeout -k 10 300 python -u tools/variant_bench.py --scene $1 --spp $2 --rounds 3 "${@:3}" 2>&1 | grep --line-buffered -v Warning | tee -a gpurun_out/ab.log || exit 1
}
run walled 1000 "$@"
run biplane 40 "$@"
run spaceship_r1 40 "$@"
run a380 40 "$@"
