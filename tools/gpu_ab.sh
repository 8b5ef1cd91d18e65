# A/B of kernel variants (lib/variants/librt_<name>.so, tools/build_variants.sh; "main" is the
# shipped library, name:VAR=VAL sets an environment knob) on the benchmark scenes, interleaved in
# one process per scene (tools/variant_bench.py).  The mesh scenes run 40 spp per launch so that
# the ~10 ms drain tail of a launch stays small.
# Usage: [SCENES="biplane spaceship_r1 a380"] tools/gpu_ab.sh name1 name2 ...   (run through gpurun)
set -o pipefail
mkdir -p gpurun_out
SCENES=${SCENES:-walled biplane spaceship_r1 a380}
for s in $SCENES; do
  spp=40; [ "$s" = walled ] && spp=1000
  timeout -k 10 300 python -u tools/variant_bench.py --scene $s --spp $spp --rounds 3 "$@" 2>&1 | grep --line-buffered -v Warning | tee -a gpurun_out/ab.log || exit 1
done
