set -o pipefail
mkdir -p gpurun_out
for s in biplane spaceship_r1; do timeout -k 10 300 python -u tools/variant_bench.py --scene $s --spp 10 --rounds 3 "$@" 2>&1 | grep -v Warning | tee -a gpurun_out/ab.log || exit 1; done
