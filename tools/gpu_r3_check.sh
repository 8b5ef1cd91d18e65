set -o pipefail
mkdir -p gpurun_out
for s in biplane spaceship_r1; do
timeout -k 10 200 python -u tools/variant_bench.py --scene $s --spp 40 --rounds 3 noquad main qnone q7w noquad7w > gpurun_out/ab_q2_$s.log 2>&1 || exit 3
grep -E "identical|variant" gpurun_out/ab_q2_$s.log
done
