# ★n2 (north_star's "KD-tree nodes and triangle slabs staged through LDS") on the current build:
# A/B of the LDS variants against the product on the mesh scenes (tools/variant_bench.py, one
# process, interleaved rounds, images checked bit-identical), then the vector-memory and LDS
# counters of each variant on a380 (rocprofv3, own passes).  Variants (tools/build_variants.sh):
#   top128   top-of-tree node cache, 128 nodes in LDS (stack kernel: 7 waves per SIMD)
#   top1024  1,024 nodes (~9 levels) with the stackless kernel (RT_DEBUG_KD_RESTART=1), whose LDS
#            holds no stack
#   slab64 / glds64  leaf triangle slabs of 64 primitives per wave, copied through VGPRs / by
#            LDS-DMA (global_load_lds_dwordx4), in the stackless kernel (RT_DEBUG_KD_RESTART=2)
# Usage (GPU box): bash tools/gpu_lds_ab.sh [tag]
set -o pipefail
TAG=${1:-r4_lds}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
V="main top128:RT_DEBUG_KD_RESTART=0 main:RT_DEBUG_KD_RESTART=1 top1024:RT_DEBUG_KD_RESTART=1 main:RT_DEBUG_KD_RESTART=2 slab64:RT_DEBUG_KD_RESTART=2 glds64:RT_DEBUG_KD_RESTART=2"
for s in a380 biplane spaceship_r1; do
  timeout -k 10 300 python -u tools/variant_bench.py --scene $s --spp 40 --rounds 3 $V > $OUT/ab_$s.log 2>&1 || { echo "ab $s failed"; tail -5 $OUT/ab_$s.log; exit 1; }
  echo "== $s"; cat $OUT/ab_$s.log
done
i=0
for v in $V; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc TA_TA_BUSY_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE --output-format csv -d $OUT/tatd_$i -o run -- \
      python3 tools/variant_bench.py --scene a380 --spp 40 --rounds 1 $v > $OUT/tatd_$i.log 2>&1 || { echo "tatd $v failed"; exit 2; }
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $OUT/sq_$i -o run -- \
      python3 tools/variant_bench.py --scene a380 --spp 40 --rounds 1 $v > $OUT/sq_$i.log 2>&1 || { echo "sq $v failed"; exit 3; }
  echo "counters $i $v ok"
done
echo lds_ab_ok
