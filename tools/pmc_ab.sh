set -o pipefail
export TMPDIR=/tmp
for v in head nopairs pairs; do
  timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU --output-format csv -d gpurun_out/pmc_$v -o run -- python3 tools/variant_bench.py --scene walled --spp 32 --rounds 1 $v > gpurun_out/pmc_$v.log 2>&1 || exit 1
  timeout -k 10 200 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_THREAD_CYCLES_VALU SQ_INSTS_VMEM_RD --output-format csv -d gpurun_out/pmc2_$v -o run -- python3 tools/variant_bench.py --scene walled --spp 32 --rounds 1 $v > gpurun_out/pmc2_$v.log 2>&1 || exit 2
done
echo ok
