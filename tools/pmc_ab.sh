#!/bin/bash
# Counter A/B of kernel variants selected by RT_DEBUG_* knobs (one library build): for each
# variant "name:VAR=VAL,..." three rocprofv3 --pmc passes (each counter group in its own run) of
# one synchronous bench step, summed over the trace kernel's dispatches per sample.
# Usage: tools/pmc_ab.sh <tag> "<bench args>" variant ...   (run through gpurun)
set -o pipefail
export TMPDIR=/tmp
TAG=$1; shift
ARGS=$1; shift
O=gpurun_out/pmcab_$TAG
mkdir -p $O
python3 -c "import sys; sys.path.insert(0, 'gpu-ray_trace-rust_amd'); from rt_amd import abi; print(abi.kernel_build_id())" > $O/build_id || exit 1
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_VALU"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU"
P3="TA_TA_BUSY_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum"
for v in "$@"; do
  name=${v%%:*}
  envs=""
  [[ "$v" == *:* ]] && envs=${v#*:}
  mkdir -p $O/$name
  for k in 1 2 3; do
    eval "C=\$P$k"
    ( IFS=',' read -ra KVS <<< "$envs"; for kv in "${KVS[@]}"; do export "$kv"; done
      timeout -s KILL 200 rocprofv3 --pmc $C --output-format csv -d $O/$name/p$k -o run -- \
        python3 bench.py $ARGS --sync --no-cpu --no-roofline --no-configs > $O/$name/p$k.log 2>&1 ) || exit $k
  done
  echo "== $name ($envs)"
  for k in 1 2 3; do python3 tools/pmc_sum.py $O/$name/p$k queue_kernel; done
done
echo pmc_ab_ok
