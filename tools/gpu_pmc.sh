#!/bin/bash
# PMC passes on a shortened bench (n=32 steps): each pass its own rocprofv3 run,
# stopping at the first pass that fails.
# usage: tools/gpu_pmc.sh TAG [PARAMSET [extra bench args]]
#   with PARAMSET set, the FETCH_SIZE/WRITE_SIZE passes also rewrite
#   profiles/traffic_PARAMSET.json (the record bench.py reports as roofline.traffic)
TAG=$1; shift
PS=$1; [ -n "$PS" ] && shift
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_$TAG
i=0
for CS in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
          "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE" \
          "SQ_INSTS_VALU_MUL_U32 SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA TCP_TOTAL_CACHE_ACCESSES_sum TCC_HIT_sum TCC_MISS_sum GRBM_COUNT" \
          "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY" \
          "FETCH_SIZE" "WRITE_SIZE" ; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $CS -d gpurun_out/pmc_$TAG/p$i -o run --output-format csv -- \
      python3 bench.py --steps 1 --warmup 0 --cpu-baseline 0 --n-override 32 ${PS:+--paramset $PS} "$@" \
      > gpurun_out/pmc_$TAG/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/pmc_$TAG/p$i.log; exit 1; }
done
python3 tools/pmc_summary.py gpurun_out/pmc_$TAG ${KPAT:-mk_step_kernel} $PS
