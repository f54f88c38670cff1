#!/bin/bash
# round 4: PMC of a step kernel (KNAME), one rocprofv3 run per pass; BARGS = the bench arguments (default: config 5)
export TMPDIR=/tmp
D=gpurun_out/pmc_${TAG}
BARGS=${BARGS:---paramset STD100_MKNTRU --q-bits 50 --stage evalacc}
K=${KNAME:-widereg2::step_kernel}
mkdir -p $D
i=0
for CS in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
          "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE" \
          "SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA TCP_TOTAL_CACHE_ACCESSES_sum TCC_HIT_sum TCC_MISS_sum GRBM_COUNT" \
          "FETCH_SIZE" "WRITE_SIZE" ; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $CS -d $D/p$i -o run --output-format csv -- \
      python3 bench.py --steps 1 --warmup 0 --cpu-baseline 0 --n-override 32 $BARGS \
      > $D/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $D/p$i.log; exit 1; }
done
python3 tools/pmc_summary.py $D $K
# instruction-cache pass (its own run; counter names per the gfx9 SQC block)
timeout -s KILL 60 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES -d $D/pic -o run --output-format csv -- \
    python3 bench.py --steps 1 --warmup 0 --cpu-baseline 0 --n-override 32 $BARGS \
    > $D/pic.log 2>&1 || { echo "icache pass failed"; tail -3 $D/pic.log; }
python3 tools/pmc_summary.py $D $K | grep SQC || true
