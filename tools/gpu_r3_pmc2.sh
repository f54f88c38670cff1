#!/bin/bash
# round 3: HBM traffic of the step2 headline kernel, default stores vs sc1 stores (FETCH/WRITE passes)
export TMPDIR=/tmp
KPAT=mk_step2_kernel bash tools/gpu_pmc.sh r3_s2b STD128_MKNTRU --stage evalacc > gpurun_out/pmc_r3_s2b.txt 2>&1 || { tail -5 gpurun_out/pmc_r3_s2b.txt; exit 1; }
tail -4 gpurun_out/pmc_r3_s2b.txt
mkdir -p gpurun_out/pmc_r3_sc1
i=0
for CS in "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  MKFHE_LIB=$PWD/mkfhe_amd/lib/variants/sc1.so timeout -k 10 240 rocprofv3 --pmc $CS -d gpurun_out/pmc_r3_sc1/p$i -o run --output-format csv -- \
      python3 bench.py --steps 1 --warmup 0 --cpu-baseline 0 --n-override 32 --stage evalacc > gpurun_out/pmc_r3_sc1/p$i.log 2>&1 || { echo "sc1 pass $i failed"; exit 1; }
done
python3 tools/pmc_summary.py gpurun_out/pmc_r3_sc1 mk_step2_kernel
