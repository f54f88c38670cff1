#!/bin/bash
# round 3: per-config v1/v2 A/B, then stochastic PC sampling of the v2 headline step kernel
export TMPDIR=/tmp
mkdir -p gpurun_out/r3
for CFG in "STD100_MKNTRU|" "STD128_MKNTRU_3|--batch 8192 --n-override 96" "STD100_MKNTRU_LWE_2|"; do
  IFS='|' read -r PS EXTRA <<< "$CFG"
  for V in 2 1; do
    MKACC_STEP=$V timeout -k 10 300 python bench.py --stage evalacc --steps 2 --warmup 1 --cpu-threads 16 --paramset $PS $EXTRA \
       > gpurun_out/r3/cfg_${PS}_v$V.json 2> gpurun_out/r3/cfg_${PS}_v$V.err || { echo "$PS v$V failed"; tail -5 gpurun_out/r3/cfg_${PS}_v$V.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/r3/cfg_${PS}_v$V.json')); print('$PS v$V', round(d['value'],1), 'us/launch', round(d['roofline']['per_launch_us'],2), 'parity', d.get('parity_checked'), d.get('parity_mismatches'))"
  done
done
timeout -k 10 240 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method stochastic --pc-sampling-unit cycles \
    --pc-sampling-interval 1048576 -d gpurun_out/r3/pcs -o run --output-format csv -- \
    python3 bench.py --stage evalacc --steps 1 --warmup 0 --cpu-baseline 0 --n-override 24 > gpurun_out/r3/pcs.log 2>&1
echo "pcs rc=$?"; tail -3 gpurun_out/r3/pcs.log; find gpurun_out/r3/pcs -type f | head; du -sh gpurun_out/r3/pcs
