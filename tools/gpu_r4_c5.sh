#!/bin/bash
# round 4: config 5 register-resident FP64 kernel -- wide parity, then A/B against the LDS-tile kernel
export TMPDIR=/tmp
O=gpurun_out/r4
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_wide.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    > $O/${TAG}_wide_parity.txt 2>&1 || { tail -40 $O/${TAG}_wide_parity.txt; exit 1; }
tail -2 $O/${TAG}_wide_parity.txt
for rep in 1 2; do
for V in 1 0; do
  MKACC_WFP_REG=$V timeout -k 10 300 python bench.py --paramset STD100_MKNTRU --q-bits 50 --stage evalacc --steps 2 --warmup 1 --cpu-threads 16 \
     > $O/${TAG}_c5_reg$V.$rep.json 2> $O/${TAG}_c5_reg$V.$rep.err || { echo "c5 reg$V failed"; tail -5 $O/${TAG}_c5_reg$V.$rep.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/${TAG}_c5_reg$V.$rep.json')); print('c5 reg$V', round(d['value'],1), 'us/launch', round(d['roofline']['per_launch_us'],2), 'parity', d.get('parity_checked'), d.get('parity_mismatches'))"
done
done
