#!/bin/bash
# round 4: two-waves-per-gate FP64 kernel (widereg2): wide parity + golden, config-5 bench A/B vs one wave per gate
export TMPDIR=/tmp
O=gpurun_out/r4
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_wide.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    > $O/${TAG}_wide_parity.txt 2>&1 || { tail -40 $O/${TAG}_wide_parity.txt; exit 1; }
tail -2 $O/${TAG}_wide_parity.txt
timeout -k 10 400 python -u -m pytest tests/test_golden.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    > $O/${TAG}_golden.txt 2>&1 || { tail -40 $O/${TAG}_golden.txt; exit 1; }
tail -2 $O/${TAG}_golden.txt
for rep in 1 2; do
for V in 1 0; do
  MKACC_WREG2=$V timeout -k 10 300 python bench.py --paramset STD100_MKNTRU --q-bits 50 --stage evalacc --steps 2 --warmup 1 --cpu-threads 16 \
     > $O/${TAG}_c5_r2$V.$rep.json 2> $O/${TAG}_c5_r2$V.$rep.err || { echo "c5 r2=$V failed"; tail -5 $O/${TAG}_c5_r2$V.$rep.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/${TAG}_c5_r2$V.$rep.json')); print('c5 wreg2=$V', round(d['value'],1), 'EvalAcc/s', round(d['roofline']['per_launch_us'],2), 'us/launch parity', d.get('parity_checked'), d.get('parity_mismatches'))"
done
done
for rep in 1 2; do
  MKFHE_LIB=$PWD/mkfhe_amd/lib/variants/w2pf1.so timeout -k 10 300 python bench.py --paramset STD100_MKNTRU --q-bits 50 --stage evalacc --steps 2 --warmup 1 --cpu-threads 16 \
     > $O/${TAG}_c5_pf1.$rep.json 2> $O/${TAG}_c5_pf1.$rep.err || { echo "c5 pf1 failed"; tail -5 $O/${TAG}_c5_pf1.$rep.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/${TAG}_c5_pf1.$rep.json')); print('c5 w2pf1', round(d['value'],1), 'EvalAcc/s', round(d['roofline']['per_launch_us'],2), 'us/launch parity', d.get('parity_checked'), d.get('parity_mismatches'))"
done
