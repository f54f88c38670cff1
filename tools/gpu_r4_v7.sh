#!/bin/bash
# round 4: FP64 issue rate vs independent work at one and two waves per SIMD, then the
# widereg offset-word / digit-plan build: wide parity + CFG5 golden, config-5 bench x2
export TMPDIR=/tmp
O=gpurun_out/r4
mkdir -p $O
timeout -k 10 120 tools/bin/ubench_dp_ilp > $O/${TAG}_ubench_dp_ilp.txt 2>&1 || { echo "ubench failed"; tail -5 $O/${TAG}_ubench_dp_ilp.txt; exit 1; }
cat $O/${TAG}_ubench_dp_ilp.txt
timeout -k 10 600 python -u -m pytest tests/test_wide.py tests/test_golden.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    > $O/${TAG}_wide_parity.txt 2>&1 || { tail -40 $O/${TAG}_wide_parity.txt; exit 1; }
tail -2 $O/${TAG}_wide_parity.txt
for rep in 1 2; do
  timeout -k 10 300 python bench.py --paramset STD100_MKNTRU --q-bits 50 --stage evalacc --steps 2 --warmup 1 --cpu-threads 16 \
     > $O/${TAG}_c5.$rep.json 2> $O/${TAG}_c5.$rep.err || { echo "c5 failed"; tail -5 $O/${TAG}_c5.$rep.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/${TAG}_c5.$rep.json')); print('c5', round(d['value'],1), 'EvalAcc/s', round(d['roofline']['per_launch_us'],2), 'us/launch parity', d.get('parity_checked'), d.get('parity_mismatches'))"
done
