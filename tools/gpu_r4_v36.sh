#!/bin/bash
# round 4: config 4, MKACC_DS_CANON=3 variant (the index party's pass sums acc[index] too) vs the default 2; then the
# variant's GPU parity tests (EvalAcc cases incl. the k=8 dg=4 shape, dscr modes, full paramsets, golden fixtures)
export TMPDIR=/tmp
O=gpurun_out/r4
mkdir -p $O
run() {  # name, env, bench args
  env $2 timeout -k 10 400 python bench.py $3 > $O/${TAG}_$1.json 2> $O/${TAG}_$1.err || { echo "$1 failed"; tail -5 $O/${TAG}_$1.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/${TAG}_$1.json')); print('$1', round(d['value'],1), round(d['ms_per_step'],2), 'ms/step', round(d['roofline']['per_launch_us'],2), 'us/step', d['roofline']['kernel'], 'parity', d.get('parity_checked'), d.get('parity_mismatches'))"
}
C4="--stage evalacc --steps 1 --warmup 1 --paramset STD128_MKNTRU_3 --batch 8192"
V=$PWD/mkfhe_amd/lib/variants
run c4_base "" "$C4"
run c4_canon3 "MKFHE_LIB=$V/canon3.so" "$C4"
run c4_base2 "" "$C4"
run c4_canon3b "MKFHE_LIB=$V/canon3.so" "$C4"
MKFHE_LIB=$V/canon3.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_golden.py -m gpu -x -q --timeout 300 \
   --timeout-method thread -p no:cacheprovider -k "evalacc or golden or STD128" > $O/${TAG}_canon3_pytest.txt 2>&1 || { tail -30 $O/${TAG}_canon3_pytest.txt; exit 1; }
tail -2 $O/${TAG}_canon3_pytest.txt
