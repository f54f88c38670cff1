#!/bin/bash
# round 4: widereg2 with wave-local LB->LC / LC->LD transposes: wide parity + golden, A/B vs all-cross, PMC
export TMPDIR=/tmp
O=gpurun_out/r4
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_wide.py tests/test_golden.py -m gpu -x -v -k "wide or CFG5" --timeout 300 --timeout-method thread -p no:cacheprovider \
    > $O/${TAG}_wide.txt 2>&1 || { tail -40 $O/${TAG}_wide.txt; exit 1; }
tail -2 $O/${TAG}_wide.txt
run() {  # name, env, bench args
  env $2 timeout -k 10 400 python bench.py $3 > $O/${TAG}_$1.json 2> $O/${TAG}_$1.err || { echo "$1 failed"; tail -5 $O/${TAG}_$1.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/${TAG}_$1.json')); print('$1', round(d['value'],1), round(d['roofline']['per_launch_us'],2), 'us/launch parity', d.get('parity_checked'), d.get('parity_mismatches'))"
}
C5="--paramset STD100_MKNTRU --q-bits 50 --stage evalacc --steps 2 --warmup 1 --cpu-threads 16"
V=$PWD/mkfhe_amd/lib/variants
for rep in 1 2; do
run c5_local$rep "MKACC_WREG2=1" "$C5"
run c5_cross$rep "MKFHE_LIB=$V/w2cross.so" "$C5"
done
TAG=$TAG bash tools/gpu_r4_pmc_c5.sh
