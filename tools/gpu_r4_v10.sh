#!/bin/bash
# round 4: mk_step3_kernel (27-bit, two waves per gate) parity + A/B on configs 4 and 2; widereg2 LC lane-map fix
export TMPDIR=/tmp
O=gpurun_out/r4
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "step_kernels" --timeout 300 --timeout-method thread -p no:cacheprovider \
    > $O/${TAG}_step_parity.txt 2>&1 || { tail -40 $O/${TAG}_step_parity.txt; exit 1; }
tail -2 $O/${TAG}_step_parity.txt
timeout -k 10 500 python -u -m pytest tests/test_golden.py tests/test_wide.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    > $O/${TAG}_golden_wide.txt 2>&1 || { tail -40 $O/${TAG}_golden_wide.txt; exit 1; }
tail -2 $O/${TAG}_golden_wide.txt
run() {  # name, env, bench args
  env $2 timeout -k 10 400 python bench.py $3 > $O/${TAG}_$1.json 2> $O/${TAG}_$1.err || { echo "$1 failed"; tail -5 $O/${TAG}_$1.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/${TAG}_$1.json')); print('$1', round(d['value'],1), round(d['roofline']['per_launch_us'],2), 'us/launch parity', d.get('parity_checked'), d.get('parity_mismatches'))"
}
C4="--stage evalacc --steps 1 --warmup 1 --cpu-threads 16 --paramset STD128_MKNTRU_3 --batch 8192"
run c4_s3 "MKACC_STEP=3" "$C4"
run c4_s1 "MKACC_STEP=1" "$C4"
run hl_s3 "MKACC_STEP=3" "--steps 3 --warmup 1 --cpu-threads 16"
run hl_s2 "MKACC_STEP=2" "--steps 3 --warmup 1 --cpu-threads 16"
run c5 "MKACC_WREG2=1" "--paramset STD100_MKNTRU --q-bits 50 --stage evalacc --steps 2 --warmup 1 --cpu-threads 16"
run c4_s3b "MKACC_STEP=3" "$C4"
run hl_s3b "MKACC_STEP=3" "--steps 3 --warmup 1 --cpu-threads 16"
