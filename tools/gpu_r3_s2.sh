#!/bin/bash
# round 3: step2 kernel parity, then v2 / v1 bench A/B (EvalAcc, headline set) + kernel stats
export TMPDIR=/tmp
mkdir -p gpurun_out/r3
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_golden.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/r3/s2_parity.txt 2>&1 || { tail -40 gpurun_out/r3/s2_parity.txt; exit 1; }
tail -2 gpurun_out/r3/s2_parity.txt
for rep in 1 2; do
for V in 2 1; do
  MKACC_STEP=$V timeout -k 10 300 python bench.py --stage evalacc --steps 2 --warmup 1 --cpu-threads 16 ${BENCH_ARGS} \
     > gpurun_out/r3/s2_v$V.$rep.json 2> gpurun_out/r3/s2_v$V.$rep.err || { echo "v$V bench failed"; tail -5 gpurun_out/r3/s2_v$V.$rep.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r3/s2_v$V.$rep.json')); print('v$V', round(d['value'],1), 'us/launch', round(d['roofline']['per_launch_us'],2), 'parity', d.get('parity_checked'), d.get('parity_mismatches'))"
done
done
