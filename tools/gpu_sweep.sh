#!/bin/bash
# parity subset, then bench lines under environment settings: each argument is
# "ENV=.. [ENV=..] -- bench args" (quoted); prints value and per-launch time
export TMPDIR=/tmp
mkdir -p gpurun_out/sweep
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py tests/test_gate.py tests/test_e2e_gpu.py -m gpu -x -q \
    -p no:cacheprovider > gpurun_out/sweep/pytest.txt 2>&1
rc=$?; tail -2 gpurun_out/sweep/pytest.txt; [ $rc -ne 0 ] && exit $rc
i=0
for spec in "$@"; do
  i=$((i+1))
  envs=${spec%%--*}; args=${spec#*--}
  env $envs timeout -k 10 300 python bench.py --cpu-baseline 0 $args > gpurun_out/sweep/r$i.json 2> gpurun_out/sweep/r$i.err \
      || { echo "FAILED: $spec"; tail -3 gpurun_out/sweep/r$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/sweep/r$i.json')); print('$spec ->', round(d['value'],1), round(d['roofline']['per_launch_us'],2))"
done
