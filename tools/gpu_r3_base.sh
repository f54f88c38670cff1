#!/bin/bash
# round 3 baseline of the split-unit build: GPU suite, smoke, headline bench, rocprof kernel stats
export TMPDIR=/tmp
mkdir -p gpurun_out/r3
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/r3/base_pytest_gpu.txt 2>&1 || { tail -30 gpurun_out/r3/base_pytest_gpu.txt; exit 1; }
tail -2 gpurun_out/r3/base_pytest_gpu.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3/base_smoke.txt 2>&1 || { cat gpurun_out/r3/base_smoke.txt; exit 1; }
cat gpurun_out/r3/base_smoke.txt
timeout -k 10 400 python bench.py > gpurun_out/r3/base_bench.json 2> gpurun_out/r3/base_bench.err || { tail -20 gpurun_out/r3/base_bench.err; exit 1; }
cat gpurun_out/r3/base_bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r3/base_prof -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --cpu-baseline 0 > gpurun_out/r3/base_prof.log 2>&1 || { tail -20 gpurun_out/r3/base_prof.log; exit 1; }
find gpurun_out/r3/base_prof -name "*kernel_stats.csv" | head -1 | xargs head -4 | cut -c1-220
