#!/bin/bash
# round 4 validation: GPU suite, smoke, headline bench, rocprof kernel stats
export TMPDIR=/tmp
O=gpurun_out/r4
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > $O/${TAG}_pytest_gpu.txt 2>&1 || { tail -40 $O/${TAG}_pytest_gpu.txt; exit 1; }
tail -2 $O/${TAG}_pytest_gpu.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/${TAG}_smoke.txt 2>&1 || { cat $O/${TAG}_smoke.txt; exit 1; }
tail -3 $O/${TAG}_smoke.txt
timeout -k 10 400 python bench.py > $O/${TAG}_bench.json 2> $O/${TAG}_bench.err || { tail -20 $O/${TAG}_bench.err; exit 1; }
cat $O/${TAG}_bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/${TAG}_prof -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --cpu-baseline 0 > $O/${TAG}_prof.log 2>&1 || { tail -20 $O/${TAG}_prof.log; exit 1; }
find $O/${TAG}_prof -name "*kernel_stats.csv" | head -1 | xargs head -4 | cut -c1-220
