#!/bin/bash
# round 3: GPU suite + smoke of the current build (no building on the box)
export TMPDIR=/tmp
mkdir -p gpurun_out/r3
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/r3/pytest_gpu.txt 2>&1
rc=$?
tail -5 gpurun_out/r3/pytest_gpu.txt
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3/smoke.txt 2>&1 || { cat gpurun_out/r3/smoke.txt; exit 1; }
cat gpurun_out/r3/smoke.txt
