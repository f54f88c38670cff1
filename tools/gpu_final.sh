#!/bin/bash
# final validation of the in-tree library: full check (suite, bench, rocprof), smoke,
# small-batch stress, fresh-key truth tables and the C++ example runs
TAG=$1
export TMPDIR=/tmp
bash tools/gpu_check.sh $TAG || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.txt 2>&1 || { echo "smoke FAILED"; tail -5 gpurun_out/smoke_$TAG.txt; exit 1; }
tail -1 gpurun_out/smoke_$TAG.txt
bash tools/gpu_lat_ab.sh $TAG 300 mkfhe_amd/lib/libmkfhe_amd.so || exit $?
bash tools/gpu_diag.sh $TAG 8 || exit $?
exit 0
