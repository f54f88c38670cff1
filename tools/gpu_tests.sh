#!/bin/bash
# usage: tools/gpu_tests.sh TAG [pytest selection...]
#   the -m gpu suite (or a selection of it) under its own time limit
TAG=$1; shift
export TMPDIR=/tmp
mkdir -p gpurun_out
SEL=${@:-tests}
timeout -k 10 800 python -u -m pytest $SEL -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/pytest_$TAG.txt 2>&1
rc=$?
tail -4 gpurun_out/pytest_$TAG.txt
exit $rc
