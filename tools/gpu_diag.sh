#!/bin/bash
# fresh-key NAND truth tables (python mirror + the C++ example), then an A/B of engine variants
# usage: tools/gpu_diag.sh TAG TRIALS [LIB.so ...]
TAG=$1; TRIALS=$2; shift 2
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/fresh_key_trials.py $TRIALS STD128_MKNTRU > gpurun_out/fk_$TAG.txt 2>&1
rc=$?; tail -3 gpurun_out/fk_$TAG.txt
case $rc in 0) ;; *) echo "fresh-key trials rc=$rc"; exit $rc;; esac
for i in 1 2 3 4 5 6; do
  timeout -k 10 120 tests/cpp/build/boolean-mkntru STD128_MKNTRU > gpurun_out/ex_${TAG}_$i.txt 2>&1
  rc=$?
  echo "example run $i rc=$rc: $(grep -o '= [01]' gpurun_out/ex_${TAG}_$i.txt | tr -d '= ' | tr -d '\n')"
  case $rc in 0|1) ;; *) exit $rc;; esac
done
if [ $# -gt 0 ]; then bash tools/gpu_ab.sh $TAG "$@" || exit $?; fi
exit 0
