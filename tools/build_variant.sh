#!/bin/bash
# usage: tools/build_variant.sh NAME [-DFLAG ...]
#   a DG=3-only engine build for A/B timing (mkfhe_amd/lib/variants/NAME.so)
NAME=$1; shift
mkdir -p mkfhe_amd/lib/variants
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -fvisibility-inlines-hidden -Wl,-Bsymbolic \
  -Wno-unused-result -Wno-pass-failed -I include -DMKACC_ONLY_DG=3 "$@" -Rpass-analysis=kernel-resource-usage \
  -o mkfhe_amd/lib/variants/$NAME.so mkfhe_amd/csrc/mkacc_engine.hip 2> mkfhe_amd/lib/variants/$NAME.res
rc=$?
grep -A9 "mk_step_kernelILi3ELi0ELb0E" mkfhe_amd/lib/variants/$NAME.res | grep -E "VGPRs( Spill)?:" | sed 's/.*remark: *//' | tr '\n' ' '
echo " [$NAME rc=$rc]"
exit $rc
