#!/bin/bash
# usage: tools/build_variant.sh NAME [-DFLAG ...]
#   an engine build with extra -D switches for A/B timing (mkfhe_amd/lib/variants/NAME.so).
#   Every digit count is instantiated, so a variant runs every test; its build
#   identity (mkacc_build_info: header/source ids and these flags) is checked by
#   mkfhe_amd._lib.load when it is loaded through MKFHE_LIB.
NAME=$1; shift
python3 -m mkfhe_amd.build --variant "$NAME" "$@" > /dev/null   # add --units a,b to recompile only those units
rc=$?
grep -A9 "mk_step2_kernelILi3ELi0ELb0E" mkfhe_amd/lib/variants/$NAME.res | grep -E "VGPRs( Spill)?:" | sed 's/.*remark: *//' | tr '\n' ' '
echo " [$NAME rc=$rc]"
# store-data / VCC hazard audit of the variant (a violation corrupts stores under load)
python3 tools/isa_audit.py mkfhe_amd/lib/variants/$NAME.so > /tmp/isa_audit_$$.txt; a=$?
tail -1 /tmp/isa_audit_$$.txt; rm -f /tmp/isa_audit_$$.txt
[ $a -eq 0 ] || rc=1
exit $rc
