// mkacc_steps.hip -- kernel translation units of the engine library.  The
// build (mkfhe_amd/build.py) compiles this file once per unit, in parallel:
//   -DMKACC_TU_DG=d -DMKACC_TU_PART=0   mk_step_kernel instantiations of digit count d (4, 5)
//   -DMKACC_TU_DG=d -DMKACC_TU_PART=1   mk_lat_kernel instantiations of digit count d (2..4)
//   -DMKACC_TU_DG=d -DMKACC_TU_PART=2   mk_step2_kernel instantiations of digit count d (2, 3), later steps
//   -DMKACC_TU_DG=d -DMKACC_TU_PART=3   the same kernel's first (KDM) step
//   -DMKACC_TU_DG=d -DMKACC_TU_PART=4   mk_quad_kernel / mk_quad_run_kernel of digit count d (2..5)
//   -DMKACC_TU_WIDE=1 / 2               64-bit word step kernels (integer / FP64 register-resident)
// and the host unit (mkacc_engine.hip) launches them through mkacc_tu.
#include "mkacc_kernels.hpp"

#if defined(MKACC_TU_WIDE)
#include "mkacc_wide.hpp"
#if MKACC_TU_WIDE == 2
#include "mkacc_fp64.hpp"
#include "mkacc_widereg2.hpp"
#endif
namespace mkacc_tu {
#if MKACC_TU_WIDE == 2
KernelPtr widereg2_step(int method, bool first) {
    if (method == XZW)
        return first ? (KernelPtr)widereg2::step_kernel<XZW, true> : (KernelPtr)widereg2::step_kernel<XZW, false>;
    return first ? (KernelPtr)widereg2::step_kernel<XZW_B, true> : (KernelPtr)widereg2::step_kernel<XZW_B, false>;
}
#else
KernelPtr wide_step(int method, bool first) {
    if (method == XZW) return first ? (KernelPtr)wide::step_kernel<XZW, true> : (KernelPtr)wide::step_kernel<XZW, false>;
    return first ? (KernelPtr)wide::step_kernel<XZW_B, true> : (KernelPtr)wide::step_kernel<XZW_B, false>;
}
#endif
}  // namespace mkacc_tu

#elif defined(MKACC_TU_DG)
#define MKACC_CAT2(a, b) a##b
#define MKACC_CAT(a, b) MKACC_CAT2(a, b)
namespace mkacc_tu {
#if MKACC_TU_PART == 0
KernelPtr MKACC_CAT(step_dg, MKACC_TU_DG)(int method, bool first, bool dscr) {
    return (KernelPtr)pick_step<MKACC_TU_DG>(method, first, dscr);
}
#elif MKACC_TU_PART == 1
KernelPtr MKACC_CAT(lat_dg, MKACC_TU_DG)(int method, bool first) {
    return (KernelPtr)pick_lat<MKACC_TU_DG>(method, first);
}
KernelPtr MKACC_CAT(latd_dg, MKACC_TU_DG)(int method, bool first) {
    return (KernelPtr)pick_latd<MKACC_TU_DG>(method, first);
}
KernelPtr MKACC_CAT(latdrun_dg, MKACC_TU_DG)(int method) { return pick_latd_run<MKACC_TU_DG>(method); }
KernelPtr MKACC_CAT(latrun_dg, MKACC_TU_DG)(int method) { return pick_lat_run<MKACC_TU_DG>(method); }
#elif MKACC_TU_PART == 2
KernelPtr MKACC_CAT(step2_dg, MKACC_TU_DG)(int method) { return (KernelPtr)pick_step2<MKACC_TU_DG, false>(method); }
#elif MKACC_TU_PART == 4
KernelPtr MKACC_CAT(quad_dg, MKACC_TU_DG)(int method, bool first, int occ) {
    return pick_quad<MKACC_TU_DG>(method, first, occ);
}
KernelPtr MKACC_CAT(quadrun_dg, MKACC_TU_DG)(int method, int occ) { return pick_quad_run<MKACC_TU_DG>(method, occ); }
#else
KernelPtr MKACC_CAT(step2f_dg, MKACC_TU_DG)(int method) { return (KernelPtr)pick_step2<MKACC_TU_DG, true>(method); }
#endif
}  // namespace mkacc_tu

#else
#error "mkacc_steps.hip is compiled with MKACC_TU_DG or MKACC_TU_WIDE (mkfhe_amd/build.py)"
#endif
