// tfg_fused_f64.hip -- the fp64 ("exact") engine's instantiations of the fused
// multi-step kernel k_fused<double, true, ...> (tfg_fused.hpp) and their launch.
//
// This translation unit is compiled with machine-level loop-invariant code
// motion off (-mllvm -disable-machine-licm; __graft_entry__.py).  With it on,
// the compiler hoists the fp64 libm polynomial constants and plane addresses
// of the step out of the step loop; the fp64 step then holds 242 VGPRs (2
// waves per SIMD) and spills 111 SGPRs into VGPR lanes.  With it off: 120
// VGPRs, 4 waves per SIMD, 77 SGPR spills, and 4096^2 x 192-step launches of
// 174.9 ms against 198.7-199.5 ms (same-box A/B, scripts/gpu_ab_all.sh).  The
// fp32 kernel runs 2 % slower without the code motion, so it stays in
// tfg_engine.hip with the default flags.  Same arithmetic either way: the
// results are bit for bit those of the same source under the default flags.
#include "tfg_fused.hpp"

namespace tfg_kern {

hipError_t launch_fused_exact(const KArgs& a, const FusedBufs& b, bool read_depths, bool catchments, bool qc_on,
                              int blocks, size_t lds, hipStream_t stream) {
  constexpr int C = kCellsPerThread;
#define TFG_ARGS a, b.uni, static_cast<const double*>(b.forc), static_cast<const double*>(b.stat), b.geo, b.catch_id, \
                 b.st, b.tot, b.ring, static_cast<double*>(b.hist), b.slab, static_cast<const double*>(b.qc)
#define TFG_LAUNCH(RD, CT, QC) \
  hipLaunchKernelGGL((k_fused<double, true, RD, CT, QC, C>), blocks, kBlock, lds, stream, TFG_ARGS)
  if (qc_on) {
    if (read_depths && catchments) TFG_LAUNCH(true, true, true);
    else if (read_depths) TFG_LAUNCH(true, false, true);
    else if (catchments) TFG_LAUNCH(false, true, true);
    else TFG_LAUNCH(false, false, true);
  } else {
    if (read_depths && catchments) TFG_LAUNCH(true, true, false);
    else if (read_depths) TFG_LAUNCH(true, false, false);
    else if (catchments) TFG_LAUNCH(false, true, false);
    else TFG_LAUNCH(false, false, false);
  }
#undef TFG_LAUNCH
#undef TFG_ARGS
  return hipGetLastError();
}

}  // namespace tfg_kern
