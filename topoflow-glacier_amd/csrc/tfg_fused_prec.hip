// tfg_fused_prec.hip -- the fp32 engine's fp64-flux form (tfg_set_flux(h,
// TFG_FLUX_F64)): the instantiations k_fused<float, false, ..., PREC = true>
// (tfg_fused.hpp, tfg::cell_step_fast) and their launch.  Its own translation
// unit so that the library's units still compile side by side (build()).
#include "tfg_fused.hpp"

namespace tfg_kern {

hipError_t launch_fused_prec(const KArgs& a, const FusedBufs& b, bool read_depths, bool catchments, bool qc_on,
                             bool nan_safe, int blocks, size_t lds, hipStream_t stream) {
  constexpr int C = kCellsPerThread;
#define TFG_ARGS a, b.uni, static_cast<const float*>(b.forc), static_cast<const float*>(b.stat), b.geo, b.catch_id, \
                 b.st, b.tot, b.ring, static_cast<float*>(b.hist), b.slab, static_cast<const float*>(b.qc)
#define TFG_LAUNCH(RD, CT, QC, NS) \
  hipLaunchKernelGGL((k_fused<float, false, RD, CT, QC, C, NS, true>), blocks, kBlock, lds, stream, TFG_ARGS)
#define TFG_LAUNCH_NS(RD, CT, QC) \
  do { if (nan_safe) TFG_LAUNCH(RD, CT, QC, true); else TFG_LAUNCH(RD, CT, QC, false); } while (0)
  if (qc_on) {
    if (read_depths && catchments) TFG_LAUNCH_NS(true, true, true);
    else if (read_depths) TFG_LAUNCH_NS(true, false, true);
    else if (catchments) TFG_LAUNCH_NS(false, true, true);
    else TFG_LAUNCH_NS(false, false, true);
  } else {
    if (read_depths && catchments) TFG_LAUNCH_NS(true, true, false);
    else if (read_depths) TFG_LAUNCH_NS(true, false, false);
    else if (catchments) TFG_LAUNCH_NS(false, true, false);
    else TFG_LAUNCH_NS(false, false, false);
  }
#undef TFG_LAUNCH_NS
#undef TFG_LAUNCH
#undef TFG_ARGS
  return hipGetLastError();
}

}  // namespace tfg_kern
