// Instantiations of the implicit-GEMM conv kernel: forward convolutions (EPI_STATS, optional lazy-BN prologue).
#include "conv_igemm_impl.h"

namespace fdt {
namespace conv {

bool launch_cases_fwd(int pro, int epi, int act, const ConvArgs& a, int BM, int BN, int BK, int kg, bool pure,
                      hipStream_t st) {
#define FDT_CONV_CASE(P_, E_, A_) \
  if (pro == P_ && epi == E_ && act == A_) { launch_tile<P_, E_, A_>(a, BM, BN, BK, kg, pure, st); return true; }
  FDT_CONV_CASE(kProNone, kEpiStats, kActNone)
  FDT_CONV_CASE(kProAffineAct, kEpiStats, kActRelu)
  FDT_CONV_CASE(kProAffineAct, kEpiStats, kActCelu)
  FDT_CONV_CASE(kProAffineAct, kEpiStats, kActNone)
  FDT_CONV_CASE(kProJoin, kEpiStats, kActRelu)
#undef FDT_CONV_CASE
  return false;
}

}  // namespace conv
}  // namespace fdt
