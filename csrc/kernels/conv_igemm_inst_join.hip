// Instantiations of the implicit-GEMM conv kernel: the dgrad that completes a residual block's output gradient + its join backward.
#include "conv_igemm_impl.h"

namespace fdt {
namespace conv {

bool launch_cases_join(int pro, int epi, int act, const ConvArgs& a, int BM, int BN, int BK, int kg, bool pure,
                      hipStream_t st) {
#define FDT_CONV_CASE(P_, E_, A_) \
  if (pro == P_ && epi == E_ && act == A_) { launch_tile<P_, E_, A_>(a, BM, BN, BK, kg, pure, st); return true; }
  FDT_CONV_CASE(kProFold, kEpiJoinBwd, kActRelu)
  FDT_CONV_CASE(kProFold, kEpiJoinBwd, kActCelu)
#undef FDT_CONV_CASE
  return false;
}

}  // namespace conv
}  // namespace fdt
