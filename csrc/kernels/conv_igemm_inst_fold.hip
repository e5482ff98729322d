// Instantiations of the implicit-GEMM conv kernel: dgrad with the BN-backward fold prologue (ACTBWD / STORE / ADD epilogues).
#include "conv_igemm_impl.h"

namespace fdt {
namespace conv {

bool launch_cases_fold(int pro, int epi, int act, const ConvArgs& a, int BM, int BN, int BK, int kg, bool pure,
                      hipStream_t st) {
#define FDT_CONV_CASE(P_, E_, A_) \
  if (pro == P_ && epi == E_ && act == A_) { launch_tile<P_, E_, A_>(a, BM, BN, BK, kg, pure, st); return true; }
  FDT_CONV_CASE(kProFold, kEpiActBwd, kActRelu)
  FDT_CONV_CASE(kProFold, kEpiActBwd, kActCelu)
  FDT_CONV_CASE(kProFold, kEpiActBwd, kActNone)
  FDT_CONV_CASE(kProFold, kEpiStore, kActNone)
  FDT_CONV_CASE(kProFold, kEpiAdd, kActNone)
#undef FDT_CONV_CASE
  return false;
}

}  // namespace conv
}  // namespace fdt
