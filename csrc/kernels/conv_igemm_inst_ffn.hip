// Instantiations of the implicit-GEMM kernel used as the transformer FFN GEMM (1x1 "conv" over
// tokens): the bias + GELU + dropout forward epilogue and the GELU-dropout backward epilogue.
#include "conv_igemm_impl.h"

namespace fdt {
namespace conv {

bool launch_cases_ffn(int pro, int epi, int act, const ConvArgs& a, int BM, int BN, int BK, int kg, bool pure,
                      hipStream_t st) {
  if (pro != kProNone || act != kActNone) return false;
  FDT_CHECK(!(epi == kEpiGeluFwd || epi == kEpiGeluBwd) || pure, "FFN epilogues: dense token GEMM only");
  if (epi == kEpiGeluFwd) { launch_tile<kProNone, kEpiGeluFwd, kActNone>(a, BM, BN, BK, kg, true, st); return true; }
  if (epi == kEpiGeluBwd) { launch_tile<kProNone, kEpiGeluBwd, kActNone>(a, BM, BN, BK, kg, true, st); return true; }
  return false;
}

}  // namespace conv
}  // namespace fdt
