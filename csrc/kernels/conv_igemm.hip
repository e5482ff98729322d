// Host launcher of the implicit-GEMM convolution kernels (kernel: conv_igemm_impl.h; the
// (prologue, epilogue, activation) instantiations: conv_igemm_inst_*.hip).
#include "conv_igemm_impl.h"

#include <algorithm>

namespace fdt {

// Python-facing launchers.  taps: list of (dh, dw, wt) triples encoded as int8 arrays.
static void conv_igemm_impl(uint64_t x, uint64_t x2, uint64_t ps, uint64_t pt, uint64_t pg, uint64_t w, uint64_t out,
                            uint64_t part, int part_rows, uint64_t ex, uint64_t es, uint64_t et, uint64_t jmask,
                            uint64_t jyb, uint64_t jout, long Nb, int Hi, int Wi, int Cx, int Ho, int Wo, int S,
                            const std::vector<int>& dh, const std::vector<int>& dw, const std::vector<int>& wt, int Cout,
                            int ldw, int Hout, int Wout, int OS, int oy, int ox, int pro, int pro_act, float pro_alpha,
                            int epi, int epi_act, float epi_alpha, int BM, int BN, int BK, int nsplit, uint64_t slab,
                            uint64_t cnt, uint64_t pt2, uint64_t pout, uint64_t pmask, int kg, uint64_t stream,
                            const LazyStats& ls1 = LazyStats{}, const LazyStats& ls2 = LazyStats{},
                            const std::vector<uint64_t>& jz = {}) {
  using namespace conv;
  ConvArgs a{};
  a.ls1 = ls1;
  a.ls2 = ls2;
  FDT_CHECK(!ls1.base || pro == kProAffineAct || pro == kProJoin, "lazy statistics need the affine / join prologue");
  FDT_CHECK(!ls2.base || pro == kProJoin, "lazy shortcut statistics: join prologue");
  a.pt2 = P<const float>(pt2);
  a.pout = P<bf16>(pout);
  a.pmask = P<uint8_t>(pmask);
  if (pro == kProJoin) {
    FDT_CHECK(x2 != 0 && pout != 0 && ((ps != 0 && pt != 0) || ls1.base) && (pg == 0 || pt2 != 0),
              "join prologue: y, r, s, t, out");
    FDT_CHECK(dh.size() == 1 && S == 1 && Hi == Ho && Wi == Wo, "join prologue: 1x1 stride-1 convolution only");
  }
  a.x = P<const bf16>(x);
  a.x2 = P<const bf16>(x2);
  a.ps = P<const float>(ps);
  a.pt = P<const float>(pt);
  a.pg = P<const float>(pg);
  a.w = P<const bf16>(w);
  a.out = P<bf16>(out);
  a.part = P<float>(part);
  a.ex = P<const bf16>(ex);
  a.es = P<const float>(es);
  a.et = P<const float>(et);
  a.jmask = P<const uint8_t>(jmask);
  a.jyb = P<const bf16>(jyb);
  a.jout = P<const bf16>(jout);
  FDT_CHECK(jz.empty() || (jz.size() == 3 && epi == kEpiJoinBwd), "jz = [] | [sb, tb, xid] (join backward z mode)");
  a.jsb = jz.empty() ? nullptr : P<const float>(jz[0]);
  a.jtb = jz.empty() ? nullptr : P<const float>(jz[1]);
  a.jx = jz.empty() ? nullptr : P<const bf16>(jz[2]);
  if (epi == kEpiJoinBwd) {
    const bool zm = es != 0;  // z mode: es / et = the residual branch's (s, t)
    FDT_CHECK(!zm || (epi_act == kActCelu && et != 0 && jz.size() == 3 && (jyb ? (jz[0] && jz[1]) : jz[2] != 0)),
              "join backward z mode (CELU): es, et and jz = [sb, tb] (BN'd shortcut) | [.., .., xid] (identity)");
    FDT_CHECK(ex != 0 && part != 0 && (jmask != 0 || jout != 0 || zm), "join backward needs y_res, slots and mask|out|z");
    FDT_CHECK(S == 1 && OS == 1 && Hout == Ho && Wout == Wo, "join backward needs a dense (stride-1) dgrad");
  }
  FDT_CHECK(Cx >= 8 && (Cx & (Cx - 1)) == 0, "Cx must be a power of two >= 8");
  FDT_CHECK(Cout % BN == 0, "Cout must be a multiple of BN");
  FDT_CHECK(dh.size() == dw.size() && dh.size() == wt.size() && dh.size() <= 12, "bad tap table");
  FDT_CHECK(ldw % 8 == 0, "weight row stride must be a multiple of 8");
  a.M = Nb * (long)Ho * Wo;
  a.Hi = Hi; a.Wi = Wi; a.Cx = Cx;
  a.log2Cx = 31 - __builtin_clz((unsigned)Cx);
  a.Ho = Ho; a.Wo = Wo; a.S = S;
  a.ntaps = (int)dh.size();
  a.K = a.ntaps * Cx;
  a.Cout = Cout; a.ldw = ldw;
  a.Hout = Hout; a.Wout = Wout; a.OS = OS; a.oy = oy; a.ox = ox;
  a.pro_act = pro_act; a.pro_alpha = pro_alpha;
  a.epi_act = epi_act; a.epi_alpha = epi_alpha;
  for (size_t i = 0; i < dh.size(); ++i) {
    a.dh[i] = (int8_t)dh[i];
    a.dw[i] = (int8_t)dw[i];
    a.wt[i] = (int8_t)wt[i];
  }
  a.Nb_HiWi_Cx_bytes = Nb * (long)Hi * Wi * Cx * 2;
  a.w_bytes = (long)Cout * ldw * 2;
  FDT_CHECK(a.Nb_HiWi_Cx_bytes < 0x7FFFFFF0L && a.w_bytes < 0x7FFFFFF0L && Nb * (long)Hout * Wout * Cout < 0x7FFFFFFFL,
            "conv operand exceeds the 2 GiB buffer-descriptor range");
  a.nbm = (int)((a.M + BM - 1) / BM);
  a.nbn = Cout / BN;
  a.det = deterministic() ? 1 : 0;
  a.wthru = conv_write_through() ? 1 : 0;
  a.dbg = conv_debug_flags();
  a.slot_mask = part ? stat_slot_mask(part_rows, a.nbm) : 0u;
  {
    const int nkt = (a.K + BK - 1) / BK;
    if (nsplit < 1 || nkt <= 1) nsplit = 1;
    if (nsplit > nkt && nkt >= 1) nsplit = nkt;
    a.kps = nsplit == 1 ? (nkt > 1 ? nkt : 1) : (nkt + nsplit - 1) / nsplit;
    a.nsplit = nsplit == 1 ? 1 : (nkt + a.kps - 1) / a.kps;  // no empty splits
    a.slab = P<float>(slab);
    a.cnt = P<int>(cnt);
    FDT_CHECK(a.nsplit == 1 || (slab != 0 && cnt != 0), "split-K needs a slab and a zeroed ticket buffer");
  }
  const bool pure = a.ntaps == 1 && dh[0] == 0 && dw[0] == 0 && wt[0] == 0 && S == 1 && Hi == Ho && Wi == Wo;
  hipStream_t st = as_stream(stream);
  if (a.M == 0) return;
  const int act = (pro == kProAffineAct || pro == kProJoin) ? pro_act : ((epi == kEpiActBwd || epi == kEpiJoinBwd) ? epi_act : 0);
  if (kg >= 5 && kg <= 8) {  // halo-staged 3x3 stride-1 loop (conv_h3.hip): prologue-free operands, no split-K
    FDT_CHECK(pro == kProNone && a.nsplit == 1, "kg 5-8 (halo 3x3): prologue-free, nsplit 1");
    FDT_CHECK(launch_h3(pro, epi, act, a, BM, BN, kg, st), "kg 5-8 (halo 3x3): unsupported tile / epilogue");
    return;
  }
  if (kg == 2 && a.nsplit > 1) kg = 1;  // K groups and split-K are alternatives (kg 4: rotated loop, any split)
  if (kg == 3 && pro != kProNone) kg = 1;  // the LDS-DMA ring cannot apply a prologue
  if (launch_cases_fwd(pro, epi, act, a, BM, BN, BK, kg, pure, st) ||
      launch_cases_fold(pro, epi, act, a, BM, BN, BK, kg, pure, st) ||
      launch_cases_join(pro, epi, act, a, BM, BN, BK, kg, pure, st) ||
      launch_cases_plain(pro, epi, act, a, BM, BN, BK, kg, pure, st) ||
      launch_cases_ffn(pro, epi, act, a, BM, BN, BK, kg, pure, st))
    return;
  FDT_CHECK(false, "unsupported (prologue, epilogue) combination");
}

void conv_igemm(uint64_t x, uint64_t x2, uint64_t ps, uint64_t pt, uint64_t pg, uint64_t w, uint64_t out, uint64_t part,
                int part_rows, uint64_t ex, uint64_t es, uint64_t et, uint64_t jmask, uint64_t jyb, uint64_t jout, long Nb, int Hi,
                int Wi, int Cx, int Ho, int Wo, int S,
                const std::vector<int>& dh, const std::vector<int>& dw, const std::vector<int>& wt, int Cout, int ldw,
                int Hout, int Wout, int OS, int oy, int ox, int pro, int pro_act, float pro_alpha, int epi, int epi_act,
                float epi_alpha, int BM, int BN, int BK, int nsplit, uint64_t slab, uint64_t cnt, int kg,
                uint64_t stream, const std::vector<uint64_t>& lz_ptr, const std::vector<double>& lz_val,
                const std::vector<uint64_t>& jz) {
  FDT_CHECK(pro != conv::kProJoin, "the join prologue goes through conv_igemm_join");
  conv_igemm_impl(x, x2, ps, pt, pg, w, out, part, part_rows, ex, es, et, jmask, jyb, jout, Nb, Hi, Wi, Cx, Ho, Wo, S, dh,
                  dw, wt, Cout, ldw, Hout, Wout, OS, oy, ox, pro, pro_act, pro_alpha, epi, epi_act, epi_alpha, BM, BN, BK,
                  nsplit, slab, cnt, 0, 0, 0, kg, stream, make_lazy(lz_ptr, lz_val), LazyStats{}, jz);
}

// Forward 1x1 convolution whose operand is the previous residual block's join (PRO_JOIN):
// y (its BN'd residual branch), r (shortcut: identity or BN'd by s2/t2), join output + ReLU
// mask stored on the way.
void conv_igemm_join(uint64_t y, uint64_t r, uint64_t s, uint64_t t, uint64_t s2, uint64_t t2, uint64_t w, uint64_t out,
                     uint64_t part, int part_rows, uint64_t jout, uint64_t jmask, long Nb, int H, int W, int Cx, int Cout,
                     int ldw, int BM, int BN, int BK, int nsplit, uint64_t slab, uint64_t cnt, int kg,
                     uint64_t stream, const std::vector<uint64_t>& lz1_ptr, const std::vector<double>& lz1_val,
                     const std::vector<uint64_t>& lz2_ptr, const std::vector<double>& lz2_val) {
  const std::vector<int> z{0};
  conv_igemm_impl(y, r, s, t, s2, w, out, part, part_rows, 0, 0, 0, 0, 0, 0, Nb, H, W, Cx, H, W, 1, z, z, z, Cout, ldw, H,
                  W, 1, 0, 0, conv::kProJoin, kActRelu, 1.f, conv::kEpiStats, 0, 1.f, BM, BN, BK, nsplit, slab, cnt, t2,
                  jout, jmask, kg, stream, make_lazy(lz1_ptr, lz1_val), make_lazy(lz2_ptr, lz2_val));
}

// Transformer FFN GEMMs on the implicit-GEMM kernel (a token GEMM is a 1x1 convolution over
// M "pixels"): out[M][N] = x[M][K] W[N][K]^T with
//   epi 5 (GELU_FWD): out = a = acc + bias[N] (bf16), out2 = h = dropout(gelu(a))
//   epi 6 (GELU_BWD): out = ga = keep*scale*gelu'(a_in)*acc, gb[N] += column sums of ga
// K must be a power of two >= 8 (d_model), N a multiple of BN.
void ffn_gemm(uint64_t x, uint64_t w, uint64_t out, long M, int K, int N, int epi, uint64_t bias, uint64_t out2,
              uint64_t a_in, uint64_t gb, float p, uint64_t seed, uint64_t seed_ptr, int BM, int BN, int BK, int kg,
              uint64_t stream) {
  using namespace conv;
  FDT_CHECK(epi == kEpiGeluFwd || epi == kEpiGeluBwd, "ffn_gemm: epi 5 (GELU_FWD) | 6 (GELU_BWD)");
  FDT_CHECK(epi != kEpiGeluFwd || (bias != 0 && out2 != 0), "GELU_FWD needs bias and the h output");
  FDT_CHECK(epi != kEpiGeluBwd || (a_in != 0 && gb != 0), "GELU_BWD needs a and the bias-gradient buffer");
  FDT_CHECK(p >= 0.f && p < 1.f, "dropout p in [0, 1)");
  FDT_CHECK(x % 16 == 0 && w % 16 == 0 && out % 16 == 0 && out2 % 16 == 0 && a_in % 16 == 0 && bias % 16 == 0,
            "ffn_gemm: 16-B aligned operands");
  ConvArgs a{};
  a.x = P<const bf16>(x);
  a.w = P<const bf16>(w);
  a.out = P<bf16>(out);
  a.ex = P<const bf16>(a_in);
  a.fbias = P<const float>(bias);
  a.out2 = P<bf16>(out2);
  a.gb = P<float>(gb);
  a.drop_thr = (uint32_t)std::min((double)p * 4294967296.0, 4294967295.0);
  a.drop_scale = 1.f / (1.f - p);
  a.drop_seed = seed;
  a.drop_seed_ptr = P<const uint64_t>(seed_ptr);
  FDT_CHECK(K >= 8 && (K & (K - 1)) == 0, "ffn_gemm: K must be a power of two >= 8");
  FDT_CHECK(N % BN == 0 && N % 8 == 0, "ffn_gemm: N must be a multiple of BN");
  a.M = M;
  a.Hi = a.Wi = a.Ho = a.Wo = a.Hout = a.Wout = 1;
  a.Cx = K;
  a.log2Cx = 31 - __builtin_clz((unsigned)K);
  a.S = a.OS = 1;
  a.ntaps = 1;
  a.K = K;
  a.Cout = N;
  a.ldw = K;
  a.Nb_HiWi_Cx_bytes = M * (long)K * 2;
  a.w_bytes = (long)N * K * 2;
  FDT_CHECK(a.Nb_HiWi_Cx_bytes < 0x7FFFFFF0L && M * (long)N < 0x7FFFFFFFL, "ffn_gemm: operand exceeds 2 GiB");
  a.nbm = (int)((M + BM - 1) / BM);
  a.nbn = N / BN;
  a.nsplit = 1;
  a.kps = (K + BK - 1) / BK;
  if (M == 0) return;
  if (launch_cases_ffn(kProNone, epi, kActNone, a, BM, BN, BK, kg, true, as_stream(stream))) return;
  FDT_CHECK(false, "ffn_gemm: no instantiation");
}

int conv_num_row_blocks(long M, int BM) { return (int)((M + BM - 1) / BM); }

void set_conv_write_through(bool on) { conv_write_through_flag() = on ? 1 : 0; }
void set_conv_debug_flags(int f) { conv_debug_flags_ref() = f; }

// split-K workspace sizes for a launch: (slab floats, ticket ints)
std::vector<long> conv_splitk_workspace(long M, int Cout, int BM, int BN, int nsplit) {
  const long tiles = ((M + BM - 1) / BM) * (long)(Cout / BN);
  return {tiles * nsplit * (BM / 64) * (BN / 64) * 16L * 256L, tiles};
}

}  // namespace fdt
