// Fused optimizer step + conv weight repack: ONE launch updates the whole flat parameter buffer
// and writes the packed bf16 layouts the implicit-GEMM convolutions read (forward wf[co][t][ci],
// dgrad wd[ci][t][co], pack_layout.h) straight from the freshly updated weights -- the separate
// pack_weights pass at the start of every forward (a read of all 23.5M fp32 conv weights and
// a write of both bf16 layouts, ~50 us at ResNet-50) disappears.
//
// Grid: [conv blocks | rest blocks]; the caller splits a model into two launches (1x1 weights +
// the rest ranges at a 4 KB LDS image, then the 3x3 / 2x2 weights at 38 KB).  A conv block owns one 32 (co) x 64 (ci) x T slice of one
// conv weight (the repack's blocking): it applies the update rule (optim_ops.h, bitwise the
// flat kernels' math) to each of its elements in flat (OIHW) order -- coalesced reads and writes
// of p / g / state -- stages the new values as bf16 in LDS and stores both packed layouts.  The
// rest blocks grid-stride over the remaining flat ranges (BN affine parameters, the classifier,
// alignment padding) with the plain per-element update.  A skipped step (found_inf) only clears
// the gradient: weights and their packed copies are unchanged.
#include "common.h"
#include "optim_ops.h"
#include "pack_layout.h"

namespace fdt {

namespace {

struct PackUpdEntry {  // int64 fields: filled from a torch int64 tensor (ops/conv_igemm.py)
  long off;            // element offset of the OIHW weight in the flat buffer
  long wf, wd;         // packed layouts (wd 0: forward layout only, e.g. the stem)
  long cout, cin, cxp, ntaps;
  long blk0;           // first block of this entry
};

struct RestRange {
  long start, len, cum;  // flat range and its first virtual index
};

template <int T, class Op>
__device__ __forceinline__ void update_block(const Op& op, const PackUpdEntry& E, int b, bf16* img) {
  const int Cout = (int)E.cout, Cin = (int)E.cin, Cxp = (int)E.cxp;
  const pack::Block k = pack::block_of(b, Cout, Cin, Cxp);
  constexpr int run = pack::kT * T;
  const long base = E.off + ((long)k.co0 * Cin + k.ci0) * T;
  // U elements per thread per trip, all their loads issued first: a block owns up to 18432
  // elements (3x3) and the LDS image limits residency to 4 blocks per CU
  constexpr int U = 4;
  const int total = k.nco * run;
  for (int e0 = threadIdx.x; e0 < total; e0 += blockDim.x * U) {
    long idx[U];
    bool ok[U];
    int slot[U];
    float v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int e = e0 + u * (int)blockDim.x;
      const int col = e / run, rem = e - col * run;
      const int cl = rem / T, t = rem - cl * T;
      ok[u] = e < total && cl < k.nci_s;
      idx[u] = base + (long)col * Cin * T + rem;
      slot[u] = e < total ? (col * T + t) * pack::kLd + cl : -1;
    }
    op.template apply<U>(idx, ok, v);
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (slot[u] >= 0) img[slot[u]] = __float2bfloat16(v[u]);
  }
  __syncthreads();
  pack::store_layouts<T>(img, k, reinterpret_cast<bf16*>(E.wf), reinterpret_cast<bf16*>(E.wd), Cout, Cxp);
}

// MAXT: the largest tap count among the launch's entries -- the LDS image is sized for it, so the
// 1x1 weights (most of the blocks) run as their own launch at 9x less LDS (more resident blocks)
template <class Op, class Args, int MAXT>
__global__ __launch_bounds__(256) void pack_update_kernel(const Args args, long n,
                                                          const PackUpdEntry* __restrict__ tab, int ntab,
                                                          long nblk_pack, const RestRange* __restrict__ rr, int nrr,
                                                          long rest_total) {
  if (Op::skipped(args)) {
    Op::on_skip(args, n);
    return;
  }
  const Op op(args);
  __shared__ bf16 img[pack::kCo * MAXT * pack::kLd];
  const long bid = blockIdx.x;
  if (bid < nblk_pack) {
    int lo = 0, hi = ntab - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (tab[mid].blk0 <= bid) lo = mid;
      else hi = mid - 1;
    }
    const PackUpdEntry E = tab[lo];
    const int b = (int)(bid - E.blk0);
    if constexpr (MAXT == 1) {
      update_block<1>(op, E, b, img);
    } else {
      if (E.ntaps == 1) update_block<1>(op, E, b, img);
      else if (E.ntaps == 9) update_block<9>(op, E, b, img);
      else update_block<4>(op, E, b, img);  // the table builder admits ntaps in {1, 4, 9}
    }
    return;
  }
  const long nb = (long)gridDim.x - nblk_pack;
  for (long v = (bid - nblk_pack) * blockDim.x + threadIdx.x; v < rest_total; v += nb * blockDim.x) {
    int lo = 0, hi = nrr - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (rr[mid].cum <= v) lo = mid;
      else hi = mid - 1;
    }
    op(rr[lo].start + (v - rr[lo].cum));
  }
}

struct PackPlan {
  const PackUpdEntry* tab;
  int ntab;
  long nblk_pack;
  const RestRange* rr;
  int nrr;
  long rest_total;
  dim3 grid() const {
    long rest_blocks = (rest_total + 255) / 256;
    rest_blocks = rest_blocks < 1 ? 1 : (rest_blocks > 1024 ? 1024 : rest_blocks);
    return dim3((unsigned)(nblk_pack + rest_blocks));
  }
};

PackPlan pack_plan(uint64_t tab, int ntab, long nblk_pack, uint64_t rr, int nrr, long rest_total) {
  FDT_CHECK((tab != 0 && ntab >= 1 && nblk_pack >= 1) || (ntab == 0 && nblk_pack == 0), "pack-update table");
  FDT_CHECK(rest_total == 0 || (rr != 0 && nrr >= 1), "pack-update rest ranges");
  FDT_CHECK(nblk_pack + 1024 < (1L << 31), "pack-update grid");
  return PackPlan{P<const PackUpdEntry>(tab), ntab, nblk_pack, P<const RestRange>(rr), nrr, rest_total};
}

}  // namespace

void madgrad_pack_step(uint64_t p, uint64_t g, uint64_t gss, uint64_t s, uint64_t x0, uint64_t shadow, long n,
                       float lr, float momentum, float wd, float eps, int decouple, long k, uint64_t kskip,
                       uint64_t gsc, uint64_t found_inf, int zero_grad, uint64_t tab, int ntab, long nblk_pack,
                       uint64_t rr, int nrr, long rest_total, int maxt, int count_skips, uint64_t stream) {
  FDT_CHECK(momentum == 0.f || x0 != 0, "x0 buffer required with momentum");
  FDT_CHECK(maxt == 1 || maxt == 9, "pack-update: maxt 1 or 9");
  const PackPlan pl = pack_plan(tab, ntab, nblk_pack, rr, nrr, rest_total);
  const opt::MadArgs a{P<float>(p), P<float>(g), P<float>(gss), P<float>(s), P<float>(x0), P<bf16>(shadow),
                       lr, momentum, wd, eps, decouple, k, P<int>(kskip), P<const float>(gsc),
                       P<const int>(found_inf), zero_grad, count_skips};
  if (maxt == 1)
    hipLaunchKernelGGL((pack_update_kernel<opt::MadOp, opt::MadArgs, 1>), pl.grid(), dim3(256), 0, as_stream(stream),
                       a, n, pl.tab, pl.ntab, pl.nblk_pack, pl.rr, pl.nrr, pl.rest_total);
  else
    hipLaunchKernelGGL((pack_update_kernel<opt::MadOp, opt::MadArgs, 9>), pl.grid(), dim3(256), 0, as_stream(stream),
                       a, n, pl.tab, pl.ntab, pl.nblk_pack, pl.rr, pl.nrr, pl.rest_total);
  FDT_LAUNCH_CHECK();
}

void sgd_pack_step(uint64_t p, uint64_t g, uint64_t buf, uint64_t shadow, long n, float lr, float momentum,
                   float dampening, float wd, int nesterov, int first, uint64_t gsc, uint64_t found_inf,
                   int zero_grad, uint64_t lr_dev, uint64_t tab, int ntab, long nblk_pack, uint64_t rr, int nrr,
                   long rest_total, int maxt, int count_skips, uint64_t stream) {
  (void)count_skips;  // SGD keeps no step counter
  FDT_CHECK(momentum == 0.f || buf != 0, "momentum buffer required");
  FDT_CHECK(maxt == 1 || maxt == 9, "pack-update: maxt 1 or 9");
  const PackPlan pl = pack_plan(tab, ntab, nblk_pack, rr, nrr, rest_total);
  const opt::SgdArgs a{P<float>(p), P<float>(g), P<float>(buf), P<bf16>(shadow), lr, momentum, dampening, wd,
                       nesterov, first, P<const float>(gsc), P<const int>(found_inf), zero_grad,
                       P<const float>(lr_dev)};
  if (maxt == 1)
    hipLaunchKernelGGL((pack_update_kernel<opt::SgdOp, opt::SgdArgs, 1>), pl.grid(), dim3(256), 0, as_stream(stream),
                       a, n, pl.tab, pl.ntab, pl.nblk_pack, pl.rr, pl.nrr, pl.rest_total);
  else
    hipLaunchKernelGGL((pack_update_kernel<opt::SgdOp, opt::SgdArgs, 9>), pl.grid(), dim3(256), 0, as_stream(stream),
                       a, n, pl.tab, pl.ntab, pl.nblk_pack, pl.rr, pl.nrr, pl.rest_total);
  FDT_LAUNCH_CHECK();
}

}  // namespace fdt
