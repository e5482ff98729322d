// Host-side launcher prototypes of every HIP kernel in csrc/kernels/*.hip.
// All pointers are device addresses passed as uint64_t (tensor.data_ptr()), `stream`
// is the raw hipStream_t of the current torch stream; launchers are asynchronous,
// allocation-free and graph-capture safe.
#pragma once
#include <cstdint>
#include <vector>

namespace fdt {
// bn_kernels.hip
void act_affine_fwd(uint64_t x, uint64_t s, uint64_t t, uint64_t out, long M, int C, int act, float alpha, int dt_in,
                    int dt_out, uint64_t stream);
int stats_num_blocks(long M, int C);
void set_ew_unroll(bool on);
void channel_stats_partial(uint64_t y, uint64_t part, long M, int C, int dt, uint64_t stream);
void stats_finalize(uint64_t part, int nb, int C, double count, int mode, float eps, float momentum, uint64_t gamma,
                    uint64_t beta, uint64_t run_mean, uint64_t run_var, uint64_t nbt, uint64_t out_s, uint64_t out_t,
                    uint64_t save_mean, uint64_t save_aux, int zero_after, uint64_t stream);
void act_bwd_reduce(uint64_t g, uint64_t x, uint64_t s, uint64_t t, uint64_t gx, uint64_t part, int part_rows, long M,
                    int C, int act, float alpha, int dt, uint64_t stream);
void reduce_partials(uint64_t part, int nb, int nq, int C, uint64_t out, int zero_after, uint64_t stream);
int partials_compact(uint64_t part, int nb, int W, int R, uint64_t out, uint64_t stream);
void stats_bwd_coef(uint64_t gs, uint64_t gt, int C, double count, int mode, float eps, uint64_t save_mean,
                    uint64_t save_aux, uint64_t gamma, uint64_t alpha, uint64_t beta, uint64_t ggamma, uint64_t gbeta,
                    uint64_t stream);
void stats_bwd_finalize(uint64_t part, int nb, int nq, int C, int a_mode, float a_eps, double a_count, uint64_t a_sm,
                        uint64_t a_sa, uint64_t a_gamma, uint64_t a_alpha, uint64_t a_beta, uint64_t a_gg,
                        uint64_t a_gb, int b_mode, float b_eps, double b_count, uint64_t b_sm, uint64_t b_sa,
                        uint64_t b_gamma, uint64_t b_alpha, uint64_t b_beta, uint64_t b_gg, uint64_t b_gb,
                        uint64_t stream);
void affine_fold(uint64_t gy, uint64_t y, uint64_t alpha, uint64_t beta, uint64_t gs, uint64_t out, long M, int C,
                 int dt, uint64_t stream);
void residual_act_fwd(uint64_t ya, uint64_t sa, uint64_t ta, uint64_t yb, uint64_t sb, uint64_t tb, uint64_t xid,
                      uint64_t out, uint64_t mask, long M, int C, int act, float alpha, int dt, uint64_t stream);
// lazy-statistics consumers (bn_math.h LazyStats): the producer's finalize runs inside them
void act_affine_lazy(uint64_t x, const std::vector<uint64_t>& lz_ptr, const std::vector<double>& lz_val, uint64_t out,
                     long M, int C, int act, float alpha, int dt, uint64_t stream);
void residual_act_lazy(uint64_t ya, const std::vector<uint64_t>& la_ptr, const std::vector<double>& la_val,
                       uint64_t yb, const std::vector<uint64_t>& lb_ptr, const std::vector<double>& lb_val,
                       uint64_t sb, uint64_t tb, uint64_t xid, uint64_t out, uint64_t mask, long M, int C, int act,
                       float alpha, int dt, uint64_t stream);
void residual_act_bwd(uint64_t g, uint64_t out, uint64_t mask, uint64_t ya, uint64_t yb, uint64_t gpre, uint64_t part,
                      int part_rows, long M, int C, int act, float alpha, int dt, uint64_t stream, int ghw,
                      const std::vector<uint64_t>& jz);
// deterministic mode (common.h): no-wrap statistics slots, ordered split-K sums
void set_deterministic_mode(bool on);
bool deterministic_mode();
// optim.hip
void grad_sumsq(uint64_t g, long n, uint64_t inv_scale, int unscale, uint64_t part, int nb, uint64_t found_inf,
                uint64_t stream);
// halo-staged 3x3 stride-1 weight gradient into per-split fp32 slabs [nsplit][Cout][9*Cx]
// (conv_wh3.hip; wgrad_reduce combines them)
void conv_wgrad_h3(uint64_t g, uint64_t x, uint64_t slab, int N, int H, int W, int Cx, int Cout, int BMC, int BNC,
                   int nsplit, int pipe, uint64_t stream);
// test aid: fill every CU's LDS with a NaN pattern (conv_h3.hip)
void lds_poison(uint64_t sink, int nblocks, uint64_t stream);
void grad_norm_finalize(uint64_t part, int nb, float max_norm, uint64_t out, uint64_t total, int phase,
                        uint64_t stream);
void sgd_step(uint64_t p, uint64_t g, uint64_t buf, uint64_t shadow, long n, float lr, float momentum, float dampening,
              float wd, int nesterov, int first, uint64_t gsc, uint64_t found_inf, int zero_grad, uint64_t lr_dev, uint64_t stream);
void madgrad_step(uint64_t p, uint64_t g, uint64_t gss, uint64_t s, uint64_t x0, uint64_t shadow, long n, float lr,
                  float momentum, float wd, float eps, int decouple, long k, uint64_t kskip, uint64_t gsc,
                  uint64_t found_inf, int zero_grad, uint64_t stream);
void mirror_madgrad_step(uint64_t p, uint64_t g, uint64_t gss, uint64_t z, uint64_t shadow, long n, float lr,
                         float momentum, float wd, float eps, int decouple, long k, uint64_t kskip, uint64_t gsc,
                         uint64_t found_inf, int zero_grad, uint64_t stream);
void adam_step(uint64_t p, uint64_t g, uint64_t m, uint64_t v, uint64_t shadow, long n, float lr, float b1, float b2,
               float eps, float wd, int adamw, long step, uint64_t kskip, uint64_t gsc, uint64_t found_inf,
               int zero_grad, uint64_t stream);
void cast_bf16(uint64_t x, uint64_t y, long n, uint64_t stream);
// fused optimizer step + conv weight repack (optim_pack.hip): tab = int64 [ntab, 8] entries
// (flat offset, wf, wd, Cout, Cin, Cxp, ntaps, first block), rr = int64 [nrr, 3] rest ranges
void madgrad_pack_step(uint64_t p, uint64_t g, uint64_t gss, uint64_t s, uint64_t x0, uint64_t shadow, long n,
                       float lr, float momentum, float wd, float eps, int decouple, long k, uint64_t kskip,
                       uint64_t gsc, uint64_t found_inf, int zero_grad, uint64_t tab, int ntab, long nblk_pack,
                       uint64_t rr, int nrr, long rest_total, int maxt, int count_skips, uint64_t stream);
void sgd_pack_step(uint64_t p, uint64_t g, uint64_t buf, uint64_t shadow, long n, float lr, float momentum,
                   float dampening, float wd, int nesterov, int first, uint64_t gsc, uint64_t found_inf,
                   int zero_grad, uint64_t lr_dev, uint64_t tab, int ntab, long nblk_pack, uint64_t rr, int nrr,
                   long rest_total, int maxt, int count_skips, uint64_t stream);
// head.hip
void head_fwd(uint64_t h, uint64_t W, uint64_t b, uint64_t pooled, uint64_t logits, int N, int HW, int C, int K,
              uint64_t stream);
void head_bwd(uint64_t dl, uint64_t W, uint64_t pooled, uint64_t dpool, uint64_t gW, uint64_t gb, int N, int HW,
              int C, int K, uint64_t stream);
// mixup.hip
void mixup_fwd(uint64_t x, uint64_t perm, uint64_t lam, uint64_t out, int b, long inner, int dt, uint64_t stream);
void mixup_bwd(uint64_t g, uint64_t x, uint64_t perm, uint64_t inv, uint64_t lam, uint64_t gx, uint64_t dlam, int b,
               long inner, int dt, uint64_t stream);
void mixup_ce_fwd(uint64_t logits, uint64_t ya, uint64_t yb, uint64_t lam, float lam_s, uint64_t loss, uint64_t glog,
                  uint64_t dlam, uint64_t meter, int B, int C, int dt, int labels64, uint64_t stream);
void mixup_prep(uint64_t y, int b, float lam, uint64_t seed, uint64_t perm, uint64_t yb, uint64_t lam_vec,
                uint64_t stream);
// layernorm.hip
void layernorm_fwd(uint64_t x, uint64_t a, uint64_t b, uint64_t y, uint64_t mean, uint64_t rstd, long rows, int d,
                   float eps, int dt_x, int dt_y, int dt_w, uint64_t stream);
void layernorm_bwd(uint64_t gy, uint64_t x, uint64_t a, uint64_t mean, uint64_t rstd, uint64_t gx, uint64_t gres,
                   uint64_t part, long rows, int d, int nblk, int dt_g, int dt_x, int dt_w, float eps, uint64_t stream);
// embedding.hip
void embedding_fwd(uint64_t ids, uint64_t types, uint64_t pos_ids, uint64_t tok, uint64_t pos, uint64_t seg,
                   uint64_t out, int B, int L, int d, float scale, int vt, int vp, int vs, uint64_t stream);
void embedding_bwd(uint64_t g, uint64_t ids, uint64_t types, uint64_t pos_ids, uint64_t gt, uint64_t gp, uint64_t gs,
                   int B, int L, int d, float scale, int vt, int vp, int vs, uint64_t stream);
// mlp.hip
void bias_relu_fwd(uint64_t pre, uint64_t b, uint64_t act, long rows, int cols, int dt, uint64_t stream);
void colsum_bf16(uint64_t x, uint64_t out, long rows, int cols, long ld, uint64_t stream);
void slab_sum_acc(uint64_t src, uint64_t dst, int s, long ld, long n, uint64_t stream);
void relu_bwd_colsum(uint64_t gact, uint64_t pre, uint64_t gpre, uint64_t gb, long rows, int cols, int dt,
                     uint64_t stream);
// augment.hip
void augment(uint64_t src, uint64_t idx, uint64_t labels_src, uint64_t labels_out, uint64_t out, int B, int H, int W,
             int C, int Cout, int pad, int do_flip, uint64_t rng, float m0, float m1, float m2, float s0, float s1,
             float s2, int nchw, int pad_norm, int dt_out, uint64_t stream);
void rng_advance(uint64_t rng, uint64_t stream);
// conv_igemm.hip
void conv_igemm(uint64_t x, uint64_t x2, uint64_t ps, uint64_t pt, uint64_t pg, uint64_t w, uint64_t out, uint64_t part,
                int part_rows, uint64_t ex, uint64_t es, uint64_t et, uint64_t jmask, uint64_t jyb, uint64_t jout, long Nb, int Hi,
                int Wi, int Cx, int Ho, int Wo, int S, const std::vector<int>& dh, const std::vector<int>& dw,
                const std::vector<int>& wt, int Cout, int ldw, int Hout, int Wout, int OS, int oy, int ox, int pro,
                int pro_act, float pro_alpha, int epi, int epi_act, float epi_alpha, int BM, int BN, int BK, int nsplit,
                uint64_t slab, uint64_t cnt, int kg, uint64_t stream, const std::vector<uint64_t>& lz_ptr,
                const std::vector<double>& lz_val, const std::vector<uint64_t>& jz);
void conv_igemm_join(uint64_t y, uint64_t r, uint64_t s, uint64_t t, uint64_t s2, uint64_t t2, uint64_t w, uint64_t out,
                     uint64_t part, int part_rows, uint64_t jout, uint64_t jmask, long Nb, int H, int W, int Cx, int Cout,
                     int ldw, int BM, int BN, int BK, int nsplit, uint64_t slab, uint64_t cnt, int kg, uint64_t stream,
                     const std::vector<uint64_t>& lz1_ptr, const std::vector<double>& lz1_val,
                     const std::vector<uint64_t>& lz2_ptr, const std::vector<double>& lz2_val);
void ffn_gemm(uint64_t x, uint64_t w, uint64_t out, long M, int K, int N, int epi, uint64_t bias, uint64_t out2,
              uint64_t a_in, uint64_t gb, float p, uint64_t seed, uint64_t seed_ptr, int BM, int BN, int BK, int kg,
              uint64_t stream);
int conv_num_row_blocks(long M, int BM);
void set_conv_write_through(bool on);
void set_conv_debug_flags(int f);
std::vector<long> conv_splitk_workspace(long M, int Cout, int BM, int BN, int nsplit);
// conv_wgrad.hip
void conv_wgrad(uint64_t g, uint64_t y, uint64_t al, uint64_t be, uint64_t gs, uint64_t x, uint64_t xs, uint64_t xt,
                uint64_t slab,
                long Nb, int Hi, int Wi, int Cx, int Ho, int Wo, int S, const std::vector<int>& dh,
                const std::vector<int>& dw, int Cout, int ldw, int act, float act_alpha, int BM, int BN, int BK,
                int nsplit, int direct, int stages, uint64_t out, uint64_t cnt, int Cin, int accumulate,
                uint64_t stream);
void wgrad_reduce(uint64_t slab, uint64_t out, int nsplit, int Cout, int Cin, int ntaps, int Cxp, int accumulate,
                  uint64_t stream);
void pack_weights(const std::vector<uint64_t>& src, const std::vector<uint64_t>& wf, const std::vector<uint64_t>& wd,
                  const std::vector<int>& cout, const std::vector<int>& cin, const std::vector<int>& cxp,
                  const std::vector<int>& ntaps, uint64_t stream);
// eigh.hip
void jacobi_eigh(uint64_t A, uint64_t w, uint64_t V, uint64_t table, int batch, int n, int max_sweeps, float tol, uint64_t stream);
// attention.hip
void attn_fwd(uint64_t q, uint64_t k, uint64_t v, const std::vector<long>& strides, uint64_t out, uint64_t lse,
              uint64_t mask, int B, int L, int H, float fill, float p_drop, uint64_t seed, uint64_t seed_ptr,
              uint64_t stream);
void attn_bwd(uint64_t q, uint64_t k, uint64_t v, const std::vector<long>& strides, uint64_t o, uint64_t dout,
              uint64_t lse, uint64_t delta, uint64_t mask, uint64_t dq, uint64_t dk, uint64_t dv, int B, int L, int H,
              float fill, float p_drop, uint64_t seed, uint64_t seed_ptr, long grad_ld, uint64_t stream);
// dropout.hip
void dropout_add_fwd(uint64_t y, uint64_t x, uint64_t out, long n, float p, uint64_t seed, uint64_t seed_ptr,
                     uint64_t stream);
void dropout_bwd(uint64_t g, uint64_t gy, long n, float p, uint64_t seed, uint64_t seed_ptr, uint64_t stream);
void gelu_dropout_fwd(uint64_t a, uint64_t h, long n, float p, uint64_t seed, uint64_t seed_ptr, uint64_t stream);
void gelu_dropout_bwd(uint64_t g, uint64_t a, uint64_t ga, long n, float p, uint64_t seed, uint64_t seed_ptr,
                      uint64_t stream);
void dropout_bwd_colsum(uint64_t g, uint64_t gy, uint64_t gb, long rows, int cols, float p, uint64_t seed,
                        uint64_t seed_ptr, uint64_t stream);
void gelu_dropout_bwd_colsum(uint64_t g, uint64_t a, uint64_t ga, uint64_t gb, long rows, int cols, float p,
                             uint64_t seed, uint64_t seed_ptr, uint64_t stream);
// ngd.hip
void ngd_sumsq(uint64_t X, long per, int G, uint64_t out, uint64_t stream);
bool ngd_small_supported(int D, int R);
bool ngd_proj_supported(int D, int R);
int ngd_mfma(int on);  // NGD projection on the matrix cores: set (on >= 0), returns the previous setting
void ngd_proj(uint64_t X, uint64_t Y, uint64_t W, uint64_t Hbuf, int G, int A, int D, int B, int R, uint64_t ip,
              uint64_t fp, uint64_t J, uint64_t HH, uint64_t stream);
long ngd_proj_hbuf_numel(int G, int A, int D, int B, int R, bool need_ip, bool need_j, bool need_hh);
void ngd_small_proj(uint64_t X, uint64_t Y, uint64_t W, int G, int A, int D, int B, int R, uint64_t sums, uint64_t J,
                    uint64_t HH, uint64_t part, uint64_t stream);
long ngd_small_part_numel(int G, int A, int D, int B, int R);
void ngd_rescale(uint64_t X, uint64_t Y, long per, int G, uint64_t ip, uint64_t fp, uint64_t stream);
long ngd_gram_slab_numel(int G, int R, int D, bool with_l);
void ngd_gram(uint64_t J, uint64_t W, uint64_t K, uint64_t L, uint64_t slab, int G, int R, int D, uint64_t stream);
void ngd_wupdate(uint64_t A, uint64_t J, uint64_t wc, uint64_t W, int G, int R, int D, uint64_t stream);
void ngd_pre_eigh(uint64_t K, uint64_t L, uint64_t d, uint64_t rho, uint64_t Z, uint64_t ise, uint64_t drho, uint64_t zs,
                  uint64_t dsum, int G, int R, float alpha, float eta, float N, float D, uint64_t stream);
void ngd_post_eigh(uint64_t c, uint64_t U, uint64_t ise, uint64_t drho, uint64_t zs, uint64_t dsum, uint64_t trXX,
                   uint64_t d, uint64_t rho, uint64_t A, uint64_t wc, int G, int R, float alpha, float eta, float N,
                   float D, uint64_t stream);
}  // namespace fdt
