// pybind11 bindings for the _fdt_native extension.  No torch headers: tensors cross the
// boundary as device addresses (uint64), which keeps the build fast (hipcc only, no
// ATen), avoids C++ ABI coupling with the torch wheel, and lets any .so built here
// load next to any torch on the box.  Python wrappers in faster_distributed_training_amd/ops
// validate shapes/dtypes on the host before calling in.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "api.h"
#include "runtime/runtime_api.h"

namespace py = pybind11;

PYBIND11_MODULE(_fdt_native, m) {
  m.doc() = "MI355X (gfx950) HIP kernels and native runtime of faster_distributed_training_amd";
  m.attr("arch") = "gfx950";
#define DEF(name) m.def(#name, &fdt::name)
  // normalisation engine
  DEF(act_affine_fwd);
  DEF(stats_num_blocks);
  DEF(channel_stats_partial);
  DEF(stats_finalize);
  DEF(act_bwd_reduce);
  DEF(reduce_partials);
  DEF(partials_compact);
  DEF(stats_bwd_coef);
  DEF(stats_bwd_finalize);
  DEF(affine_fold);
  DEF(residual_act_fwd);
  DEF(residual_act_bwd);
  DEF(set_deterministic_mode);
  DEF(deterministic_mode);
  // implicit-GEMM convolution engine
  DEF(conv_igemm);
  DEF(conv_num_row_blocks);
  DEF(conv_splitk_workspace);
  DEF(conv_wgrad);
  DEF(wgrad_reduce);
  DEF(pack_weights);
  DEF(jacobi_eigh);
  DEF(ngd_pre_eigh);
  DEF(ngd_sumsq);
  DEF(ngd_small_supported);
  DEF(ngd_small_proj);
  DEF(ngd_small_part_numel);
  DEF(ngd_proj_supported);
  DEF(ngd_proj);
  DEF(ngd_proj_hbuf_numel);
  DEF(ngd_rescale);
  DEF(ngd_post_eigh);
  DEF(attn_fwd);
  DEF(attn_bwd);
  // optimizers
  DEF(grad_sumsq);
  DEF(grad_norm_finalize);
  DEF(sgd_step);
  DEF(madgrad_step);
  DEF(mirror_madgrad_step);
  DEF(adam_step);
  DEF(cast_bf16);
  // mixup
  DEF(mixup_fwd);
  DEF(mixup_bwd);
  DEF(mixup_ce_fwd);
  // transformer
  DEF(layernorm_fwd);
  DEF(layernorm_bwd);
  DEF(embedding_fwd);
  DEF(embedding_bwd);
  DEF(bias_relu_fwd);
  DEF(relu_bwd_colsum);
  DEF(colsum_bf16);
  DEF(slab_sum_acc);
  DEF(dropout_add_fwd);
  DEF(dropout_bwd);
  DEF(gelu_dropout_fwd);
  DEF(gelu_dropout_bwd);
  // data
  DEF(augment);
  DEF(rng_advance);
#undef DEF
  fdt::register_runtime(m);
}
