"""Transformer sublayer fusions on the GPU: the skip-path gradient handed from
``dropout_add``'s backward into the LayerNorm backward kernel (ops/layernorm.ResidualGrad)
gives the same input / parameter gradients as autograd summing the two paths."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("kind", ["ffn", "attention"])
def test_residual_grad_handoff_matches_autograd_sum(cuda, kind):
    from faster_distributed_training_amd.models import transformer as T
    from faster_distributed_training_amd.ops import dropout as D
    from faster_distributed_training_amd.ops import layernorm as LN
    torch.manual_seed(0)
    m = (T.sublayerConnectionFFN(512, 1024, 0.0, 0.0) if kind == "ffn"
         else T.sublayerConnectionAttention(8, 512, 0.0, 0.0)).to(cuda)
    # 4096 tokens: every linear takes the engine path (ops/linear._Linear) in both runs, so the
    # bias gradients fused into the dropout kernels (fused run) and the linear's own column
    # sums (unfused run) both sum the same bf16 gradient in fp32
    x = torch.randn(16, 256, 512, device=cuda, requires_grad=True)
    g = torch.randn(16, 256, 512, device=cuda)

    def run(fused):
        x.grad = None
        for p in m.parameters():
            p.grad = None
        if fused:
            with torch.autocast("cuda", dtype=torch.bfloat16):
                out = m(x)
        else:  # same kernels, no hand-off: autograd sums the skip and LayerNorm gradients
            res = LN.ResidualGrad()
            with torch.autocast("cuda", dtype=torch.bfloat16):
                y = m.layernorm(x, None)
                y = m.ffn(y) if kind == "ffn" else m.multiheads(y, y, y, None)
                out = D.dropout_add(y, x, 0.0, True, None)
            assert not res.armed
        out.backward(g)
        return x.grad.clone(), [p.grad.clone() for p in m.parameters()]

    gx0, gp0 = run(False)
    gx1, gp1 = run(True)
    assert torch.allclose(gx1, gx0, rtol=1e-5, atol=1e-5), (gx1 - gx0).abs().max()
    for a, b in zip(gp1, gp0):
        assert torch.allclose(a, b, rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("p", [0.0, 0.1])
@pytest.mark.parametrize("direct", [False, True])
def test_ffn_fused_epilogues_match_unfused(cuda, p, direct):
    """ops/ffn.py (w_1 GEMM with the bias + GELU + dropout epilogue, w_2's data gradient with
    the GELU-dropout backward + b_1 column sums) against the unfused composition (hipBLASLt
    GEMMs + standalone dropout kernels) on the same dropout draw."""
    from faster_distributed_training_amd.models import transformer as T
    from faster_distributed_training_amd.ops import ffn
    from faster_distributed_training_amd.ops.linear import enable_direct_grads
    torch.manual_seed(0)
    m = T.PositionalWiseFFN(512, 1024, p).to(cuda)
    x = torch.randn(8, 1024, 512, device=cuda).to(torch.bfloat16).requires_grad_(True)
    g = torch.randn(8, 1024, 512, device=cuda)
    ffn.FUSED = True
    assert ffn.fusable(x, 512, 1024)

    def run(fused):
        ffn.FUSED = fused
        x.grad = None
        for q in m.parameters():
            q.grad = torch.full_like(q, 0.5) if direct else None
        enable_direct_grads(m.parameters(), direct)
        torch.manual_seed(5)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = m(x)
        y.float().backward(g)
        torch.cuda.synchronize()
        return y.detach().float(), x.grad.float().clone(), [q.grad.clone() for q in m.parameters()]

    try:
        y0, gx0, gp0 = run(False)
        y1, gx1, gp1 = run(True)
    finally:
        ffn.FUSED = True
        enable_direct_grads(m.parameters(), False)

    def rel(a, b):
        return ((a - b).norm() / b.norm()).item()
    assert rel(y1, y0) < 1e-2, rel(y1, y0)
    assert rel(gx1, gx0) < 2e-2, rel(gx1, gx0)
    for a_, b_, name in zip(gp1, gp0, ["w1", "b1", "w2", "b2"]):
        assert rel(a_, b_) < 2e-2, (name, rel(a_, b_))
