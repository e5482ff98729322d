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
