"""ops/linear.py: split-K fp32 weight gradient vs an fp32 PyTorch reference."""
import pytest
import torch
import torch.nn.functional as F

from faster_distributed_training_amd.ops.linear import _splits, linear


def rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def test_split_choice():
    assert _splits(32768) == 16
    assert _splits(8192) == 8
    assert _splits(3000) == 2
    assert _splits(1000) == 1


def test_cpu_falls_back_to_f_linear():
    x = torch.randn(5, 7, 16, requires_grad=True)
    w = torch.randn(8, 16, requires_grad=True)
    b = torch.randn(8, requires_grad=True)
    y = linear(x, w, b)
    assert torch.equal(y, F.linear(x, w, b))


@pytest.mark.gpu
@pytest.mark.parametrize("fin,fout,bias", [(512, 1536, True), (1024, 512, False)])
def test_linear_autocast_grads(cuda, fin, fout, bias):
    torch.manual_seed(0)
    x = torch.randn(64, 128, fin, device=cuda, requires_grad=True)
    w = (torch.randn(fout, fin, device=cuda) / fin ** 0.5).requires_grad_()
    b = torch.randn(fout, device=cuda, requires_grad=True) if bias else None
    g = torch.randn(64, 128, fout, device=cuda)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = linear(x, w, b)
    assert y.dtype == torch.bfloat16
    y.backward(g.to(y.dtype))
    # fp32 reference on the same bf16-rounded operands
    xr = x.detach().to(torch.bfloat16).float().requires_grad_()
    wr = w.detach().to(torch.bfloat16).float().requires_grad_()
    br = b.detach().to(torch.bfloat16).float().requires_grad_() if bias else None
    yr = F.linear(xr, wr, br)
    yr.backward(g.to(torch.bfloat16).float())
    assert rel(y, yr) < 1e-2
    assert w.grad.dtype == torch.float32 and rel(w.grad, wr.grad) < 1e-4
    assert rel(x.grad, xr.grad) < 1e-2
    if bias:
        assert rel(b.grad, br.grad) < 1e-4
