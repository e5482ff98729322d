"""Convergence parity of the bf16 HIP engine with the fp32 PyTorch path over 300 optimizer
steps on a learnable synthetic CIFAR task (scripts/convergence.py; VERDICT r3 #7b, r4 #7).

The error budget is what bf16 arithmetic alone costs: a third run, plain PyTorch under bf16
autocast (FDT_NATIVE=0) from the same weights on the same batches.  The engine must land at
most twice as far from the fp32 run as that run does (plus a small epsilon: half the fp32 loss,
at most 0.05), on the HELD-OUT loss and accuracy of the final weights (medians over five seeds
of every arm), or twice the fp32 run's own seed-to-seed spread if that is larger.  (The per-step training losses
at the end are heavy-tailed -- 0.005-0.17 step to step in every arm -- so their tail mean or
median swung by 5-8x between repeats of identical code, profiles/r5/convergence_flaky.txt;
the held-out loss of the final weights is a smooth function of them.)  Every run must also
have learned the task (training-loss tail median below half the initial loss).  ResNet-18 (both optimizers) and ResNet-50 at batch 128, i.e. through the
shipped tile table's batch-128 entries (the 8-GPU per-GPU batch).  Real CIFAR-10 is not
available offline: parity on it is unpinned (reference README.md:56-73)."""
import os
import sys

import pytest

pytestmark = pytest.mark.gpu

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# Every arm runs from SEEDS different initial weights / batch orders (the same seeds in every
# arm) and is compared by its median over them.  profiles/r6/convergence_ablation.txt (ResNet-18 /
# MADGRAD, 5 seeds, 6 arms): single held-out cross entropies range 0.012-0.13 in EVERY arm --
# fp32 0.035-0.084 (median 0.056), PyTorch bf16 autocast 0.015-0.075 (0.032), the engine 0.015-0.13
# (0.035), the engine with the round-5 CELU derivative 0.012-0.041 (0.037), engine + PyTorch
# MADGRAD 0.025-0.065, PyTorch + HIP MADGRAD 0.027-0.125 -- and the engine-trained weights give
# the same loss through the fp32 eval forward (trained running statistics included).  The
# round-5 "engine gap" (three repeats of ONE seed) was this spread, not a systematic offset; the
# CELU-join derivative (now exp(z/alpha) from the fp32 pre-activation) is pinned by its own
# kernel test (tests/test_conv_kernels.py::test_celu_join_backward_uses_preactivation).
SEEDS = 5
EPS_LOSS_REL = 0.5    # slack, relative to the fp32 median held-out cross entropy ...
EPS_LOSS_MAX = 0.05   # ... and never above this (absolute)
EPS_ACC = 0.02        # 20 of 1024 held-out samples


@pytest.mark.parametrize("opt,arch", [("madgrad", "resnet18"), ("ngd", "resnet18"), ("madgrad", "resnet50")])
@pytest.mark.timeout(900)
def test_engine_converges_like_fp32_reference(cuda, opt, arch):
    from scripts.convergence import compare
    r = compare(opt, 300, arch=arch, bs=128, repeats=SEEDS, seeds=True)
    print({k: v for k, v in r.items() if not k.endswith("curve")})
    # every run learns the task ...
    for k in ("reference_final_loss", "engine_final_loss", "bf16_torch_final_loss"):
        assert r[k] < 0.5 * r["initial_loss"], (k, r[k])
    # ... and the engine lands as close to fp32 as bf16 arithmetic or fp32's own spread allows
    d_loss = abs(r["engine_test_loss"] - r["reference_test_loss"])
    b_loss = max(abs(r["bf16_torch_test_loss"] - r["reference_test_loss"]), r["reference_spread_loss"])
    eps = min(EPS_LOSS_MAX, EPS_LOSS_REL * r["reference_test_loss"])
    assert d_loss <= 2 * b_loss + eps, (d_loss, b_loss, eps)
    d_acc = abs(r["engine_test_acc"] - r["reference_test_acc"])
    b_acc = max(abs(r["bf16_torch_test_acc"] - r["reference_test_acc"]), r["reference_spread_acc"])
    assert d_acc <= 2 * b_acc + EPS_ACC, (d_acc, b_acc)
