"""The fused ResNet engine (ops/resnet_fused.py) against the fp32 PyTorch reference model
(same weights), on an MI355X."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def _pair(arch, cuda):
    from faster_distributed_training_amd.models import resnet as R
    torch.manual_seed(0)
    m_ref = getattr(R, arch)(10).to(cuda)
    m_eng = getattr(R, arch)(10).to(cuda)
    m_eng.load_state_dict(m_ref.state_dict())
    m_ref.fast_path = False
    m_eng.fast_path = True
    return m_ref, m_eng


@pytest.mark.parametrize("arch,det", [("resnet18", False), ("resnet50", False), ("resnet50", True)])
def test_engine_train_step_matches_reference(cuda, arch, det):
    """bf16 engine vs the fp32 reference: logits within 2x the error of the reference run
    under bf16 autocast; every parameter gradient closely aligned; BN running statistics
    updated identically.  det: the deterministic-mode reductions (--deterministic)."""
    from faster_distributed_training_amd.ops import _native
    _native.set_deterministic(det)
    try:
        _train_step_vs_reference(cuda, arch)
    finally:
        _native.set_deterministic(False)


@pytest.mark.parametrize("arch", ["resnet50"])
def test_engine_at_shipped_batch128_config(cuda, arch):
    """The per-GPU batch of the 8-GPU run (128) through the tile table the bench uses
    (ops/conv_tuned.json, batch-128 entries: split-K, K groups): every conv launch takes a
    tuned entry, split-K and K-group launches are among them, and the step still matches the
    fp32 reference within the bf16-autocast budget (VERDICT r3 #7a)."""
    from faster_distributed_training_amd.ops import conv_igemm as CI
    CI.LAUNCH_LOG = []
    try:
        _train_step_vs_reference(cuda, arch, batch=128)
        log = list(CI.LAUNCH_LOG)
    finally:
        CI.LAUNCH_LOG = None
    convs = [e for e in log if e[1].startswith("128:")]
    # every launch tuned, or a halo 3x3 loop (forward / data gradient kg 5-8, weight gradient
    # "kg" 9: chosen by geometry, not by the table)
    assert convs and all(e[2] or e[5] in (5, 6, 7, 8, 9) for e in convs), [e for e in convs if not e[2]][:5]
    assert any(e[4] > 1 for e in convs), "no split-K launch"
    assert any(e[5] == 2 for e in convs), "no K-group launch"
    print(f"{len(convs)} conv launches, {sum(e[4] > 1 for e in convs)} split-K, {sum(e[5] == 2 for e in convs)} K-group")


def _train_step_vs_reference(cuda, arch, batch=64):
    m_ref, m_eng = _pair(arch, cuda)
    torch.backends.cudnn.allow_tf32 = False
    torch.manual_seed(1)
    x = torch.randn(batch, 3, 32, 32, device=cuda)
    y = torch.randint(0, 10, (batch,), device=cuda)
    m_rb = _pair(arch, cuda)[0]
    m_rb.load_state_dict(m_ref.state_dict())
    with torch.autocast("cuda", dtype=torch.bfloat16):
        out_rb = m_rb(x)
    out_r = m_ref(x)
    out_e = m_eng(x)
    e_ref, e_eng = rel(out_rb, out_r), rel(out_e, out_r)
    assert e_eng < max(2.0 * e_ref, 3e-2), (e_eng, e_ref)
    F.cross_entropy(out_r.float(), y).backward()
    F.cross_entropy(out_e.float(), y).backward()
    F.cross_entropy(out_rb.float(), y).backward()

    # Every parameter's gradient -- conv weights, BN affines, the fc weight and bias -- must be
    # within 2x the relative error of the reference model's own bf16-autocast gradient (plus a
    # small absolute floor for parameters whose autocast gradient happens to be near exact).
    # Gradients behind many normalised layers (the stem weight, BN betas) are small residuals
    # of large cancelling terms, so their bf16 errors are large in both runs; the bound is
    # relative to what bf16 itself loses on each parameter.
    worst = []
    for (n, pr), (_, pe), (_, pb) in zip(m_ref.named_parameters(), m_eng.named_parameters(),
                                         m_rb.named_parameters()):
        assert pe.grad is not None, n
        e_e, e_b = rel(pe.grad, pr.grad), rel(pb.grad, pr.grad)
        worst.append((e_e / max(e_b, 1e-6), n, e_e, e_b))
        # fc.bias: sum over the batch of softmax - onehot, the most cancellation-heavy
        # gradient (its bf16 error varies run to run with the engine's atomic statistics)
        assert e_e <= max(2.0 * e_b, 1.5e-2 if n == "fc.bias" else 5e-3), (n, e_e, e_b)
    worst.sort(reverse=True)
    print("worst engine/autocast gradient error ratios:", [(n, round(r, 2)) for r, n, _, _ in worst[:5]])
    # BN running statistics: within 2x what the bf16-autocast reference run's own update misses
    # (plus 1e-3: running_var of channels whose batch variance is ~exact in both)
    for (n, br), (_, be), (_, bb) in zip(m_ref.named_buffers(), m_eng.named_buffers(), m_rb.named_buffers()):
        if br.dtype.is_floating_point:
            assert rel(be, br) <= max(2.0 * rel(bb, br), 1e-3), (n, rel(be, br), rel(bb, br))
        else:
            assert int(be) == int(br), n


@pytest.mark.parametrize("arch", ["resnet18", "resnet50"])
def test_engine_eval_matches_reference(cuda, arch):
    m_ref, m_eng = _pair(arch, cuda)
    m_ref.eval()
    m_eng.eval()
    x = torch.randn(32, 3, 32, 32, device=cuda)
    with torch.no_grad():
        out_r = m_ref(x)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            out_rb = m_ref(x)
        e_eng, e_ref = rel(m_eng(x), out_r), rel(out_rb, out_r)
    # fresh running stats (mean 0, var 1) leave the strided-block activations
    # un-normalised in eval, which amplifies rounding: budget relative to bf16 autocast
    assert e_eng < max(2.0 * e_ref, 3e-2), (e_eng, e_ref)


@pytest.mark.parametrize("arch", ["resnet18", "resnet50"])
def test_engine_eval_after_training_matches_fp32(cuda, arch):
    """Eval with TRAINED running statistics: 50 engine training steps
    (SGD + momentum on a learnable random-label-free task), then the engine's eval forward vs
    the fp32 PyTorch eval of the same weights and buffers, within 2x the error of PyTorch's own
    bf16-autocast eval of them."""
    m_ref, m_eng = _pair(arch, cuda)
    torch.manual_seed(2)
    protos = torch.randn(10, 3, 32, 32, device=cuda)
    opt = torch.optim.SGD(m_eng.parameters(), lr=0.02, momentum=0.9)
    m_eng.train()
    for _ in range(50):
        y = torch.randint(0, 10, (64,), device=cuda)
        x = protos[y] + 0.5 * torch.randn(64, 3, 32, 32, device=cuda)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            out = m_eng(x)
        F.cross_entropy(out.float(), y).backward()
        opt.step()
        opt.zero_grad(set_to_none=True)
    m_ref.load_state_dict(m_eng.state_dict())
    rv = [b for n, b in m_ref.named_buffers() if n.endswith("running_var")]
    assert any(float((v - 1).abs().max()) > 0.05 for v in rv), "running statistics did not move"
    m_ref.eval()
    m_eng.eval()
    y = torch.randint(0, 10, (128,), device=cuda)
    x = protos[y] + 0.5 * torch.randn(128, 3, 32, 32, device=cuda)
    with torch.no_grad():
        out_r = m_ref(x)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            out_rb = m_ref(x)
            out_e = m_eng(x)
    e_eng, e_ref = rel(out_e, out_r), rel(out_rb, out_r)
    assert e_eng < max(2.0 * e_ref, 1e-2), (e_eng, e_ref)
    assert (out_e.float().argmax(1) == out_r.argmax(1)).float().mean() > 0.97


def test_engine_grad_ready_hooks_fire(cuda):
    from faster_distributed_training_amd.models import resnet as R
    from faster_distributed_training_amd.ops.resnet_fused import register_grad_ready_hook
    m = R.resnet50(10).to(cuda)
    m.fast_path = True
    seen = []
    hs = [register_grad_ready_hook(p, lambda q: seen.append(id(q))) for p in m.parameters()]
    hs += [p.register_post_accumulate_grad_hook(lambda q: seen.append(id(q))) for p in m.parameters()]
    x = torch.randn(8, 3, 32, 32, device=cuda)
    F.cross_entropy(m(x).float(), torch.randint(0, 10, (8,), device=cuda)).backward()
    torch.cuda.synchronize()
    assert sorted(seen) == sorted(id(p) for p in m.parameters())
    for h in hs:
        h.remove()


def test_engine_training_reduces_loss(cuda):
    from faster_distributed_training_amd.models import resnet as R
    from faster_distributed_training_amd.optim.flat_optim import SGD
    from faster_distributed_training_amd.utils.flat import FlatParams
    torch.manual_seed(0)
    m = R.resnet18(10).to(cuda)
    m.fast_path = True
    flat = FlatParams(m, device=cuda)
    opt = SGD(flat, lr=0.05, momentum=0.9)
    x = torch.randn(32, 3, 32, 32, device=cuda)
    y = torch.randint(0, 10, (32,), device=cuda)
    losses = []
    for _ in range(15):
        loss = F.cross_entropy(m(x).float(), y)
        loss.backward()
        opt.step()
        losses.append(loss.item())
    assert losses[-1] < 0.5 * losses[0], losses


def test_transformer_train_step_on_gpu(cuda):
    """A short AG-News-shaped run of the full transformer trainer on the GPU path
    (LayerNorm / embedding / FusedMLP / mixup kernels)."""
    from faster_distributed_training_amd.train.transformer_trainer import TransformerConfig, TransformerTrainer
    cfg = TransformerConfig(batch_size=32, synthetic=True, eval=False, plot=False, ngd=True, epoch=1,
                            steps_per_epoch=3, length_buckets=(128,), extra={"subset_stride": 50})
    tr = TransformerTrainer(cfg)
    losses = []
    it = iter(tr.train_loader)
    for _ in range(3):
        losses.append(float(tr.train_step(*next(it))))
    assert all(l == l and l < 10 for l in losses), losses


def test_engine_hip_graph_replay_matches_eager(cuda):
    """Body captured as HIP graphs (step 1 eager warm-up, step 2 capture, step 3 replay)
    gives the eager engine's logits and gradients, up to the run-to-run noise of the
    engine's fp32-atomic statistics (measured here as eager vs eager)."""
    from faster_distributed_training_amd.models import resnet as R
    from faster_distributed_training_amd.utils.flat import FlatParams
    torch.manual_seed(0)
    m = R.resnet50(10).to(cuda)
    m.fast_path = True
    flat = FlatParams(m, device=cuda)
    g = torch.Generator().manual_seed(4)
    x = torch.randn(64, 3, 32, 32, generator=g).to(cuda)
    y = torch.randint(0, 10, (64,), generator=g).to(cuda)

    def step():
        flat.grad.zero_()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            out = m(x)
        F.cross_entropy(out.float(), y).backward()
        torch.cuda.synchronize()
        return out.detach().float().clone(), flat.grad.clone()

    m.graph_engine = False
    o1, g1 = step()
    o2, g2 = step()
    m.graph_engine = True
    for _ in range(3):
        og, gg = step()
    st = list(m._plan._graphs.values())[0]
    assert st.stage == "ready" and len(st.segments) == 1
    og2, gg2 = step()  # another replay
    noise_o, noise_g = rel(o2, o1), rel(g2, g1)
    assert rel(og, o1) <= 3 * noise_o + 2e-3, (rel(og, o1), noise_o)
    assert rel(gg, g1) <= 3 * noise_g + 2e-3, (rel(gg, g1), noise_g)
    assert rel(og2, og) <= 3 * noise_o + 2e-3


@pytest.mark.parametrize("N,K,C,HW", [(64, 10, 2048, 16), (1024, 10, 2048, 16), (96, 20, 512, 16), (512, 32, 256, 49)])
def test_fused_head_kernels_match_fp32(cuda, N, K, C, HW):
    """head_fwd / head_bwd (csrc/kernels/head.hip) against the fp32 PyTorch head
    fc(mean_hw(body)) and its gradients."""
    from faster_distributed_training_amd.ops import _native
    nat = _native.native()
    g = torch.Generator(device=cuda).manual_seed(N + K)
    body = torch.randn(N, HW, C, device=cuda, generator=g).relu().to(torch.bfloat16)
    W = torch.randn(K, C, device=cuda, generator=g) * C ** -0.5
    b = torch.randn(K, device=cuda, generator=g)
    pooled = torch.empty(N, C, device=cuda, dtype=torch.bfloat16)
    logits = torch.empty(N, K, device=cuda, dtype=torch.bfloat16)
    nat.head_fwd(body.data_ptr(), W.data_ptr(), b.data_ptr(), pooled.data_ptr(), logits.data_ptr(), N, HW, C, K,
                 torch.cuda.current_stream().cuda_stream)
    p_ref = body.float().mean(1)
    l_ref = p_ref @ W.t() + b
    assert rel(pooled, p_ref) < 4e-3
    assert rel(logits, l_ref) < 1e-2, rel(logits, l_ref)
    dl = torch.randn(N, K, device=cuda, generator=g).to(torch.bfloat16)
    gW0 = torch.randn(K, C, device=cuda, generator=g)
    gb0 = torch.randn(K, device=cuda, generator=g)
    gW, gb = gW0.clone(), gb0.clone()
    dpool = torch.empty(N, C, device=cuda, dtype=torch.bfloat16)
    nat.head_bwd(dl.data_ptr(), W.data_ptr(), pooled.data_ptr(), dpool.data_ptr(), gW.data_ptr(), gb.data_ptr(),
                 N, HW, C, K, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert rel(dpool, dl.float() @ W / HW) < 1e-2
    assert rel(gW - gW0, dl.float().t() @ p_ref) < 1e-2
    assert rel(gb - gb0, dl.float().sum(0)) < 1e-4


def test_engine_fused_head_matches_pytorch_head(cuda):
    """Under bf16 autocast the engine runs the classifier head itself (FUSED_HEAD); its
    logits and every gradient match the PyTorch head (mean + F.linear) on the same engine
    (deterministic mode: identical bodies), and the fc gradients fire the engine's
    grad-ready hooks exactly once.  The loss is linear in the logits (fixed bf16 weights R)
    so both heads see the same logit gradient."""
    from faster_distributed_training_amd.models import resnet as R
    from faster_distributed_training_amd.ops import _native
    from faster_distributed_training_amd.ops import resnet_fused as rf
    from faster_distributed_training_amd.ops.resnet_fused import register_grad_ready_hook
    torch.manual_seed(0)
    m = R.resnet50(10).to(cuda)
    m.fast_path = True
    x = torch.randn(64, 3, 32, 32, device=cuda)
    r = torch.randn(64, 10, device=cuda).to(torch.bfloat16).float()

    def step():
        m.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            out = m(x)
        (out.float() * r).sum().backward()
        torch.cuda.synchronize()
        return out.detach().float(), {n: p.grad.clone() for n, p in m.named_parameters()}

    saved = rf.FUSED_HEAD
    _native.set_deterministic(True)
    try:
        rf.FUSED_HEAD = False
        o1, g1 = step()
        assert not m._plan.head_on
        rf.FUSED_HEAD = True
        seen = []
        hs = [register_grad_ready_hook(p, lambda q: seen.append(id(q))) for p in (m.fc.weight, m.fc.bias)]
        of, gf = step()
        assert m._plan.head_on
        assert sorted(seen) == sorted([id(m.fc.weight), id(m.fc.bias)])
        for h in hs:
            h.remove()
    finally:
        rf.FUSED_HEAD = saved
        _native.set_deterministic(False)
    assert rel(of, o1) < 1e-2, rel(of, o1)
    errs = {n: rel(gf[n], g1[n]) for n in g1}
    print("worst fused-head gradient differences:", sorted(errs.items(), key=lambda kv: -kv[1])[:4])
    # (the PyTorch head rounds its weight / bias gradients to bf16, the fused head does not)
    assert errs["fc.weight"] < 1e-2 and errs["fc.bias"] < 1e-2, (errs["fc.weight"], errs["fc.bias"])
    assert max(v for n, v in errs.items() if not n.startswith("fc.")) < 1e-3
    flat_f = torch.cat([gf[n].flatten() for n in g1])
    flat_1 = torch.cat([g1[n].flatten() for n in g1])
    assert rel(flat_f, flat_1) < 2e-2, rel(flat_f, flat_1)
