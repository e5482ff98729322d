"""Numerics of the hand-written implicit-GEMM conv kernels (fwd / dgrad / wgrad) against a
plain PyTorch fp32 reference of the same op (inputs rounded to bf16 on both sides)."""
import pytest
import torch
import torch.nn.functional as F

from faster_distributed_training_amd.ops import conv_igemm as ci

pytestmark = pytest.mark.gpu

BF = torch.bfloat16


_p = ci._p


def rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def act_ref(z, act, alpha):
    if act == 1:
        return torch.relu(z)
    if act == 2:
        return F.celu(z, alpha)
    return z


def make(shape_nhwc, dev, scale=1.0):
    return (torch.randn(*shape_nhwc, device=dev) * scale).to(BF)


def nchw(x):
    return x.permute(0, 3, 1, 2).float()


def nhwc(x):
    return x.permute(0, 2, 3, 1)


def padc(x, c):
    if x.shape[-1] == c:
        return x.contiguous()
    return F.pad(x, (0, c - x.shape[-1])).contiguous()


FWD_CASES = [
    # (N, H, Cin, Cout, k, stride, pad)
    (4, 8, 64, 128, 1, 1, 0),
    (2, 8, 64, 64, 3, 1, 1),
    (2, 16, 128, 128, 3, 2, 1),
    (2, 8, 64, 256, 1, 2, 0),
    (2, 8, 3, 64, 3, 1, 1),     # stem (Cin padded to 8)
    (3, 5, 64, 64, 3, 1, 1),    # M tail (75 rows)
    (2, 4, 512, 512, 3, 1, 1),
]


@pytest.mark.parametrize("case", FWD_CASES)
@pytest.mark.parametrize("mode", ["plain", "relu", "celu"])
def test_conv_fwd(cuda, case, mode):
    N, H, Cin, Cout, k, stride, pad = case
    torch.manual_seed(0)
    shp = ci.ConvShape(Cin, Cout, k, stride, pad)
    x = padc(make((N, H, H, Cin), cuda), shp.cxp)
    w = torch.randn(Cout, Cin, k, k, device=cuda) / (Cin * k * k) ** 0.5
    wf, wd = ci.alloc_packed(shp, cuda, dgrad=Cin >= 8)
    ci.pack_weights([(w, wf, wd, shp)])
    if mode == "plain":
        s = t = None
        act, alpha = 0, 1.0
        a = x[..., :Cin].float()
    else:
        s = torch.rand(shp.cxp, device=cuda) + 0.5
        t = torch.randn(shp.cxp, device=cuda) * 0.3
        act, alpha = (1, 1.0) if mode == "relu" else (2, 0.075)
        a = act_ref(x.float() * s + t, act, alpha).to(BF).float()[..., :Cin]
    for tile, ns in [(None, None), ((64, 64, 64), 1), ((64, 64, 64), 3), ((128, 64, 32), None),
                     ((128, 128, 64), 2), ((256, 128, 32), None), ((256, 64, 64), 1), ((64, 64, 128), 1),
                     ((64, 64, 128), 3), ((128, 64, 128), 2), ((64, 128, 128), None)]:
        if tile and Cout % tile[1]:
            continue
        y, part = ci.conv_fwd(x, wf, shp, s, t, act, alpha, tile=tile, nsplit=ns)
        ref = nhwc(F.conv2d(nchw(a), w.to(BF).float(), stride=stride, padding=pad))
        assert rel(y, ref) < 1e-2, (tile, rel(y, ref))
        ps = part.sum(0)
        yf = ref.reshape(-1, Cout)
        assert rel(ps[0], yf.sum(0)) < 2e-3
        assert rel(ps[1], (yf * yf).sum(0)) < 2e-3


@pytest.mark.parametrize("case", [(4, 8, 256, 64), (2, 8, 512, 128), (3, 5, 256, 256), (2, 4, 1024, 512)])
@pytest.mark.parametrize("proj", [False, True])
def test_conv_fwd_join_prologue(cuda, case, proj):
    """PRO_JOIN: the 1x1 conv of relu(y*s + t + (r*s2 + t2 | r)) -- the previous residual
    block's join -- plus the stored join output and its ReLU bit mask, against fp32 PyTorch
    (the join rounded to bf16 like the standalone kernel stores it)."""
    N, H, C, Cout = case
    torch.manual_seed(3)
    shp = ci.ConvShape(C, Cout, 1, 1, 0)
    y, r = make((N, H, H, C), cuda), make((N, H, H, C), cuda)
    s = torch.rand(C, device=cuda) + 0.5
    t = torch.randn(C, device=cuda) * 0.3
    s2 = torch.rand(C, device=cuda) + 0.5 if proj else None
    t2 = torch.randn(C, device=cuda) * 0.3 if proj else None
    w = torch.randn(Cout, C, 1, 1, device=cuda) / C ** 0.5
    wf, _ = ci.alloc_packed(shp, cuda, dgrad=False)
    ci.pack_weights([(w, wf, None, shp)])
    sc = r.float() * s2 + t2 if proj else r.float()
    joined = torch.relu(y.float() * s + t + sc)
    a = joined.to(BF).float()
    ref = nhwc(F.conv2d(nchw(a), w.to(BF).float()))
    want_mask = (joined.reshape(-1, 8) > 0).to(torch.int32)
    want_mask = (want_mask << torch.arange(8, device=cuda, dtype=torch.int32)).sum(1).to(torch.uint8)
    for tile, ns in [(None, None), ((64, 64, 64), 1), ((128, 64, 32), 3), ((128, 128, 32), None),
                     ((64, 128, 128), 2), ((64, 64, 128), 1), ((128, 128, 64), 1), ((64, 128, 64), 1),
                     ((128, 256, 64), 1), ((64, 256, 64), 2), ((128, 256, 32), 1)]:
        if tile and Cout % tile[1]:
            continue
        jout = torch.full_like(y, float("nan"))
        jmask = torch.zeros(y.numel() // 8, device=cuda, dtype=torch.uint8)
        out, part = ci.conv_fwd_join(y, r, s, t, s2, t2, wf, shp, jout, jmask, tile=tile, nsplit=ns)
        assert rel(out, ref) < 1e-2, (tile, rel(out, ref))
        # (fma vs separate roundings of y*s + t: at most one bf16 ulp apart)
        assert ((jout.float() - a).abs() <= a.abs() * 2 ** -7 + 1e-6).all(), (tile, (jout.float() - a).abs().max())
        assert (jmask != want_mask).float().mean().item() < 1e-3, tile
        ps = part.sum(0)
        yf = ref.reshape(-1, Cout)
        assert rel(ps[0], yf.sum(0)) < 2e-3 and rel(ps[1], (yf * yf).sum(0)) < 2e-3


DGRAD_CASES = [
    (4, 8, 64, 128, 1, 1, 0),
    (2, 8, 64, 64, 3, 1, 1),
    (2, 16, 128, 128, 3, 2, 1),
    (2, 8, 64, 256, 1, 2, 0),
    (3, 5, 64, 64, 3, 1, 1),
]


@pytest.mark.parametrize("case", DGRAD_CASES)
@pytest.mark.parametrize("epi", ["store", "add", "actbwd"])
def test_conv_dgrad(cuda, case, epi):
    N, H, Cin, Cout, k, stride, pad = case
    torch.manual_seed(1)
    shp = ci.ConvShape(Cin, Cout, k, stride, pad)
    w = torch.randn(Cout, Cin, k, k, device=cuda) / (Cin * k * k) ** 0.5
    wf, wd = ci.alloc_packed(shp, cuda)
    ci.pack_weights([(w, wf, wd, shp)])
    Ho, Wo = ci.out_hw(H, H, shp)
    g = make((N, Ho, Wo, Cout), cuda)
    y = make((N, Ho, Wo, Cout), cuda)
    al = torch.randn(Cout, device=cuda) * 0.1
    be = torch.randn(Cout, device=cuda) * 0.1
    gt = (g.float() + al + be * y.float()).to(BF).float()
    ref = nhwc(torch.nn.grad.conv2d_input((N, Cin, H, H), w.to(BF).float(), nchw(gt), stride=stride, padding=pad))
    xs = (N, H, H, Cin)
    if epi == "store":
        for tile, ns in [(None, None), ((64, 64, 32), 1), ((64, 64, 32), 4), ((128, 64, 64), 2),
                         ((64, 64, 128), 2), ((64, 128, 128), 1)]:
            if tile and Cin % tile[1]:
                continue
            out, _ = ci.conv_dgrad(g, y, al, be, wd, shp, xs, epi=ci.EPI_STORE, tile=tile, nsplit=ns)
            assert rel(out, ref) < 1e-2, (tile, ns)
    elif epi == "add":
        prev = make(xs, cuda)
        for ns in (1, 3):
            out = prev.clone()
            ci.conv_dgrad(g, y, al, be, wd, shp, xs, epi=ci.EPI_ADD, out=out, nsplit=ns)
            assert rel(out, ref + prev.float()) < 1e-2, ns
    else:
        ex = make(xs, cuda)
        es = torch.rand(Cin, device=cuda) + 0.5
        et = torch.randn(Cin, device=cuda) * 0.3
        z = ex.float() * es + et
        gp = ref * (z > 0).float()
        for ns in (1, 4):
            out, part = ci.conv_dgrad(g, y, al, be, wd, shp, xs, epi=ci.EPI_ACTBWD, ex=ex, es=es, et=et, act=1,
                                      nsplit=ns)
            assert rel(out, gp * es) < 1e-2, ns
            ps = part.sum(0)
            assert rel(ps[0], (gp * ex.float()).reshape(-1, Cin).sum(0)) < 1e-2
            assert rel(ps[1], gp.reshape(-1, Cin).sum(0)) < 1e-2


# halo-staged 3x3 loop (kg 5, csrc/kernels/conv_h3.hip): (N, H, Cin, Cout) -- whole image rows
# per 256-pixel tile (H 32 / 16), whole images (H 8 / 4), BN 128 and 64
H3_CASES = [(1, 32, 64, 64), (2, 16, 128, 128), (4, 8, 256, 256), (16, 4, 512, 512), (2, 16, 64, 128),
            (4, 8, 128, 64), (32, 4, 64, 128)]


@pytest.mark.parametrize("case", H3_CASES)
@pytest.mark.parametrize("kg", [5, 6, 7, 8])
@pytest.mark.parametrize("loop", ["dma", "dma64"])  # 128 / 64 output channels per workgroup
def test_h3_conv_fwd(cuda, case, kg, loop, monkeypatch):
    if kg == 8 and (loop == "dma64" or case[3] % 128):
        pytest.skip("kg 8: 256 x 128 tiles only")
    """Forward 3x3 on a materialised operand through the halo loop: output and BN statistics
    against fp32 PyTorch, and the implicit-GEMM kernel on the same inputs."""
    monkeypatch.setattr(ci, "H3_LOOP", loop)
    N, H, Cin, Cout = case
    torch.manual_seed(7)
    shp = ci.ConvShape(Cin, Cout, 3, 1, 1)
    x = make((N, H, H, Cin), cuda)
    w = torch.randn(Cout, Cin, 3, 3, device=cuda) / (Cin * 9) ** 0.5
    wf, wd = ci.alloc_packed(shp, cuda)
    ci.pack_weights([(w, wf, wd, shp)])
    assert ci.h3_tile(N, H, H, shp, ci.PRO_NONE, Cout, force=True) is not None
    y, part = ci.conv_fwd(x, wf, shp, kg=kg)
    ref = nhwc(F.conv2d(nchw(x), w.to(BF).float(), padding=1))
    assert rel(y, ref) < 1e-2, rel(y, ref)
    assert ((y.float() - ref).abs() <= ref.abs() * 2 ** -7 + 2e-3 * ref.abs().max()).float().mean() > 0.999
    ps = part.sum(0)
    yf = ref.reshape(-1, Cout)
    assert rel(ps[0], yf.sum(0)) < 2e-3
    assert rel(ps[1], (yf * yf).sum(0)) < 2e-3
    y1, _ = ci.conv_fwd(x, wf, shp, tile=(128, 64, 32), kg=1)
    assert rel(y, y1) < 1e-2


@pytest.mark.parametrize("case", H3_CASES)
@pytest.mark.parametrize("epi", ["store", "actbwd_relu", "actbwd_celu"])
@pytest.mark.parametrize("kg", [5, 6, 7, 8])
@pytest.mark.parametrize("loop", ["dma", "dma64"])
def test_h3_conv_dgrad(cuda, case, epi, kg, loop, monkeypatch):
    if kg == 8 and (loop == "dma64" or case[2] % 128):
        pytest.skip("kg 8: 256 x 128 tiles only")
    """Stride-1 3x3 data gradient of a pre-folded gradient through the halo loop (flipped taps):
    plain store and the producer's activation backward + statistics, against fp32 PyTorch."""
    monkeypatch.setattr(ci, "H3_LOOP", loop)
    N, H, Cin, Cout = case
    torch.manual_seed(8)
    shp = ci.ConvShape(Cin, Cout, 3, 1, 1)
    w = torch.randn(Cout, Cin, 3, 3, device=cuda) / (Cin * 9) ** 0.5
    wf, wd = ci.alloc_packed(shp, cuda)
    ci.pack_weights([(w, wf, wd, shp)])
    g = make((N, H, H, Cout), cuda)
    ref = nhwc(torch.nn.grad.conv2d_input((N, Cin, H, H), w.to(BF).float(), nchw(g.float()), padding=1))
    xs = (N, H, H, Cin)
    if epi == "store":
        out, _ = ci.conv_dgrad(g, None, None, None, wd, shp, xs, epi=ci.EPI_STORE, kg=kg)
        assert rel(out, ref) < 1e-2
        return
    act, alpha = (1, 1.0) if epi == "actbwd_relu" else (2, 0.075)
    ex = make(xs, cuda)
    es = torch.rand(Cin, device=cuda) + 0.5
    et = torch.randn(Cin, device=cuda) * 0.3
    z = ex.float() * es + et
    d = (z > 0).float() if act == 1 else torch.where(z > 0, torch.ones_like(z), torch.exp(z / alpha))
    gp = ref * d
    out, part = ci.conv_dgrad(g, None, None, None, wd, shp, xs, epi=ci.EPI_ACTBWD, ex=ex, es=es, et=et, act=act,
                              alpha=alpha, kg=kg)
    assert rel(out, gp * es) < 1e-2
    ps = part.sum(0)
    assert rel(ps[0], (gp * ex.float()).reshape(-1, Cin).sum(0)) < 1e-2
    assert rel(ps[1], gp.reshape(-1, Cin).sum(0)) < 1e-2


H3S2_CASES = [(4, 32, 128, 128), (8, 16, 256, 256), (16, 8, 512, 512), (4, 16, 64, 64), (4, 32, 64, 128)]


@pytest.mark.parametrize("case", H3S2_CASES)
@pytest.mark.parametrize("epi", ["store", "actbwd_relu"])
def test_h3_conv_dgrad_stride2_classes(cuda, case, epi):
    """Stride-2 3x3 data gradient whose 2- and 4-tap output-parity classes run through the halo
    loop (kg 6, the class grid = the output-gradient grid, scattered to every other pixel), the
    1-tap class through the implicit GEMM: against fp32 PyTorch."""
    N, Hx, Cin, Cout = case
    torch.manual_seed(11)
    shp = ci.ConvShape(Cin, Cout, 3, 2, 1)
    w = torch.randn(Cout, Cin, 3, 3, device=cuda) / (Cin * 9) ** 0.5
    wf, wd = ci.alloc_packed(shp, cuda)
    ci.pack_weights([(w, wf, wd, shp)])
    Hy = Hx // 2
    g = make((N, Hy, Hy, Cout), cuda)
    ref = nhwc(torch.nn.grad.conv2d_input((N, Cin, Hx, Hx), w.to(BF).float(), nchw(g.float()), stride=2, padding=1))
    xs = (N, Hx, Hx, Cin)
    ci.LAUNCH_LOG = []
    try:
        if epi == "store":
            out, _ = ci.conv_dgrad(g, None, None, None, wd, shp, xs, epi=ci.EPI_STORE, kg=6)
            assert rel(out, ref) < 1e-2, rel(out, ref)
        else:
            ex = make(xs, cuda)
            es = torch.rand(Cin, device=cuda) + 0.5
            et = torch.randn(Cin, device=cuda) * 0.3
            gp = ref * ((ex.float() * es + et) > 0).float()
            out, part = ci.conv_dgrad(g, None, None, None, wd, shp, xs, epi=ci.EPI_ACTBWD, ex=ex, es=es, et=et, act=1,
                                      kg=6)
            assert rel(out, gp * es) < 1e-2
            ps = part.sum(0)
            assert rel(ps[0], (gp * ex.float()).reshape(-1, Cin).sum(0)) < 1e-2
            assert rel(ps[1], gp.reshape(-1, Cin).sum(0)) < 1e-2
        log = list(ci.LAUNCH_LOG)
    finally:
        ci.LAUNCH_LOG = None
    assert sum(1 for e in log if e[0] == "dgrad" and e[5] == 6) == 3, log  # the 2-, 2- and 4-tap classes


WH3_CASES = [(2, 32, 64, 64), (4, 16, 128, 128), (4, 8, 256, 256), (16, 4, 512, 512), (2, 16, 64, 128),
             (4, 8, 128, 64), (32, 4, 64, 128), (8, 32, 64, 64)]


@pytest.mark.parametrize("case", WH3_CASES)
@pytest.mark.parametrize("wgs", [256, 7])
@pytest.mark.parametrize("variant", ["default", "pipe", "ts2"])
def test_h3_conv_wgrad(cuda, case, wgs, variant, monkeypatch):
    """Halo-staged 3x3 weight gradient (conv_wh3.hip) against fp32 PyTorch and the implicit-GEMM
    weight gradient, fresh and accumulating; ``wgs`` 7: few workgroups -> long pixel ranges per
    split (uneven last split); variants: register-pipelined fragments, the tap split over two
    waves per block."""
    monkeypatch.setattr(ci, "WH3_WGS", wgs)
    monkeypatch.setattr(ci, "WH3_PIPE", variant == "pipe")
    monkeypatch.setattr(ci, "WH3_TS", 2 if variant == "ts2" else 1)
    N, H, Cin, Cout = case
    torch.manual_seed(9)
    shp = ci.ConvShape(Cin, Cout, 3, 1, 1)
    x = make((N, H, H, Cin), cuda)
    g = make((N, H, H, Cout), cuda)
    assert ci.wh3_plan(N, H, H, shp, Cin, force=True) is not None
    ref = torch.nn.grad.conv2d_weight(nchw(x.float()), (Cout, Cin, 3, 3), nchw(g.float()), padding=1)
    out = torch.zeros(Cout, Cin, 3, 3, device=cuda)
    ci.conv_wgrad(g, None, None, None, x, shp, out, h3=True)
    assert rel(out, ref) < 2e-3, rel(out, ref)
    old = torch.zeros_like(out)
    ci.conv_wgrad(g, None, None, None, x, shp, old, h3=False)
    assert rel(out, old) < 2e-3
    ci.conv_wgrad(g, None, None, None, x, shp, out, accumulate=True, h3=True)
    assert rel(out, 2 * ref) < 2e-3


WGRAD_CASES = [
    (4, 8, 64, 128, 1, 1, 0),
    (2, 8, 64, 64, 3, 1, 1),
    (2, 16, 128, 128, 3, 2, 1),
    (2, 8, 64, 256, 1, 2, 0),
    (2, 8, 3, 64, 3, 1, 1),
    (3, 5, 64, 64, 3, 1, 1),
]


@pytest.mark.parametrize("case", WGRAD_CASES)
@pytest.mark.parametrize("mode", ["plain", "affine"])
@pytest.mark.parametrize("variant", ["default", "fused_reduce_stages4"])
def test_conv_wgrad(cuda, case, mode, variant, monkeypatch):
    """variant fused_reduce_stages4: the splits combined in-kernel by each tile's last arriver
    (no wgrad_reduce launch) and 4 register-staged K tiles in flight."""
    if variant != "default":
        monkeypatch.setattr(ci, "WG_FUSED_REDUCE", True)
        monkeypatch.setattr(ci, "WG_STAGES", 4)
    N, H, Cin, Cout, k, stride, pad = case
    torch.manual_seed(2)
    shp = ci.ConvShape(Cin, Cout, k, stride, pad)
    x = padc(make((N, H, H, Cin), cuda), shp.cxp)
    Ho, Wo = ci.out_hw(H, H, shp)
    g = make((N, Ho, Wo, Cout), cuda)
    y = make((N, Ho, Wo, Cout), cuda)
    if mode == "plain":
        al = be = xs = xt = None
        act = 0
        gt = g.float()
        a = x.float()[..., :Cin]
    else:
        al = torch.randn(Cout, device=cuda) * 0.1
        be = torch.randn(Cout, device=cuda) * 0.1
        xs = torch.rand(shp.cxp, device=cuda) + 0.5
        xt = torch.randn(shp.cxp, device=cuda) * 0.3
        act = 1
        gt = (g.float() + al + be * y.float()).to(BF).float()
        a = torch.relu(x.float() * xs + xt).to(BF).float()[..., :Cin]
    ref = torch.nn.grad.conv2d_weight(nchw(a), (Cout, Cin, k, k), nchw(gt), stride=stride, padding=pad)
    # split counts <= 8 take the channel-major reduce for unpadded 3x3 layers, 12 the column form
    for ns, tile in [(1, None), (3, None), (2, (64, 64, 32)), (1, (128, 128, 64)), (12, None)]:
        if tile and Cout % tile[0]:
            continue
        out = torch.empty(Cout, Cin, k, k, device=cuda)
        ci.conv_wgrad(g, y, al, be, x, shp, out, xs, xt, act, nsplit=ns, tile=tile)
        assert rel(out, ref) < 5e-3, (ns, tile, rel(out, ref))
        prev = torch.randn_like(out)
        acc = prev.clone()
        ci.conv_wgrad(g, y, al, be, x, shp, acc, xs, xt, act, nsplit=ns, tile=tile, accumulate=True)
        assert rel(acc - prev, ref) < 5e-3, (ns, tile, "accumulate")


@pytest.mark.parametrize("cout,cin,k", [(64, 3, 3), (256, 64, 1), (512, 512, 3), (48, 72, 3), (2048, 512, 1)])
def test_pack_weights_layouts(cuda, cout, cin, k):
    """fp32 OIHW -> bf16 forward layout [Cout][taps][Cxp] (zero channel padding) and dgrad
    layout [Cin][taps][Cout], against torch permutes."""
    shp = ci.ConvShape(cin, cout, k, 1, k // 2)
    w = torch.randn(cout, cin, k, k, device=cuda)
    wf, wd = ci.alloc_packed(shp, cuda, dgrad=True)
    ci.pack_weights([(w, wf, wd, shp)])
    wb = w.to(BF)
    ref_f = torch.zeros(cout, k * k, shp.cxp, device=cuda, dtype=BF)
    ref_f[:, :, :cin] = wb.permute(0, 2, 3, 1).reshape(cout, k * k, cin)
    assert torch.equal(wf.view(cout, k * k, shp.cxp), ref_f)
    ref_d = wb.permute(1, 2, 3, 0).reshape(cin, k * k, cout)
    assert torch.equal(wd.view(cin, k * k, cout)[:cin], ref_d)


@pytest.mark.parametrize("case", [(4, 8, 64, 128, 1, 1, 0), (2, 8, 64, 64, 3, 1, 1), (2, 8, 64, 256, 1, 2, 0)])
def test_fold_gradient_scale(cuda, case):
    """PRO_FOLD with a per-channel gradient scale gs (the residual join stores ONE
    gradient; each branch folds in its own BN scale): g*gs + al + be*y in dgrad and wgrad."""
    N, H, Cin, Cout, k, stride, pad = case
    torch.manual_seed(3)
    shp = ci.ConvShape(Cin, Cout, k, stride, pad)
    w = torch.randn(Cout, Cin, k, k, device=cuda) / (Cin * k * k) ** 0.5
    wf, wd = ci.alloc_packed(shp, cuda)
    ci.pack_weights([(w, wf, wd, shp)])
    Ho, Wo = ci.out_hw(H, H, shp)
    g = make((N, Ho, Wo, Cout), cuda)
    y = make((N, Ho, Wo, Cout), cuda)
    al = torch.randn(Cout, device=cuda) * 0.1
    be = torch.randn(Cout, device=cuda) * 0.1
    gs = torch.rand(Cout, device=cuda) + 0.5
    gt = (g.float() * gs + al + be * y.float()).to(BF).float()
    xs_shape = (N, H, H, Cin)
    ref = nhwc(torch.nn.grad.conv2d_input((N, Cin, H, H), w.to(BF).float(), nchw(gt), stride=stride, padding=pad))
    for ns in (1, 3):
        out, _ = ci.conv_dgrad(g, y, al, be, wd, shp, xs_shape, epi=ci.EPI_STORE, nsplit=ns, gs=gs)
        assert rel(out, ref) < 1e-2, ns
    x = padc(make(xs_shape, cuda), shp.cxp)
    refw = torch.nn.grad.conv2d_weight(nchw(x.float()[..., :Cin]), (Cout, Cin, k, k), nchw(gt), stride=stride,
                                       padding=pad)
    for ns in (1, 2):
        outw = torch.empty(Cout, Cin, k, k, device=cuda)
        ci.conv_wgrad(g, y, al, be, x, shp, outw, nsplit=ns, gs=gs)
        assert rel(outw, refw) < 5e-3, ns


@pytest.mark.parametrize("case", [(4, 8, 64, 256, 1, 1, 0), (3, 5, 128, 64, 1, 1, 0), (2, 4, 512, 1024, 1, 1, 0)])
@pytest.mark.parametrize("join", ["relu_mask", "relu_mask_shortcut", "celu_z", "celu_z_shortcut"])
@pytest.mark.parametrize("ns", [1, 3])
def test_conv_dgrad_join_backward(cuda, case, join, ns):
    """EPI_JOINBWD: the dgrad that completes a block-output gradient also runs that block's
    residual-join backward: g_pre = (prev + dA) * act'(z) stored in place, slots
    (sum g_pre*y_res, sum g_pre, sum g_pre*y_sc).  CELU joins: the oracle is the fp32
    derivative exp(z/alpha) of the fp32 pre-activation z = ya*sa + ta + (yb*sb + tb | xid)
    (reference nn.CELU autograd, resnet.py:188-190) -- NOT a formula of the bf16 join output."""
    from faster_distributed_training_amd.ops import _native
    nat = _native.native()
    N, H, Cin, Cout, k, stride, pad = case
    torch.manual_seed(5)
    shp = ci.ConvShape(Cin, Cout, k, stride, pad)
    w = torch.randn(Cout, Cin, k, k, device=cuda) / (Cin * k * k) ** 0.5
    wf, wd = ci.alloc_packed(shp, cuda)
    ci.pack_weights([(w, wf, wd, shp)])
    g = make((N, H, H, Cout), cuda)
    y = make((N, H, H, Cout), cuda)
    al = torch.randn(Cout, device=cuda) * 0.1
    be = torch.randn(Cout, device=cuda) * 0.1
    gt = (g.float() + al + be * y.float()).to(BF).float()
    xs = (N, H, H, Cin)
    dA = nhwc(torch.nn.grad.conv2d_input((N, Cin, H, H), w.to(BF).float(), nchw(gt), stride=1, padding=pad))
    prev = make(xs, cuda)
    ya = make(xs, cuda)
    yb = make(xs, cuda) if join.endswith("shortcut") else None
    zkw = {}
    if join.startswith("celu"):
        act, alpha = 2, 0.075
        mask = None
        sa = torch.rand(Cin, device=cuda) * 0.5 + 0.2
        ta = torch.randn(Cin, device=cuda) * 0.3 - 0.3   # most of z negative: the CELU tail
        if yb is not None:
            sb = torch.rand(Cin, device=cuda) * 0.5 + 0.2
            tb = torch.randn(Cin, device=cuda) * 0.2
            z = ya.float() * sa + ta + (yb.float() * sb + tb)
            zkw = dict(es=sa, et=ta, jz=(sb, tb, None))
        else:
            xid = make(xs, cuda)
            z = ya.float() * sa + ta + xid.float()
            zkw = dict(es=sa, et=ta, jz=(None, None, xid))
        assert (z < -0.5).float().mean() > 0.2  # the regime the bf16-output formula gets wrong
        dact = torch.where(z > 0, torch.ones_like(z), torch.exp(z.double() / alpha).float())
    else:
        out_join = make(xs, cuda)
        act, alpha = 1, 1.0
        dact = (out_join.float() > 0).float()
        mask = torch.empty(out_join.numel() // 8, device=cuda, dtype=torch.uint8)
        # the forward join kernel's mask: residual_act_fwd with y_a = out, s = 1, t = 0, x = 0
        one, zero = torch.ones(Cin, device=cuda), torch.zeros(Cin, device=cuda)
        tmp = torch.empty_like(out_join)
        nat.residual_act_fwd(out_join.data_ptr(), one.data_ptr(), zero.data_ptr(), 0, 0, 0,
                             torch.zeros_like(out_join).data_ptr(), tmp.data_ptr(), mask.data_ptr(),
                             N * H * H, Cin, 1, 1.0, 1, _native.stream_ptr())
    gp = (prev.float() + dA) * dact
    part = ci.stat_slots(3, Cin, cuda)
    out = prev.clone()
    ci.conv_dgrad(g, y, al, be, wd, shp, xs, epi=ci.EPI_JOINBWD, out=out, ex=ya, part=part, act=act, alpha=alpha,
                  jmask=mask, jyb=yb, nsplit=ns, **zkw)
    # elementwise: bf16 rounding of the stored g_pre (and of dA's bf16 operand) only
    err = (out.float() - gp).abs()
    assert (err <= gp.abs() * 2 ** -7 + dact * 1e-3 + 1e-7).float().mean() > 0.999, err.max()
    assert rel(out, gp) < 1e-2
    ps = part.sum(0)
    assert rel(ps[0], (gp * ya.float()).reshape(-1, Cin).sum(0)) < 1e-2
    assert rel(ps[1], gp.reshape(-1, Cin).sum(0)) < 1e-2
    if yb is not None:
        assert rel(ps[2], (gp * yb.float()).reshape(-1, Cin).sum(0)) < 1e-2
    else:
        assert torch.count_nonzero(ps[2]).item() == 0


@pytest.mark.parametrize("shortcut", [False, True])
def test_celu_join_backward_uses_preactivation(cuda, shortcut):
    """The standalone join backward (residual_act_bwd, the last block / strided blocks) in z mode
    matches the fp32 exp(z/alpha) oracle on the CELU tail, and the legacy derivative from the
    bf16 OUTPUT (1 + o/alpha) does not -- the round-5 ResNet-18 convergence gap
    (profiles/r6/convergence_ablation.txt)."""
    from faster_distributed_training_amd.ops import _native
    nat = _native.native()
    torch.manual_seed(11)
    N, H, C, alpha = 4, 8, 64, 0.075
    M = N * H * H
    ya, g = make((N, H, H, C), cuda), make((N, H, H, C), cuda)
    sa = torch.rand(C, device=cuda) * 0.5 + 0.2
    ta = torch.randn(C, device=cuda) * 0.3 - 0.4
    yb = make((N, H, H, C), cuda) if shortcut else None
    sb = torch.rand(C, device=cuda) * 0.5 + 0.2 if shortcut else None
    tb = torch.randn(C, device=cuda) * 0.2 if shortcut else None
    xid = None if shortcut else make((N, H, H, C), cuda)
    # the forward join (bf16 output o), as the engine runs it
    out = torch.empty_like(ya)
    nat.residual_act_fwd(ya.data_ptr(), sa.data_ptr(), ta.data_ptr(), _p(yb), _p(sb), _p(tb),
                         0 if shortcut else xid.data_ptr(), out.data_ptr(), 0, M, C, 2, alpha, 1,
                         _native.stream_ptr())
    z = ya.float() * sa + ta + (yb.float() * sb + tb if shortcut else xid.float())
    want = g.float() * torch.where(z > 0, torch.ones_like(z), torch.exp(z.double() / alpha).float())

    def run(jz):
        gpre = torch.empty_like(ya)
        part = ci.stat_slots(3, C, cuda)
        nat.residual_act_bwd(g.data_ptr(), 0 if jz else out.data_ptr(), 0, ya.data_ptr(), _p(yb), gpre.data_ptr(),
                             part.data_ptr(), part.shape[0], M, C, 2, alpha, 1, _native.stream_ptr(), 0,
                             [_p(v) for v in jz] if jz else [])
        return gpre.float(), part.sum(0)

    tail = z < -0.5
    assert tail.float().mean() > 0.2
    got, ps = run([sa, ta, sb, tb, xid])
    tol = want.abs() * 2 ** -7 + 1e-7
    assert ((got - want).abs() <= tol).float().mean() > 0.999
    assert rel(ps[1], want.reshape(-1, C).sum(0)) < 1e-2
    assert rel(ps[0], (want * ya.float()).reshape(-1, C).sum(0)) < 1e-2
    legacy, _ = run(None)
    # on the tail the output-based derivative is mostly wrong by more than bf16 rounding ...
    assert ((legacy - want).abs() > tol)[tail].float().mean() > 0.5
    # ... including sign flips of g (o rounded below -alpha)
    assert ((legacy * want) < 0)[tail].any()


def test_strided_dgrad_store_writes_every_parity_class(cuda):
    """A 1x1 stride-2 dgrad with EPI_STORE must write zeros in the parity classes it has no
    taps for (the engine's shortcut dgrad is the first writer of the block-input gradient)."""
    shp = ci.ConvShape(64, 256, 1, 2, 0)
    w = torch.randn(256, 64, 1, 1, device=cuda) / 8
    wf, wd = ci.alloc_packed(shp, cuda)
    ci.pack_weights([(w, wf, wd, shp)])
    g = make((2, 4, 4, 256), cuda)
    xs = (2, 8, 8, 64)
    out = torch.full(xs, float("nan"), device=cuda, dtype=BF)
    ci.conv_dgrad(g, None, None, None, wd, shp, xs, epi=ci.EPI_STORE, out=out)
    ref = nhwc(torch.nn.grad.conv2d_input((2, 64, 8, 8), w.to(BF).float(), nchw(g), stride=2, padding=0))
    assert torch.isfinite(out.float()).all() and rel(out, ref) < 1e-2


@pytest.mark.parametrize("tile", [(64, 64, 64), (128, 64, 64), (64, 128, 64), (128, 128, 64), (64, 64, 128)])
def test_kgroups_match_reference(cuda, tile):
    """K groups (kg=2: 8-wave workgroups whose halves take alternate K tiles, partial sums
    handed over in LDS) for the forward conv with/without the lazy-BN prologue, the join
    prologue and the folded dgrad with the activation-backward epilogue, odd and even K-tile
    counts, against fp32 PyTorch; the statistics slots too."""
    torch.manual_seed(7)
    for (N, H, Cin, Cout, k, stride, pad) in [(2, 8, 64, 128, 3, 1, 1), (2, 4, 512, 128, 3, 1, 1),
                                             (3, 5, 256, 128, 1, 1, 0), (2, 8, 64, 256, 1, 2, 0)]:
        if Cout % tile[1]:
            continue
        shp = ci.ConvShape(Cin, Cout, k, stride, pad)
        x = padc(make((N, H, H, Cin), cuda), shp.cxp)
        w = torch.randn(Cout, Cin, k, k, device=cuda) / (Cin * k * k) ** 0.5
        wf, wd = ci.alloc_packed(shp, cuda)
        ci.pack_weights([(w, wf, wd, shp)])
        s = torch.rand(Cin, device=cuda) + 0.5
        t = torch.randn(Cin, device=cuda) * 0.3
        for pro in ("plain", "relu"):
            a = x.float() if pro == "plain" else torch.relu(x.float() * s + t).to(BF).float()
            ref = nhwc(F.conv2d(nchw(a), w.to(BF).float(), stride=stride, padding=pad))
            y, part = ci.conv_fwd(x, wf, shp, None if pro == "plain" else s, None if pro == "plain" else t,
                                  0 if pro == "plain" else 1, 1.0, tile=tile, nsplit=1, kg=2)
            assert rel(y, ref) < 1e-2, (tile, pro, rel(y, ref))
            ps, yf = part.sum(0), ref.reshape(-1, Cout)
            assert rel(ps[0], yf.sum(0)) < 2e-3 and rel(ps[1], (yf * yf).sum(0)) < 2e-3
        # dgrad: fold prologue + ReLU activation backward epilogue
        Ho, Wo = ci.out_hw(H, H, shp)
        g, yy = make((N, Ho, Wo, Cout), cuda), make((N, Ho, Wo, Cout), cuda)
        al, be = torch.randn(Cout, device=cuda) * 0.1, torch.randn(Cout, device=cuda) * 0.1
        gt = (g.float() + al + be * yy.float()).to(BF).float()
        dref = nhwc(torch.nn.grad.conv2d_input((N, Cin, H, H), w.to(BF).float(), nchw(gt), stride=stride,
                                               padding=pad))
        if Cin % tile[1] == 0:
            xs = (N, H, H, Cin)
            out, _ = ci.conv_dgrad(g, yy, al, be, wd, shp, xs, epi=ci.EPI_STORE, tile=tile, nsplit=1, kg=2)
            assert rel(out, dref) < 1e-2, (tile, "dgrad")
            ex = make(xs, cuda)
            es, et = torch.rand(Cin, device=cuda) + 0.5, torch.randn(Cin, device=cuda) * 0.3
            gp = dref * ((ex.float() * es + et) > 0).float()
            out, part = ci.conv_dgrad(g, yy, al, be, wd, shp, xs, epi=ci.EPI_ACTBWD, ex=ex, es=es, et=et, act=1,
                                      tile=tile, nsplit=1, kg=2)
            assert rel(out, gp * es) < 1e-2, (tile, "actbwd")
            ps = part.sum(0)
            assert rel(ps[0], (gp * ex.float()).reshape(-1, Cin).sum(0)) < 1e-2
            assert rel(ps[1], gp.reshape(-1, Cin).sum(0)) < 1e-2
        # join prologue (1x1 stride-1 only)
        if k == 1 and stride == 1:
            yj, rj = make((N, H, H, Cin), cuda), make((N, H, H, Cin), cuda)
            joined = torch.relu(yj.float() * s + t + rj.float())
            jref = nhwc(F.conv2d(nchw(joined.to(BF).float()), w.to(BF).float()))
            jout = torch.empty_like(yj)
            jmask = torch.zeros(yj.numel() // 8, device=cuda, dtype=torch.uint8)
            out, _ = ci.conv_fwd_join(yj, rj, s, t, None, None, wf, shp, jout, jmask, tile=tile, nsplit=1, kg=2)
            assert rel(out, jref) < 1e-2, (tile, "join")
            assert rel(jout, joined) < 1e-2



@pytest.mark.parametrize("tile", [(128, 128, 32), (64, 64, 32), (128, 64, 64), (64, 128, 64), (256, 64, 64),
                                  (64, 64, 128)])
@pytest.mark.parametrize("nsplit", [1, 2])
def test_lds_dma_ring_matches_register_path(cuda, tile, nsplit):
    """kg=3 (operand tiles staged global -> LDS by LDS-DMA into a 3-buffer ring) runs the same
    MFMA sequence as the register-staged path: bitwise-equal forward / dgrad outputs for 3x3
    (padding taps, strides) and 1x1 convolutions, split-K included, and both within bf16
    tolerance of fp32 PyTorch."""
    torch.manual_seed(11)
    for (N, H, Cin, Cout, k, stride, pad) in [(2, 8, 64, 128, 3, 1, 1), (2, 9, 128, 256, 3, 2, 1),
                                             (3, 5, 256, 128, 1, 1, 0), (2, 4, 512, 512, 3, 1, 1)]:
        if Cout % tile[1]:
            continue
        shp = ci.ConvShape(Cin, Cout, k, stride, pad)
        x = padc(make((N, H, H, Cin), cuda), shp.cxp)
        w = torch.randn(Cout, Cin, k, k, device=cuda) / (Cin * k * k) ** 0.5
        wf, wd = ci.alloc_packed(shp, cuda)
        ci.pack_weights([(w, wf, wd, shp)])
        ref = nhwc(F.conv2d(nchw(x.float()), w.to(BF).float(), stride=stride, padding=pad))
        y1, p1 = ci.conv_fwd(x, wf, shp, tile=tile, nsplit=nsplit, kg=1)
        y3, p3 = ci.conv_fwd(x, wf, shp, tile=tile, nsplit=nsplit, kg=3)
        assert rel(y3, ref) < 1e-2, (tile, "fwd", rel(y3, ref))
        assert torch.equal(y1, y3), (tile, "fwd bitwise", (y1.float() - y3.float()).abs().max().item())
        assert torch.equal(p1, p3)
        if Cin % tile[1]:
            continue
        Ho, Wo = ci.out_hw(H, H, shp)
        g = make((N, Ho, Wo, Cout), cuda)
        xs = (N, H, H, Cin)
        dref = nhwc(torch.nn.grad.conv2d_input((N, Cin, H, H), w.to(BF).float(), nchw(g), stride=stride,
                                               padding=pad))
        d1, _ = ci.conv_dgrad(g, None, None, None, wd, shp, xs, epi=ci.EPI_STORE, tile=tile, nsplit=nsplit, kg=1)
        d3, _ = ci.conv_dgrad(g, None, None, None, wd, shp, xs, epi=ci.EPI_STORE, tile=tile, nsplit=nsplit, kg=3)
        assert rel(d3, dref) < 1e-2, (tile, "dgrad", rel(d3, dref))
        assert torch.equal(d1, d3), (tile, "dgrad bitwise")
        ex = make(xs, cuda)
        es, et = torch.rand(Cin, device=cuda) + 0.5, torch.randn(Cin, device=cuda) * 0.3
        a1, q1 = ci.conv_dgrad(g, None, None, None, wd, shp, xs, epi=ci.EPI_ACTBWD, ex=ex, es=es, et=et, act=1,
                               tile=tile, nsplit=nsplit, kg=1)
        a3, q3 = ci.conv_dgrad(g, None, None, None, wd, shp, xs, epi=ci.EPI_ACTBWD, ex=ex, es=es, et=et, act=1,
                               tile=tile, nsplit=nsplit, kg=3)
        assert torch.equal(a1, a3) and torch.equal(q1, q3), (tile, "actbwd bitwise")
