"""NGD optimizer steps replayed as HIP graphs (optim/ngd.py NGD._graph_step) against eager
steps from the same state -- review r2 5b: replays had drifted 2-4 % after update steps."""
import pytest
import torch
import torch.nn as nn

pytestmark = pytest.mark.gpu


def _opt(cuda, graphs):
    from faster_distributed_training_amd.optim.ngd import NGD
    from faster_distributed_training_amd.utils.flat import FlatParams
    torch.manual_seed(0)
    m = nn.Sequential(nn.Conv2d(64, 64, 3), nn.Conv2d(64, 128, 1), nn.Linear(256, 512), nn.Linear(512, 96)).to(cuda)
    flat = FlatParams(m, device=cuda)
    opt = NGD(flat, lr=0.05, momentum=0.9, weight_decay=1e-4)
    opt.graphs = graphs  # (the graph path is opt-in: FDT_NGD_GRAPHS=1)
    return flat, opt


def test_ngd_graph_replay_matches_eager_over_three_update_periods(cuda):
    fa, oa = _opt(cuda, False)
    fb, ob = _opt(cuda, True)
    gen = torch.Generator().manual_seed(1)
    coef = torch.ones((), device=cuda)  # a static clip coefficient, like GradClipper's
    for step in range(10 + 3 * 4 + 2):  # initialisation schedule, then three update periods
        if step == 15:
            for o in (oa, ob):  # a scheduler changing the learning rate between replays
                o.param_groups[0]["lr"] = 0.02
        if step >= 17:
            for o in (oa, ob):  # ... and the momentum every step (OneCycleLR's cycle_momentum)
                o.param_groups[0]["momentum"] = 0.85 + 0.01 * (step % 5)
        g = (torch.randn(fa.numel, generator=gen) * 1e-2).to(cuda)
        fa.grad.copy_(g)
        fb.grad.copy_(g)
        coef.fill_(0.5 + 0.01 * step)
        oa.step(grad_scale=coef)
        ob.step(grad_scale=coef)
        oa.sync_state()
        ob.sync_state()
        torch.cuda.synchronize()
        err = ((fa.data - fb.data).abs().max() / fa.data.abs().max()).item()
        assert err <= 1e-6, (step, err)
    assert ob.graph_replays == 14 and oa.graph_replays == 0
    assert {k[0] for k in ob._gcache} == {True, False} and len(ob._gcache) == 2  # captured once per kind
    for (sa, _), (sb, _) in zip(oa.groups, ob.groups):
        for (_, xa), (_, xb) in zip(sa.axes, sb.axes):
            assert xa.t == xb.t and torch.allclose(xa.W, xb.W, rtol=1e-5, atol=1e-7)
