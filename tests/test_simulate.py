"""bench.py --simulate-world N --simulate-rank R (parallel/simulate.py): one rank of a world-N
job rehearsed in one process -- rank / world as the framework sees them, collectives replaced by
same-sized local operations, and the sharded paths sized for world N."""
import json
import os
import subprocess
import sys

import pytest
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def test_simulated_collectives_and_identity():
    from faster_distributed_training_amd.parallel import simulate
    simulate.install(2, 4)
    try:
        assert dist.is_initialized() and dist.get_rank() == 2 and dist.get_world_size() == 4
        t = torch.ones(6)
        dist.all_reduce(t)
        assert torch.equal(t, torch.full((6,), 4.0))  # SUM of 4 similar contributions
        m = torch.arange(6.0)
        dist.all_reduce(m, op=dist.ReduceOp.MAX)
        assert torch.equal(m, torch.arange(6.0))
        inp = torch.arange(8.0)
        out = torch.empty(2)
        dist.reduce_scatter_tensor(out, inp, op=dist.ReduceOp.AVG)
        assert torch.equal(out, torch.tensor([4.0, 5.0]))  # rank 2's slice
        full = torch.zeros(8)
        w = dist.all_gather_into_tensor(full, torch.tensor([7.0, 9.0]), async_op=True)
        w.wait()
        assert torch.equal(full, torch.tensor([0, 0, 0, 0, 7.0, 9.0, 0, 0]))
        b = simulate.comm_bytes()
        assert b["all_reduce"] == 6 * 4 * 2 and b["reduce_scatter"] == 32 and b["all_gather"] == 32
    finally:
        simulate.uninstall()
    assert not dist.is_initialized()


@pytest.mark.timeout(600)
def test_bench_simulate_rank_runs_the_sharded_path():
    """The per-rank step of the 8-GPU sharded-NGD configuration, rank 5: batch 1024/8-style
    share, 1/8 owner shard, bucketed reducer -- one JSON record marked as simulated."""
    env = dict(os.environ, FDT_NATIVE="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--simulate-world", "8", "--simulate-rank", "5",
                        "--steps", "1", "--warmup", "1", "--global-batch", "32", "--arch", "resnet18", "--ngd"],
                       capture_output=True, text=True, env=env, timeout=580)
    assert r.returncode == 0, r.stderr[-2000:]
    rec = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert rec["simulated"]["world"] == 8 and rec["simulated"]["rank"] == 5 and rec["n_gpus"] == 1
    assert rec["simulated"]["per_rank_batch"] == 4 and rec["dist_world"] == 8
    assert rec["config"]["parallelism"] == "dp8" and "owner" in rec["config"]["optimizer_sharding"]
    from faster_distributed_training_amd.models import resnet as R
    n = sum(p.numel() for p in R.resnet18(10).parameters())
    assert rec["config"]["owner_shard_numel"] < n / 4  # ~1/8 of the parameters (balanced by NGD cost)
    cb = rec["simulated"]["comm_bytes_first_step"]
    assert cb["all_reduce"] > 0 and cb["all_gather"] > 0


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_simulated_world8_transformer_step_with_graph_comm_check(cuda):
    """Rank 3 of a simulated world-8 transformer run on the GPU: ZeRO-2 sharded NGD, bucket
    all-reduces captured into the step graph, the in-run capture check, and the recapture after
    it (which used to reuse the dropped graphs' private pool and trip the caching allocator's
    use-count assert -- a crash the first real 8-GPU transformer run would have hit)."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--model", "transformer", "--simulate-world",
                        "8", "--simulate-rank", "3", "--steps", "4", "--warmup", "6"],
                       capture_output=True, text=True, timeout=580)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert rec["simulated"]["rank"] == 3 and rec["config"]["hip_graphs"]
    assert rec["config"].get("graph_comm", "").startswith("capture"), rec["config"]


def test_comm_watch_drain_only_for_nccl(monkeypatch):
    """parallel/graphs.drain_comm_watch: before a capture that can take collectives, eager RCCL
    collectives are finished and RCCL's watchdog gets one polling interval; without an nccl
    process group (here: none, then a simulated gloo rank) it returns at once."""
    import time
    from faster_distributed_training_amd.parallel import graphs as G
    from faster_distributed_training_amd.parallel import simulate as S
    slept = []
    monkeypatch.setattr(time, "sleep", lambda s: slept.append(s))
    G.drain_comm_watch()
    assert slept == []
    S.install(0, 2)
    try:
        assert dist.get_backend() == ("nccl" if torch.cuda.is_available() else "gloo")
        G.drain_comm_watch()
        assert slept == ([0.25] if torch.cuda.is_available() else [])
    finally:
        S.uninstall()
