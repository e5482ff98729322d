#!/usr/bin/env python3
"""Headline benchmark: ResNet-50 (CIFAR stem) training throughput, global batch 1024, DDP.

BASELINE.json metric: "images/sec (whole node) ResNet-50 bs=1024 DDP at 1/2/4/8 MI355X;
epoch time".  Reference number: ~680 img/s (derived from the reference's
published epoch time with its tricks enabled).

    python bench.py                               # 1 GPU, defaults
    python bench.py --gpus 8                      # starts 8 ranks itself (child torchrun)
    python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
        --master-port 29500 bench.py --gpus 8 --steps 50 --warmup 10

One timed step = the full reference training step on synthetic CIFAR-shaped data and
random-init weights: device-resident batch + GPU augmentation (crop/flip/normalise),
input mixup, forward + mixup cross-entropy + backward (HIP engine, bf16), bucketed RCCL
gradient all-reduce overlapped with backward, grad-norm clip (10.0), MADGRAD step
(the reference's default optimizer for this path, resnet50_test.py:493).  Global batch is
fixed at 1024 (per-GPU 1024/N, strong scaling).  W warmup steps are
untimed; exactly K steps are timed between barrier + device synchronisation on both
sides; the MAX time over ranks is reported.  Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

BASELINE_IMG_S = 680.0  # ~680 img/s (reference w/ tricks, ~73 s/epoch)
METRIC = "images/sec (whole node) ResNet-50 bs=1024 DDP at 1/2/4/8 MI355X; epoch time"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=8)
    ap.add_argument("--global-batch", type=int, default=1024)
    ap.add_argument("--arch", default="resnet50")
    ap.add_argument("--optimizer", default="madgrad")
    ap.add_argument("--ngd", action="store_true")
    ap.add_argument("--meta_learning", action="store_true")
    ap.add_argument("--fsdp", action="store_true")
    ap.add_argument("--fsdp-param-dtype", default="bf16", choices=["bf16", "fp32"],
                    help="--fsdp: parameter all-gather wire / compute-copy precision (masters stay fp32)")
    ap.add_argument("--fsdp-offload", action="store_true",
                    help="--fsdp: shards + optimizer state in pinned host memory (the reference's CPUOffload; eager)")
    ap.add_argument("--fsdp-offload-optimizer", default="device", choices=["device", "host"],
                    help="--fsdp-offload: optimizer on the GPU over the staged shard, or on the host (reference)")
    ap.add_argument("--fsdp-wrap", default="model", choices=["sublayer", "model"],
                    help="--model transformer --fsdp: wrap units (sublayers, or the whole model as one unit "
                         "like the reference's FSDP(model))")
    ap.add_argument("--fsdp-schedule", default="full_shard", choices=["full_shard", "shard_grad_op"],
                    help="--fsdp: FULL_SHARD (reshard after forward, re-gather in backward) or SHARD_GRAD_OP")
    ap.add_argument("--sharded-ngd", action="store_true",
                    help="with --ngd at N=1: run the sharded-NGD data-parallel path over a world-1 group")
    ap.add_argument("--ddp", action="store_true",
                    help="at N=1: run the DDP bucket reducer over a world-1 group (graph cuts + all-reduce actions "
                         "of the multi-GPU path, without the communication time)")
    ap.add_argument("--precision", default="bf16")
    ap.add_argument("--bucket-mb", type=float, default=25.0)
    ap.add_argument("--first-bucket-mb", type=float, default=None,
                    help="ResNet DDP / sharded NGD: size of the first (classifier-side) bucket (default: the "
                         "trainer's)")
    ap.add_argument("--comm-dtype", default="fp32")
    ap.add_argument("--no-native", action="store_true", help="ablation: plain PyTorch ops (w/o tricks)")
    ap.add_argument("--profile-steps", type=int, default=0)
    ap.add_argument("--no-graphs", action="store_true", help="ablation: launch the engine's kernels eagerly")
    ap.add_argument("--deterministic", action="store_true", help="bitwise-repeatable engine reductions (cost probe)")
    ap.add_argument("--model", default="resnet50", choices=["resnet50", "transformer"],
                    help="transformer: secondary benchmark (BASELINE.json config 4, AG-News-shaped)")
    ap.add_argument("--simulate-world", type=int, default=0,
                    help="rehearse ONE rank of a world-N job on this GPU (parallel/simulate.py): rank R's batch "
                         "share, optimizer / FSDP shards, bucket plan and graph replay, collectives replaced by "
                         "same-sized local copies (no xGMI time); the record is per-rank, not a scaling point")
    ap.add_argument("--simulate-rank", type=int, default=0)
    ap.add_argument("--seq-buckets", default="128,256",
                    help="transformer: padded-length buckets (a batch pads to the smallest bucket >= its longest "
                         "sample; the largest bucket must cover the longest sample, so nothing is truncated)")
    return ap.parse_args()


def _launch_ranks(n: int) -> int:
    """``--gpus N`` (N > 1) without a launcher: start N ranks ourselves, one process per GPU,
    as a CHILD ``torch.distributed.run`` (never an exec, and before anything here touches the
    GPU), relay rank 0's JSON line and return the child's exit code.  Same contract as the
    reference's launcher (/root/reference/run_distributed.sh:2-3), which always starts its
    ranks itself."""
    import socket
    import subprocess
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    proc = subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True, env=env)
    for line in proc.stdout:  # rank 0's record -> our stdout, anything else -> stderr
        if line.startswith("{") and '"metric"' in line:
            sys.stdout.write(line)
            sys.stdout.flush()
        else:
            sys.stderr.write(line)
    return proc.wait()


def main():
    args = parse()
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is None and args.gpus > 1:
        sys.exit(_launch_ranks(args.gpus))
    if world_env is not None and int(world_env) != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but this launcher started WORLD_SIZE={world_env} ranks")
    if args.no_native:
        os.environ["FDT_NATIVE"] = "0"
    if args.simulate_world:
        assert world_env is None and args.gpus == 1, "--simulate-world runs in ONE process on one GPU"
        from faster_distributed_training_amd.parallel import simulate
        simulate.install(args.simulate_rank, args.simulate_world)
    if args.model == "transformer":
        return bench_transformer(args)
    import torch
    import torch.distributed as dist

    from faster_distributed_training_amd.train.resnet_trainer import ResNetConfig, ResNetTrainer

    n = args.simulate_world or int(os.environ.get("WORLD_SIZE", "1"))
    gb = args.global_batch
    assert gb % n == 0, "global batch must divide evenly over ranks"
    cfg = ResNetConfig(arch=args.arch, bs=gb // n, synthetic=True, eval=False, plot=False,
                       distributed=n > 1, ngd=args.ngd, meta_learning=args.meta_learning,
                       optimizer="ngd" if args.ngd else args.optimizer, fsdp=args.fsdp,
                       precision=args.precision, bucket_mb=args.bucket_mb, comm_dtype=args.comm_dtype,
                       fast_path=False if args.no_native else None, graphs=not args.no_graphs,
                       deterministic=args.deterministic, force_sharded=args.sharded_ngd, force_ddp=args.ddp,
                       fsdp_param_dtype=args.fsdp_param_dtype, fsdp_schedule=args.fsdp_schedule,
                       fsdp_offload=args.fsdp_offload, fsdp_offload_optimizer=args.fsdp_offload_optimizer,
                       **({} if args.first_bucket_mb is None else {"first_bucket_mb": args.first_bucket_mb}))
    tr = ResNetTrainer(cfg)
    dev = tr.device
    cuda = dev.type == "cuda"

    def batches():
        while True:
            for b in tr.train_loader:
                yield b

    it = batches()
    tr.model.train()

    def sync():
        if cuda:
            torch.cuda.synchronize()
        if dist.is_initialized():
            from faster_distributed_training_amd.parallel.dist import barrier
            barrier()
            if cuda:
                torch.cuda.synchronize()

    # The engine captures its body into HIP graphs on the 2nd training step (1st = eager
    # warm-up); make sure that one-time capture is never inside the timed window.
    graphs = cuda and not args.no_graphs and not args.no_native
    untimed = max(args.warmup, 3) if graphs else args.warmup
    for i in range(untimed):
        x, y = next(it)
        tr.train_step(x, y)
        if i == 0:
            _first_step_comm()
    sync()
    stager = getattr(tr.train_loader, "stager", None)
    w0 = stager.wait_s if stager is not None else 0.0
    t0 = time.perf_counter()
    for _ in range(args.steps):
        x, y = next(it)
        tr.train_step(x, y)
    host = time.perf_counter() - t0  # host submission time of the K steps (no sync inside)
    waited = (stager.wait_s - w0) if stager is not None else 0.0
    sync()
    elapsed = time.perf_counter() - t0
    if dist.is_initialized():
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev if cuda else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ms = elapsed / args.steps * 1e3
    value = gb * args.steps / elapsed
    native = (os.environ.get("FDT_NATIVE", "1") != "0") and cuda
    rec = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "images/sec",
        "n_gpus": n,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms, 3),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": round(value / BASELINE_IMG_S, 2),
        "dtype": args.precision,
        "data": "synthetic (CIFAR-10-shaped uint8, GPU augmentation), random-init weights",
        "config": {"model": f"{args.arch} (CIFAR stem, 10 classes)", "global_batch": gb, "seq_len": None,
                   "image_size": 32, "parallelism": f"{'fsdp' if args.fsdp else 'dp'}{n}",
                   "optimizer": "ngd" if args.ngd else args.optimizer, "mixup": "meta" if args.meta_learning else "input",
                   "native_kernels": native, "hip_graphs": graphs, "deterministic": args.deterministic},
        "epoch_time_s": round(50000.0 / value, 3),
        "host_ms_per_step": round(host / args.steps * 1e3, 3),
        "host_busy_ms_per_step": round((host - waited) / args.steps * 1e3, 3),
        "peak_mem_gb": round(torch.cuda.max_memory_allocated() / 2**30, 2) if cuda else None,
    }
    _sharding_fields(tr, rec)
    _dist_fields(rec)
    if tr.rank == 0 or rec.get("simulated"):
        print(json.dumps(rec), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


_COMM0 = None


def _first_step_comm():
    """Collective bytes of the first (eager) step of a simulated rank: later steps replay graphs,
    whose captured collectives never reach the Python counters."""
    global _COMM0
    from faster_distributed_training_amd.parallel import simulate
    if simulate.active() is not None and _COMM0 is None:
        _COMM0 = simulate.comm_bytes()


def _dist_fields(rec):
    """The process group that actually ran: its size (must equal n_gpus) and backend."""
    import torch.distributed as dist
    from faster_distributed_training_amd.parallel import simulate
    sim = simulate.active()
    if sim is not None:
        # one GPU played rank R of world N: a per-rank step time, not a scaling point
        rec["metric"] = f"simulated per-rank step: rank {sim.rank} of world {sim.world} on one GPU ({rec['metric']})"
        rec["n_gpus"] = 1
        rec["simulated"] = {"world": sim.world, "rank": sim.rank, "per_rank_batch": rec["config"]["global_batch"] // sim.world,
                            "comm_bytes_first_step": _COMM0,
                            "note": "collectives replaced by same-sized local copies; xGMI transfer time not included"}
        rec["dist_world"] = sim.world
        rec["backend"] = f"simulated({dist.get_backend()})"
        return
    if dist.is_initialized():
        rec["dist_world"] = dist.get_world_size()
        rec["backend"] = dist.get_backend()
    else:
        rec["dist_world"] = 1
        rec["backend"] = None
    assert rec["dist_world"] == rec["n_gpus"], (rec["dist_world"], rec["n_gpus"])


def _sharding_fields(tr, rec):
    """Record which data-parallel path actually ran (FSDP units / ZeRO-2 / bucket reducer) and
    whether the NGD step ran as HIP-graph replays."""
    import torch
    cfg = rec["config"]
    if hasattr(tr.optimizer, "graph_replays"):
        cfg["ngd_graph_replays"] = int(tr.optimizer.graph_replays)
        cfg["ngd_graph_kinds"] = len(tr.optimizer._gcache)
    if tr.reducer is not None:
        cfg["ddp_buckets"] = len(tr.reducer.buckets)
        plan = getattr(tr.model, "_plan", None)
        states = list(getattr(plan, "_graphs", {}).values()) if plan is not None else []
        if states and states[0].segments:
            from faster_distributed_training_amd.parallel import graphs
            cfg["bwd_graph_segments"] = len(states[0].segments)
            cfg["bwd_captured_collectives"] = int(getattr(states[0].rec, "captured", 0))
            cfg["graph_comm"] = graphs.comm_status()
    if tr.reducer is not None or getattr(tr, "zero", None) is not None:
        from faster_distributed_training_amd.parallel import graphs
        cfg["graph_comm"] = graphs.comm_status()
    if tr.fsdp is not None:
        cfg["fsdp_units"] = len(tr.fsdp.units)
        cfg["fsdp_wrap"] = "model" if len(tr.fsdp.units) == 1 and tr.fsdp.units[0].name == "" else "per-unit"
        cfg["fsdp_peak_full_bytes"] = int(tr.fsdp.peak_full_bytes)
        cfg["fsdp_shard_numel"] = int(tr.fsdp.space.numel)
        cfg["fsdp_static_graphs"] = bool(tr.fsdp.static)
        # what actually ran: the static ring is FULL_SHARD; static without it SHARD_GRAD_OP;
        # eager FSDP reshards after forward (FULL_SHARD)
        cfg["fsdp_schedule"] = "shard_grad_op" if (tr.fsdp.static and not tr.fsdp.ring) else "full_shard"
        cfg["fsdp_param_dtype"] = str(tr.fsdp.param_dtype or torch.float32).replace("torch.", "")
        cfg["fsdp_offload"] = bool(tr.fsdp.offload)
        if tr.fsdp.offload:
            cfg["fsdp_offload_optimizer"] = "device" if tr.fsdp.opt_on_device else "host"
    elif tr.zero is not None:
        cfg["optimizer_sharding"] = "ngd-owner-shards (bucketed all-reduce overlapped with backward + all-gather)"
        cfg["owner_shard_numel"] = int(tr.zero.view.numel)
        cfg["ddp_buckets"] = len(tr.zero.buckets)
    elif tr.reducer is not None:
        cfg["ddp_buckets"] = len(tr.reducer.buckets)


def bench_transformer(args):
    """Transformer text classifier (6 layers, d 512, vocab 30522), AG-News-shaped synthetic
    batches padded to a length bucket (never truncated: the reference pads to the longest
    sample), global batch 256 (reference: 64 x 4 GPUs), NGD optimizer (run_distributed.sh:3),
    bf16."""
    import torch
    import torch.distributed as dist

    from faster_distributed_training_amd.train.transformer_trainer import TransformerConfig, TransformerTrainer

    world = args.simulate_world or int(os.environ.get("WORLD_SIZE", "1"))
    gb = 256 if args.global_batch == 1024 else args.global_batch
    assert gb % world == 0
    buckets = tuple(sorted(int(b) for b in args.seq_buckets.split(",")))
    cfg = TransformerConfig(batch_size=gb // world, synthetic=True, eval=False, plot=False, distributed=world > 1,
                            ngd=True, precision=args.precision, length_buckets=buckets,
                            bucket_mb=args.bucket_mb, fsdp=args.fsdp, epoch=1, fsdp_param_dtype=args.fsdp_param_dtype,
                            fsdp_schedule=args.fsdp_schedule, fsdp_wrap=args.fsdp_wrap,
                            fsdp_offload=args.fsdp_offload, fsdp_offload_optimizer=args.fsdp_offload_optimizer)
    tr = TransformerTrainer(cfg)
    longest = int(tr.train_loader.store.lengths.max())
    assert longest <= buckets[-1], f"largest bucket {buckets[-1]} would truncate samples of length {longest}"
    dev = tr.device
    cuda = dev.type == "cuda"
    it = iter(tr.train_loader)
    tr.model.train()

    def sync():
        if cuda:
            torch.cuda.synchronize()
        if dist.is_initialized():
            from faster_distributed_training_amd.parallel.dist import barrier
            barrier()

    for i in range(args.warmup):
        tr.train_step(*next(it))
        if i == 0:
            _first_step_comm()
    sync()
    t0 = time.perf_counter()
    stager = getattr(tr.train_loader, "stager", None)
    w0 = stager.wait_s if stager is not None else 0.0
    for _ in range(args.steps):
        tr.train_step(*next(it))
    host = time.perf_counter() - t0
    waited = (stager.wait_s - w0) if stager is not None else 0.0
    sync()
    elapsed = time.perf_counter() - t0
    if dist.is_initialized():
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev if cuda else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    value = gb * args.steps / elapsed
    rec = {"metric": "samples/sec (whole node) Transformer AG-News-shaped bs=256", "value": round(value, 2),
           "unit": "samples/sec", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
           "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True, "scaling": "strong",
           "vs_baseline": round(value / 66.0, 2), "dtype": args.precision,
           "data": "synthetic (AG-News-shaped token batches), random-init weights",
           "config": {"model": "transformer 6x512 (vocab 30522)", "global_batch": gb, "seq_len": list(buckets),
                      "truncation": "none (pad to the smallest bucket >= the batch's longest sample)",
                      "parallelism": f"{'fsdp' if args.fsdp else 'dp'}{world}", "optimizer": "ngd"},
           "peak_mem_gb": round(torch.cuda.max_memory_allocated() / 2**30, 2) if cuda else None,
           "host_ms_per_step": round(host / args.steps * 1e3, 3),
           # host_ms minus the time the training thread sat blocked on the staging ring's
           # backpressure (waiting for the GPU to free a slot): the host's own work per step
           "host_busy_ms_per_step": round((host - waited) / args.steps * 1e3, 3)}
    rec["config"]["hip_graphs"] = bool(tr._graphs_on()) if cuda else False
    _sharding_fields(tr, rec)
    _dist_fields(rec)
    if tr.rank == 0 or rec.get("simulated"):
        print(json.dumps(rec), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
