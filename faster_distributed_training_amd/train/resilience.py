"""Failure handling around the training loop (survey §5: failure detection / checkpoint-
resume; the reference only keeps a best-accuracy, weights-only checkpoint and relies on
GradScaler's inf skip, resnet50_test.py:541-548, 664-690).

* ``save_last`` / ``restore_last``: a rolling full-state checkpoint (``*_last.pth``) written
  at the end of every epoch by rank 0 -- model (reference schema, so the reference loader
  reads it), optimizer (flat state incl. NGD preconditioners), scheduler, loss scaler,
  best accuracy, global step, and every RNG stream (python, numpy, torch CPU / device, the
  device data loader's counter RNG) so a resumed run continues the same random sequence.
  Loads use ``weights_only=True``; numpy/python RNG states are stored as tensors/ints.
* per-rank state lives in ``*_last.rank{r}.pth`` next to the main file (every rank writes
  its own): the RNG streams (seeded per rank, so restoring rank 0's on every rank would make
  all ranks draw the same mixup / augmentation / dropout randomness) and, when the optimizer
  state is sharded (FSDP / sharded NGD), that rank's optimizer shard.  A resume must use the
  same world size (checked).
* ``--auto_resume``: at start-up a trainer restores ``*_last.pth`` if present and continues
  with the next epoch -- combined with ``torchrun --max-restarts N`` (run_distributed.sh)
  a crashed or killed rank restarts the job from the last completed epoch.
* ``maybe_inject_fault``: fault-injection hook for tests (``FDT_FAULT_STEP=k`` raises on
  global step k, optionally only on ``FDT_FAULT_RANK``).
* Non-finite gradients (the device-side check in ``GradClipper``) make the optimizer
  kernels skip the update without a host sync; trainers count skipped steps per epoch.
"""
from __future__ import annotations

import os
import random

import numpy as np
import torch

from . import checkpoint as ckpt


class InjectedFault(RuntimeError):
    pass


def maybe_inject_fault(global_step: int, rank: int = 0):
    s = os.environ.get("FDT_FAULT_STEP")
    if s is None or int(s) != global_step:
        return
    r = os.environ.get("FDT_FAULT_RANK")
    if r is not None and int(r) != rank:
        return
    raise InjectedFault(f"injected fault at step {global_step} on rank {rank}")


def last_path(best_path: str) -> str:
    root, ext = os.path.splitext(best_path)
    return root.replace("_ckpt", "") + "_last" + ext


def _rng_state(trainer):
    py = random.getstate()
    npst = np.random.get_state()
    st = {"py_version": int(py[0]), "py_state": torch.tensor(py[1], dtype=torch.int64),
          "np_keys": torch.from_numpy(np.asarray(npst[1], dtype=np.int64)), "np_pos": int(npst[2]),
          "np_has_gauss": int(npst[3]), "np_gauss": float(npst[4]),
          "torch_cpu": torch.get_rng_state()}
    if torch.cuda.is_available() and trainer.device.type == "cuda":
        st["torch_cuda"] = torch.cuda.get_rng_state(trainer.device)
    ld = getattr(trainer, "train_loader", None)
    if ld is not None and isinstance(getattr(ld, "rng", None), torch.Tensor):
        st["loader_rng"] = ld.rng.detach().cpu()
    if ld is not None and isinstance(getattr(ld, "_cpu_gen", None), torch.Generator):
        st["loader_cpu_gen"] = ld._cpu_gen.get_state()
    return st


def _set_rng_state(trainer, st):
    random.setstate((st["py_version"], tuple(int(v) for v in st["py_state"].tolist()), None))
    np.random.set_state(("MT19937", st["np_keys"].numpy().astype(np.uint32), st["np_pos"], st["np_has_gauss"],
                         st["np_gauss"]))
    torch.set_rng_state(st["torch_cpu"])
    if "torch_cuda" in st and trainer.device.type == "cuda":
        torch.cuda.set_rng_state(st["torch_cuda"], trainer.device)
    ld = getattr(trainer, "train_loader", None)
    if ld is not None and "loader_rng" in st:
        ld.rng.copy_(st["loader_rng"].to(ld.rng.device))
    if ld is not None and "loader_cpu_gen" in st:
        ld._cpu_gen.set_state(st["loader_cpu_gen"])


def rank_path(path: str, rank: int, epoch: int | None = None) -> str:
    """Per-rank file of the save after ``epoch`` (epoch-tagged: a crash between the rank
    files and the main file leaves the previous save's rank files intact)."""
    root, ext = os.path.splitext(path)
    tag = "" if epoch is None else f".e{int(epoch)}"
    return f"{root}.rank{rank}{tag}{ext}"


def _sharded(trainer) -> bool:
    """Optimizer state differs per rank: FSDP shards, ZeRO-2 sharded NGD (``trainer.zero``),
    or any other sharder the trainer holds."""
    return (getattr(trainer, "sharder", None) is not None or getattr(trainer, "fsdp", None) is not None
            or getattr(trainer, "zero", None) is not None
            or bool(getattr(getattr(trainer, "optimizer", None), "sharded", False)))


def _drop_stale_rank_files(path: str, rank: int, keep_epoch: int):
    root, ext = os.path.splitext(path)
    d = os.path.dirname(os.path.abspath(path))
    prefix = os.path.basename(f"{root}.rank{rank}.e")
    for f in os.listdir(d):
        if f.startswith(prefix) and f.endswith(ext) and f != os.path.basename(rank_path(path, rank, keep_epoch)):
            try:
                os.remove(os.path.join(d, f))
            except OSError:
                pass


def _optimizer_state(trainer):
    st = {"optimizer": trainer.optimizer.state_dict()}
    ngd = getattr(trainer.optimizer, "ngd_state_dict", None)
    if ngd is not None:
        st["ngd"] = ngd()
    return st


def _load_optimizer_state(trainer, ck):
    trainer.optimizer.load_state_dict(ck["optimizer"])
    if "ngd" in ck and hasattr(trainer.optimizer, "load_ngd_state_dict"):
        trainer.optimizer.load_ngd_state_dict(ck["ngd"])


def save_last(trainer, epoch: int):
    """Full training state after ``epoch`` completed: every rank writes its rank file, rank 0
    the main file, then all ranks barrier."""
    from ..parallel.dist import barrier
    rank, world = int(getattr(trainer, "rank", 0)), int(getattr(trainer, "world", 1))
    step = int(trainer.global_step)
    mine = {"rng": _rng_state(trainer), "rank": rank, "world": world, "epoch": int(epoch), "global_step": step}
    sharded = _sharded(trainer)
    if sharded:
        mine.update(_optimizer_state(trainer))
    path = rank_path(trainer.last_path, rank, epoch)
    os.makedirs(os.path.dirname(os.path.abspath(path)) or ".", exist_ok=True)
    torch.save(mine, path + ".tmp")
    os.replace(path + ".tmp", path)
    barrier()  # every rank file of this save exists before the main file names it
    extra = {"global_step": step, "best_acc": float(trainer.best_acc), "world": world,
             "sharded_optimizer": sharded, "last": True, "rank_files": "epoch_tagged"}
    if not sharded:
        extra.update(_optimizer_state(trainer))
    if getattr(trainer, "scheduler", None) is not None:
        extra["scheduler"] = trainer.scheduler.state_dict()
    if getattr(trainer, "scaler", None) is not None:
        extra["scaler"] = trainer.scaler.state_dict()
    meta = getattr(trainer, "meta", None)
    if meta is not None:
        extra["meta"] = {k: v.detach().cpu() for k, v in meta.state_dict().items()}
    acc = trainer.testing_acc[-1] if getattr(trainer, "testing_acc", None) else 0.0
    ckpt.save_checkpoint(trainer.last_path, trainer.model, acc, epoch, module_prefix=False, extra=extra)
    _drop_stale_rank_files(trainer.last_path, rank, epoch)  # (after the main file's commit + barrier)


def restore_last(trainer) -> bool:
    """Restore ``trainer.last_path`` if it exists; sets ``start_epoch`` to the epoch after
    the saved one.  Returns whether a checkpoint was restored."""
    path = trainer.last_path
    if not os.path.isfile(path):
        return False
    ck = ckpt.load_checkpoint(path)
    rank, world = int(getattr(trainer, "rank", 0)), int(getattr(trainer, "world", 1))
    if int(ck.get("world", world)) != world:
        raise RuntimeError(f"{path} was written by {ck['world']} ranks; resume with the same world size "
                           f"(this run has {world})")
    rp = rank_path(path, rank, int(ck["epoch"]))
    if not os.path.isfile(rp) and ck.get("rank_files") != "epoch_tagged":
        rp = rank_path(path, rank)  # written before rank files were epoch-tagged (untagged names)
    mine = ckpt.load_checkpoint(rp) if os.path.isfile(rp) else None
    if mine is not None and (int(mine.get("epoch", -1)) != int(ck["epoch"])
                             or int(mine.get("global_step", -1)) != int(ck.get("global_step", 0))):
        raise RuntimeError(f"{rp} (epoch {mine.get('epoch')}, step {mine.get('global_step')}) does not belong to "
                           f"{path} (epoch {ck['epoch']}, step {ck.get('global_step')})")
    if ck.get("sharded_optimizer", False) != _sharded(trainer):
        raise RuntimeError(f"{path}: optimizer sharding differs from this run's (--fsdp / sharded NGD)")
    ckpt.load_model_state(trainer.model, ck["net"])
    if hasattr(trainer.flat, "refresh_shadow"):
        trainer.flat.refresh_shadow()
    if ck.get("sharded_optimizer", False):
        if mine is None:
            raise FileNotFoundError(f"missing per-rank optimizer shard {rp}")
        _load_optimizer_state(trainer, mine)
    else:
        _load_optimizer_state(trainer, ck)
    if "scheduler" in ck and getattr(trainer, "scheduler", None) is not None:
        trainer.scheduler.load_state_dict(ck["scheduler"])
    if "scaler" in ck and getattr(trainer, "scaler", None) is not None:
        trainer.scaler.load_state_dict(ck["scaler"])
    if "meta" in ck and getattr(trainer, "meta", None) is not None:
        trainer.meta.load_state_dict(ck["meta"])
    trainer.global_step = int(ck.get("global_step", 0))
    trainer.best_acc = max(float(trainer.best_acc), float(ck.get("best_acc", 0.0)))
    trainer.start_epoch = int(ck["epoch"]) + 1
    rng = mine["rng"] if mine is not None else ck.get("rng")  # (older files: rank 0's only)
    if rng is not None:
        _set_rng_state(trainer, rng)
    return True
