"""Metrics / logging / plotting (survey C2, C3, §5 observability).

* ``DeviceMeter``: per-step loss / lambda-weighted accuracy accumulated ON DEVICE (the
  reference syncs 4-5 times per batch for its tqdm descriptor, ``resnet50_test.py:550-566``);
  read once per epoch (or every ``log_interval`` steps), all-reduced in one collective.
* ``StepTimer``: HIP-event timing of steps/phases, read once per epoch.
* ``JsonlLogger``: rank-0 JSON-lines metrics (step, epoch, img/s, loss, acc, peak mem).
* ``draw_graph``: the reference's matplotlib curves (``utils.py:54-69``), rank 0 only
  (the reference wrote the same PNG from every rank, Q16).
"""
from __future__ import annotations

import json
import os
import time

import numpy as np
import torch

from ..utils.env import is_rank0


class DeviceMeter:
    """Device-side training accumulators [loss sum, correct, samples]: no host sync per step.
    The fused mixup cross-entropy kernel can add into ``acc`` itself (sets ``fused``); then
    ``update`` only counts the step."""

    def __init__(self, device):
        self.device = device
        self.reset()

    def reset(self):
        # zeroed in place once allocated: a captured training step (the transformer's loss
        # kernel inside its HIP graph) keeps adding into this buffer's address
        if getattr(self, "acc", None) is None:
            self.acc = torch.zeros(3, device=self.device, dtype=torch.float32)
        else:
            self.acc.zero_()
        self.steps = 0
        self.fused = False

    @property
    def loss(self):
        return self.acc[0]

    @property
    def correct(self):
        return self.acc[1]

    @property
    def total(self):
        return self.acc[2]

    @torch.no_grad()
    def update(self, loss, logits, y_a, y_b=None, lam=1.0):
        self.steps += 1
        if self.fused:  # the loss kernel already accumulated this step
            self.fused = False
            return
        pred = logits.argmax(1)
        if y_b is None:
            corr = (pred == y_a).sum().float()
        elif isinstance(lam, torch.Tensor) and lam.numel() > 1:
            lv = lam.reshape(-1).float()
            corr = (lv * (pred == y_a).float()).sum() + ((1 - lv) * (pred == y_b).float()).sum()
        else:
            lv = float(lam)
            corr = lv * (pred == y_a).sum().float() + (1 - lv) * (pred == y_b).sum().float()
        self.acc[0] += loss.detach().float().reshape(())
        self.acc[1] += corr
        self.acc[2] += float(logits.shape[0])

    def reduced(self):
        from ..parallel.dist import all_reduce_metrics
        t = self.acc.clone()
        all_reduce_metrics(t)
        loss, correct, total = t.tolist()
        from ..parallel.dist import world
        steps = max(1, self.steps)
        return {"loss": loss / steps / world(), "acc": 100.0 * correct / max(total, 1.0),
                "correct": correct, "total": total}


class StepTimer:
    """Wall-clock + HIP-event timer (events recorded on the current stream, resolved
    lazily: no synchronisation inside the timed loop)."""

    def __init__(self, cuda: bool):
        self.cuda = cuda
        self.events = []

    def mark(self):
        if self.cuda:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            self.events.append(e)
        else:
            self.events.append(time.perf_counter())

    def intervals_ms(self):
        if len(self.events) < 2:
            return []
        if self.cuda:
            torch.cuda.synchronize()
            return [a.elapsed_time(b) for a, b in zip(self.events[:-1], self.events[1:])]
        return [(b - a) * 1e3 for a, b in zip(self.events[:-1], self.events[1:])]


class JsonlLogger:
    def __init__(self, path: str | None):
        self.path = path if is_rank0() else None
        if self.path:
            os.makedirs(os.path.dirname(os.path.abspath(self.path)), exist_ok=True)

    def log(self, **kw):
        if self.path:
            kw.setdefault("time", time.time())
            with open(self.path, "a") as f:
                f.write(json.dumps(kw) + "\n")


def peak_memory_gb(device=None) -> float:
    if torch.cuda.is_available():
        return torch.cuda.max_memory_allocated(device) / 1024**3
    return 0.0


def draw_graph(xs, ys, labels, title, metric, out_dir="."):
    """Reference ``draw_graph`` (``utils.py:54-69``): writes ``<title>.png``."""
    if not is_rank0():
        return None
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    plt.figure(figsize=(12, 8))
    if isinstance(xs[0], (list, np.ndarray)):
        for x_list, y_list, label in zip(xs, ys, labels):
            plt.plot(x_list, y_list, label=label, linewidth=2)
        plt.xticks(xs[0])
    else:
        plt.plot(xs, ys, label=labels, linewidth=2)
        plt.xticks(xs)
    plt.xlabel("Epoch/Iteration")
    plt.ylabel(metric)
    plt.title(title)
    plt.legend()
    plt.grid()
    path = os.path.join(out_dir, title + ".png")
    plt.savefig(path)
    plt.close()
    return path


class PhaseProfiler:
    """``--profile_steps K`` (survey §5 tracing): per-phase device time of the first K train
    steps from HIP events (one synchronisation at the end, none inside the steps), plus
    roctx ranges around each phase so a ``rocprofv3 --marker-trace`` / timeline shows the
    phase structure.  Phases are marked in order by the trainer: ``mark("fwd")`` etc."""

    def __init__(self, steps: int, cuda: bool, logger=None, skip: int = 3):
        # skip: steps left unprofiled first (eager warm-up + HIP-graph capture of the engine)
        self.steps, self.cuda, self.logger = int(steps), cuda, logger
        self.skip = int(skip) if steps > 0 else 0
        self.done = 0
        self.records = []  # per step: [(phase, start_event, end_event)]
        self._cur = None
        self._open = None
        try:
            from torch.cuda import nvtx  # roctx on ROCm builds
            self._nvtx = nvtx if cuda else None
        except Exception:  # noqa: BLE001 - tracing is optional
            self._nvtx = None

    @property
    def active(self):
        return self.done < self.steps

    def _event(self):
        e = torch.cuda.Event(enable_timing=True) if self.cuda else None
        if e is not None:
            e.record()
        return e if e is not None else time.perf_counter()

    def begin_step(self):
        if not self.active:
            return
        if self.skip > 0:
            self.skip -= 1
            self._cur = None
            return
        self._cur = []
        self._open = None

    def mark(self, phase: str):
        """Close the open phase (if any) and open ``phase``."""
        if not self.active or self._cur is None:
            return
        now = self._event()
        if self._open is not None:
            self._cur.append((self._open[0], self._open[1], now))
            if self._nvtx is not None:
                self._nvtx.range_pop()
        self._open = (phase, now)
        if self._nvtx is not None:
            self._nvtx.range_push(phase)

    def end_step(self):
        if not self.active or self._cur is None:
            return
        self.mark("_end")
        if self._nvtx is not None:
            self._nvtx.range_pop()
        self.records.append(self._cur)
        self._cur = None
        self.done += 1
        if self.done == self.steps:
            self.report()

    def summary(self):
        if self.cuda:
            torch.cuda.synchronize()
        tot = {}
        for rec in self.records:
            for ph, a, b in rec:
                ms = a.elapsed_time(b) if self.cuda else (b - a) * 1e3
                tot[ph] = tot.get(ph, 0.0) + ms
        n = max(1, len(self.records))
        return {ph: round(v / n, 4) for ph, v in tot.items()}

    def report(self):
        s = self.summary()
        from ..utils.env import print0
        print0("profile (device ms/step over %d steps): %s" % (len(self.records), json.dumps(s)))
        if self.logger is not None:
            self.logger.log(profile_ms_per_step=s, profile_steps=len(self.records))
