"""Failure handling (survey §5): full-state "last" checkpoint + auto-resume reproduces an
uninterrupted run exactly, fault injection + CLI auto-resume, the non-finite step guard,
and the phase profiler.  CPU (plain-PyTorch path), small ResNet-18 steps."""
import os
import subprocess
import sys

import torch

from faster_distributed_training_amd.train.resnet_trainer import ResNetConfig, ResNetTrainer

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _cfg(tmp_path, **kw):
    base = dict(arch="resnet18", bs=8, epoch=1, synthetic=True, eval=False, plot=False, steps_per_epoch=2,
                checkpoint_dir=str(tmp_path), optimizer="madgrad", seed=7)
    base.update(kw)
    return ResNetConfig(**base)


def _params(tr):
    return tr.flat.data.detach().clone()


def test_auto_resume_reproduces_uninterrupted_run(tmp_path):
    # A: three epochs straight
    a = ResNetTrainer(_cfg(tmp_path / "a", epoch=3)).fit()
    # B: two epochs with the rolling full-state checkpoint, then a fresh process-like
    # trainer that auto-resumes and runs the third
    b1 = ResNetTrainer(_cfg(tmp_path / "b", epoch=2, save_last=True)).fit()
    assert os.path.isfile(b1.last_path)
    b2 = ResNetTrainer(_cfg(tmp_path / "b", epoch=1, auto_resume=True))
    assert b2.start_epoch == 2 and b2.global_step == b1.global_step
    b2.fit()
    assert torch.equal(_params(a), _params(b2)), (_params(a) - _params(b2)).abs().max()
    sa, sb = a.optimizer.state_dict()["flat_state"], b2.optimizer.state_dict()["flat_state"]
    assert sa.keys() == sb.keys() and all(torch.equal(sa[k], sb[k]) for k in sa)


def test_auto_resume_ngd_state(tmp_path):
    b1 = ResNetTrainer(_cfg(tmp_path, epoch=1, save_last=True, ngd=True, optimizer="ngd")).fit()
    b2 = ResNetTrainer(_cfg(tmp_path, epoch=1, auto_resume=True, ngd=True, optimizer="ngd"))
    s1, s2 = b1.optimizer.ngd_state_dict(), b2.optimizer.ngd_state_dict()
    assert len(s1) == len(s2) > 0
    for g1, g2 in zip(s1, s2):
        for x, y in zip(g1, g2):
            assert x["t"] == y["t"] and torch.equal(x["W"], y["W"]) and torch.equal(x["d"], y["d"])


def test_nonfinite_step_is_skipped(tmp_path):
    tr = ResNetTrainer(_cfg(tmp_path))
    x, y = next(iter(tr.train_loader))
    before = _params(tr)
    tr.train_step(torch.full_like(x, float("nan")), y)
    assert torch.equal(before, _params(tr)), "a non-finite step must not touch the parameters"
    assert int(tr.skipped) == 1
    tr.train_step(x, y)
    assert not torch.equal(before, _params(tr)) and int(tr.skipped) == 1


def test_phase_profiler_reports(tmp_path):
    tr = ResNetTrainer(_cfg(tmp_path, profile_steps=2))
    it = iter(tr.train_loader)
    for _ in range(3 + 3):  # 3 warm-up steps are skipped
        tr.train_step(*next(it))
    s = tr.profiler.summary()
    assert {"mixup", "forward", "loss", "backward", "grad_sync", "optimizer"} <= set(s)
    assert all(v >= 0 for v in s.values()) and len(tr.profiler.records) == 2


def test_cli_fault_injection_then_auto_resume(tmp_path):
    env = dict(os.environ, FDT_NATIVE="0", PYTHONPATH=ROOT, FDT_FAULT_STEP="3")
    args = [sys.executable, os.path.join(ROOT, "resnet50_test.py"), "--arch", "resnet18", "--synthetic", "--bs", "8",
            "--epoch", "3", "--steps", "2", "--no_eval", "--no_plot", "--checkpoint_dir", str(tmp_path),
            "--auto_resume", "--log", str(tmp_path / "log.jsonl")]
    r = subprocess.run(args, cwd=tmp_path, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode != 0 and "injected fault at step 3" in (r.stderr + r.stdout)
    assert os.path.isfile(tmp_path / "resnet_last.pth")  # epoch 0 completed and was saved
    env.pop("FDT_FAULT_STEP")
    r = subprocess.run(args, cwd=tmp_path, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "auto-resume" in r.stdout and "continuing at epoch 1" in r.stdout
    ck = torch.load(tmp_path / "resnet_last.pth", weights_only=True)
    assert ck["epoch"] == 3 and ck["global_step"] == 8  # resumed run: epochs 1..3, 2 steps each


def test_transformer_auto_resume(tmp_path):
    from faster_distributed_training_amd.train.transformer_trainer import TransformerConfig, TransformerTrainer

    def cfg(**kw):
        base = dict(batch_size=8, epoch=1, synthetic=True, eval=False, plot=False, steps_per_epoch=2, n_layers=1,
                    d_model=64, heads=4, d_ff=128, d_hidden=128, length_buckets=(32,), checkpoint_dir=str(tmp_path),
                    optimizer="mirror_madgrad", seed=3, profile_steps=1,
                    extra={"scheduler": "multistep"})  # OneCycle's length depends on --epoch
        base.update(kw)
        return TransformerConfig(**base)
    a = TransformerTrainer(cfg(epoch=2, checkpoint_dir=str(tmp_path / "a"))).fit()
    TransformerTrainer(cfg(epoch=1, save_last=True)).fit()
    b = TransformerTrainer(cfg(epoch=1, auto_resume=True))
    assert b.start_epoch == 1
    b.fit()
    assert torch.equal(a.flat.data, b.flat.data)
