"""End-to-end CLI runs on the CPU (BASELINE.json config 1 "plumbing"), checkpoint written
in the reference schema and resumed."""
import os
import subprocess
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, cwd, timeout=600):
    env = dict(os.environ, FDT_NATIVE="0", PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable] + args, cwd=cwd, env=env, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return r.stdout


def test_resnet_cli_train_checkpoint_resume(tmp_path):
    cli = os.path.join(ROOT, "resnet50_test.py")
    common = ["--synthetic", "--arch", "resnet18", "--bs", "16", "--epoch", "1", "--steps", "2",
              "--subset_stride", "100", "--no_plot", "--meta_learning", "--ngd", "--lr", "0.01"]
    out = _run([cli] + common, tmp_path)
    assert "epoch 0:" in out and "test epoch 0" in out
    ck = torch.load(tmp_path / "checkpoint" / "resnet_ckpt.pth", weights_only=True)
    assert set(ck) >= {"net", "acc", "epoch"} and ck["epoch"] == 0
    out2 = _run([cli, "--resume"] + common, tmp_path)
    assert "epoch 0:" in out2  # the reference re-runs the saved epoch on resume


def test_transformer_cli_train_checkpoint(tmp_path):
    cli = os.path.join(ROOT, "transformer_test.py")
    out = _run([cli, "--synthetic", "-b", "16", "--epoch", "1", "--steps", "3", "--eval_steps", "2", "--layers", "2",
                "--d_model", "64", "--no_plot", "--ngd"], tmp_path)
    assert "epoch 0:" in out and "test epoch 0" in out
    ck = torch.load(tmp_path / "checkpoint" / "transformer_ckpt.pth", weights_only=True)
    assert "net" in ck and any(k.startswith("classifier.classifier.W1") for k in ck["net"])


def test_tuning_scripts_parse(tmp_path):
    out = _run([os.path.join(ROOT, "tuning", "resnet50_tuning.py"), "--synthetic", "--arch", "resnet18", "--bs", "8",
                "--epoch", "1", "--steps", "1", "--no_eval", "--no_plot", "--subset_stride", "200"], tmp_path)
    assert "epoch 0:" in out


def test_run_distributed_script_is_valid_bash():
    r = subprocess.run(["bash", "-n", os.path.join(ROOT, "run_distributed.sh")], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
