"""End-to-end CLI runs on the CPU (BASELINE.json config 1 "plumbing"), checkpoint written
in the reference schema and resumed."""
import json
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


# ---------------------------------------------------------------- multi-rank entry points
# The driver's scaling run launches bench.py under torchrun with one rank per GPU; these run
# the same entry points with 2 gloo ranks on the CPU (reference run_distributed.sh:2-3,
# utils.py:20-23 setup_norank), so the first multi-rank execution is not the driver's.

_PORT = [29600 + (os.getpid() % 200) * 2]


def _port():
    _PORT[0] += 1
    return _PORT[0]


def _torchrun(args, cwd, nproc=2, timeout=900):
    env = dict(os.environ, FDT_NATIVE="0", PYTHONPATH=ROOT, OMP_NUM_THREADS="2", MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr", "127.0.0.1", "--master-port", str(_port())] + args
    r = subprocess.run(cmd, cwd=cwd, env=env, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return r.stdout


def _bench_lines(out):
    return [json.loads(l) for l in out.splitlines() if l.startswith("{")]


@pytest.mark.parametrize("extra,par,opt", [([], "dp2", "madgrad"),
                                           (["--ngd", "--meta_learning"], "dp2", "ngd"),
                                           (["--fsdp"], "fsdp2", "madgrad")])
def test_bench_two_ranks_torchrun(tmp_path, extra, par, opt):
    out = _torchrun([os.path.join(ROOT, "bench.py"), "--gpus", "2", "--arch", "resnet18", "--global-batch", "16",
                     "--steps", "2", "--warmup", "1"] + extra, tmp_path)
    lines = _bench_lines(out)
    assert len(lines) == 1, out  # rank 0 only
    rec = lines[0]
    assert rec["n_gpus"] == 2 and rec["steps"] == 2 and rec["config"]["parallelism"] == par
    assert rec["dist_world"] == 2
    assert rec["config"]["optimizer"] == opt and rec["config"]["global_batch"] == 16
    assert rec["value"] > 0 and rec["ms_per_step"] > 0
    if "--fsdp" in extra:
        assert rec["config"]["fsdp_units"] > 1


def test_bench_launches_its_own_ranks(tmp_path):
    """``python bench.py --gpus 2`` with no launcher starts 2 ranks itself (child torchrun)
    and relays exactly one JSON line naming a 2-rank process group."""
    env = dict(os.environ, FDT_NATIVE="0", PYTHONPATH=ROOT, OMP_NUM_THREADS="2")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--arch", "resnet18",
                        "--global-batch", "16", "--steps", "2", "--warmup", "1"], cwd=tmp_path, env=env,
                       capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.strip()]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["dist_world"] == 2 and rec["backend"] == "gloo"
    assert rec["config"]["parallelism"] == "dp2"


def test_bench_refuses_world_size_mismatch(tmp_path):
    env = dict(os.environ, FDT_NATIVE="0", PYTHONPATH=ROOT, WORLD_SIZE="2", RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4", "--steps", "1"], cwd=tmp_path,
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode != 0 and "WORLD_SIZE=2" in r.stderr


def test_bench_transformer_two_ranks_torchrun(tmp_path):
    out = _torchrun([os.path.join(ROOT, "bench.py"), "--gpus", "2", "--model", "transformer", "--global-batch", "8",
                     "--steps", "2", "--warmup", "1"], tmp_path)
    lines = _bench_lines(out)
    assert len(lines) == 1 and lines[0]["n_gpus"] == 2 and lines[0]["config"]["parallelism"] == "dp2", out


def test_run_distributed_two_ranks(tmp_path):
    env = dict(os.environ, FDT_NATIVE="0", NGPU="2", MASTER_PORT=str(_port()), OMP_NUM_THREADS="2",
               PYTHONPATH=ROOT)
    common = ["--synthetic", "--epoch", "1", "--steps", "2", "--no_plot", "--checkpoint_dir", str(tmp_path / "ck")]
    r = subprocess.run(["bash", os.path.join(ROOT, "run_distributed.sh"), "resnet", "--arch", "resnet18", "--bs", "8",
                        "--subset_stride", "100"] + common, cwd=tmp_path, env=env, capture_output=True, text=True,
                       timeout=900)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "epoch 0:" in r.stdout and "test epoch 0" in r.stdout
    ck = torch.load(tmp_path / "ck" / "resnet_ckpt.pth", weights_only=True)
    assert all(k.startswith("module.") for k in ck["net"])  # DDP-wrapped schema, like the reference
    env["MASTER_PORT"] = str(_port())
    r = subprocess.run(["bash", os.path.join(ROOT, "run_distributed.sh"), "transformer", "--batch_size", "4",
                        "--layers", "2", "--d_model", "64", "--eval_steps", "2"] + common, cwd=tmp_path, env=env,
                       capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "epoch 0:" in r.stdout


def test_transformer_distributed_faithful_is_fsdp_offload(tmp_path):
    """The reference's ``transformer_test.py --distributed`` is FSDP(whole model) with
    CPUOffload(offload_params=True) (reference transformer_test.py:387-392); ``--faithful``
    selects exactly that path (printed), and it ends where eager FSDP without offload ends."""
    cli = os.path.join(ROOT, "transformer_test.py")
    common = ["--synthetic", "-b", "4", "--epoch", "1", "--steps", "2", "--eval_steps", "1", "--layers", "2",
              "--d_model", "64", "--no_plot", "--ngd", "--distributed", "--faithful"]
    out = _torchrun([cli] + common + ["--checkpoint_dir", str(tmp_path / "off")], tmp_path)
    assert "distributed path: FSDP full_shard (whole model as one unit, eager, CPU offload" in out, out[-2000:]
    assert "the reference's FSDP(model, CPUOffload)" in out
    out2 = _torchrun([cli] + common + ["--fsdp", "--checkpoint_dir", str(tmp_path / "dev")], tmp_path)
    assert "CPU offload" not in out2 and "distributed path: FSDP full_shard (whole model as one unit" in out2
    a = torch.load(tmp_path / "off" / "transformer_ckpt.pth", weights_only=True)["net"]
    b = torch.load(tmp_path / "dev" / "transformer_ckpt.pth", weights_only=True)["net"]
    assert a.keys() == b.keys()
    for k in a:
        assert torch.allclose(a[k].float(), b[k].float(), atol=1e-6, rtol=0), k
