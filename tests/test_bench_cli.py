"""bench.py's launch contract, on the CPU: --gpus N must
run exactly N ranks -- started by bench.py itself when torchrun's env is
absent -- and a world / GPU-count mismatch must fail non-zero instead of
printing a line for fewer GPUs than asked."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _run(args, **env):
    e = {k: v for k, v in os.environ.items()
         if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
    e.update(env)
    return subprocess.run([sys.executable, BENCH] + args, env=e, capture_output=True, text=True,
                          timeout=120)


def test_world_mismatch_fails():
    r = _run(["--gpus", "2", "--steps", "1", "--warmup", "0"], WORLD_SIZE="1")
    assert r.returncode != 0
    assert "--gpus 2 but the process group has 1 rank" in r.stderr


def test_self_launch_starts_n_ranks_and_checks_gpus():
    """No torchrun env: bench.py starts 2 ranks (they rendezvous over gloo on
    this GPU-less host) and each refuses to run with fewer GPUs than ranks."""
    import torch
    if torch.cuda.device_count() >= 2:  # (a multi-GPU host would run the bench)
        return
    r = _run(["--gpus", "2", "--steps", "1", "--warmup", "0"])
    assert r.returncode != 0
    assert r.stderr.count("--gpus 2 needs 2 visible GPUs") == 2, r.stderr
    assert "rank exit codes" in r.stderr


def test_gpus_must_be_positive():
    r = _run(["--gpus", "0"])
    assert r.returncode != 0
