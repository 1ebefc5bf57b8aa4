"""bench.py's `--gpus N` contract on the CPU box: N GPUs or a non-zero exit, never a silent 1-GPU run.

* `--gpus 2` with no launcher and fewer than 2 visible GPUs exits non-zero before touching a GPU
  (with enough GPUs it starts torch.distributed.run with 2 ranks itself: tests/test_bench_dist.py);
* under a launcher, WORLD_SIZE must equal --gpus.
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(args, env_extra=None):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], cwd=ROOT, env=env,
                          capture_output=True, text=True, timeout=120)


def test_gpus_more_than_visible_fails():
    out = run(["--gpus", "2", "--steps", "1", "--warmup", "0"], {"HIP_VISIBLE_DEVICES": ""})
    assert out.returncode != 0
    assert "--gpus 2" in out.stderr and "visible" in out.stderr
    assert not [ln for ln in out.stdout.splitlines() if ln.startswith("{")]


def test_world_size_mismatch_fails():
    out = run(["--gpus", "2", "--steps", "1", "--warmup", "0"],
              {"WORLD_SIZE": "3", "RANK": "0", "LOCAL_RANK": "0"})
    assert out.returncode != 0
    assert "WORLD_SIZE=3" in out.stderr


def test_one_device_needs_gloo():
    out = run(["--gpus", "2", "--one-device", "--steps", "1", "--warmup", "0"])
    assert out.returncode != 0
    assert "gloo" in out.stderr
