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


def test_telemetry_degrades_to_a_note():
    """bench.GpuTelemetry without a readable GPU (this CPU box): the clock and power fields are None and
    the reason is in the line; starting, stopping and closing it never raise."""
    sys.path.insert(0, ROOT)
    import bench

    t = bench.GpuTelemetry(0)
    t.start()
    t.stop()
    s = t.summary()
    t.close()
    assert s["sclk_mhz_mean"] is None and s["power_w_mean"] is None and s["power_cap_w"] is None
    assert isinstance(s["telemetry"], str) and s["telemetry"]


def test_rank_digests_skip_other_layouts():
    """bench.rank_digests checks only the layout tests/golden/rank_digest.json was made for (L 1350,
    stride 1408, ranks 0-7, at least 2^16 slots); anything else says why it was skipped (no GPU needed)."""
    sys.path.insert(0, ROOT)
    import bench

    assert bench.rank_digests(None, None, None, None, 1408, 1 << 20, 1350, 0, None, verify=False)["digest_skipped"]
    for stride, n, L, rank in ((1472, 1 << 20, 1350, 0), (1408, 1 << 15, 1350, 0), (1408, 1 << 20, 1349, 0),
                               (1408, 1 << 20, 1350, 8)):
        d = bench.rank_digests(None, None, None, None, stride, n, L, rank, None)
        assert d["sealed_digest_ok"] is None and d["digest_skipped"] == "not the golden's layout"
