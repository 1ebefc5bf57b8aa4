"""bench.py's multi-rank path on real hardware: two ranks launched the way the driver launches N GPUs
(python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N), each sealing and opening
its own shard with no data-path collective; barrier + max-over-ranks timing; rank 0 prints the one
JSON line.  A 1-GPU box cannot host two RCCL ranks, so this rehearsal puts both ranks on cuda:0 over
gloo (--one-device --dist-backend gloo); the RCCL variant is the same code with device_id per rank.
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _digests_ok(line: dict, prefix: int) -> None:
    """Every rank hashed its own arena prefix against tests/golden/rank_digest.json after the timed loop
    (seeds 0x5EED0001 + r): the timed state, one more seal, the open back."""
    per = line["per_gpu"]
    assert all(g["sealed_digest_ok"] is True and g["opened_digest_ok"] is True for g in per), per
    assert line["sealed_digest_ok"] is True and line["opened_digest_ok"] is True
    assert line["digest_prefix"] == prefix


def test_bench_two_ranks_one_device():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", "29533", os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "3", "--warmup", "1", "--packets", "65536", "--dist-backend", "gloo",
           "--one-device"]
    out = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout  # rank 0 only
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["status_ok"] is True and line["steps"] == 3
    assert line["scaling"] == "weak" and line["config"]["packets_per_gpu"] == 65536
    assert "cpu_baseline" not in line  # rank 0 at N=1 only
    assert line["value"] > 0
    per = line["per_gpu"]  # each rank's own rate, gathered after the timed region
    assert [g["rank"] for g in per] == [0, 1] and all(g["packets"] == 65536 and g["GiB_s"] > 0 for g in per)
    assert line["per_gpu_GiB_s"]["min"] <= line["per_gpu_GiB_s"]["max"]
    assert line["dist_backend"] == "gloo"
    _digests_ok(line, 1 << 16)


def test_bench_config4_two_ranks_one_device():
    """The driver's N > 1 default: config 4 (64 x 2^20 x 1350 B in total) sharded over the ranks, here 2
    ranks x 2^25 packets (47 GB of slots each) on cuda:0 over gloo; strong scaling over the fixed total."""
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", "29534", os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "2", "--warmup", "1", "--settle-ms", "0", "--dist-backend", "gloo",
           "--one-device"]
    out = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=400)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout
    line = json.loads(lines[0])
    assert line["status_ok"] is True and line["scaling"] == "strong"
    assert line["config"]["packets_total"] == 64 << 20 and line["config"]["packets_per_gpu"] == 32 << 20
    assert line["config"]["workload"].startswith("config4")
    assert [g["packets"] for g in line["per_gpu"]] == [32 << 20, 32 << 20]
    _digests_ok(line, 1 << 20)  # each rank's first 2^20 slots of its 2^25-packet shard


def test_bench_rccl_process_group_one_rank():
    """The RCCL branch of bench.py (init_process_group("nccl", device_id=...), the device-tensor
    all_reduce of the step time and the all_gather of the per-rank figures) on real hardware: one rank
    under torch.distributed.run, as the driver launches each rank of an N-GPU node."""
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr", "127.0.0.1", "--master-port", "29535", os.path.join(ROOT, "bench.py"),
           "--gpus", "1", "--steps", "3", "--warmup", "1", "--packets", "65536", "--settle-ms", "0",
           "--no-extra", "--no-cpu-baseline"]
    out = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout
    line = json.loads(lines[0])
    assert line["dist_backend"] == "nccl" and line["status_ok"] is True and line["n_gpus"] == 1
    assert len(line["per_gpu"]) == 1 and line["per_gpu"][0]["packets"] == 65536
    _digests_ok(line, 1 << 16)


def test_bench_gpus_flag_spawns_ranks():
    """`python bench.py --gpus 2` with no launcher around it starts the two ranks itself (here both on
    cuda:0 over gloo) and reports n_gpus 2 -- the flag can no longer silently measure one GPU."""
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["OMP_NUM_THREADS"] = "1"
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1",
           "--packets", "65536", "--settle-ms", "0", "--dist-backend", "gloo", "--one-device"]
    out = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["status_ok"] is True and line["config"]["packets_per_gpu"] == 65536


def test_bench_eight_ranks_one_device():
    """The driver's N = 8 launch rehearsed on one GPU: eight ranks (torch.distributed.run
    --nproc-per-node 8, the driver's command with --one-device --dist-backend gloo) each seal and open
    their own 2^18-packet shard; barrier + max-over-ranks timing, per-GPU figures from all eight ranks,
    one JSON line from rank 0 (main.go:72-75: quantum's independent workers; here one rank per GPU)."""
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=8",
           "--master-addr", "127.0.0.1", "--master-port", "29536", os.path.join(ROOT, "bench.py"),
           "--gpus", "8", "--steps", "3", "--warmup", "1", "--packets", "262144", "--settle-ms", "0",
           "--dist-backend", "gloo", "--one-device"]
    out = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout
    line = json.loads(lines[0])
    assert line["n_gpus"] == 8 and line["status_ok"] is True and line["scaling"] == "weak"
    assert line["config"]["packets_per_gpu"] == 262144 and line["config"]["packets_total"] == 8 * 262144
    per = line["per_gpu"]
    assert [g["rank"] for g in per] == list(range(8)) and all(g["packets"] == 262144 and g["GiB_s"] > 0 for g in per)
    assert line["value"] > 0 and line["dist_backend"] == "gloo"
    _digests_ok(line, 1 << 18)  # ranks 0..7, each against its own seeds
