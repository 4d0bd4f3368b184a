"""bench.py's launch contract on CPU: `--gpus N` without a launcher resolves to
an N-process torch.distributed.run child (rendezvous on 127.0.0.1), a launcher whose WORLD_SIZE
differs from --gpus is an error rather than a silent one-GPU run, and the CPU baseline runs at the
cores the cgroup quota grants."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True,
                          text=True, env=env, timeout=120)


@pytest.mark.parametrize("n", [2, 8])
def test_gpus_n_resolves_to_n_process_launch(n):
    r = _run(["--gpus", str(n), "--steps", "5", "--warmup", "2", "--print-launch"])
    assert r.returncode == 0, r.stderr
    lines = [x for x in r.stdout.splitlines() if x.strip()]
    assert len(lines) == 1
    d = json.loads(lines[0])
    cmd = d["launch"]
    assert d["world_size"] == n
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=%d" % n in cmd and "--nnodes=1" in cmd and "--master-addr=127.0.0.1" in cmd
    tail = cmd[cmd.index(os.path.join(ROOT, "bench.py")) + 1:]
    assert tail == ["--gpus", str(n), "--steps", "5", "--warmup", "2"]


def test_world_size_mismatch_is_an_error():
    r = _run(["--gpus", "2"], {"WORLD_SIZE": "4", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2 and "WORLD_SIZE" in r.stderr and r.stdout == ""


def test_side_benches_refuse_multi_gpu():
    r = _run(["--gpus", "2", "--config", "upsert"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2


def test_cpu_baseline_threads_follow_the_quota():
    sys.path.insert(0, ROOT)
    import bench
    assert bench.cpu_threads(256, 16.0) == 16
    assert bench.cpu_threads(256, 15.5) == 16
    assert bench.cpu_threads(8, 16.0) == 8
    assert bench.cpu_threads(8, None) == 8
    assert bench.cpu_threads(4, 0.5) == 1
