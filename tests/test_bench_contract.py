"""bench.py's launch contract (CPU): a multi-GPU request is either a torchrun world of
that size or a torchrun child launch; a single process never reports N GPUs."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_mismatched_world_size_is_refused():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4"], env=env, cwd=ROOT,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 2 and "WORLD_SIZE=2" in r.stderr
    assert "{" not in r.stdout  # no bench line


def test_gpus_without_torchrun_relaunches_n_ranks(monkeypatch):
    seen = {}

    def fake_run(cmd, *a, **kw):
        seen["cmd"] = cmd

        class R:
            returncode = 0
        return R()
    monkeypatch.setattr(bench.subprocess, "run", fake_run)
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "8", "--steps", "7", "--warmup", "2"])
    try:
        bench.main()
    except SystemExit as e:
        assert e.code == 0
    cmd = seen["cmd"]
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "127.0.0.1" in cmd
    i = cmd.index(os.path.abspath(bench.__file__))
    assert cmd[i + 1:] == ["--gpus", "8", "--steps", "7", "--warmup", "2"]


def test_host_cores_reports_the_affinity_set():
    cores, detail = bench.host_cores()
    assert 1 <= cores <= len(os.sched_getaffinity(0))
    assert detail["sched_getaffinity"] == len(os.sched_getaffinity(0))
