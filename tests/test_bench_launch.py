"""bench.py's rank launcher: `bench.py --gpus N` without a
launcher starts N rank processes itself; with one, --gpus must agree with
WORLD_SIZE.  The reference's batch loop this spreads over the node is
src/pipeline.py:376-393.  CPU only: the plan is checked, nothing is launched
on a GPU."""
from __future__ import annotations

import importlib.util
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", ROOT / "bench.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


B = _bench()


def test_single_rank_runs_in_process():
    assert B.rank_launch_plan(1, {}, 1, "nccl", []) is None
    assert B.rank_launch_plan(1, {}, 0, "nccl", []) is None  # CPU box: the run itself fails later


def test_under_launcher_world_size_must_agree():
    assert B.rank_launch_plan(2, {"WORLD_SIZE": "2"}, 8, "nccl", []) is None
    with pytest.raises(B.LaunchError, match="WORLD_SIZE=2"):
        B.rank_launch_plan(4, {"WORLD_SIZE": "2"}, 8, "nccl", [])
    with pytest.raises(B.LaunchError, match="WORLD_SIZE=8"):
        B.rank_launch_plan(1, {"WORLD_SIZE": "8"}, 8, "nccl", [])


def test_nccl_needs_one_gpu_per_rank():
    with pytest.raises(B.LaunchError, match="only 1 GPU"):
        B.rank_launch_plan(8, {}, 1, "nccl", ["--gpus", "8"])
    with pytest.raises(B.LaunchError, match="no GPU"):
        B.rank_launch_plan(2, {}, 0, "gloo", ["--gpus", "2"])
    with pytest.raises(B.LaunchError):
        B.rank_launch_plan(0, {}, 8, "nccl", [])


def test_launch_command_and_env():
    argv = ["--gpus", "8", "--steps", "5", "--warmup", "2"]
    cmd, env = B.rank_launch_plan(8, {"PATH": "/usr/bin"}, 8, "nccl", argv, port=lambda: 29511)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--nnodes=1" in cmd
    assert "--master-addr=127.0.0.1" in cmd and "--master-port=29511" in cmd
    i = cmd.index(str((ROOT / "bench.py").resolve()))
    assert cmd[i + 1:] == argv            # the ranks see the same arguments (WORLD_SIZE = --gpus)
    assert env["HSA_ENABLE_IPC_MODE_LEGACY"] == "0" and env["PATH"] == "/usr/bin"
    assert "WORLD_SIZE" not in env        # set per rank by the launcher, not by us
    # gloo rehearsal: two ranks on one GPU
    cmd, _ = B.rank_launch_plan(2, {}, 1, "gloo", ["--gpus", "2", "--dist-backend", "gloo"],
                                port=lambda: 29512)
    assert "--nproc-per-node=2" in cmd


def test_placement_never_reports_ranks_as_gpus():
    assert B.placement(1, 1) == {"n_gpus": 1, "world_size": 1, "ranks_per_gpu": 1.0}
    assert B.placement(2, 1) == {"n_gpus": 1, "world_size": 2, "ranks_per_gpu": 2.0}
    assert B.placement(8, 8) == {"n_gpus": 8, "world_size": 8, "ranks_per_gpu": 1.0}
    assert B.placement(4, 8)["n_gpus"] == 4


def test_cli_refuses_more_gpus_than_visible():
    # this container has no GPU: --gpus 3 over RCCL must fail loudly, exit 2,
    # before any rank is started
    p = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "3"],
                       capture_output=True, text=True, timeout=120,
                       env={k: v for k, v in __import__("os").environ.items() if k != "WORLD_SIZE"})
    assert p.returncode == 2, p.stderr[-500:]
    assert "GPU" in p.stderr and p.stdout == ""


def test_relay_keeps_only_the_json_line_on_stdout():
    import io
    script = ("print('[Gloo] Rank 0 is connected to 1 peer ranks.'); "
              "print('{\"metric\": \"m\", \"value\": 1}'); import sys; sys.exit(3)")
    out, err = io.StringIO(), io.StringIO()
    rc = B.relay_ranks([sys.executable, "-c", script], dict(__import__("os").environ), out, err)
    assert rc == 3
    assert out.getvalue() == '{"metric": "m", "value": 1}\n'
    assert "[Gloo]" in err.getvalue()
