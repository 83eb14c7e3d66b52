"""bench.py --gpus N: the rank launcher (CPU; no GPU call anywhere here).

The driver's scaling run calls `bench.py --gpus N`; without torchrun's
environment bench.py must start the N ranks itself (a torch.distributed.run
child, the replacement for the reference's <=4-replica loop,
/root/reference/train.py:62-78), refuse a node with fewer GPUs, and refuse a
world that does not match --gpus."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import bench  # noqa: E402


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "NSTL_DP")}
    env.update(kw)
    return env


def test_rank_launch_cmd():
    class A:
        gpus = 8
    cmd = bench.rank_launch_cmd(A, ["--gpus", "8", "--steps", "5"], 29501)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    i = cmd.index("--nproc-per-node")
    assert cmd[i + 1] == "8"
    assert cmd[cmd.index("--nnodes") + 1] == "1"
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[cmd.index("--master-port") + 1] == "29501"
    assert cmd[-4:] == ["--gpus", "8", "--steps", "5"]
    assert cmd[-5] == os.path.join(REPO, "bench.py")


def test_gpus_without_enough_devices_fails_clearly():
    """No GPU in this container: `bench.py --gpus 2` stops before starting ranks."""
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2"], env=_env(),
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 2, r.stderr[-2000:]
    assert "needs 2 GPUs" in r.stderr
    assert r.stdout.strip() == ""


def test_world_mismatch_raises():
    """One rank of a torchrun world of 2 given --gpus 4: refused before any GPU work."""
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "4"],
                       env=_env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0"), capture_output=True, text=True,
                       timeout=300)
    assert r.returncode != 0
    assert "world of 2" in r.stderr


def test_run_ranks_relays_and_stops_a_stalled_child():
    code = ("import sys, time; print('{\"value\": 1}', flush=True); "
            "print('progress', file=sys.stderr, flush=True); time.sleep(60)")
    rc, out, tail, why = bench._run_ranks([sys.executable, "-c", code], dict(os.environ), stall_s=3, limit_s=30)
    assert rc is None and "no output" in why
    assert json.loads(out[0]) == {"value": 1}
    assert tail == ["progress"]
    rc, out, tail, why = bench._run_ranks([sys.executable, "-c", "print('{}')"], dict(os.environ), 30, 30)
    assert rc == 0 and why is None and out == ["{}\n"]


def test_launch_falls_back_to_zero1(monkeypatch):
    """The first attempt (default exchange) fails: a second one runs NSTL_DP=zero1
    and the relayed line says so."""
    calls = []

    def fake_run(cmd, env, stall_s, limit_s):
        calls.append(env["NSTL_DP"])
        assert env["NSTL_BENCH_SELF_LAUNCH"] == "1"
        if env["NSTL_DP"] == "zero1_push":
            return 1, [], ["PushTimeout: copies to rank(s) [3] not landed"], None
        return 0, ['{"value": 5.0, "config": {"gradient_exchange": "zero1"}}\n'], [], None

    class A:
        gpus = 2
        launch_stall_s = 10
        launch_limit_s = 10
    monkeypatch.setattr(bench, "_run_ranks", fake_run)
    monkeypatch.setattr(bench.torch.cuda, "device_count", lambda: 8)
    monkeypatch.delenv("NSTL_DP", raising=False)
    printed = []
    monkeypatch.setattr("builtins.print", lambda s, **kw: printed.append(s))
    assert bench.launch_ranks(A, ["--gpus", "2"]) == 0
    assert calls == ["zero1_push", "zero1"]
    line = json.loads(printed[-1])
    assert line["value"] == 5.0
    assert "zero1_push attempt failed" in line["config"]["dp_fallback"]
    assert [a["NSTL_DP"] for a in line["launch"]["attempts"]] == ["zero1_push", "zero1"]
