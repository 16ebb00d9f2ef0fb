"""bench.py --gpus N without a launcher: the parent builds a
torch.distributed.run child for N ranks on 127.0.0.1, never imports torch (so
it cannot touch the GPU before spawning), relays rank 0's JSON line and exits
with the child's status; --gpus beyond the visible GPUs and --gpus != WORLD_SIZE
under a launcher are errors.  The parent runs in a fresh interpreter so that
`sys.modules` shows exactly what it imported."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

PARENT = r"""
import io, json, sys
sys.path.insert(0, {repo!r})
import bench

class FakeProc:
    def __init__(self, cmd, env, stdout, text):
        FakeProc.seen = (cmd, env)
        self.stdout = iter(["torchrun noise\n", {line!r} + "\n"])
        self.returncode = {rc}
    def wait(self):
        return self.returncode
    def send_signal(self, s):
        pass

out = io.StringIO()
rc = bench.maybe_launch({argv!r}, out, popen=FakeProc)
cmd, env = FakeProc.seen
print(json.dumps({{"rc": rc, "cmd": cmd, "env_ipc": env.get("HSA_ENABLE_IPC_MODE_LEGACY"),
                  "env_world": env.get("WORLD_SIZE"), "relayed": out.getvalue(),
                  "torch_imported": any(m == "torch" or m.startswith("torch.") for m in sys.modules)}}))
"""


def _run_parent(argv, env_extra, line='{"metric": "m", "value": 1.0}', rc=0):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra)
    code = PARENT.format(repo=REPO, argv=argv, line=line, rc=rc)
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, timeout=120)
    return p


def test_parent_spawns_torchrun_child_without_importing_torch():
    argv = ["--gpus", "4", "--steps", "7", "--warmup", "2", "--workload", "c2"]
    p = _run_parent(argv, {"FVP_BENCH_VISIBLE_GPUS": "8"})
    assert p.returncode == 0, p.stderr
    r = json.loads(p.stdout.strip().splitlines()[-1])
    cmd = r["cmd"]
    assert cmd[0] == sys.executable and cmd[1:3] == ["-m", "torch.distributed.run"]
    i = cmd.index("--nproc-per-node")
    assert cmd[i + 1] == "4"
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[cmd.index("--nnodes") + 1] == "1"
    assert int(cmd[cmd.index("--master-port") + 1]) > 0
    script = cmd.index(os.path.join(REPO, "bench.py"))
    assert cmd[script + 1:] == argv  # the same command line for every rank
    assert r["env_ipc"] == "0" and r["env_world"] is None
    assert r["relayed"].strip() == '{"metric": "m", "value": 1.0}'  # rank 0's line, nothing else
    assert r["rc"] == 0
    assert not r["torch_imported"], "the launching parent imported torch before spawning"


def test_child_failure_is_the_parent_exit_status():
    p = _run_parent(["--gpus", "2"], {"FVP_BENCH_VISIBLE_GPUS": "2"}, line="not json", rc=3)
    r = json.loads(p.stdout.strip().splitlines()[-1])
    assert r["rc"] == 3 and r["relayed"] == ""


def test_missing_result_line_is_an_error():
    p = _run_parent(["--gpus", "2"], {"FVP_BENCH_VISIBLE_GPUS": "2"}, line="no result", rc=0)
    r = json.loads(p.stdout.strip().splitlines()[-1])
    assert r["rc"] == 1


def test_more_gpus_than_visible_is_refused_before_spawning():
    p = _run_parent(["--gpus", "8"], {"FVP_BENCH_VISIBLE_GPUS": "1"})
    assert p.returncode != 0
    assert "--gpus 8 but 1 visible GPU(s)" in p.stderr
    assert "FakeProc" not in p.stdout


def test_gloo_rehearsal_skips_the_device_count():
    p = _run_parent(["--gpus", "2"], {"FVP_BENCH_BACKEND": "gloo", "FVP_BENCH_VISIBLE_GPUS": "1"})
    assert p.returncode == 0, p.stderr
    r = json.loads(p.stdout.strip().splitlines()[-1])
    assert r["cmd"][r["cmd"].index("--nproc-per-node") + 1] == "2"


def test_single_gpu_and_launched_ranks_do_not_spawn():
    sys.path.insert(0, REPO)
    import bench

    def boom(*a, **k):
        raise AssertionError("spawned")

    assert bench.maybe_launch(["--gpus", "1"], None, popen=boom) is None
    os.environ["WORLD_SIZE"] = "2"
    try:
        assert bench.maybe_launch(["--gpus", "2"], None, popen=boom) is None
    finally:
        del os.environ["WORLD_SIZE"]


def test_gpus_must_match_the_launchers_world_size():
    sys.path.insert(0, REPO)
    import bench

    args = bench.parse(["--gpus", "8"])
    bench.check_world(args, {"WORLD_SIZE": "8"})
    bench.check_world(bench.parse(["--gpus", "1"]), {})
    with pytest.raises(SystemExit, match="--gpus 8 but the launcher started WORLD_SIZE=2"):
        bench.check_world(args, {"WORLD_SIZE": "2"})
