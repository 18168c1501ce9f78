"""bench.py's multi-rank launch contract (CPU; no GPU is touched):
`bench.py --gpus N` without torch.distributed.run starts N ranks itself (a
child torch.distributed.run, as the reference's train.py:184-186 spawns its
workers), and never silently measures fewer ranks than asked."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def test_launcher_command_line():
    import bench
    cmd = bench.launcher_command(8, 29555, ["--gpus", "8", "--steps", "20", "--warmup", "5"])
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    i = cmd.index("--nproc-per-node")
    assert cmd[i + 1] == "8"
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[cmd.index("--master-port") + 1] == "29555"
    assert "--nnodes=1" in cmd
    assert cmd[-7].endswith("bench.py") and cmd[-6:] == ["--gpus", "8", "--steps", "20", "--warmup", "5"]


def _run(args, env_extra):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "DROID_BENCH_ONE_DEVICE"):
        env.pop(k, None)
    env.update(env_extra)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, cwd=ROOT,
                          stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=300)


def test_gpus_without_devices_fails_instead_of_running_one_rank():
    # this container has no GPU: asking for 2 must fail before any rank starts
    r = _run(["--gpus", "2", "--steps", "1", "--warmup", "0"], {"HIP_VISIBLE_DEVICES": ""})
    assert r.returncode == 2, r.stderr.decode()[-2000:]
    assert b"visible GPU" in r.stderr
    assert r.stdout.strip() == b""


def test_world_size_mismatch_is_an_error():
    r = _run(["--gpus", "4", "--steps", "1", "--warmup", "0"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2
    assert b"--gpus 4 but WORLD_SIZE 2" in r.stderr
