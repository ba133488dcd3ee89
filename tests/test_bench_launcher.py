"""bench.py's own N-GPU launcher (no GPU needed): `bench.py --gpus N` with N > 1 and no WORLD_SIZE starts the N rank
processes itself as a child torch.distributed.run on 127.0.0.1, after checking that N devices are visible
(--rehearse-gloo: every rank on cuda:0, no device count needed); inside a rank, --gpus must equal WORLD_SIZE."""
import json
import os
import subprocess
import sys

from conftest import ROOT

BENCH = os.path.join(ROOT, "bench.py")


def run(args, env_extra=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, BENCH] + args, capture_output=True, text=True, timeout=300, env=env)


def test_launch_command_for_rehearsal():
    r = run(["--gpus", "2", "--rehearse-gloo", "--steps", "3", "--launch-dry-run"])
    assert r.returncode == 0, r.stderr
    cmd = json.loads(r.stdout.strip().splitlines()[-1])["launch"]
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=2" in cmd and "--nnodes=1" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert any(a.startswith("--master-port=") and int(a.split("=")[1]) > 0 for a in cmd)
    i = cmd.index(BENCH)
    assert cmd[i + 1:] == ["--gpus", "2", "--rehearse-gloo", "--steps", "3", "--launch-dry-run"]


def test_too_few_devices_fails_before_launch():
    r = run(["--gpus", "2", "--launch-dry-run"], {"HIP_VISIBLE_DEVICES": "", "CUDA_VISIBLE_DEVICES": ""})
    assert r.returncode == 3 and "GPU(s) visible" in r.stderr, (r.returncode, r.stderr)
    assert "launch" not in r.stdout


def test_bad_gpu_count():
    r = run(["--gpus", "0"])
    assert r.returncode == 2 and "--gpus must be >= 1" in r.stderr


def test_rank_world_size_mismatch():
    # a rank of a 2-process job asked for 4 GPUs: refuses before any GPU work
    r = run(["--gpus", "4", "--no-cpu-baseline"], {"WORLD_SIZE": "2", "RANK": "1", "LOCAL_RANK": "1",
                                                  "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": "29999"})
    assert r.returncode == 3 and "WORLD_SIZE=2" in r.stderr, (r.returncode, r.stderr)
