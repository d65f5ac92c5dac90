"""CPU tests of bench.py's N-rank launcher: `python bench.py --gpus N` started
as one process runs N ranks (torch.distributed.run child), `--gpus 1` stays one process, and too
few GPUs is a non-zero exit with a message rather than a silent 1-rank run."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(kw)
    return env


def test_launch_cmd_shape():
    sys.path.insert(0, ROOT)
    import bench
    cmd = bench.rank_launch_cmd(["--gpus", "8", "--steps", "3"], 8, 29511)
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--nnodes=1" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[cmd.index("--master-port") + 1] == "29511"
    assert cmd[-4:] == ["--gpus", "8", "--steps", "3"]
    assert os.path.samefile(cmd[-5], BENCH)


@pytest.mark.parametrize("n", [2, 3])
def test_gpus_n_reaches_n_ranks(n):
    """--gpus N without WORLD_SIZE: the child job has N ranks in one process group (gloo probe:
    the rendezvous and one all-reduce, no ISDF build)."""
    r = subprocess.run([sys.executable, BENCH, "--gpus", str(n)], capture_output=True, text=True,
                       timeout=240, env=_env(FISDF_BENCH_PROBE="1", OMP_NUM_THREADS="1"))
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout        # rank 0 only
    out = lines[0]
    assert out["probe"] and out["n_gpus"] == n and out["world_env"] == n
    assert out["allreduce_sum"] == float(n) and out["gpus_arg"] == n


def test_gpus_1_is_one_process():
    """--gpus 1 does not start a child: the probe runs in this very process as a 1-rank group."""
    r = subprocess.run([sys.executable, BENCH, "--gpus", "1"], capture_output=True, text=True,
                       timeout=240, env=_env(FISDF_BENCH_PROBE="1", WORLD_SIZE="1", RANK="0",
                                             LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                                             MASTER_PORT="29517"))
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["n_gpus"] == 1


def test_too_few_gpus_fails_loudly():
    """RCCL needs one GPU per rank: with fewer visible devices the bench exits non-zero with a
    message (here no GPU at all; on the 1-GPU box --gpus 2 does the same)."""
    import torch
    if torch.cuda.device_count() >= 2:
        pytest.skip("enough GPUs for a 2-rank run")
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2"], capture_output=True, text=True,
                       timeout=240, env=_env())
    assert r.returncode != 0
    assert "needs 2 visible GPUs" in r.stderr
    assert not r.stdout.strip()
