"""bench.py's multi-GPU entry point on CPU: ``--gpus N`` launches N ranks itself (torch.distributed.run
child, rendezvous on 127.0.0.1) and every mismatch between the requested and the available world
fails loudly instead of silently measuring one rank."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env=None, timeout=240):
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + args, cwd=REPO, env=e,
                          capture_output=True, text=True, timeout=timeout)


@pytest.mark.parametrize("n", [2, 3])
def test_gpus_flag_launches_n_ranks(n):
    r = _run(["--workload", "plumbing", "--gpus", str(n)])
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == n
    assert sorted(tuple(x) for x in line["ranks"]) == [(i, i, n) for i in range(n)]
    assert line["max_over_ranks"] == float(n)


def test_single_rank_default():
    r = _run(["--workload", "plumbing"])
    assert r.returncode == 0, r.stderr[-2000:]
    assert json.loads(r.stdout.strip().splitlines()[-1])["ranks"] == [[0, 0, 1]]


def test_world_size_mismatch_fails():
    r = _run(["--workload", "plumbing", "--gpus", "4"], env={"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0 and "WORLD_SIZE=2" in r.stderr


def test_more_gpus_than_visible_fails():
    # no GPU in this container: asking the extraction bench for 2 GPUs must exit non-zero, before any GPU call
    r = _run(["--gpus", "2", "--steps", "1", "--warmup", "0"], env={"HIP_VISIBLE_DEVICES": ""})
    assert r.returncode != 0 and "visible GPU" in r.stderr
