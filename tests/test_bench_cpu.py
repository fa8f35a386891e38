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


def _fake_topology(tmp_path, n_cpu, n_gpu):
    root = tmp_path / "nodes"
    for i in range(n_cpu + n_gpu):
        d = root / str(i)
        d.mkdir(parents=True)
        simds = 0 if i < n_cpu else 1024
        (d / "properties").write_text(f"cpu_cores_count {16 if i < n_cpu else 0}\nsimd_count {simds}\n"
                                      f"gfx_target_version {0 if i < n_cpu else 90500}\n")
    return str(root)


def test_count_visible_gpus_from_kfd_topology(tmp_path):
    sys.path.insert(0, REPO)
    import bench
    topo = _fake_topology(tmp_path, 2, 8)
    assert bench.count_visible_gpus(topo, env={}) == 8
    assert bench.count_visible_gpus(topo, env={"ROCR_VISIBLE_DEVICES": "0,1,2,3"}) == 4
    assert bench.count_visible_gpus(topo, env={"ROCR_VISIBLE_DEVICES": "0,1,2,3", "HIP_VISIBLE_DEVICES": "1"}) == 1
    assert bench.count_visible_gpus(topo, env={"HIP_VISIBLE_DEVICES": ""}) == 0
    assert bench.count_visible_gpus(str(tmp_path / "absent"), env={}) == 0


def test_launcher_parent_never_initialises_hip(tmp_path):
    """the --gpus N parent spawns the torch.distributed.run child without any HIP
    call — torch.cuda.device_count / lazy init are made to raise, and the runtime must still be
    uninitialised at spawn time."""
    topo = _fake_topology(tmp_path, 1, 8)
    code = f"""
import sys, subprocess, torch
sys.path.insert(0, {REPO!r})
import bench
def boom(*a, **k):
    raise RuntimeError("HIP touched before spawn")
torch.cuda.device_count = boom
torch.cuda.init = boom
torch.cuda._lazy_init = boom
bench.KFD_TOPOLOGY = {topo!r}
seen = {{}}
def fake_call(cmd):
    seen["cmd"] = cmd
    seen["initialised"] = torch.cuda.is_initialized()
    return 0
subprocess.call = fake_call
sys.argv = ["bench.py", "--gpus", "8", "--steps", "1"]
rc = bench.launch_ranks(bench.parse_args(sys.argv[1:]))
assert rc == 0 and seen["initialised"] is False, seen
assert "--nproc-per-node=8" in seen["cmd"] and "--master-addr=127.0.0.1" in seen["cmd"], seen["cmd"]
print("ok")
"""
    e = {k: v for k, v in os.environ.items()
         if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "HIP_VISIBLE_DEVICES",
                      "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES")}
    r = subprocess.run([sys.executable, "-c", code], cwd=REPO, env=e, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stderr[-2000:]
