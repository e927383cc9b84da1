"""bench.py --gpus N (BASELINE config 4's command): outside a torch.distributed
launch the script starts one rank process per GPU itself, before it touches
the GPU, and refuses (non-zero exit, nothing run) when fewer than N GPUs are
visible -- the process-per-worker shape of
baseline_exps/run_planning_exps.py:378-380."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _bench():
    import importlib
    return importlib.import_module("bench")


def test_launch_plan_env_and_argv():
    b = _bench()
    plan = b.launch_plan(4, ["--gpus", "4", "--steps", "2"], 29511,
                         base_env={"PATH": "/usr/bin", "RANK": "7"})
    assert len(plan) == 4
    for r, (argv, env) in enumerate(plan):
        assert argv[0] == sys.executable and argv[-4:] == ["--gpus", "4", "--steps", "2"]
        assert os.path.basename(argv[-5]) == "bench.py"
        assert (env["RANK"], env["LOCAL_RANK"], env["WORLD_SIZE"]) == (str(r), str(r), "4")
        assert (env["MASTER_ADDR"], env["MASTER_PORT"]) == ("127.0.0.1", "29511")
        assert env["HSA_ENABLE_IPC_MODE_LEGACY"] == "0" and env["PATH"] == "/usr/bin"


def _run(args, env=None):
    e = dict(os.environ)
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args,
                          capture_output=True, text=True, env=e, timeout=300, cwd=ROOT)


@pytest.mark.skipif(__import__("torch").cuda.device_count() >= 2, reason="needs < 2 GPUs")
def test_more_gpus_than_visible_fails_before_running():
    r = _run(["--gpus", "2", "--steps", "1"])
    assert r.returncode != 0
    assert "needs 2 visible GPUs" in r.stderr and "nothing was run" in r.stderr
    assert r.stdout.strip() == ""


def test_gpus_disagreeing_with_world_size_fails():
    r = _run(["--gpus", "3"], env={"WORLD_SIZE": "2", "RANK": "0"})
    assert r.returncode != 0 and "--gpus 3 but WORLD_SIZE=2" in r.stderr


@pytest.mark.gpu
def test_gpus_2_on_a_one_gpu_box_exits_nonzero():
    import torch
    if torch.cuda.device_count() != 1:
        pytest.skip("one-GPU box")
    r = _run(["--gpus", "2", "--trees", "256", "--sims", "64", "--steps", "1",
              "--no-cpu-baseline"])
    assert r.returncode != 0 and "needs 2 visible GPUs" in r.stderr, r.stderr[-2000:]


@pytest.mark.gpu
def test_two_ranks_sharing_one_gpu_print_one_line():
    """The launcher, rendezvous, exchange (all-gather + device merge), barrier
    and max-over-ranks timing of N = 2 ranks, both on GPU 0 over gloo (one
    GPU here; the measurement uses nccl = RCCL, one GPU per rank): rank 0
    prints one JSON line with n_gpus 2 and the whole job's simulations."""
    r = _run(["--gpus", "2", "--dist-backend", "gloo", "--share-gpu", "--trees", "512",
              "--sims", "256", "--steps", "2", "--warmup", "1", "--no-cpu-baseline"])
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["collective"] == "gloo"
    assert d["config"]["counted_sims_per_step"] == 2 * 512 * 256
    assert d["value"] > 0 and d["config"]["rccl_ranks"] is None
