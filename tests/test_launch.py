"""bench.py / parallel.launch: `--gpus N` really runs N ranks, one per device (VERDICT r3 missing #1).

The planning rules are checked as a pure function; the spawn path end to end on the CPU oracle
engine over gloo (`--device cpu`), the same code path a GPU run takes up to the device binding.
"""
import json
import os
import subprocess
import sys

import pytest

from macbf_gnn_amd.parallel import launch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_plan_standalone_spawns_n_ranks():
    p = launch.plan(4, environ={}, device_count=8)
    assert (p.action, p.ranks, p.share_devices) == ("spawn", 4, False)
    assert launch.plan(None, environ={}, device_count=1).action == "run"
    assert launch.plan(1, environ={}, device_count=1).ranks == 1


def test_plan_rejects_too_few_devices_under_rccl():
    with pytest.raises(SystemExit) as e:
        launch.plan(2, environ={}, device_count=1)
    assert "needs 2 HIP devices" in str(e.value)
    with pytest.raises(SystemExit):
        launch.plan(1, environ={}, device_count=0)


def test_plan_gloo_rehearsal_shares_devices():
    p = launch.plan(8, environ={"MACBF_DP_BACKEND": "gloo"}, device_count=1)
    assert (p.action, p.ranks, p.share_devices) == ("spawn", 8, True)
    q = launch.plan(8, environ={"MACBF_DP_BACKEND": "gloo", "WORLD_SIZE": "8", "RANK": "5", "LOCAL_RANK": "5"},
                    device_count=1)
    assert launch.device_index(q, 1) == 0


def test_plan_under_launcher_checks_world_and_device():
    env = {"WORLD_SIZE": "4", "RANK": "2", "LOCAL_RANK": "2"}
    p = launch.plan(4, environ=env, device_count=8)
    assert (p.action, p.ranks, p.rank, launch.device_index(p, 8)) == ("run", 4, 2, 2)
    assert launch.plan(None, environ=env, device_count=8).ranks == 4
    with pytest.raises(SystemExit) as e:
        launch.plan(8, environ=env, device_count=8)
    assert "WORLD_SIZE=4" in str(e.value)
    with pytest.raises(SystemExit) as e:        # rank 2 of 4 on a 2-device box: no device of its own
        launch.plan(4, environ=env, device_count=2)
    assert "no device of its own" in str(e.value)


def test_spawn_cmd_is_one_torchrun_child():
    cmd = launch.spawn_cmd("/x/bench.py", ["--gpus", "8", "--steps", "3"], 8, port=1234)
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--master-addr=127.0.0.1" in cmd
    assert cmd[-4:] == ["--gpus", "8", "--steps", "3"]


def _bench(args, extra_env=None, timeout=300):
    env = dict(os.environ, OMP_NUM_THREADS="1", **(extra_env or {}))
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=timeout)
    return r


@pytest.mark.timeout(600)
def test_bench_gpus2_spawns_two_ranks_cpu():
    r = _bench(["--gpus", "2", "--device", "cpu", "--agents", "10", "--envs", "2", "--steps", "1",
                "--warmup", "0", "--inner_loops", "4"], {"MACBF_DP_BACKEND": "gloo"})
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout          # rank 0 only
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["world"] == 2 and out["dp_backend"] == "gloo"
    assert out["config"]["parallelism"] == "dp2" and out["config"]["global_batch"] == 4
    assert out["scaling"] == "weak"             # an explicit --envs is per rank
    assert len(out["device_ids"]) == 2


@pytest.mark.timeout(600)
def test_bench_default_is_the_stated_config_strong_scaled_cpu():
    """Without --envs / --weak, bench.py runs BASELINE config #3 as stated: 64 envs over ALL ranks
    (32 per rank at --gpus 2), reported as strong scaling with global_batch 64."""
    r = _bench(["--gpus", "2", "--device", "cpu", "--agents", "6", "--steps", "1", "--warmup", "0",
                "--inner_loops", "2"], {"MACBF_DP_BACKEND": "gloo"})
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    assert out["scaling"] == "strong" and out["config"]["global_batch"] == 64
    assert out["config"]["envs_per_gpu"] == 32 and out["config"]["parallelism"] == "dp2"


@pytest.mark.timeout(300)
def test_bench_world_mismatch_fails_fast():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0", OMP_NUM_THREADS="1")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4", "--device", "cpu"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode != 0 and "WORLD_SIZE=2" in r.stderr
