"""bench.py's launch contract (BASELINE.json metric "1/2/4/8-GPU"): `--gpus N` starts N ranks
when no launcher did, and refuses a launcher whose WORLD_SIZE disagrees with --gpus."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(REPO, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(kw)
    return env


def test_world_size_mismatch_is_an_error():
    """A launcher's WORLD_SIZE that disagrees with --gpus exits non-zero before any GPU call."""
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--no-cpu-baseline"],
                       env=_env(WORLD_SIZE="3", RANK="0", LOCAL_RANK="0"), capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 2, r.stderr
    assert "WORLD_SIZE=3" in r.stderr


@pytest.mark.gpu
def test_gpus_flag_spawns_ranks(cuda):
    """`bench.py --gpus 2` with no launcher runs two ranks (here both on cuda:0 over gloo, the
    one-GPU rehearsal of the driver's multi-GPU run) and rank 0 reports n_gpus = 2."""
    r = subprocess.run([sys.executable, "-u", BENCH, "--gpus", "2", "--same-device", "--dist-backend",
                        "gloo", "--steps", "2", "--warmup", "1", "--bags", "4", "--no-cpu-baseline",
                        "--busy-seconds", "1", "--no-calibration"],
                       env=_env(), capture_output=True, text=True, timeout=600, cwd=REPO)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2
    assert out["config"]["global_batch_bags"] == 8
    assert out["value"] > 0


def test_cpu_baseline_core_count_has_provenance():
    """cpu_baseline times the reference on every CPU this process may use: its affinity mask,
    capped by the cgroup CPU quota; the line records both (verdict r04, item 7)."""
    sys.path.insert(0, REPO)
    import bench
    n, prov = bench.host_cores()
    assert prov["affinity_cpus"] == len(os.sched_getaffinity(0))
    assert 1 <= n <= prov["affinity_cpus"]
    if prov["cgroup_cpu_quota"] is not None:
        assert n <= max(1, int(prov["cgroup_cpu_quota"]))
