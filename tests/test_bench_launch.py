"""bench.py's multi-GPU launch plumbing on the CPU (no GPU is touched): `python3 bench.py --gpus N`
without a launcher spawns N rank processes with torchrun's environment, the ranks form one gloo
group, and rank 0 reports N; a launcher whose world disagrees with --gpus is an error."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _run(args, env=None, timeout=180):
    e = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    e.update(env or {})
    return subprocess.run([sys.executable, BENCH] + args, env=e, capture_output=True, text=True, timeout=timeout)


@pytest.mark.timeout(240)
@pytest.mark.parametrize("n", [2, 3])
def test_gpus_n_spawns_n_ranks(n):
    p = _run(["--gpus", str(n), "--world-check"])
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout  # only rank 0 prints
    d = json.loads(lines[0])
    assert d["n_gpus"] == n and d["requested_gpus"] == n and d["group_size"] == n
    assert d["rank_sum"] == n * (n - 1) // 2  # every rank joined exactly once
    assert d["master"].startswith("127.0.0.1:")


@pytest.mark.timeout(120)
def test_single_gpu_runs_in_process():
    p = _run(["--gpus", "1", "--world-check"])
    assert p.returncode == 0, p.stderr[-2000:]
    d = json.loads([l for l in p.stdout.splitlines() if l.startswith("{")][0])
    assert d["n_gpus"] == 1 and d["group_size"] == 1


@pytest.mark.timeout(120)
def test_world_mismatch_is_an_error():
    p = _run(["--gpus", "4", "--world-check"], env={"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert p.returncode != 0
    assert "launcher started 2 ranks" in (p.stderr + p.stdout)


@pytest.mark.timeout(240)
@pytest.mark.parametrize("inject", ["fail", "group", "conservation"])
def test_c5_failure_fails_the_run(inject):
    """At N > 1 the C5 exchange's outcome is agreed by every rank: a rank whose merge raises, or a
    group smaller than --gpus, puts "c5_ok": false in the line and the run exits non-zero (the line
    used to keep the error in extra.c5_flow_reduce and exit 0)."""
    p = _run(["--gpus", "2", "--world-check"], env={"FB_C5_INJECT": inject})
    assert p.returncode != 0, p.stdout
    d = json.loads([l for l in p.stdout.splitlines() if l.startswith("{")][0])
    c5 = d["extra"]["c5_flow_reduce"]
    assert d["c5_ok"] is False and "error" in c5
    assert c5["failed_ranks"] == ([1] if inject == "fail" else [0, 1])
    if inject == "conservation":
        assert "conservation violated: payload_bytes" in c5["error"]


@pytest.mark.timeout(240)
def test_c5_success_keeps_rc_zero():
    p = _run(["--gpus", "2", "--world-check"])
    assert p.returncode == 0, p.stderr[-2000:]
    d = json.loads([l for l in p.stdout.splitlines() if l.startswith("{")][0])
    assert d["c5_ok"] is True and d["extra"]["c5_flow_reduce"]["ranks_in_group"] == 2


def test_c5_conservation_checks():
    sys.path.insert(0, ROOT)
    import bench
    sums = dict(packets=10, payload_bytes=640, ip_bytes=1040)
    ok = bench.c5_conservation(sums, dict(sums), [6, 5], 9, 9)
    assert ok["packets"] == 10 and ok["local_flows"] == [6, 5]
    for merged, local, g, u, what in ((dict(sums, packets=9), [6, 5], 9, 9, "packets"),
                                      (sums, [6, 5], 12, 12, "outside"),
                                      (sums, [6, 5], 5, 5, "outside"),
                                      (sums, [6, 5], 9, 8, "distinct keys")):
        with pytest.raises(RuntimeError) as e:
            bench.c5_conservation(merged, sums, local, g, u)
        assert what in str(e.value)
