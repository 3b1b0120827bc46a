"""CPU: `bench.py --gpus N` launches N rank processes by itself (no torchrun), one device per rank,
and refuses a WORLD_SIZE that differs from --gpus. FD_BENCH_LAUNCH_CHECK=1 makes the ranks report
their layout over gloo without touching a GPU."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                           "MASTER_PORT", "LOCAL_WORLD_SIZE")}
    env.update(FD_BENCH_LAUNCH_CHECK="1", **kw)
    return env


def test_self_launch_two_ranks():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], capture_output=True,
                       text=True, timeout=240, env=_env(FD_BENCH_LAUNCH_CHECK_DEVICES="2"))
    assert r.returncode == 0, r.stderr[-2000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(line) == 1, r.stdout  # rank 0 prints the only line
    out = json.loads(line[0])
    assert out["n_gpus"] == 2 and out["requested_gpus"] == 2
    assert sorted(x["rank"] for x in out["ranks"]) == [0, 1]
    assert sorted(x["device"] for x in out["ranks"]) == [0, 1]  # distinct devices
    assert len({x["pid"] for x in out["ranks"]}) == 2
    assert out["process_group"] == {"backend": "gloo", "world_size": 2}
    assert all(x["device_count"] == 2 for x in out["ranks"])
    # strong-scaled legs: the ranks' blocks partition each global batch (configs[3] 256, configs[4] 512)
    for leg, total in out["strong_global_batch"].items():
        spans = sorted(tuple(x["strong_blocks"][leg]) for x in out["ranks"])
        assert spans[0][0] == 0 and spans[-1][1] == total and spans[0][1] == spans[1][0], (leg, spans)
    assert out["strong_global_batch"] == {"config4_lsd_map": 256, "config5_superpoint": 512}


def test_self_launch_four_ranks_strong_blocks():
    """Four gloo ranks rehearse an N=4 scaling run: distinct devices, and each strong-scaled leg's
    global batch split into four contiguous equal blocks."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4"], capture_output=True,
                       text=True, timeout=240, env=_env(FD_BENCH_LAUNCH_CHECK_DEVICES="4"))
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    assert out["process_group"]["world_size"] == 4
    assert sorted(x["device"] for x in out["ranks"]) == [0, 1, 2, 3]
    for leg, total in out["strong_global_batch"].items():
        spans = sorted(tuple(x["strong_blocks"][leg]) for x in out["ranks"])
        assert [e - s for s, e in spans] == [total // 4] * 4
        assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))


def test_world_size_must_match_gpus():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1"], capture_output=True,
                       text=True, timeout=120,
                       env=_env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT="1"))
    assert r.returncode != 0 and "WORLD_SIZE=2 but --gpus 1" in r.stderr
