"""CPU: the committed round profiles are re-derivable from the committed PMC summary
(tools/make_round_profiles.py), and bench.py's roofline traffic / issue numbers read those files."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_traffic_and_sq_regenerate():
    tag = "r02"
    summary = os.path.join(ROOT, "profiles", f"{tag}_pmc_summary.csv")
    committed_t = json.load(open(os.path.join(ROOT, "profiles", f"{tag}_traffic.json")))
    committed_q = json.load(open(os.path.join(ROOT, "profiles", f"{tag}_sq.json")))
    # regenerate under a scratch tag, compare, clean up
    scratch = "zz_test_regen"
    try:
        subprocess.run([sys.executable, os.path.join(ROOT, "tools", "make_round_profiles.py"), summary, scratch],
                       check=True, capture_output=True)
        t = json.load(open(os.path.join(ROOT, "profiles", f"{scratch}_traffic.json")))
        q = json.load(open(os.path.join(ROOT, "profiles", f"{scratch}_sq.json")))
    finally:
        for suf in ("traffic", "sq"):
            p = os.path.join(ROOT, "profiles", f"{scratch}_{suf}.json")
            if os.path.exists(p):
                os.remove(p)
    for k, v in committed_t.items():
        if k == "_what":
            continue
        assert t[k] == v, k
    for k, v in committed_q.items():
        if k == "_what":
            continue
        assert q[k] == v, k


def test_bench_reads_round_files():
    sys.path.insert(0, ROOT)
    import bench

    traffic, src = bench.measured_traffic("northstar_k_corner")
    assert traffic and src.endswith("_traffic.json")
    issue = bench.north_star_issue()
    assert issue and 0.0 < issue["simd_valu_utilisation"] < 1.0
