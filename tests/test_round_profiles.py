"""CPU: the committed round profiles are re-derivable from the committed PMC summary
(tools/make_round_profiles.py), and bench.py's roofline traffic / issue numbers read those files."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _latest_tag():
    tags = sorted(f.split("_")[0] for f in os.listdir(os.path.join(ROOT, "profiles")) if f.endswith("_pmc_summary.csv"))
    return tags[-1]


def _subset_equal(committed, regenerated, path=""):
    """Every value the committed file holds is regenerated identically (the generator may add fields,
    and an older round's run may hold counters the current pass list no longer collects)."""
    if isinstance(committed, dict):
        for k, v in committed.items():
            if k == "_what":
                continue
            if k not in regenerated and path.endswith("counters"):
                continue
            assert k in regenerated, path + "/" + k
            _subset_equal(v, regenerated[k], path + "/" + k)
    else:
        assert committed == regenerated, path


def test_traffic_and_sq_regenerate():
    tag = _latest_tag()
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
    _subset_equal(committed_t, t)
    _subset_equal(committed_q, q)


def test_bench_reads_round_files():
    sys.path.insert(0, ROOT)
    import bench

    traffic, src = bench.measured_traffic("northstar_k_corner")
    assert traffic and src.endswith("_traffic.json")
    issue = bench.north_star_issue()
    assert issue and 0.0 < issue["simd_valu_utilisation"] < 1.0


def test_bench_ref_extract_matches_sources(monkeypatch):
    """profiles/<tag>_bench_ref.json (what the GPU box reads instead of the csv / txt profiles, which its
    upload skips) gives bench.py the same rocprof kernel rows and k_select phase clocks as the files."""
    sys.path.insert(0, ROOT)
    import bench

    from_files = (bench.rocprof_kernel("headline", "k_select<"), bench.rocprof_kernel("roofline_kernel", "k_corner"),
                  bench.select_phase_cycles())
    assert all(from_files)
    monkeypatch.setattr(bench, "KSTATS_FILE", None)
    monkeypatch.setattr(bench, "STAMPS_FILE", None)
    from_ref = (bench.rocprof_kernel("headline", "k_select<"), bench.rocprof_kernel("roofline_kernel", "k_corner"),
                bench.select_phase_cycles())
    assert from_ref == from_files
