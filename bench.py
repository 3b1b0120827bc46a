#!/usr/bin/env python3
"""Throughput bench of the MI355X feature-detection hot path (one JSON line on rank 0).

Workload (BASELINE.json metric "Mpix/s corner-response+NMS, 640x480 gray batch"; configs[1]):
Harris response + 4-neighbour NMS + grid (greedy min-distance) selection on 640x480 u8 frames,
dist 20, need 200, thr 30, `--batch` frames per GPU per step (default 1, as configs[1]). A step is
one fd_points_detect over the batch with frames resident in HBM. Steps are replayed from a hipGraph
that cycles over `--pool` distinct frames (every step re-does all the work on a different frame).

Multi-GPU (torchrun, one process per GPU): frames are independent, so every rank processes its own
batch (weak scaling) with no collective on the data path; only the timing barrier / max-reduce uses
the process group. value = pixels processed by all ranks / max-over-ranks time.

Also reported: the roofline of the per-pixel kernel (HIP-event timed, algorithmic bytes = 1 B/px of
frame input; traffic = measured FETCH_SIZE from profiles/r03_traffic.json), the north-star shape
(Shi-Tomasi 1920x1080 batch 256), and the CPU baseline (the oracle restatement on a bounded sample of
the same workload: single thread, and a pool of up to 16 threads).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
# (SuperPoint leg: MIOpen's solver search is set up in superpoint.SuperPointDetector.Initialize.)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip-level parameters)
MFMA_PEAK_TFLOPS_FP16 = 2500.0  # dense BF16/FP16 MFMA (MI355X_MICROARCH.md: ~2.5 PF dense, no sparsity)
# HBM traffic per launch measured with rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes) and
# corrected by the calibrated gfx950 factor (tools/gpu_traffic.sh, tools/calib/fetch_calib.hip).
# (tools/gpu_round_pmc.sh + tools/make_round_profiles.py write both files)


def latest_profile(suffix):
    """profiles/rNN_<suffix> of the latest round that committed one (None if none)."""
    d = os.path.join(ROOT, "profiles")
    try:
        c = sorted(f for f in os.listdir(d) if f.startswith("r") and f.endswith("_" + suffix))
    except OSError:
        return None
    return os.path.join(d, c[-1]) if c else None


TRAFFIC_FILE = latest_profile("traffic.json")
SQ_FILE = latest_profile("sq.json")
KSTATS_FILE = latest_profile("bench_kernel_stats.csv")  # rocprofv3 --kernel-trace of bench.py, by bench leg
STAMPS_FILE = latest_profile("select_stamps.txt")  # k_select phase clocks (FD_SELECT_STAMPS) at the headline
# the two above in one JSON (tools/make_bench_ref.py): the GPU box's upload skips profiles/*.csv / *.txt
REF_FILE = latest_profile("bench_ref.json")


def _bench_ref():
    try:
        with open(REF_FILE or "") as fh:
            return json.load(fh)
    except (OSError, ValueError):
        return {}


def rocprof_kernel(phase_name, name_part):
    """(avg us, calls, source) of a kernel in a bench leg of the committed rocprofv3 summary, or None."""
    import csv

    rows, src = None, None
    try:
        with open(KSTATS_FILE or "") as fh:
            rows = [r for r in csv.reader(l for l in fh if not l.startswith("#"))][1:]
        src = os.path.relpath(KSTATS_FILE, ROOT)
    except OSError:
        ref = _bench_ref()
        rows, src = ref.get("kernel_stats"), ref.get("kernel_stats_source")
    for r in rows or []:
        if len(r) >= 4 and r[0] == "fdbench:" + phase_name and name_part in r[1]:
            return float(r[3]), int(r[2]), src
    return None


def select_phase_cycles():
    """k_select's phase clocks of the first headline frame in the committed stamps file (FD_SELECT_STAMPS;
    tools/select_stamps.py), or None: {phase: cycles} and the greedy scan's share of the total."""
    src = os.path.relpath(STAMPS_FILE, ROOT) if STAMPS_FILE else None
    try:
        with open(STAMPS_FILE or "") as fh:
            lines = fh.readlines()
    except OSError:
        ref = _bench_ref()
        lines, src = ref.get("select_stamps_lines") or [], ref.get("select_stamps_source")
    try:
        i = next(k for k, l in enumerate(lines) if l.startswith("k_select cycles:"))
    except StopIteration:
        return None
    toks = lines[i].replace("|", " ").split()[2:]
    ph = {}
    for k, v in zip(toks[0::2], toks[1::2]):
        if v.isdigit() and k not in ("subkeys", "chunks", "descents", "subchunks"):
            ph[k] = int(v)
    # the wave-serial scan (fine slots 26 / 27: its first batch and the others) when the line below has them
    fine = lines[i + 1].split()[1:] if i + 1 < len(lines) and lines[i + 1].strip().startswith("fine:") else []
    if len(fine) >= 12 and all(f.isdigit() for f in fine):
        ph["scan_first_batch"] = int(fine[10])
        ph["scan_other_batches"] = int(fine[11])
    tot = sum(ph.values())
    serial = ph.get("greedy", 0) + ph.get("scan_first_batch", 0) + ph.get("scan_other_batches", 0)
    return {"source": src, "cycles": ph,
            "greedy_share": round(serial / tot, 3) if tot else None}


def north_star_issue():
    """What bounds the north-star kernel, from the committed SQ counter pass (None if absent)."""
    try:
        with open(SQ_FILE or "") as fh:
            q = json.load(fh)["ns_sq"]
    except (OSError, KeyError, ValueError):
        return None
    c = q.get("counters", {})
    slots = c.get("SQ_INSTS_VALU", 0.0) - c.get("SQ_ACTIVE_INST_VALU2", 0.0)  # dual-issued pairs share a slot
    return {"source": os.path.relpath(SQ_FILE, ROOT),
            "valu_issue_slots_per_launch": slots or None,
            "valu_issue_slot_busy": q.get("valu_issue_slot_busy"),
            "simd_valu_utilisation": q["simd_valu_utilisation"],
            "waves_resident_per_simd": q["waves_resident_per_simd"],
            "wave_time_issue_stalled": q["wave_time_issue_stalled"],
            "note": ("VALU issue-slot bound: one quad-cycle issue slot per wave64 VALU instruction (dual-issued "
                     "pairs share one; measured per opcode class in profiles/r03_valu_probe.txt), busy = "
                     "(SQ_INSTS_VALU - SQ_ACTIVE_INST_VALU2) x 4 / (1024 SIMDs x kernel cycles); HBM is ~10 % "
                     "-- DESIGN.md section 5")}


SIMDS, CLOCK_GHZ = 1024, 2.4  # 256 CUs x 4 SIMDs; peak engine clock (MI355X_MICROARCH.md)


def valu_floor(issue, pixels, kernel_ms):
    """The north-star kernel against its VALU issue-slot floor: one quad-cycle slot per wave64 VALU
    instruction (dual-issued pairs one), all SIMDs at the peak clock; and the slot budget per pixel that
    70 % of the HBM read roofline (1 B/px) would leave."""
    if not issue or not issue.get("valu_issue_slots_per_launch"):
        return None
    slots = issue["valu_issue_slots_per_launch"]
    floor_ms = slots * 4 / SIMDS / (CLOCK_GHZ * 1e9) * 1e3
    slot_rate = SIMDS * CLOCK_GHZ * 1e9 / 4
    return {"issue_slots_per_px": round(slots / pixels, 4), "lane_slots_per_px": round(64 * slots / pixels, 1),
            "floor_ms": round(floor_ms, 4), "frac": round(floor_ms / kernel_ms, 4),
            "hbm70_slots_per_px": round(slot_rate / (0.7 * HBM_PEAK_GBS * 1e9), 4),
            "note": "VALU issue-slot floor at the peak clock vs the measured kernel time; 70 % of the HBM read "
                    "roofline would need <= hbm70_slots_per_px wave issue slots per pixel (DESIGN.md section 5)"}


def measured_traffic(key):
    try:
        with open(TRAFFIC_FILE or "") as fh:
            t = json.load(fh)
        return int(t[key]["read_bytes_corrected"]), os.path.relpath(TRAFFIC_FILE, ROOT)
    except (OSError, KeyError, ValueError):
        return None, None


def cpu_model():
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"
KIND = {"harris": 0, "shi_tomasi": 1, "fast": 2}
THR = {"harris": 30.0, "shi_tomasi": 40.0, "fast": 10.0}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--warmup", type=int, default=20)
    p.add_argument("--detector", default="harris", choices=list(KIND))
    p.add_argument("--rows", type=int, default=480)
    p.add_argument("--cols", type=int, default=640)
    p.add_argument("--batch", type=int, default=1, help="frames per GPU per step")
    p.add_argument("--pool", type=int, default=16, help="distinct frame batches cycled by the graph")
    p.add_argument("--need", type=int, default=200)
    p.add_argument("--dist", type=int, default=20)
    p.add_argument("--pattern", default="noise", choices=["noise", "checker"])
    p.add_argument("--no-graph", action="store_true")
    p.add_argument("--no-north-star", action="store_true")
    p.add_argument("--no-config3", action="store_true", help="skip the FAST + BRIEF (configs[2]) leg")
    p.add_argument("--no-lsd", action="store_true", help="skip the LSD map (configs[3]) leg")
    p.add_argument("--no-superpoint", action="store_true", help="skip the SuperPoint (configs[4]) leg")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=10.0)
    return p.parse_args()


def make_frames(torch, pattern, n, rows, cols, seed, device, period=16):
    """Seeded synthetic u8 frames generated on the GPU (noise, or period-px 60/180 checker + U[-10,10])."""
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    if pattern == "noise":
        return torch.randint(0, 256, (n, rows, cols), generator=g, device=device, dtype=torch.int32).to(torch.uint8)
    r = torch.arange(rows, device=device).view(1, rows, 1) // period
    c = torch.arange(cols, device=device).view(1, 1, cols) // period
    base = torch.where(((r + c) % 2) == 1, 180, 60)
    noise = torch.randint(-10, 11, (n, rows, cols), generator=g, device=device, dtype=torch.int32)
    return (base + noise).clamp(0, 255).to(torch.uint8)


def timed_graph(torch, fn, steps, warmup, use_graph, per_graph, barrier=None):
    """Run fn(i) (i = step index) `warmup` then `steps` times; returns seconds for the timed steps.

    With graphs, `per_graph` consecutive steps are captured into one hipGraph and replayed. The timed
    region is bracketed by barrier() (all ranks) + device synchronisation on both sides."""
    def fence():
        torch.cuda.synchronize()
        if barrier is not None:
            barrier()
        torch.cuda.synchronize()

    if not use_graph:
        for i in range(warmup):
            fn(i)
        fence()
        t0 = time.perf_counter()
        for i in range(steps):
            fn(i)
        fence()
        return time.perf_counter() - t0, steps
    for i in range(max(warmup, 1)):  # eager warmup also sizes the library workspace
        fn(i)
    torch.cuda.synchronize()
    # Exactly `steps` steps: reps replays of a graph of per_graph steps + one graph of the remainder
    # (per_graph 0: all steps in one graph, cycling the pool inside it -- one graph launch in the timed
    # region, up to 1024 steps).
    per_graph = max(1, min(per_graph if per_graph > 0 else 1024, steps))
    reps, rem = divmod(steps, per_graph)
    graphs = []
    for n in (per_graph, rem):
        if n == 0:
            graphs.append(None)
            continue
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for i in range(n):
                fn(i)
        g.replay()  # untimed: first replay uploads the graph
        torch.cuda.synchronize()
        graphs.append(g)
    fence()
    t0 = time.perf_counter()
    for _ in range(reps):
        graphs[0].replay()
    if graphs[1] is not None:
        graphs[1].replay()
    fence()
    return time.perf_counter() - t0, reps * per_graph + rem


def kernel_time_ms(torch, fd, frames_pool, kind, thr, reps=50):
    """Average duration of the per-pixel kernel alone, HIP events on the stream it is launched on
    (torch's current stream, which the library context follows).

    A launch of a small frame batch is shorter than the host's per-call overhead, so back-to-back
    calls would time the host. When the output lists fit, the reps are fd_points_response_append
    calls (the kernel alone, no count reset; each rep appends after the previous) captured in one
    HIP graph and replayed between the events. Otherwise (the north-star batch, ~0.7 ms a launch)
    plain fd_points_response calls, whose 1-word count memset is noise at that size.
    """
    b, r, c = frames_pool[0].shape
    base = r * c if kind == "fast" else r * c // 2 + 64
    dev = frames_pool[0].device
    graph = b * base * (reps + 3) * 8 <= (1 << 30)
    cap = base * (reps + 3) if graph else base
    out = (torch.empty((b, cap), dtype=torch.float32, device=dev), torch.empty((b, cap), dtype=torch.int32, device=dev),
           torch.empty((b,), dtype=torch.int32, device=dev))
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if graph:
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            out[2].zero_()
            for i in range(3):
                fd.point_response(kind, frames_pool[i % len(frames_pool)], thr, out=out, append=True)
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for i in range(reps):
                fd.point_response(kind, frames_pool[i % len(frames_pool)], thr, out=out, append=True)
        out[2].zero_()
        torch.cuda.synchronize()
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        del g
        return ms
    for i in range(3):
        fd.point_response(kind, frames_pool[i % len(frames_pool)], thr, out=out)
    torch.cuda.synchronize()
    e0.record()
    for i in range(reps):
        fd.point_response(kind, frames_pool[i % len(frames_pool)], thr, out=out)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def run_config(torch, fd, dev, detector, rows, cols, batch, pool, need, dist, pattern, steps, warmup, use_graph,
               seed, barrier=None, ties="raster", frames_pool=None):
    if frames_pool is None:
        frames_pool = [make_frames(torch, pattern, batch, rows, cols, seed + 7919 * i, dev) for i in range(pool)]
    thr = THR[detector]
    stride = max(need, 1) + 1
    xy = torch.empty((batch, stride, 2), dtype=torch.float32, device=dev)
    cnt = torch.empty((batch,), dtype=torch.int32, device=dev)
    ctx = fd.default_context(dev.index or 0)
    ctx.reserve(KIND[detector], batch, rows, cols)

    def step(i):
        fd.detect_points(detector, frames_pool[i % pool], need, dist, thr, out=(xy, cnt), ctx=ctx, ties=ties)

    secs, done = timed_graph(torch, step, steps, warmup, use_graph, per_graph=0, barrier=barrier)
    return secs, done, frames_pool, (xy, cnt)


def tie_frames(fd, dev, detector, frames_pool, need, dist):
    """Frames of a timed pool whose selection scan met equal responses (FD_FRAME_TIES after a raster-order
    run): only those can differ from the reference's std::sort order, which ties="reference" restores
    with a host re-selection. Returns (tied frames, frames)."""
    ctx = fd.default_context(dev.index or 0)
    tied = total = 0
    for f in frames_pool:
        fd.detect_points(detector, f, need, dist, THR[detector], ctx=ctx, ties="raster")
        st = ctx.frame_status(f.shape[0])
        tied += int(((st & fd.points.FRAME_TIES) != 0).sum())
        total += f.shape[0]
    return tied, total


def tie_report(torch, fd, dev, detector, frames_pool, need, dist, steps=10, raster_ms=None):
    """The leg's tie count; when nonzero the same workload is also timed with ties="reference" (the
    reference's std::sort order on the GPU: k_select_reference emulates libstdc++'s introsort over the
    visited prefix), replayed from a hipGraph like the raster steps, and the frames it had to leave to
    the host (FD_FRAME_UNRESOLVED: the introsort's heapsort fallback) are counted."""
    tied, total = tie_frames(fd, dev, detector, frames_pool, need, dist)
    rep = {"tie_frames": tied, "frames_checked": total,
           "timed_order": "raster (equal to the reference order on every frame without FD_FRAME_TIES)"}
    if tied:
        b, rows, cols = frames_pool[0].shape
        secs, done, _, _ = run_config(torch, fd, dev, detector, rows, cols, b, len(frames_pool), need, dist, None,
                                      steps, 2, True, 0, ties="reference", frames_pool=frames_pool)
        ms = secs / done * 1e3
        rep["reference_order_ms_per_step"] = round(ms, 5)
        rep["reference_order_mpix_s"] = round(done * b * rows * cols / secs / 1e6, 1)
        rep["reference_order_graph"] = True
        if raster_ms:
            rep["reference_vs_raster_step"] = round(ms / raster_ms, 3)
        ctx = fd.default_context(dev.index or 0)
        unresolved = resolved = 0
        for f in frames_pool:
            fd.detect_points(detector, f, need, dist, THR[detector], ctx=ctx, ties="reference")
            st = ctx.frame_status(f.shape[0])
            unresolved += int(((st & fd.points.FRAME_UNRESOLVED) != 0).sum())
            resolved += int(((st & fd.points.FRAME_RESOLVED) != 0).sum())
        rep["reference_resolved_on_gpu"] = resolved
        rep["reference_unresolved_frames"] = unresolved
    return rep


def run_pipelined(torch, fd, dev, detector, rows, cols, need, dist, pattern, seed, nctx=2, pool=16, reps=20):
    """Serving variant of the headline (reported beside it, never as `value`): the same batch-1 calls,
    but consecutive frames alternate between `nctx` contexts, each with its own workspace and stream,
    so that one frame's per-pixel kernel overlaps the previous frame's single-workgroup selection.
    One hipGraph holds `pool` calls as `nctx` independent branches (forked from and joined to the
    capturing stream); returns (ms per frame, frames)."""
    frames_pool = [make_frames(torch, pattern, 1, rows, cols, seed + 7919 * i, dev) for i in range(pool)]
    thr = THR[detector]
    stride = max(need, 1) + 1
    ctxs = [fd.Context(dev.index or 0) for _ in range(nctx)]
    for c in ctxs:
        c.reserve(KIND[detector], 1, rows, cols)
    outs = [(torch.empty((1, stride, 2), dtype=torch.float32, device=dev),
             torch.empty((1,), dtype=torch.int32, device=dev)) for _ in range(nctx)]
    streams = [torch.cuda.Stream(device=dev) for _ in range(nctx)]

    def run_all():
        main = torch.cuda.current_stream()  # the capturing stream inside torch.cuda.graph
        for s in streams:
            s.wait_stream(main)
        for i in range(pool):
            k = i % nctx
            with torch.cuda.stream(streams[k]):
                fd.detect_points(detector, frames_pool[i], need, dist, thr, out=outs[k], ctx=ctxs[k], ties="raster")
        for s in streams:
            main.wait_stream(s)

    run_all()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        run_all()
    g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        g.replay()
    torch.cuda.synchronize()
    secs = time.perf_counter() - t0
    del g
    for c in ctxs:
        c.close()
    return secs / (reps * pool) * 1e3, reps * pool


def run_config3(torch, fd, dev, seed, batch=64, rows=720, cols=1280, need=200, dist=20, steps=20, reps=20):
    """FAST-12 (thr 10) + greedy selection + steered BRIEF-256 on the selected keypoints, all on the
    device: the detector writes keypoints/counts, the descriptor kernel reads them in place."""
    pool = [make_frames(torch, "noise", batch, rows, cols, seed + 7919 * i, dev) for i in range(2)]
    stride = need + 1
    xy = torch.empty((batch, stride, 2), dtype=torch.float32, device=dev)
    cnt = torch.empty((batch,), dtype=torch.int32, device=dev)
    bits = torch.empty((batch, stride, 8), dtype=torch.int32, device=dev)
    ctx = fd.default_context(dev.index or 0)
    ctx.reserve(fd.FD_FAST, batch, rows, cols)

    def step(i):
        fd.detect_points("fast", pool[i % 2], need, dist, THR["fast"], out=(xy, cnt), ctx=ctx, ties="raster")
        fd.brief_compute(pool[i % 2], xy, cnt, length=256, half_patch_size=8, out=bits, ctx=ctx)

    secs, done = timed_graph(torch, step, steps, 2, True, per_graph=2)
    # the descriptor kernel alone: reps launches captured in one graph (keypoints from the last step)
    fd.detect_points("fast", pool[0], need, dist, THR["fast"], out=(xy, cnt), ctx=ctx, ties="raster")
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fd.brief_compute(pool[0], xy, cnt, length=256, half_patch_size=8, out=bits, ctx=ctx)
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    brief_ms = e0.elapsed_time(e1) / reps
    kp = int(cnt.sum().item())
    px = batch * rows * cols
    ties = tie_report(torch, fd, dev, "fast", pool, need, dist, steps=4, raster_ms=secs / done * 1e3)
    if "reference_order_ms_per_step" in ties:
        ties["reference_order_note"] = "detect + select only (no BRIEF)"
    return {
        "workload": f"fast (thr 10) + grid NMS (need {need}, dist {dist}) + BRIEF-256 (half 8, bilinear), "
                    f"{cols}x{rows} gray noise, batch {batch}/GPU (BASELINE configs[2])",
        "mpix_s": round(done * px / secs / 1e6, 1), "ms_per_step": round(secs / done * 1e3, 4),
        "keypoints_per_step": kp, "brief_kernel_ms": round(brief_ms, 4),
        "brief_keypoints_per_s": round(kp / (brief_ms * 1e-3), 1), "ties": ties,
    }


class phase:
    """roctx range around one leg of the bench (torch.cuda.nvtx on ROCm): rocprofv3 --marker-trace
    records it, and tools/rocpd_summary.py --phases attributes each kernel to the leg it ran in."""

    def __init__(self, torch, name):
        self.torch, self.name = torch, name

    def __enter__(self):
        self.torch.cuda.synchronize()
        print(f"[bench] {self.name}", file=sys.stderr, flush=True)  # progress (stdout keeps the one JSON line)
        try:
            self.torch.cuda.nvtx.range_push("fdbench:" + self.name)
        except Exception:
            pass
        return self

    def __exit__(self, *exc):
        self.torch.cuda.synchronize()
        try:
            self.torch.cuda.nvtx.range_pop()
        except Exception:
            pass
        return False


def graph_time_ms(torch, fn, reps):
    """Average time of fn() replayed `reps` times from one captured hipGraph (HIP events)."""
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    del g
    return e0.elapsed_time(e1) / reps


def _line_threads():
    import multiprocessing

    n = multiprocessing.cpu_count()
    lease = os.environ.get("OMP_NUM_THREADS")
    if lease and lease.isdigit() and int(lease) > 0:
        n = min(n, int(lease))
    return int(os.environ.get("FD_LINE_THREADS", n))


def run_lsd(torch, fd, dev, seed, batch=256, rows=1080, cols=1920, reps=5, line_reps=3, global_batch=None,
            barrier=None, max_fn=None):
    """BASELINE configs[3]: LSD level-line map (norm, angle, valid + column-major valid list) on
    structured 64-px checker frames, all on the device (the host region growing is not timed).

    Strong scaling: this rank's contiguous block (`batch` frames) of the global 256-frame batch. With
    ranks, the map is also timed wall-clock between barriers (max over ranks) -> the whole job's rate."""
    global_batch = global_batch or batch
    frames = make_frames(torch, "checker", batch, rows, cols, seed, dev, period=64)
    out = fd.lsd_map(frames)
    torch.cuda.synchronize()
    valid = int(out[4].sum().item())
    ms = graph_time_ms(torch, lambda: fd.lsd_map(frames, out=out), reps)
    job_ms = None
    if max_fn is not None:
        job_ms = ranked_time_ms(torch, lambda: fd.lsd_map(frames, out=out), reps, barrier, max_fn)
    px = batch * rows * cols
    mpx = batch * (rows - 1) * (cols - 1)
    alg = px + 9 * mpx + 4 * valid  # read u8 frame; write norm f32 + angle f32 + valid u8; 4 B per listed pixel
    del out
    # Whole line detector (FeatureLineDetector::DetectGoodFeatures for every frame): GPU compact map,
    # lists over PCIe, region growing + rectangles on host worker threads (fd_lsd_lines).
    segs = fd.lsd_lines(frames, max_lines=2048)  # warm (workspace, pinned buffers, threads)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(line_reps):
        segs = fd.lsd_lines(frames, max_lines=2048)
    line_s = (time.perf_counter() - t0) / line_reps
    n_lines = sum(len(x) for x in segs)
    del frames
    lines = {"ms_per_batch": round(line_s * 1e3, 3), "frames_per_s": round(batch / line_s, 1),
             "lines_per_s": round(n_lines / line_s, 1), "lines_per_batch": n_lines,
             "mpix_s": round(px / line_s / 1e6, 1), "host_threads": _line_threads(),
             "note": "fd_lsd_lines: GPU level-line map (compact lists) + D2H + host region growing on worker threads"}
    res = {
        "workload": f"LSD level-line map, {cols}x{rows} gray 64-px checker + noise, global batch {global_batch} "
                    f"frame-sharded over the ranks ({batch} on this rank; BASELINE configs[3]); whole line detector "
                    "under 'lines'",
        "scaling": "strong", "global_batch": global_batch, "frames_this_rank": batch,
        "ms_per_batch": round(ms, 4), "mpix_s": round(px / (ms * 1e-3) / 1e6, 1), "valid_pixels": valid,
        "kernels": "k_lsd_map + k_lsd_scan + k_lsd_scatter",
        "roofline": {"bound": "hbm", "achieved": round(alg / (ms * 1e-3) / 1e9, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(alg / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                     "bytes_per_launch": alg},
        "lines": lines,
    }
    if job_ms is not None:
        res["job"] = {"ms_per_global_batch": round(job_ms, 4),
                      "mpix_s": round(global_batch * rows * cols / (job_ms * 1e-3) / 1e6, 1),
                      "note": "all ranks' blocks, wall clock between barriers, max over ranks"}
    return res


def ranked_time_ms(torch, fn, reps, barrier, max_fn):
    """Wall time per call of fn() over all ranks: `reps` calls replayed from one hipGraph per rank,
    bracketed by barrier + device synchronisation on both sides, max over ranks (ms)."""
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()

    def fence():
        torch.cuda.synchronize()
        if barrier is not None:
            barrier()
        torch.cuda.synchronize()

    fence()
    t0 = time.perf_counter()
    g.replay()
    fence()
    el = time.perf_counter() - t0
    del g
    return max_fn(el) / reps * 1e3


def copy_bandwidth(torch, dev, nbytes=1 << 30, reps=5):
    """Measured device-to-device copy bandwidth (read + write bytes / time): the practical HBM ceiling.
    A float4 (16 B per lane) nontemporal grid-stride copy kernel (tools/calib/copy_kernel.hip, the form
    MI355X_MICROARCH.md measures at ~6.3 TB/s); torch's copy_ beside it for comparison."""
    import ctypes

    a = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    b = torch.empty_like(a)
    out = {"torch_copy_gbs": round(2 * nbytes / (graph_time_ms(torch, lambda: b.copy_(a), reps) * 1e-3) / 1e9, 1)}
    so = os.path.join(ROOT, "tools", "calib", "libcopybw.so")
    if os.path.exists(so):
        lib = ctypes.CDLL(so)
        for name, key in (("fdcal_copy16", "kernel_copy_nt_gbs"), ("fdcal_copy16_flat", "kernel_copy_gbs")):
            fn = getattr(lib, name)
            fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]

            def kcopy(fn=fn):
                rc = fn(b.data_ptr(), a.data_ptr(), nbytes, torch.cuda.current_stream().cuda_stream)
                assert rc == 0, rc

            out[key] = round(2 * nbytes / (graph_time_ms(torch, kcopy, reps) * 1e-3) / 1e9, 1)
        # write-only, and the LSD map's traffic shape: 1 B read + 9 B written per pixel (its bytes without its
        # arithmetic), each as a nontemporal grid-stride kernel and a flat default-policy one
        npx = nbytes // 10 // 64 * 64
        nrm = b[:4 * npx]
        ang = a[:4 * npx]  # (the copy source is free now)
        src, val = a[4 * npx:5 * npx], a[5 * npx:6 * npx]
        for name, key in (("fdcal_fill16", "kernel_fill_nt_gbs"), ("fdcal_fill16_flat", "kernel_fill_gbs")):
            fill = getattr(lib, name)
            fill.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
            out[key] = round(nbytes / (graph_time_ms(
                torch, lambda fill=fill: fill(b.data_ptr(), nbytes, torch.cuda.current_stream().cuda_stream), reps)
                * 1e-3) / 1e9, 1)
        for name, key in (("fdcal_lsd_shape", "lsd_shape_nt_gbs"), ("fdcal_lsd_shape_flat", "lsd_shape_flat_gbs")):
            shape = getattr(lib, name)
            shape.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_size_t, ctypes.c_void_p]
            out[key] = round(10 * npx / (graph_time_ms(
                torch, lambda shape=shape: shape(src.data_ptr(), nrm.data_ptr(), ang.data_ptr(), val.data_ptr(), npx,
                                                 torch.cuda.current_stream().cuda_stream), reps) * 1e-3) / 1e9, 1)
        out["lsd_shape_gbs"] = max(out["lsd_shape_nt_gbs"], out["lsd_shape_flat_gbs"])
    del a, b
    out["device_copy_gbs"] = max(v for k, v in out.items() if "copy" in k)
    return out


def run_end_to_end(torch, fd, args, seconds=3.0):
    """PCIe-inclusive rate of the headline workload: host frames staged by the library, features
    copied back (what the C++ drop-in class does per call). Reported beside `value`, never as it."""
    import numpy as np

    frames = make_frames(torch, args.pattern, 16, args.rows, args.cols, 31337, torch.device("cuda")).cpu().numpy()
    fd.detect_points(args.detector, frames[0], args.need, args.dist, THR[args.detector], ties="raster")
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        fd.detect_points(args.detector, frames[n % len(frames)], args.need, args.dist, THR[args.detector],
                         ties="raster")
        n += 1
    el = time.perf_counter() - t0
    return {"mpix_s": round(n * args.rows * args.cols / el / 1e6, 1), "ms_per_frame": round(el / n * 1e3, 4),
            "frames": n, "note": "host numpy frame -> H2D staging -> detect -> D2H features, synchronous per frame"}


def run_ingest(torch, fd, args, seconds=3.0, batch=16, depth=3):
    """PCIe-inclusive rate through the pipelined ingest (fd_ingest_*): host frames
    written into pinned slots, uploads overlapped with detection, features copied back. Reported beside
    `value`, never as it."""
    frames = make_frames(torch, args.pattern, 2 * batch, args.rows, args.cols, 31338, torch.device("cuda")).cpu().numpy()
    ing = fd.Ingest(args.detector, args.rows, args.cols, batch=batch, depth=depth, need=args.need,
                    min_feature_distance=args.dist, min_valid_response=THR[args.detector])
    n, k, t0 = 0, 0, None
    while True:
        slot = k % depth
        if k >= depth:
            ing.wait(slot)
            n += batch
        if t0 is None and k == depth:  # timing starts with the pipeline full
            t0, n = time.perf_counter(), 0
        if t0 is not None and time.perf_counter() - t0 >= seconds:
            break
        ing.frames(slot)[:] = frames[(k % 2) * batch:(k % 2 + 1) * batch]
        ing.submit(slot)
        k += 1
    el = time.perf_counter() - t0
    for j in range(k - depth + 1, k):  # drain
        if j >= 0:
            ing.wait(j % depth)
    ing.close()
    return {"mpix_s": round(n * args.rows * args.cols / el / 1e6, 1), "frames_per_s": round(n / el, 1),
            "batch": batch, "depth": depth,
            "note": "host numpy frames -> pinned slot (memcpy) -> H2D on a copy stream overlapped with detect -> "
                    "D2H features; host fill included"}


def conv_flops(net, rows, cols):
    """Dense multiply-add FLOPs (2 per MAC) of every Conv2d of the network for one rows x cols frame."""
    from torch import nn

    total, scale = 0, {"1": 1, "2": 2, "3": 4, "4": 8, "P": 8, "D": 8}
    for name, m in net.named_modules():
        if isinstance(m, nn.Conv2d):
            f = scale[name[4]]  # conv1a -> '1', convPa -> 'P'
            h, w = rows // f, cols // f
            total += 2 * h * w * m.in_channels * m.out_channels * m.kernel_size[0] * m.kernel_size[1]
    return total


def run_superpoint(torch, fd, dev, seed, batch=64, rows=480, cols=640, steps=10, global_batch=None, chunk=64,
                   barrier=None, max_fn=None):
    """BASELINE configs[4]: SuperPoint fp16 on 640x480, a global batch of 512 frames frame-sharded over
    the ranks (strong scaling: `batch` = this rank's block, run as network batches of `chunk`): network
    (PyTorch-ROCm, MIOpen convs), then GPU selection + descriptors (fd_nn_select / fd_nn_descriptors)."""
    from feature_detector_amd import superpoint as spm

    global_batch = global_batch or batch
    det = spm.SuperPointDetector(spm.Options(kComputeDescriptors=True, kMaxImageRows=rows, kMaxImageCols=cols),
                                 device=dev.index or 0)
    det.Initialize()
    frames = make_frames(torch, "noise", batch, rows, cols, seed, dev)
    chunks = [frames[i:i + chunk] for i in range(0, batch, chunk)]

    def step():
        for c in chunks:
            res = det.DetectGoodFeaturesWithDescriptor(c)
        return res

    for _ in range(2):
        step()

    def fence():
        torch.cuda.synchronize()
        if barrier is not None:
            barrier()
        torch.cuda.synchronize()

    fence()
    t0 = time.perf_counter()
    for _ in range(steps):
        xy, cnt, d = step()
    fence()
    el = (time.perf_counter() - t0) / steps
    job_s = max_fn(el) if max_fn is not None else el
    first = chunks[0]
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(steps):
        heat, desc = det.InferenceSession(first)
    e1.record()
    torch.cuda.synchronize()
    net_ms = e0.elapsed_time(e1) / steps
    xy, cnt, d = det.DetectGoodFeaturesWithDescriptor(first)
    post_ms = graph_time_ms(torch, lambda: (spm.nn_select(heat, det.options(), out=(xy, cnt)),
                                            spm.nn_descriptors(desc, xy, cnt, out=d)), 10)
    nb = len(first)
    flops = conv_flops(det.net, rows, cols) * nb
    return {
        "workload": f"SuperPoint (random weights, fp16 convs) + heatmap selection (thr 0.1, dist 15, max 240) + "
                    f"256-d descriptors, {cols}x{rows} noise, global batch {global_batch} frame-sharded over the "
                    f"ranks ({batch} on this rank, network batches of {chunk}; BASELINE configs[4])",
        "scaling": "strong", "global_batch": global_batch, "frames_this_rank": batch,
        "ms_per_step": round(el * 1e3, 3), "frames_per_s": round(batch / el, 1),
        "mpix_s": round(batch * rows * cols / el / 1e6, 1),
        "job": {"ms_per_global_batch": round(job_s * 1e3, 3), "frames_per_s": round(global_batch / job_s, 1),
                "note": "all ranks' blocks, wall clock between barriers, max over ranks"},
        "network_ms": round(net_ms, 3), "network_batch": nb,
        "postprocess_ms": round(post_ms, 4), "features_per_frame": round(float(cnt.float().mean().item()), 1),
        "network_roofline": {"bound": "mfma", "achieved": round(flops / (net_ms * 1e-3) / 1e12, 1),
                             "peak": MFMA_PEAK_TFLOPS_FP16, "unit": "TFLOP/s",
                             "frac": round(flops / (net_ms * 1e-3) / 1e12 / MFMA_PEAK_TFLOPS_FP16, 4),
                             "flops_per_step": flops},
    }


def cpu_workers():
    """Threads for the CPU pool leg: the CPUs this process may run on, capped by the lease's thread
    budget (the GPU box exports OMP_NUM_THREADS=16: its CPU share, although nproc shows the whole
    host). Returns (workers, visible logical CPUs, cap source)."""
    try:
        visible = len(os.sched_getaffinity(0))
    except AttributeError:
        visible = os.cpu_count() or 1
    lease = os.environ.get("OMP_NUM_THREADS")
    if lease and lease.isdigit() and int(lease) > 0:
        return min(visible, int(lease)), visible, f"OMP_NUM_THREADS={lease} (lease CPU share)"
    return visible, visible, "sched_getaffinity"


def cpu_leg(work, px_per_item, seconds, unit="Mpix/s", label="", kind="port"):
    """Time work(i, tls) (one item = one frame, tls = per-thread state) on 1 thread, then on a pool of
    cpu_workers() threads, each for about `seconds` of wall time (ctypes releases the GIL, so the
    pool scales). Returns (single-thread baseline dict, pool baseline dict)."""
    import threading
    from concurrent.futures import ThreadPoolExecutor

    def run_for(tls, deadline, start):
        n = 0
        while time.perf_counter() < deadline:
            work(start + n, tls)
            n += 1
        return n

    tls0 = {}
    work(0, tls0)  # warm (allocations, page faults)
    t0 = time.perf_counter()
    n1 = run_for(tls0, t0 + seconds, 0)
    el1 = time.perf_counter() - t0
    workers, visible, cap = cpu_workers()
    barrier = threading.Barrier(workers)

    def pooled(w):
        tls = {}
        work(w, tls)
        barrier.wait()
        t = time.perf_counter()
        n = run_for(tls, t + seconds, 1000 * w)
        return n, time.perf_counter() - t

    with ThreadPoolExecutor(workers) as ex:
        res = list(ex.map(pooled, range(workers)))
    n2 = sum(r[0] for r in res)
    el2 = max(r[1] for r in res)
    host = f"host {cpu_model()}, {visible} logical CPUs visible"
    single = {"value": round(n1 * px_per_item / el1 / 1e6, 3), "unit": unit, "cores": 1, "kind": kind,
              "sample": f"{n1} frames in {el1:.1f} s on 1 thread: {label}; {host}"}
    pool = {"value": round(n2 * px_per_item / el2 / 1e6, 3), "unit": unit, "cores": workers, "kind": kind,
            "sample": f"{n2} frames in {el2:.1f} s over {workers} threads ({cap}), one detector state per "
                      f"thread: {label}; {host}"}
    return single, pool


def cpu_frames(torch, dev, pattern, n, rows, cols, seed, period=16):
    return make_frames(torch, pattern, n, rows, cols, seed, dev, period).cpu().numpy()


def launch_ranks(n):
    """`bench.py --gpus N` without torchrun: start N rank processes (one GPU each) and wait for them.
    The parent never touches the GPU (only the ranks do), so no GPU context is inherited or exec'd."""
    import socket
    import subprocess

    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rcs = [p.wait() for p in procs]
    bad = [rc for rc in rcs if rc != 0]
    return bad[0] if bad else 0


# Global batches of the strong-scaled legs (BASELINE configs[3]: 256 frames over the GPUs; configs[4]:
# 512 frames over the GPUs): each rank takes its contiguous block (shard.shard_range).
STRONG_GLOBAL = {"config4_lsd_map": 256, "config5_superpoint": 512}


def strong_blocks(world, rank):
    from feature_detector_amd.shard import shard_range

    return {leg: shard_range(n, rank, world) for leg, n in STRONG_GLOBAL.items()}


def rank_layout(dist, world, rank, local, device, device_count):
    """Every rank's placement, gathered to all ranks over the process group (control plane only)."""
    me = {"rank": rank, "local_rank": local, "device": device, "device_count": device_count, "pid": os.getpid(),
          "strong_blocks": strong_blocks(world, rank)}
    if world == 1:
        return [me], {"backend": None, "world_size": 1}
    objs = [None] * world
    dist.all_gather_object(objs, me)
    return objs, {"backend": dist.get_backend(), "world_size": dist.get_world_size()}


def launch_check(args, world, rank, local):
    """FD_BENCH_LAUNCH_CHECK=1: the rank layout without any GPU work (the CPU tests use it with gloo):
    every rank reports its device index and its blocks of the strong-scaled legs; rank 0 prints one
    JSON line in the bench's own `ranks` / `process_group` format."""
    import torch.distributed as dist

    ndev = int(os.environ.get("FD_BENCH_LAUNCH_CHECK_DEVICES", "0")) or world
    dist.init_process_group("gloo")
    objs, pg = rank_layout(dist, world, rank, local, local % ndev, ndev)
    if rank == 0:
        print(json.dumps({"n_gpus": world, "requested_gpus": args.gpus, "ranks": objs, "process_group": pg,
                          "strong_global_batch": STRONG_GLOBAL}), flush=True)
    dist.destroy_process_group()


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))  # self-launch: one rank process per GPU
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}; launch one rank per GPU")
    if os.environ.get("FD_BENCH_LAUNCH_CHECK") == "1":
        return launch_check(args, world, rank, local)
    import torch
    import torch.distributed as dist

    # Control-plane collectives only (barrier, timing max): RCCL by default; FD_BENCH_BACKEND=gloo
    # rehearses N>1 on fewer GPUs (ranks then share devices round-robin).
    backend = os.environ.get("FD_BENCH_BACKEND", "nccl")
    ndev = torch.cuda.device_count()
    if backend == "nccl" and world > ndev:
        raise SystemExit(f"bench.py: {world} ranks but {ndev} visible GPUs (RCCL needs one GPU per rank; "
                         "FD_BENCH_BACKEND=gloo rehearses more ranks than GPUs)")
    dev_index = local % max(ndev, 1)
    torch.cuda.set_device(dev_index)
    dev = torch.device("cuda", dev_index)
    if world > 1:
        dist.init_process_group(backend)
    import feature_detector_amd as fd
    from feature_detector_amd.shard import max_over_ranks

    fd.load()

    # ---- headline workload (per rank: its own frames; weak scaling) -------------------------------
    barrier = dist.barrier if world > 1 else None
    with phase(torch, "headline"):
        secs, done, pool, _ = run_config(torch, fd, dev, args.detector, args.rows, args.cols, args.batch, args.pool,
                                         args.need, args.dist, args.pattern, args.steps, args.warmup,
                                         not args.no_graph, seed=1234 + 1000003 * rank, barrier=barrier)
    secs_max = max_over_ranks(secs, dist if world > 1 else None, dev if backend == "nccl" else None)
    px_step = args.batch * args.rows * args.cols
    value = world * done * px_step / secs_max / 1e6  # Mpix/s, all ranks
    ms_per_step = secs_max / done * 1e3

    # ---- per-kernel timing for the roofline (rank-local, same stream) -----------------------------
    with phase(torch, "roofline_kernel"):
        k_ms = kernel_time_ms(torch, fd, pool, args.detector, THR[args.detector])
    k_bytes = px_step  # algorithmic: 1 B/px frame read
    kernels = {"corner_or_fast_ms": k_ms, "step_ms": ms_per_step}
    # the remainder of a step is the per-frame selection (one workgroup per frame)
    sel_ms = max(ms_per_step - k_ms, 0.0)
    kernels["select_and_rest_ms"] = sel_ms
    dominant = "k_corner" if args.detector != "fast" else "k_fast"
    if sel_ms > k_ms:
        dominant_note = ("k_select (per-frame greedy selection, one workgroup per frame) dominates the step at this "
                         "batch; roofline below is for the per-pixel kernel")
    else:
        dominant_note = f"{dominant} dominates the step"
    achieved = k_bytes / (k_ms * 1e-3) / 1e9
    traffic, traffic_src = (measured_traffic("bench_k_corner") if (args.detector == "harris" and args.rows == 480
                                                                     and args.cols == 640 and args.batch == 1)
                            else (None, None))
    ties_headline = tie_report(torch, fd, dev, args.detector, pool, args.need, args.dist, raster_ms=ms_per_step)
    roofline = {"kernel": dominant, "bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
                "bytes_per_launch": k_bytes, "avg_launch_ms": round(k_ms, 5), "note": dominant_note}
    if traffic_src:
        roofline["traffic_source"] = (traffic_src + ": FETCH_SIZE x calibrated 2.0; at batch 1 short tiles re-read "
                                      "their halo rows and the level-0 histogram atomics are memory-side")
    # The same kernel in the committed rocprofv3 summary of this bench command: its roofline_kernel leg
    # (the launches timed above: agrees with avg_launch_ms), and its duration inside the headline step
    # (shorter: there it follows k_select instead of another K1 append).
    kname = "k_corner<" if args.detector != "fast" else "k_fast<"
    rp = rocprof_kernel("roofline_kernel", kname)
    rs = rocprof_kernel("headline", kname)
    if rp:
        roofline["rocprof"] = {"source": rp[2], "phase": "fdbench:roofline_kernel", "avg_us": rp[0], "calls": rp[1],
                               "frac": round(k_bytes / (rp[0] * 1e-6) / 1e9 / HBM_PEAK_GBS, 5)}
    if rs:
        roofline["in_step"] = {"source": rs[2], "phase": "fdbench:headline", "avg_us": rs[0],
                               "frac": round(k_bytes / (rs[0] * 1e-6) / 1e9 / HBM_PEAK_GBS, 5)}
    # the step's dominant kernel is latency-bound (one workgroup per frame): its time, in core clocks, and
    # where those go (phase clocks of the headline frame)
    sel = rocprof_kernel("headline", "k_select<")
    latency = {"kernel": "k_select", "bound": "latency (one 1024-thread workgroup per frame)",
               "avg_us": sel[0] if sel else None, "source": sel[2] if sel else None,
               "cycles_at_peak_clock": round(sel[0] * CLOCK_GHZ * 1e3) if sel else None,
               "phases": select_phase_cycles()}
    del pool

    out = {
        "metric": "Mpix/s corner-response+NMS, 640x480 gray batch, 1/2/4/8 MI355X",
        "value": round(value, 2), "unit": "Mpix/s", "n_gpus": world, "steps": done, "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 5), "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "u8->i32/f32", "data": "synthetic (seeded u8 %s frames generated on GPU)" % args.pattern,
        "config": {"workload": f"{args.detector} response+NMS + grid NMS (greedy min-distance select), "
                               f"{args.cols}x{args.rows} gray, batch {args.batch}/GPU (BASELINE configs[1])",
                   "detector": args.detector, "rows": args.rows, "cols": args.cols, "global_batch": args.batch * world,
                   "need": args.need, "min_feature_distance": args.dist, "min_valid_response": THR[args.detector],
                   "parallelism": f"frame-sharded x{world} (no collective)", "graph": not args.no_graph},
        "roofline": roofline,
        "latency": latency,
        "kernels": kernels,
        "ties": ties_headline,
    }
    if args.batch == 1 and not args.no_graph:
        with phase(torch, "headline_pipelined"):
            p_ms, p_frames = run_pipelined(torch, fd, dev, args.detector, args.rows, args.cols, args.need, args.dist,
                                           args.pattern, seed=4321 + rank, nctx=4)
        out["headline_pipelined"] = {
            "workload": "same batch-1 calls, consecutive frames round-robin over 4 contexts/streams (up to 4 "
                        "requests in flight: per-pixel kernels overlap other frames' single-workgroup selections; "
                        "tools/pipe_sweep.py: 1/2/3/4/6 contexts); not `value`", "contexts": 4,
            "ms_per_frame": round(p_ms, 5), "mpix_s": round(args.rows * args.cols / (p_ms * 1e-3) / 1e6, 1),
            "frames": p_frames}

    # ---- north-star shape: Shi-Tomasi 1920x1080 batch 256 (kernel roofline) -----------------------
    if not args.no_north_star:
        ns_batch = 256
        with phase(torch, "north_star"):
            s2, d2, pool2, _ = run_config(torch, fd, dev, "shi_tomasi", 1080, 1920, ns_batch, 2, 200, 20, "noise",
                                          10, 2, False, seed=99 + rank)
        with phase(torch, "north_star_kernel"):
            kms = kernel_time_ms(torch, fd, pool2, "shi_tomasi", 40.0, reps=10)
        with phase(torch, "north_star_ties"):
            ties_ns = tie_report(torch, fd, dev, "shi_tomasi", pool2, 200, 20, steps=4, raster_ms=s2 / d2 * 1e3)
        del pool2
        with phase(torch, "north_star_kernel_checker"):
            pool3 = [make_frames(torch, "checker", ns_batch, 1080, 1920, 199 + rank + 7919 * i, dev) for i in range(2)]
            kms_checker = kernel_time_ms(torch, fd, pool3, "shi_tomasi", 40.0, reps=10)
            del pool3
        kb = ns_batch * 1080 * 1920
        ach = kb / (kms * 1e-3) / 1e9
        ns_issue = north_star_issue()
        out["north_star"] = {
            "workload": "shi_tomasi response+NMS + grid NMS, 1920x1080 gray, batch 256/GPU, noise",
            "mpix_s_per_gpu": round(d2 * kb / s2 / 1e6, 1), "ms_per_step": round(s2 / d2 * 1e3, 4),
            "kernel": "k_corner_lp<ShiTomasi, 4 px/lane>", "kernel_ms": round(kms, 4),
            "kernel_mpix_s": round(kb / (kms * 1e-3) / 1e6, 1),
            "kernel_ms_checker": round(kms_checker, 4),
            "roofline": {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(ach / HBM_PEAK_GBS, 4), "bytes_per_launch": kb,
                         "traffic": measured_traffic("northstar_k_corner")[0],
                         # the bound that binds: VALU issue slots (SQ pass of the same kernel, profiles/)
                         "valu_frac": ns_issue["valu_issue_slot_busy"] if ns_issue else None,
                         "valu": valu_floor(ns_issue, kb, kms)},
            "issue": ns_issue,
            "ties": ties_ns,
        }

    # ---- BASELINE configs[2]: FAST-12 + BRIEF-256, 1280x720 batch 64 (detect -> describe on device) --
    if not args.no_config3:
        with phase(torch, "config3_fast_brief"):
            out["config3_fast_brief"] = run_config3(torch, fd, dev, seed=777 + rank)

    # ---- BASELINE configs[4]: SuperPoint, 640x480, 64 frames per GPU --------------------------------
    # (strong scaling: the global batch split over the ranks; every rank's block, device and the process
    # group's own world size go into the line)
    blocks = strong_blocks(world, rank)
    max_fn = (lambda v: max_over_ranks(v, dist if world > 1 else None, dev if backend == "nccl" else None))
    if not args.no_superpoint:
        s0, e0 = blocks["config5_superpoint"]
        with phase(torch, "config5_superpoint"):
            out["config5_superpoint"] = run_superpoint(torch, fd, dev, seed=5151 + 7 * s0, batch=e0 - s0,
                                                       global_batch=STRONG_GLOBAL["config5_superpoint"],
                                                       barrier=barrier, max_fn=max_fn)

    # ---- BASELINE configs[3]: LSD map, 1920x1080, 256 frames over the ranks ------------------------
    if not args.no_lsd:
        s0, e0 = blocks["config4_lsd_map"]
        with phase(torch, "config4_lsd_map"):
            out["config4_lsd_map"] = run_lsd(torch, fd, dev, seed=4242 + 7 * s0, batch=e0 - s0,
                                             global_batch=STRONG_GLOBAL["config4_lsd_map"], barrier=barrier,
                                             max_fn=max_fn)
    out["ranks"], out["process_group"] = rank_layout(dist, world, rank, local, dev_index, ndev)
    with phase(torch, "device_copy"):
        cb = copy_bandwidth(torch, dev)
        out["device_copy_gbs"] = cb.pop("device_copy_gbs")
        out["device_copy"] = cb
        lsd = out.get("config4_lsd_map")
        if lsd and cb.get("lsd_shape_gbs"):  # the map against a kernel that moves the same bytes and nothing else
            lsd["roofline"]["shape_ceiling_gbs"] = cb["lsd_shape_gbs"]
            lsd["roofline"]["frac_of_shape_ceiling"] = round(lsd["roofline"]["achieved"] / cb["lsd_shape_gbs"], 4)
    if world == 1:
        with phase(torch, "end_to_end"):
            out["end_to_end_host_frames"] = run_end_to_end(torch, fd, args)
            out["end_to_end_ingest"] = run_ingest(torch, fd, args)

    # ---- CPU baselines beside every leg: rank 0 at N=1, bounded samples of the same workloads ------
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from oracle import oracle as O

        O.lib()
        sec = args.cpu_seconds
        leg = max(2.0, sec / 2.5)

        def refflow(kind_name, frames, dist_, need_):
            def work(i, tls):
                det = tls.setdefault("det", O.RefFlowDetector())
                det.detect(KIND[kind_name], frames[i % len(frames)], dist_, THR[kind_name], need_)
            return work

        frames = cpu_frames(torch, dev, args.pattern, 64, args.rows, args.cols, 4242)
        flow = ("reference data flow (oracle/fd_oracle_refflow.cpp: float sliding sums, dense response map, "
                "std::sort, int32 mask), g++ -O3 like the reference build")
        out["cpu_baseline"], out["cpu_baseline_pool"] = cpu_leg(
            refflow(args.detector, frames, args.dist, args.need), args.rows * args.cols, sec,
            label=f"{args.detector} DetectGoodFeatures {args.cols}x{args.rows} {args.pattern}, dist {args.dist}, "
                  f"need {args.need}; {flow}")
        del frames
        if "north_star" in out:
            for pat in ("noise", "checker"):
                fr = cpu_frames(torch, dev, pat, 8, 1080, 1920, 99)
                b1, bp = cpu_leg(refflow("shi_tomasi", fr, 20, 200), 1080 * 1920, leg,
                                 label=f"shi_tomasi DetectGoodFeatures 1920x1080 {pat}, dist 20, need 200; {flow}")
                key = "" if pat == "noise" else "_checker"
                out["north_star"]["cpu_baseline" + key], out["north_star"]["cpu_baseline_pool" + key] = b1, bp
        if "config3_fast_brief" in out:
            fr = cpu_frames(torch, dev, "noise", 8, 720, 1280, 777)

            def fast_brief(i, tls):
                det = tls.setdefault("det", O.RefFlowDetector())
                img = fr[i % len(fr)]
                kp = det.detect(KIND["fast"], img, 20, THR["fast"], 200)
                O.brief(img, kp, 256, 8, 0)

            out["config3_fast_brief"]["cpu_baseline"], out["config3_fast_brief"]["cpu_baseline_pool"] = cpu_leg(
                fast_brief, 720 * 1280, leg,
                label="FAST thr 10 DetectGoodFeatures (reference data flow) + BRIEF-256 per keypoint "
                      "(oracle restatement), 1280x720 noise, dist 20, need 200")
        if "config4_lsd_map" in out:
            fr = cpu_frames(torch, dev, "checker", 8, 1080, 1920, 4242, period=64)

            def lsd(i, tls):
                img = fr[i % len(fr)]
                nrm, _, _, idx = O.lsd_map(img)
                O.lsd_sort(nrm, idx)

            out["config4_lsd_map"]["cpu_baseline"], out["config4_lsd_map"]["cpu_baseline_pool"] = cpu_leg(
                lsd, 1080 * 1920, leg,
                label="ComputeLineLevelAngleMap restatement (maps + column-major valid list + std::sort by norm), "
                      "1920x1080 64-px checker")

            def lines(i, tls):
                O.lsd_lines(fr[i % len(fr)])

            lb, lp = cpu_leg(lines, 1080 * 1920, leg,
                             label="FeatureLineDetector::DetectGoodFeatures restatement (oracle/fd_oracle_lines.cpp, "
                                   "the reference's data structures), 1920x1080 64-px checker")
            out["config4_lsd_map"]["lines"]["cpu_baseline"], out["config4_lsd_map"]["lines"]["cpu_baseline_pool"] = lb, lp
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
