"""Tile-geometry sweep for the per-pixel kernel (tuning aid): times point_response / detect_points
for several FD_TARGET_WAVES / FD_TILE_MULT settings, each in a fresh process (the geometry is read at
call time from the environment, so one process per setting keeps the runs independent)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import sys, json, torch
sys.path.insert(0, %r)
import feature_detector_amd as fd
kind, rows, cols, batch, mode = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), sys.argv[5]
g = torch.Generator(device="cuda"); g.manual_seed(7)
fr = torch.randint(0, 256, (batch, rows, cols), generator=g, device="cuda", dtype=torch.int32).to(torch.uint8)
thr = {"harris": 30.0, "shi_tomasi": 40.0, "fast": 10.0}[kind]
def run():
    if mode == "response": fd.point_response(kind, fr, thr)
    else: fd.detect_points(kind, fr, 200, 20, thr)
for _ in range(3): run()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(10): run()
e1.record(); torch.cuda.synchronize()
print(json.dumps({"ms": e0.elapsed_time(e1) / 10}))
''' % ROOT

def main():
    kind, rows, cols, batch, mode = sys.argv[1:6]
    for tw in [int(x) for x in sys.argv[6].split(",")]:
        for mult in [int(x) for x in sys.argv[7].split(",")]:
            env = dict(os.environ, FD_TARGET_WAVES=str(tw), FD_TILE_MULT=str(mult))
            out = subprocess.run([sys.executable, "-c", CHILD, kind, rows, cols, batch, mode], env=env,
                                 capture_output=True, text=True, timeout=300)
            line = out.stdout.strip().splitlines()[-1] if out.returncode == 0 else "ERR " + out.stderr[-300:]
            print(kind, rows, cols, batch, mode, "target_waves", tw, "mult", mult, line, flush=True)
            if out.returncode != 0:
                return 1
    return 0

if __name__ == "__main__":
    sys.exit(main())
