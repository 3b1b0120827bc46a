"""Diagnostic: k_corner_lp candidate lists (fd_points_response) and detect features against the oracle
for each lane width (FD_PX), on image.png and seeded noise / checker frames. Prints mismatch details."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import feature_detector_amd as fd  # noqa: E402
from oracle import oracle as O  # noqa: E402
from tests.conftest import _read_png_gray as read_png_gray  # noqa: E402

KIND = {"harris": 0, "shi_tomasi": 1}
THR = {"harris": 30.0, "shi_tomasi": 40.0}
imgs = {"image.png": read_png_gray(os.path.join(ROOT, "tests", "golden", "image.png")),
        "noise480": O.make_frame("noise", 7, 480, 640), "checker720": O.make_frame("checker", 8, 720, 1280)}
bad = 0
for px in sys.argv[1:] or ["2", "4", "8"]:
    os.environ["FD_PX"] = px
    for iname, img in imgs.items():
        for name in ("harris", "shi_tomasi"):
            rows, cols = img.shape
            dev = torch.from_numpy(img[None].copy()).cuda()
            resp, idx, cnt = fd.point_response(name, dev, THR[name])
            torch.cuda.synchronize()
            n = int(cnt.cpu()[0])
            gi = idx[0, :n].cpu().numpy().astype(np.int64)
            gr = resp[0, :n].cpu().numpy()
            er, ex, ey = O.nms(O.response_map(img, KIND[name], THR[name], None), THR[name])
            ei = ey.astype(np.int64) * cols + ex
            o = np.argsort(gi, kind="stable")
            same = len(gi) == len(ei) and np.array_equal(gi[o], ei) and np.array_equal(gr[o].view(np.uint32), er.view(np.uint32))
            msg = f"px={px} {iname} {name}: cands {n} vs {len(ei)} {'OK' if same else 'DIFF'}"
            if not same:
                bad += 1
                gs, es = set(gi.tolist()), set(ei.tolist())
                extra, miss = sorted(gs - es)[:8], sorted(es - gs)[:8]
                msg += f" extra {[(i % cols, i // cols) for i in extra]} missing {[(i % cols, i // cols) for i in miss]}"
                if len(gs) != len(gi):
                    msg += f" dup {len(gi) - len(gs)}"
                if not extra and not miss and len(gs) == len(gi):
                    d = np.nonzero(gr[o].view(np.uint32) != er.view(np.uint32))[0][:5]
                    msg += f" value diffs at {[(int(ei[k] % cols), int(ei[k] // cols), float(gr[o][k]), float(er[k])) for k in d]}"
            res = fd.detect_points(name, img, 200, 20, THR[name], ties="raster")
            exp, _ = O.detect(KIND[name], img, 20, THR[name], 200, sort_mode=1)
            got = res.features(0)
            fsame = np.array_equal(got, exp)
            msg += f" | features {len(got)} vs {len(exp)} {'OK' if fsame else 'DIFF'}"
            if not fsame:
                bad += 1
                k = next((i for i in range(min(len(got), len(exp))) if not np.array_equal(got[i], exp[i])), None)
                msg += f" first diff at {k}: {got[k] if k is not None else None} vs {exp[k] if k is not None else None}"
            print(msg, flush=True)
print("bad", bad)
