"""Diagnostic: print k_select phase clocks (FD_SELECT_STAMPS=1) for the bench shapes."""
import os, sys
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import numpy as np, torch
import feature_detector_amd as fd
from oracle import oracle as O
img = O.make_frame("noise", 1234, 480, 640)
for name, thr in (("harris", 30.0), ("shi_tomasi", 40.0), ("fast", 10.0)):
    for _ in range(3):
        fd.detect_points(name, img, 200, 20, thr)
img = O.make_frame("noise", 1234, 1080, 1920)
for name, thr in (("shi_tomasi", 40.0), ("fast", 10.0)):
    for _ in range(2):
        fd.detect_points(name, img, 200, 20, thr)
