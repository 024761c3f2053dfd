"""Generate tests/golden/frames_avg152.npz with the CPU oracle (the restated reference algorithm).

Frames (float32, [x*H + y] RGBA) of avg152T1_LR, the reference transfer function:
  VRC + TEST x {default steady camera, key-X reset camera} at 100x100x100, and 64x48x64 (non-square).
Plus per-ray VRC sample dumps for 8 pixels and the N_in sample counts.  These pin the GPU path on
boxes where the oracle is rebuilt anyway, and guard the oracle itself against regressions.
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402
from volumerenderingproject_amd import volumes  # noqa: E402


def main():
    vol, hdr = volumes.avg152()
    cal = hdr["cal_max"]
    oct_ = O.OracleOctree(vol)
    tf = O.default_tf()
    out = {}
    for (W, H, S) in [(100, 100, 100), (64, 48, 64)]:
        for camn in ["default", "oblique"]:
            cam = O.camera_default(W, H) if camn == "default" else O.camera_oblique(W, H)
            p = O.params(W, H, S)
            out[f"vrc_{W}x{H}x{S}_{camn}"] = oct_.render_vrc(cal, tf, p, cam)
            out[f"test_{W}x{H}x{S}_{camn}"] = O.render_test(vol, cal, tf, p, cam)
            out[f"nin_{W}x{H}x{S}_{camn}"] = np.array(oct_.count_in_samples(p, cam), np.int64)
    W, H, S = 100, 100, 100
    p = O.params(W, H, S)
    cam = O.camera_default(W, H)
    pix = [(50, 50), (30, 60), (70, 40), (10, 10), (99, 99), (45, 80), (55, 20), (62, 62)]
    out["ray_pixels"] = np.array(pix, np.int32)
    out["ray_samples"] = np.stack([oct_.ray_samples(cal, tf, p, cam, x, y) for x, y in pix])
    np.savez_compressed(os.path.join(ROOT, "tests", "golden", "frames_avg152.npz"), **out)
    print({k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()
