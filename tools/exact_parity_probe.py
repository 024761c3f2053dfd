"""Max |GPU - oracle| of the exact (back-to-front) VRC and TEST frames at the parity sizes, and
whether they are bitwise equal (diagnostic for the contraction-off model)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import numpy as np  # noqa: E402
import oracle as O  # noqa: E402
import volumerenderingproject_amd as vr  # noqa: E402
from volumerenderingproject_amd import volumes  # noqa: E402

vol, hdr = volumes.avg152()
cal = hdr["cal_max"]
r = vr.VolumeRenderer(vol, cal, device=0)
octree = O.OracleOctree(vol)
for W, H, S in [(100, 100, 100), (64, 48, 64), (37, 91, 150), (120, 90, 333), (300, 300, 300)]:
    for camera in ("default", "oblique"):
        ocam = O.camera_default(W, H) if camera == "default" else O.camera_oblique(W, H)
        cam = vr.default_camera(W, H) if camera == "default" else vr.reset_camera()
        ref = octree.render_vrc(cal, O.default_tf(), O.params(W, H, S), ocam)
        got = r.render(vr.default_params(W, H, S), cam)
        reft = O.render_test(vol, cal, O.default_tf(), O.params(W, H, S), ocam)
        gott = r.render(vr.default_params(W, H, S, mode=vr.VR_MODE_TEST), cam)
        gotf = r.render(vr.default_params(W, H, S, mode=vr.VR_MODE_TEST, flags=3), cam)
        print(f"{W}x{H}x{S} {camera}: VRC max {np.abs(got - ref).max():.3g} bitwise {np.array_equal(got, ref)} "
              f"| TEST max {np.abs(gott - reft).max():.3g} bitwise {np.array_equal(gott, reft)} "
              f"(n diff {(gott != reft).sum()}) | TEST ess+ert max {np.abs(gotf - reft).max():.3g}", flush=True)
