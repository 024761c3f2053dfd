"""Seeded random views against the oracle: cameras on a sphere around the volume (re-derived with
processInput's formulas, myApp.cu:1105-1112, on both sides), odd frame sizes and sample counts,
every compositing mode.  Exact and ESS-only frames are bitwise the oracle's (the reference's
back-to-front blend, kernel.cu:194-225); ESS + ERT and ERT alone within 1e-4; TEST exact bitwise
(kernel.cu:72-187).  Covers the general-view paths (padded leaf maps, lazy empty-space tests,
empty-cell skipping of exact frames) on views no other test picks."""
import math

import numpy as np
import pytest

import volumerenderingproject_amd as vr
from test_gpu_parity import assert_bitwise

pytestmark = pytest.mark.gpu

TOL = 1e-4
E, T = vr.VR_FLAG_ESS, vr.VR_FLAG_ERT


def random_views(n, seed):
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        W, H = int(rng.integers(17, 97)), int(rng.integers(13, 81))
        S = int(rng.integers(20, 320))
        th, ph = rng.uniform(0, 2 * math.pi), rng.uniform(-1.2, 1.2)
        dist = rng.uniform(0.7, 1.3)
        pos = (dist * math.cos(ph) * math.sin(th), dist * math.sin(ph), dist * math.cos(ph) * math.cos(th))
        up = (0.0, 1.0, 0.0) if abs(ph) < 1.0 else (1.0, 0.0, 0.0)
        out.append((W, H, S, pos, up))
    return out


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_random_views_match_oracle(avg152, avg152_octree, oracle_mod, seed):
    vol, cal = avg152
    O = oracle_mod
    r = vr.VolumeRenderer(vol, cal, device=0)
    try:
        for i, (W, H, S, pos, up) in enumerate(random_views(16, seed)):
            p = vr.default_params(W, H, S)
            cam = vr.derive_camera(pos, up, p.real_screen_width, p.real_screen_height)
            op = O.params(W, H, S)
            ocam = O.camera_derive(pos, up, op.real_screen_width, op.real_screen_height)
            ref = avg152_octree.render_vrc(cal, O.default_tf(), op, ocam)
            for flags in (0, E):
                assert_bitwise(r.render(vr.default_params(W, H, S, flags=flags), cam), ref)
            for flags in (E | T, T):
                got = r.render(vr.default_params(W, H, S, flags=flags), cam)
                assert np.abs(got - ref).max() <= TOL, (i, flags)
            if i % 3 == 0:
                tref = O.render_test(vol, cal, O.default_tf(), op, ocam)
                assert_bitwise(r.render(vr.default_params(W, H, S, mode=vr.VR_MODE_TEST), cam), tref)
    finally:
        r.close()
