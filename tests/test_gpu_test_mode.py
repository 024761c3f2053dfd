"""TEST mode (getColorFromNF, kernel.cu:72-187) on the GPU: the axis plane march and C3 size.

Views along a volume axis (the reference's default camera looks along z) march plane by plane
(test_axis_kernel: the corner planes carried from sample to sample and memoised on their class
tuple; along x and y too, with the per-plane values the reference's y-x-z lerp order allows).  That is the same arithmetic on the same values as the per-sample evaluation, so its exact
(back-to-front) frames must equal the generic TEST march (vr_options.test_plane_march = 0) and the
oracle's (the restated reference) bit for bit; front-to-back ERT frames are held to the 1e-4
tolerance (the two marches check ERT at different batch boundaries).  At C3 size
(1920x1080x500, BASELINE.json configs[2]) the whole frame is checked through size-independent
properties and a column sample against the oracle.
"""
import numpy as np
import pytest

import volumerenderingproject_amd as vr
from test_gpu_parity import assert_bitwise

pytestmark = pytest.mark.gpu

E, T = vr.VR_FLAG_ESS, vr.VR_FLAG_ERT
TOL = 1e-4


def z_cameras(W, H):
    """Views whose inverse view keeps two coordinates fixed along the ray (the plane march's
    condition) -- along z, x and y, both directions each -- and one that does not (the oblique
    reset camera: generic march in both builds)."""
    up = tuple(vr.default_camera(W, H).up)
    rsw, rsh = 2.0, 2.0 * H / W
    return {
        "default": vr.default_camera(W, H),
        "behind": vr.derive_camera((0.0, 0.0, -1.0), up, rsw, rsh),     # looking along +z: p_z grows
        "zoomed": vr.derive_camera((0.0, 0.0, 0.45), up, rsw, rsh),     # starts inside the volume box
        "far": vr.derive_camera((0.0, 0.0, 2.5), up, rsw, rsh),
        "x": vr.derive_camera((1.0, 0.0, 0.0), (0.0, 1.0, 0.0), rsw, rsh),     # along -x
        "x_back": vr.derive_camera((-1.0, 0.0, 0.0), (0.0, 1.0, 0.0), rsw, rsh),
        "y": vr.derive_camera((0.0, 1.0, 0.0), (0.0, 0.0, 1.0), rsw, rsh),     # along -y
        "y_back": vr.derive_camera((0.0, -0.6, 0.0), (0.0, 0.0, 1.0), rsw, rsh),   # inside the box
        "oblique": vr.reset_camera(),
    }


@pytest.mark.parametrize("W,H,S", [(64, 48, 64), (127, 95, 37), (200, 150, 1000), (300, 300, 300)])
def test_plane_march_equals_generic(avg152, W, H, S):
    vol, cal = avg152
    a = vr.VolumeRenderer(vol, cal, device=0)
    b = vr.VolumeRenderer(vol, cal, device=0, options=vr.default_options(test_plane_march=0))
    for name, cam in z_cameras(W, H).items():
        exact = None
        for flags in (0, E, T, E | T):
            p = vr.default_params(W, H, S, mode=vr.VR_MODE_TEST, flags=flags)
            fa, fb = a.render(p, cam), b.render(p, cam)
            if flags & T:
                # front to back, ERT checked once per batch: the two marches batch differently, so
                # each is held to the ERT tolerance against the exact frame, not to the other
                assert np.abs(fa - exact).max() <= TOL and np.abs(fb - exact).max() <= TOL, (name, flags)
            else:
                assert np.array_equal(fa, fb), (name, flags, float(np.abs(fa - fb).max()))
                exact = fa
    a.close()
    b.close()


def test_plane_march_mni_and_tile_output(mni_standin):
    """The MNI stand-in (step 0.87 voxel per sample at S = 500) and tile-buffer output (farming)."""
    import torch
    vol, cal = mni_standin
    W, H, S = 480, 270, 500
    a = vr.VolumeRenderer(vol, cal, device=0)
    b = vr.VolumeRenderer(vol, cal, device=0, options=vr.default_options(test_plane_march=0))
    cams = z_cameras(W, H)
    for name in ("default", "behind", "zoomed", "x", "y_back"):
        ex = a.render(vr.default_params(W, H, S, mode=vr.VR_MODE_TEST), cams[name])
        assert np.array_equal(ex, b.render(vr.default_params(W, H, S, mode=vr.VR_MODE_TEST), cams[name])), name
        p = vr.default_params(W, H, S, mode=vr.VR_MODE_TEST, flags=E | T)
        assert np.abs(a.render(p, cams[name]) - ex).max() <= TOL, name
    p = vr.default_params(W, H, S, mode=vr.VR_MODE_TEST, flags=E | T)
    tiles = torch.zeros((8, 64 * 64, 3), dtype=torch.float32, device="cuda:0")
    ref = a.render(p, cams["default"])
    n = a.render_tiles(p, cams["default"], 64, 64, 3, 5, tiles.data_ptr(), rgb=True)
    nty = (H + 63) // 64
    got = tiles.cpu().numpy()
    for k in range(n):
        t = 3 + 5 * k
        tx, ty = divmod(t, nty)
        blk = got[k].reshape(64, 64, 3)
        x1, y1 = min(W, tx * 64 + 64), min(H, ty * 64 + 64)
        assert np.array_equal(blk[:x1 - tx * 64, :y1 - ty * 64], ref[tx * 64:x1, ty * 64:y1, :3])
    a.close()
    b.close()


def test_plane_march_cube_wrap_and_tf_variants(oracle_mod):
    """A cube-filling random volume (corner rows wrap into the next row / slab at the upper faces;
    corners past the last voxel are the idx < total guard) and a TF whose class 0 is opaque (the
    plane march does not apply: generic march) against the oracle, bitwise in exact mode."""
    O = oracle_mod
    rng = np.random.default_rng(7)
    vol = rng.integers(0, 256, size=(40, 33, 47)).astype(np.float32)
    W, H, S = 90, 70, 160
    tfs = [vr.default_transfer_function(),
           [(0.0, 1.0, (0.1, 0.2, 0.3, 0.05)), (0.3, 0.6, (0.9, 0.5, 0.1, 0.4))]]
    for tf in tfs:
        with vr.VolumeRenderer(vol, 255.0, tf=tf, device=0) as r:
            views = [((0.0, 0.0, 1.0), (0.0, 1.0, 0.0)), ((1.0, 0.0, 0.0), (0.0, 1.0, 0.0)),
                     ((0.0, -1.0, 0.0), (0.0, 0.0, 1.0))]
            cams = [(vr.default_camera(W, H), O.camera_default(W, H))]
            cams += [(vr.derive_camera(pos, upv, 2.0, 2.0 * H / W), O.camera_derive(pos, upv, 2.0, 2.0 * H / W))
                     for pos, upv in views[1:]]
            for cam, ocam in cams:
                ref = O.render_test(vol, 255.0, O.tf_array(tf), O.params(W, H, S), ocam)
                got = r.render(vr.default_params(W, H, S, mode=vr.VR_MODE_TEST), cam)
                assert_bitwise(got, ref)
                fast = r.render(vr.default_params(W, H, S, mode=vr.VR_MODE_TEST, flags=E | T), cam)
                assert np.abs(fast - ref).max() <= TOL


@pytest.mark.parametrize("camera", ["default", "oblique"])
def test_c3_test_mode_1920x1080(mni_standin, oracle_mod, camera):
    """C3 in TEST mode (verdict r2 item 4): whole frame ESS == exact bitwise, ESS + ERT within 1e-4
    of exact, alpha = 1, background where rays miss; 17 columns against the oracle bitwise (exact)
    and within 1e-4 (ESS + ERT).  kernel.cu:72-187, :194-225."""
    import torch
    vol, cal = mni_standin
    W, H, S = 1920, 1080, 500
    O = oracle_mod
    r = vr.VolumeRenderer(vol, cal, device=0)
    cam = vr.default_camera(W, H) if camera == "default" else vr.reset_camera()
    out = {}
    for name, fl in (("exact", 0), ("ess", E), ("fast", E | T)):
        t = torch.empty((W, H, 4), dtype=torch.float32, device="cuda:0")
        r.render_device(vr.default_params(W, H, S, mode=vr.VR_MODE_TEST, flags=fl), cam, t.data_ptr())
        out[name] = t
    assert torch.equal(out["ess"], out["exact"])
    assert (out["fast"] - out["exact"]).abs().max().item() <= TOL
    assert torch.all(out["exact"][..., 3] == 1.0)
    miss = (out["exact"][..., :3] == torch.tensor([0.2, 0.2, 0.2], device="cuda:0")).all(-1)
    assert miss.any() and not miss.all()
    xs = sorted(set(int(x) for x in np.linspace(0, W - 1, 17).round()))
    ocam = O.camera_default(W, H) if camera == "default" else O.camera_oblique(W, H)
    ref = O.render_test_columns(vol, cal, O.default_tf(), O.params(W, H, S), ocam, xs)
    assert_bitwise(out["exact"][xs].cpu().numpy(), ref)
    assert np.abs(out["fast"][xs].cpu().numpy() - ref).max() <= TOL
    r.close()


def _orbit_views(W, H, n=3):
    """General (non-axis) views: the oblique reset camera and a few orbit positions."""
    import math
    cams = {"oblique": vr.reset_camera()}
    up = (0.0, 1.0, 0.0)
    for i in range(n):
        a = 0.4 + 1.9 * i
        pos = (math.cos(a) * 0.9, 0.35 * (i - 1), math.sin(a) * 0.9)
        cams[f"orbit{i}"] = vr.derive_camera(pos, up, 2.0, 2.0 * H / W)
    return cams


@pytest.mark.parametrize("n_tf", [4, 10, 20])
def test_corner_volumes_are_exact(avg152, oracle_mod, n_tf):
    """The general TEST march's corner volumes (vr_options.test_corners): per voxel the 8 corner
    classes at the TF's class width, x-major (0: 16 / 32 / 64 bits for 4 / 10 / 20 intervals) or in
    4^3-voxel bricks (3), 64 bits x-major (1) and none -- four corner-row dword gathers (2) -- render the same
    frames bit for bit in every mode, on avg152 and on a cube-filling random volume whose corner rows
    wrap into the next row / slab (the reference's flat-index read, kernel.cu:130-155); the exact
    frames equal the oracle's.  Front to back (ERT) with 2-bit corner classes (<= 4 intervals: modes 0
    and 3) the march reads the plane table instead of the TF (round 6): those two modes agree bit for
    bit, the 64-bit and dword modes (1, 2: TF reads and lerps) bit for bit, and the two pairs, and each
    against the oracle's exact frame, within the ERT tolerance."""
    from test_gpu_parity import _tf_n
    O = oracle_mod
    tf = _tf_n(n_tf)
    rng = np.random.default_rng(11)
    vols = [avg152, (rng.integers(0, 256, size=(37, 30, 41)).astype(np.float32), 255.0)]
    W, H, S = 96, 72, 180
    for vol, cal in vols:
        rs = [vr.VolumeRenderer(vol, cal, tf=tf, device=0, options=vr.default_options(test_corners=m))
              for m in (0, 1, 2, 3)]
        for name, cam in _orbit_views(W, H).items():
            ref = O.render_test(vol, cal, O.tf_array(tf), O.params(W, H, S), O.camera_oblique(W, H)) \
                if name == "oblique" else None
            for flags in (0, E, T, E | T):
                p = vr.default_params(W, H, S, mode=vr.VR_MODE_TEST, flags=flags)
                got = [r.render(p, cam) for r in rs]
                if (flags & T) and n_tf <= 4:   # plane table in modes 0 and 3
                    assert_bitwise(got[3], got[0])
                    assert_bitwise(got[2], got[1])
                    assert np.abs(got[0] - got[1]).max() <= TOL
                else:
                    for g in got[1:]:
                        assert_bitwise(g, got[0])
                if ref is not None:
                    if flags & T:
                        assert max(float(np.abs(g - ref).max()) for g in got) <= TOL
                    else:
                        assert_bitwise(got[0], ref)
        for r in rs:
            r.close()


def test_long_rays_general_test_march(avg152, oracle_mod):
    """the general TEST march's per-frame position table is bounded (16 B per sample in
    LDS); rays longer than the bound compute the same expressions per sample.  S = 9000 (past the
    table) renders, bitwise against the oracle in exact mode and within 1e-4 with ESS + ERT, and
    S = 4000 (the table) agrees with the oracle too."""
    vol, cal = avg152
    O = oracle_mod
    W, H = 20, 14
    with vr.VolumeRenderer(vol, cal, device=0) as r:
        for S in (4000, 9000):
            ref = O.render_test(vol, cal, O.default_tf(), O.params(W, H, S), O.camera_oblique(W, H))
            got = r.render(vr.default_params(W, H, S, mode=vr.VR_MODE_TEST), vr.reset_camera())
            assert_bitwise(got, ref)
            fast = r.render(vr.default_params(W, H, S, mode=vr.VR_MODE_TEST, flags=E | T), vr.reset_camera())
            assert np.abs(fast - ref).max() <= TOL


@pytest.mark.parametrize("camera", ["default", "oblique"])
def test_count_work_test_mode(avg152, camera):
    """vr_count_work in TEST mode (the roofline numerator of TEST bench lines): the counting pass
    renders vr_render's frame; the corner-row dword march reads 4 B per gather; the compact corner
    volume (2 B entries at the default TF) reads fewer bytes for the same samples evaluated; ESS and
    ERT only remove work."""
    import torch
    vol, cal = avg152
    W, H, S = 128, 96, 200
    cam = vr.default_camera(W, H) if camera == "default" else vr.reset_camera()
    r0 = vr.VolumeRenderer(vol, cal, device=0)
    r2 = vr.VolumeRenderer(vol, cal, device=0, options=vr.default_options(test_corners=2))
    prev = None
    for flags in (0, E, E | T):
        p = vr.default_params(W, H, S, mode=vr.VR_MODE_TEST, flags=flags)
        w0, w2 = r0.count_work(p, cam), r2.count_work(p, cam)
        for w in (w0, w2):
            assert w["gathers"] > 0 and w["bytes"] > 0 and w["samples"] > 0
        if camera == "oblique":
            assert w2["bytes"] == 4 * w2["gathers"]
            if flags & T:   # (the plane table's front-to-back colours round differently: ERT may end a
                            #  ray a batch apart)
                assert abs(w0["samples"] - w2["samples"]) <= 0.001 * w2["samples"]
            else:
                assert w0["samples"] == w2["samples"]
            assert w0["bytes"] < w2["bytes"] // 4
        if prev is not None:
            assert w0["samples"] <= prev
        prev = w0["samples"]
    # the counting pass leaves vr_render's frame in the context: same frame as a plain render (general
    # views front to back: the plane table of r0 against r2's TF reads, within the ERT tolerance)
    p = vr.default_params(W, H, S, mode=vr.VR_MODE_TEST, flags=E | T)
    if camera == "oblique":
        assert np.abs(r0.render(p, cam) - r2.render(p, cam)).max() <= TOL
    else:
        assert_bitwise(r0.render(p, cam), r2.render(p, cam))
    r0.close()
    r2.close()


def test_count_work_vrc_matches_count_marched(avg152):
    """vr_count_work on VRC frames: the gathers and samples of vr_count_marched, and 1 B per class
    gather on a 32-bit volume (no run words)."""
    vol, cal = avg152
    W, H, S = 120, 90, 160
    with vr.VolumeRenderer(vol, cal, device=0) as r:
        for cam in (vr.default_camera(W, H), vr.reset_camera()):
            for flags in (0, E | T):
                p = vr.default_params(W, H, S, flags=flags)
                g, n = r.count_marched(p, cam)
                w = r.count_work(p, cam)
                assert (w["gathers"], w["samples"]) == (g, n) and w["bytes"] == g


def test_test_mode_screen_cull_is_exact(mni_standin):
    """TEST whole frames cull the work tiles off the dataset box's projection (its bounding
    rectangle and, for general views, its hull: vr_api.cpp project_box_test through M^-1 of
    getColorFromNF's matrices) into background-only workgroups: every mode and view renders the frame
    of the unculled march (cull = 0) bit for bit, and the farm's visible tiles (vr_visible_tiles)
    keep every tile with a non-background pixel."""
    vol, cal = mni_standin
    W, H, S = 400, 240, 200
    a = vr.VolumeRenderer(vol, cal, device=0)
    b = vr.VolumeRenderer(vol, cal, device=0, options=vr.default_options(cull=0))
    cams = dict(z_cameras(W, H))
    cams.update(_orbit_views(W, H))
    far = vr.derive_camera((0.0, 0.0, 2.5), tuple(vr.default_camera(W, H).up), 2.0, 2.0 * H / W)
    cams["far"] = far
    for name, cam in cams.items():
        for flags in (0, E, T, E | T):
            p = vr.default_params(W, H, S, mode=vr.VR_MODE_TEST, flags=flags)
            fa = a.render(p, cam)
            assert_bitwise(fa, b.render(p, cam))
            if flags == (E | T):
                bg = np.array([0.2, 0.2, 0.2], np.float32)
                vis = set(int(t) for t in a.visible_tiles(p, cam, 64, 64))
                nty = (H + 63) // 64
                for tx in range((W + 63) // 64):
                    for ty in range(nty):
                        blk = fa[tx * 64:(tx + 1) * 64, ty * 64:(ty + 1) * 64, :3]
                        if not np.all(blk == bg):
                            assert tx * nty + ty in vis, (name, tx, ty)
    a.close()
    b.close()


def test_test_axis_tables_follow_view_and_stream(avg152):
    """TEST axis views stage the march axis's per-view tables that the host builds once per view and
    stream (make_test_axis_table; uploaded when an input changes): in one context, views, flags, S
    and sizes changing from frame to frame and two caller streams alternating with the context's own
    give bit for bit the frames of the generic march (test_plane_march = 0), which has no such table."""
    import torch
    vol, cal = avg152
    a = vr.VolumeRenderer(vol, cal, device=0)
    b = vr.VolumeRenderer(vol, cal, device=0, options=vr.default_options(test_plane_march=0))
    try:
        seq = []
        for W, H, S in ((96, 72, 120), (64, 48, 300)):
            cams = z_cameras(W, H)
            for name in ("default", "x", "default", "y_back", "behind", "default"):
                for flags in (0, E):
                    seq.append((W, H, S, flags, name, cams[name]))
        s1, s2 = torch.cuda.Stream(device=0), torch.cuda.Stream(device=0)
        streams = (None, s1, s2, s1, None)
        for i, (W, H, S, flags, name, cam) in enumerate(seq):
            st = streams[i % len(streams)]
            a.set_stream(st.cuda_stream if st is not None else 0)
            p = vr.default_params(W, H, S, mode=vr.VR_MODE_TEST, flags=flags)
            fa = a.render(p, cam)
            assert np.array_equal(fa, b.render(p, cam)), (i, W, H, S, flags, name)
    finally:
        a.set_stream(0)
        a.close()
        b.close()


def test_stream_caches_survive_destroyed_streams(avg152):
    """the per-stream caches (AXIS1 view tables, work lists, TEST axis tables) of streams a
    caller has since destroyed.  Twelve caller streams, each used for a TEST axis frame and a VRC
    frame, switched away from and destroyed: past the eighth the caches of the other streams are
    retired behind the context's live streams (no wait on a dead handle), and every frame stays bit
    for bit the frame of a context that never left its own stream."""
    import ctypes
    import torch  # noqa: F401  (loads the HIP runtime libvr shares)
    hip = ctypes.CDLL("libamdhip64.so.7")
    vol, cal = avg152
    W, H, S = 64, 48, 120
    cam = vr.default_camera(W, H)
    pt = vr.default_params(W, H, S, mode=vr.VR_MODE_TEST, flags=E)
    pv = vr.default_params(W, H, S, flags=E | T)
    with vr.VolumeRenderer(vol, cal, device=0) as ref, vr.VolumeRenderer(vol, cal, device=0) as a:
        want_t, want_v = ref.render(pt, cam), ref.render(pv, cam)
        for i in range(12):
            s = ctypes.c_void_p()
            assert hip.hipStreamCreate(ctypes.byref(s)) == 0
            a.set_stream(s.value)
            assert np.array_equal(a.render(pt, cam), want_t), i
            assert np.array_equal(a.render(pv, cam), want_v), i
            a.set_stream(0)
            assert hip.hipStreamDestroy(s) == 0
        assert np.array_equal(a.render(pt, cam), want_t)
        assert np.array_equal(a.render(pv, cam), want_v)
