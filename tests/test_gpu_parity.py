"""HIP kernels vs the CPU oracle (the restated reference algorithm), through the C-ABI.

Tolerance: 1e-4 per channel (north_star) for the fast front-to-back modes (ERT).  The exact
back-to-front mode (the reference's blendSampleColors order) is BITWISE equal to the oracle: both
evaluate the reference's arithmetic as written, each float operation rounded, no contraction
(DESIGN.md section 2).  ESS alone must be BITWISE equal to the exact mode (it only skips alpha-0
samples).
"""
import ctypes

import numpy as np
import pytest

import volumerenderingproject_amd as vr
from volumerenderingproject_amd import volumes

pytestmark = pytest.mark.gpu

TOL = 1e-4
VR_EINVAL = -1   # include/vr_api.h


@pytest.fixture(scope="module")
def r152(avg152):
    vol, cal = avg152
    r = vr.VolumeRenderer(vol, cal, device=0)
    yield r
    r.close()


def assert_bitwise(got, ref):
    assert got.shape == ref.shape
    d = np.abs(got - ref)
    assert np.array_equal(got, ref), f"max |diff| {d.max():.3g} at {np.unravel_index(d.argmax(), d.shape)}, " \
                                     f"{int((d > 0).sum())} values differ"


def oracle_vrc(oracle_mod, octree, cal, W, H, S, camera="default"):
    O = oracle_mod
    cam = O.camera_default(W, H) if camera == "default" else O.camera_oblique(W, H)
    return octree.render_vrc(cal, O.default_tf(), O.params(W, H, S), cam)


def oracle_test(oracle_mod, vol, cal, W, H, S, camera="default"):
    O = oracle_mod
    cam = O.camera_default(W, H) if camera == "default" else O.camera_oblique(W, H)
    return O.render_test(vol, cal, O.default_tf(), O.params(W, H, S), cam)


def cam_of(W, H, camera):
    return vr.default_camera(W, H) if camera == "default" else vr.reset_camera()


@pytest.mark.parametrize("camera", ["default", "oblique"])
@pytest.mark.parametrize("W,H,S", [(100, 100, 100), (64, 48, 64), (37, 91, 150), (300, 300, 300)])
def test_vrc_exact_matches_oracle(r152, avg152, avg152_octree, oracle_mod, W, H, S, camera):
    vol, cal = avg152
    ref = oracle_vrc(oracle_mod, avg152_octree, cal, W, H, S, camera)
    got = r152.render(vr.default_params(W, H, S), cam_of(W, H, camera))
    assert got.shape == ref.shape
    assert np.all(got[..., 3] == 1.0)
    assert_bitwise(got, ref)


@pytest.mark.parametrize("camera", ["default", "oblique"])
@pytest.mark.parametrize("W,H,S", [(100, 100, 100), (64, 48, 64), (300, 300, 300)])
def test_vrc_ess_bitwise_and_ert_within_tol(r152, avg152, avg152_octree, oracle_mod, W, H, S, camera):
    vol, cal = avg152
    cam = cam_of(W, H, camera)
    exact = r152.render(vr.default_params(W, H, S), cam)
    ess = r152.render(vr.default_params(W, H, S, flags=vr.VR_FLAG_ESS), cam)
    assert np.array_equal(exact, ess)          # skipping alpha-0 samples is exact
    ref = oracle_vrc(oracle_mod, avg152_octree, cal, W, H, S, camera)
    for flags in (vr.VR_FLAG_ERT, vr.VR_FLAG_ESS | vr.VR_FLAG_ERT):
        got = r152.render(vr.default_params(W, H, S, flags=flags), cam)
        assert np.abs(got - ref).max() <= TOL, flags


@pytest.mark.parametrize("camera", ["default", "oblique"])
@pytest.mark.parametrize("W,H,S", [(100, 100, 100), (64, 48, 64), (120, 90, 333)])
def test_test_mode_matches_oracle(r152, avg152, oracle_mod, W, H, S, camera):
    vol, cal = avg152
    ref = oracle_test(oracle_mod, vol, cal, W, H, S, camera)
    cam = cam_of(W, H, camera)
    exact = r152.render(vr.default_params(W, H, S, mode=vr.VR_MODE_TEST), cam)
    assert_bitwise(exact, ref)
    ess = r152.render(vr.default_params(W, H, S, mode=vr.VR_MODE_TEST, flags=vr.VR_FLAG_ESS), cam)
    assert np.array_equal(ess, exact)           # TEST macro cells skip only alpha-0 samples
    for flags in (vr.VR_FLAG_ERT, vr.VR_FLAG_ESS | vr.VR_FLAG_ERT):
        got = r152.render(vr.default_params(W, H, S, mode=vr.VR_MODE_TEST, flags=flags), cam)
        assert np.abs(got - ref).max() <= TOL, flags


def test_count_samples_matches_oracle(r152, avg152_octree, oracle_mod):
    for W, H, S, camera in [(100, 100, 100, "default"), (64, 48, 64, "oblique"), (120, 90, 200, "default")]:
        O = oracle_mod
        ocam = O.camera_default(W, H) if camera == "default" else O.camera_oblique(W, H)
        ref = avg152_octree.count_in_samples(O.params(W, H, S), ocam)
        got = r152.count_samples(vr.default_params(W, H, S), cam_of(W, H, camera))
        assert got == ref, (W, H, S, camera)
    # the survey's figure for C1: 88,200 in-dataset samples at 100x100x100
    assert r152.count_samples(vr.default_params(100, 100, 100), vr.default_camera(100, 100)) == 88200


@pytest.mark.parametrize("rgb", [False, True])
def test_tiles_assemble_equals_frame(r152, rgb):
    """Tile renders + assembly == the whole frame, bitwise; rgb: VR_OUT_RGB 3-float tile pixels."""
    import torch
    W, H, S = 200, 136, 120
    ch = 3 if rgb else 4
    p = vr.default_params(W, H, S, flags=vr.VR_FLAG_ESS | vr.VR_FLAG_ERT)
    cam = vr.default_camera(W, H)
    full = r152.render(p, cam)
    for world, tw, th in [(1, 64, 64), (3, 64, 64), (4, 32, 48)]:
        from volumerenderingproject_amd.renderer import tiles_per_rank
        mt = max(tiles_per_rank(W, H, tw, th, r, world) for r in range(world))
        tiles = torch.zeros((world, mt, tw * th, ch), dtype=torch.float32, device="cuda:0")
        for rank in range(world):
            n = r152.render_tiles(p, cam, tw, th, rank, world, tiles[rank].data_ptr(), rgb=rgb)
            assert n == tiles_per_rank(W, H, tw, th, rank, world)
        frame = torch.zeros((W, H, 4), dtype=torch.float32, device="cuda:0")
        r152.assemble_tiles(W, H, tw, th, world, mt, tiles.data_ptr(), frame.data_ptr(), rgb=rgb)
        assert np.array_equal(frame.cpu().numpy(), full), (world, tw, th)
        # the kernels write exactly the layout volumerenderingproject_amd.distributed states
        from volumerenderingproject_amd import distributed as D
        for rank in range(world):
            n = tiles_per_rank(W, H, tw, th, rank, world)
            ref = D.tiles_from_frame(full, tw, th, rank, world, channels=ch)
            got = tiles[rank, :n].cpu().numpy()
            for k in range(n):   # pixels outside the frame are left untouched by the kernel
                t = rank + k * world
                tx, ty = divmod(t, D.grid(W, H, tw, th)[1])
                w, h = min(tw, W - tx * tw), min(th, H - ty * th)
                assert np.array_equal(got[k].reshape(tw, th, ch)[:w, :h], ref[k].reshape(tw, th, ch)[:w, :h])


@pytest.mark.parametrize("camera", ["default", "oblique", "conic", "conic_oblique"])
def test_visible_tiles_are_conservative(r152, oracle_mod, camera):
    """Every pixel of a tile vr_visible_tiles drops is exactly the background (all four views)."""
    W, H, S = 400, 260, 150
    flags = vr.VR_FLAG_ESS | vr.VR_FLAG_ERT
    if camera.startswith("conic"):
        rsw, rsh, cam, _ = conic_setup(oracle_mod, W, H, "default" if camera == "conic" else "oblique")
        p = vr.default_params(W, H, S, flags=flags | vr.VR_FLAG_CONIC)
        p.real_screen_width, p.real_screen_height = rsw, rsh
    else:
        p, cam = vr.default_params(W, H, S, flags=flags), cam_of(W, H, camera)
    full = r152.render(p, cam)
    bg = np.array(list(p.background), np.float32)
    for tw, th in [(64, 64), (16, 32)]:
        ids = set(r152.visible_tiles(p, cam, tw, th).tolist())
        ntx, nty = -(-W // tw), -(-H // th)
        assert 0 < len(ids) <= ntx * nty
        for t in range(ntx * nty):
            if t not in ids:
                tx, ty = divmod(t, nty)
                assert np.all(full[tx * tw:(tx + 1) * tw, ty * th:(ty + 1) * th] == bg), (camera, t)
    if camera == "default":      # the box covers a minority of the screen: real culling
        assert len(r152.visible_tiles(p, cam, 64, 64)) < 0.6 * (-(-W // 64)) * (-(-H // 64))
    # TEST mode (round 5: the box projected through getColorFromNF's matrices): the tiles it drops
    # are exactly the background of the TEST frame too
    pt = vr.default_params(W, H, S, mode=vr.VR_MODE_TEST)
    ct = cam_of(W, H, camera) if not camera.startswith("conic") else cam_of(W, H, "default")
    tfull = r152.render(pt, ct)
    ids = set(r152.visible_tiles(pt, ct, 64, 64).tolist())
    nty = -(-H // 64)
    assert 0 < len(ids) <= (-(-W // 64)) * nty
    for t in range((-(-W // 64)) * nty):
        if t not in ids:
            tx, ty = divmod(t, nty)
            assert np.all(tfull[tx * 64:(tx + 1) * 64, ty * 64:(ty + 1) * 64] == bg), ("TEST", camera, t)


@pytest.mark.parametrize("rgb", [False, True])
def test_tile_list_render_assemble_equals_frame(r152, rgb):
    import torch
    W, H, S = 300, 200, 120
    ch = 3 if rgb else 4
    p = vr.default_params(W, H, S, flags=vr.VR_FLAG_ESS | vr.VR_FLAG_ERT)
    cam = vr.default_camera(W, H)
    full = r152.render(p, cam)
    bg = list(p.background)
    for world, tw, th in [(1, 64, 64), (3, 64, 64), (2, 32, 48)]:
        ids = r152.visible_tiles(p, cam, tw, th)
        mt = -(-len(ids) // world)
        tiles = torch.zeros((world, mt, tw * th, ch), dtype=torch.float32, device="cuda:0")
        for rank in range(world):
            n = r152.render_tile_list(p, cam, tw, th, ids, rank, world, tiles[rank].data_ptr(), rgb=rgb)
            assert n == len(ids[rank::world])
        frame = torch.full((W, H, 4), -7.0, dtype=torch.float32, device="cuda:0")
        r152.assemble_tile_list(W, H, tw, th, ids, world, mt, tiles.data_ptr(), bg, frame.data_ptr(), rgb=rgb)
        assert np.array_equal(frame.cpu().numpy(), full), (world, tw, th)
    with pytest.raises(vr.VRError):
        r152.render_tile_list(p, cam, 64, 64, [10 ** 6], 0, 1, tiles.data_ptr())


@pytest.mark.parametrize("w0", [1.0, 2.5, 1e6])
def test_weighted_plan_render_assemble_slots_equals_frame(r152, w0):
    """The multi-GPU farm's data path on one GPU: each rank's share of a weighted plan rendered with
    vr_render_tile_list (RGB tiles) into its block range, vr_assemble_tile_slots == the frame."""
    import torch
    from volumerenderingproject_amd import distributed as D
    W, H, S, T = 300, 200, 120, 32
    p = vr.default_params(W, H, S, flags=vr.VR_FLAG_ESS | vr.VR_FLAG_ERT)
    cam = vr.default_camera(W, H)
    full = r152.render(p, cam)
    ids = [int(t) for t in r152.visible_tiles(p, cam, T, T)]
    for world in (2, 3):
        lists = D.weighted_lists(ids, world, w0)
        tiles, slots, mt = D.plan_slots(lists)
        blocks = torch.zeros((world * mt, T * T, 3), dtype=torch.float32, device="cuda:0")
        for rank, L in enumerate(lists):
            if L:
                n = r152.render_tile_list(p, cam, T, T, L, 0, 1, blocks[rank * mt].data_ptr(), rgb=True)
                assert n == len(L)
        frame = torch.full((W, H, 4), -3.0, dtype=torch.float32, device="cuda:0")
        r152.assemble_tile_slots(W, H, T, T, tiles, slots, world * mt, blocks.data_ptr(), list(p.background),
                                 frame.data_ptr(), rgb=True)
        assert np.array_equal(frame.cpu().numpy(), full), (world, w0)
    with pytest.raises(vr.VRError):   # a tile listed twice
        r152.assemble_tile_slots(W, H, T, T, [ids[0], ids[0]], [0, 1], 2, blocks.data_ptr(), list(p.background),
                                 frame.data_ptr(), rgb=True)


def test_tile_farm_pipelined_streams_single_rank(r152):
    """TileFarm's pipelined GPU path (render on the main stream, assembly on the second stream after
    the render event, double-buffered blocks) over a one-rank process group: every step's frame,
    completed one step later, equals vr_render's frame bitwise."""
    import socket
    import torch
    import torch.distributed as dist
    from volumerenderingproject_amd.distributed import TileFarm
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    try:
        W, H, S = 300, 200, 120
        p = vr.default_params(W, H, S, flags=vr.VR_FLAG_ESS | vr.VR_FLAG_ERT)
        cams = [vr.default_camera(W, H), vr.reset_camera()]
        refs = [r152.render(p, c) for c in cams]
        for c, ref in zip(cams, refs):
            farm = TileFarm.for_renderer(r152, W, H, 0, 1, p, c, tile=32, device=0)
            assert farm.pipelined and farm.asm_stream is not None
            for i in range(4):
                farm.step()
            out = farm.drain()
            # no device-wide sync: .cpu() runs on the current stream, which drain() ordered after
            # the assembly on the farm's second stream
            assert np.array_equal(out.cpu().numpy(), ref)
            # a full batch, read right away through step()'s frame, while the next batch renders
            for i in range(farm.B):
                f = farm.step()
            first = f.cpu().numpy()
            for i in range(farm.B):
                farm.step()
            assert np.array_equal(first, ref) and np.array_equal(f.cpu().numpy(), ref)
            farm.drain()
            torch.cuda.synchronize()
    finally:
        dist.destroy_process_group()
        torch.cuda.synchronize()
        torch.cuda.set_stream(torch.cuda.default_stream())
        r152.set_stream(0)


def test_device_output_and_timing(r152):
    import torch
    W, H, S = 128, 96, 100
    p = vr.default_params(W, H, S)
    cam = vr.default_camera(W, H)
    host = r152.render(p, cam)
    out = torch.empty((W, H, 4), dtype=torch.float32, device="cuda:0")
    r152.timing_enable(True)
    r152.render_device(p, cam, out.data_ptr(), asynchronous=True)
    r152.synchronize()
    t = r152.timing_read()
    r152.timing_enable(False)
    assert t.launches == 1 and t.total_ms > 0
    assert np.array_equal(out.cpu().numpy(), host)


def test_transfer_function_update(r152, avg152, avg152_octree, oracle_mod):
    vol, cal = avg152
    tf = [(0.0, 1.0, (0.0, 0.0, 0.0, 0.0)), (0.2, 0.6, (0.1, 0.9, 0.3, 0.25)), (0.5, 0.55, (1.0, 0.0, 0.0, 0.9))]
    r152.set_transfer_function(tf)
    try:
        W, H, S = 80, 80, 120
        O = oracle_mod
        ref = avg152_octree.render_vrc(cal, O.tf_array(tf), O.params(W, H, S), O.camera_default(W, H))
        got = r152.render(vr.default_params(W, H, S, flags=vr.VR_FLAG_ESS), vr.default_camera(W, H))
        assert_bitwise(got, ref)
        reft = O.render_test(vol, cal, O.tf_array(tf), O.params(W, H, S), O.camera_default(W, H))
        gott = r152.render(vr.default_params(W, H, S, mode=vr.VR_MODE_TEST), vr.default_camera(W, H))
        assert_bitwise(gott, reft)
    finally:
        r152.set_transfer_function(vr.default_transfer_function())


def test_opaque_zero_class_disables_clipping(avg152, avg152_octree, oracle_mod):
    """TF(0).a > 0: samples outside the dataset are visible, so clipping/ESS must not apply."""
    vol, cal = avg152
    tf = [(0.0, 1.0, (0.1, 0.2, 0.3, 0.05)), (0.3, 0.5, (0.9, 0.9, 0.9, 0.5))]
    W, H, S = 60, 70, 90
    O = oracle_mod
    ref = avg152_octree.render_vrc(cal, O.tf_array(tf), O.params(W, H, S), O.camera_default(W, H))
    with vr.VolumeRenderer(vol, cal, tf=tf) as r:
        assert r.info.zero_transparent == 0
        for flags in (0, vr.VR_FLAG_ESS, vr.VR_FLAG_ESS | vr.VR_FLAG_ERT):
            got = r.render(vr.default_params(W, H, S, flags=flags), vr.default_camera(W, H))
            assert np.abs(got - ref).max() <= TOL


def test_mni_standin_c2_properties(mni_standin, oracle_mod):
    """C2 geometry (700x700, S=500) on the MNI stand-in: ESS bitwise == exact, ERT within 1e-4,
    and a half-resolution frame against the oracle."""
    vol, cal = mni_standin
    with vr.VolumeRenderer(vol, cal) as r:
        W, H, S = 700, 700, 500
        cam = vr.default_camera(W, H)
        exact = r.render(vr.default_params(W, H, S), cam)
        ess = r.render(vr.default_params(W, H, S, flags=vr.VR_FLAG_ESS), cam)
        assert np.array_equal(exact, ess)
        fast = r.render(vr.default_params(W, H, S, flags=vr.VR_FLAG_ESS | vr.VR_FLAG_ERT), cam)
        assert np.abs(fast - exact).max() <= TOL
        oct_ = oracle_mod.OracleOctree(vol)
        W2, H2, S2 = 175, 175, 125
        ref = oracle_vrc(oracle_mod, oct_, cal, W2, H2, S2)
        got = r.render(vr.default_params(W2, H2, S2, flags=vr.VR_FLAG_ESS), vr.default_camera(W2, H2))
        assert_bitwise(got, ref)


def test_against_committed_golden_frames(r152):
    """The committed oracle frames (tests/golden/frames_avg152.npz) reproduced through the C-ABI."""
    import os
    from conftest import GOLDEN
    g = np.load(os.path.join(GOLDEN, "frames_avg152.npz"))
    for (W, H, S) in [(100, 100, 100), (64, 48, 64)]:
        for camn in ["default", "oblique"]:
            cam = cam_of(W, H, camn)
            for flags in (0, vr.VR_FLAG_ESS):
                got = r152.render(vr.default_params(W, H, S, flags=flags), cam)
                assert_bitwise(got, g[f"vrc_{W}x{H}x{S}_{camn}"])
            got = r152.render(vr.default_params(W, H, S, flags=vr.VR_FLAG_ESS | vr.VR_FLAG_ERT), cam)
            assert np.abs(got - g[f"vrc_{W}x{H}x{S}_{camn}"]).max() <= TOL
            got = r152.render(vr.default_params(W, H, S, mode=vr.VR_MODE_TEST), cam)
            assert_bitwise(got, g[f"test_{W}x{H}x{S}_{camn}"])
            assert r152.count_samples(vr.default_params(W, H, S), cam) == int(g[f"nin_{W}x{H}x{S}_{camn}"])


@pytest.mark.parametrize("camera", ["default", "oblique"])
def test_shading_stage_matches_oracle(r152, avg152, avg152_octree, oracle_mod, camera):
    """Opt-in gradient + Phong (VR_FLAG_SHADE).  No reference counterpart exists, so
    parity is against the oracle's own restatement of the definition (parity unpinned)."""
    vol, cal = avg152
    W, H, S = 96, 80, 120
    O = oracle_mod
    sh = (0.3, 0.7, 0.2, 16.0)
    ocam = O.camera_default(W, H) if camera == "default" else O.camera_oblique(W, H)
    ref = avg152_octree.render_vrc_shaded(cal, O.default_tf(), O.params(W, H, S), ocam, sh)
    plain = avg152_octree.render_vrc(cal, O.default_tf(), O.params(W, H, S), ocam)
    assert np.abs(ref - plain).max() > 1e-2                     # shading changes the frame
    for flags in (vr.VR_FLAG_SHADE, vr.VR_FLAG_SHADE | vr.VR_FLAG_ESS, vr.VR_FLAG_SHADE | vr.VR_FLAG_ESS | vr.VR_FLAG_ERT):
        p = vr.default_params(W, H, S, flags=flags)
        p.shade_ambient, p.shade_diffuse, p.shade_specular, p.shade_shininess = sh
        got = r152.render(p, cam_of(W, H, camera))
        tol = TOL if flags & vr.VR_FLAG_ERT else 1e-5
        assert np.abs(got - ref).max() <= tol, flags
    with pytest.raises(vr.VRError):
        r152.render(vr.default_params(W, H, S, mode=vr.VR_MODE_TEST, flags=vr.VR_FLAG_SHADE), cam_of(W, H, camera))


@pytest.mark.parametrize("shape", [(64, 64, 64), (128, 100, 128), (32, 17, 32)])
def test_cube_filling_volumes(oracle_mod, shape):
    """Volumes whose longest side is a power of two fill the octree cube (box = [0, 1)), so the clip
    margin reaches outside the cube -- the case that exposed the ESS jump bug at 512^3 / 2048^3."""
    O = oracle_mod
    rng = np.random.default_rng(shape[1])
    vol = rng.integers(0, 256, size=shape).astype(np.float32)
    vol[vol < 120] = 0                                  # empty space for ESS to skip
    octree = O.OracleOctree(vol)
    r = vr.VolumeRenderer(vol, 255.0, device=0)
    for camera in ("default", "oblique"):
        for W, H, S in [(64, 48, 97), (50, 50, 256)]:
            ocam = O.camera_default(W, H) if camera == "default" else O.camera_oblique(W, H)
            ref = octree.render_vrc(255.0, O.default_tf(), O.params(W, H, S), ocam)
            cam = cam_of(W, H, camera)
            exact = r.render(vr.default_params(W, H, S), cam)
            assert_bitwise(exact, ref)
            assert np.array_equal(r.render(vr.default_params(W, H, S, flags=vr.VR_FLAG_ESS), cam), exact)
            fast = r.render(vr.default_params(W, H, S, flags=vr.VR_FLAG_ESS | vr.VR_FLAG_ERT), cam)
            assert np.abs(fast - ref).max() <= TOL
            # TEST mode on the same volume: corner indices wrap at the upper faces (kernel.cu:92-160)
            tref = O.render_test(vol, 255.0, O.default_tf(), O.params(W, H, S), ocam)
            texact = r.render(vr.default_params(W, H, S, mode=vr.VR_MODE_TEST), cam)
            assert_bitwise(texact, tref)
            tess = r.render(vr.default_params(W, H, S, mode=vr.VR_MODE_TEST, flags=vr.VR_FLAG_ESS), cam)
            assert np.array_equal(tess, texact)
    r.close()


def conic_setup(O, W, H, camera):
    """Conic screen of utils.h:57 (rsw = 2 tan(pi/4) * vpd) and the conic top-left corner."""
    import math
    vpd = 2.0
    rsw = float(np.float32(np.float32(2 * math.tan(np.float32(math.pi / 4))) * np.float32(vpd)))
    rsh = float(np.float32(np.float32(rsw) * np.float32(H) / np.float32(W)))
    if camera == "default":
        pos, up = (0.0, 0.0, 1.0), tuple(vr.default_camera(W, H).up)
    else:
        pos, up = (0.456607, 0.693644, -0.55711), (0.868199, -0.484147, 0.108777)
    return rsw, rsh, vr.derive_camera_conic(pos, up, rsw, rsh, vpd), O.camera_derive_conic(pos, up, rsw, rsh, vpd)


@pytest.mark.parametrize("camera", ["default", "oblique"])
def test_conic_projection_matches_oracle(r152, avg152, avg152_octree, oracle_mod, camera):
    """VR_FLAG_CONIC: perspective rays of kernel.cu:30-34 / :53-54 (disabled in the reference build,
    utils.h:28 -- parity against the oracle's restatement of those lines)."""
    vol, cal = avg152
    O = oracle_mod
    W, H, S = 90, 70, 160
    rsw, rsh, cam, ocam = conic_setup(O, W, H, camera)
    op = O.params(W, H, S)
    op.real_screen_width, op.real_screen_height, op.conic = rsw, rsh, 1
    ref = avg152_octree.render_vrc(cal, O.default_tf(), op, ocam)
    ortho = avg152_octree.render_vrc(cal, O.default_tf(), O.params(W, H, S), ocam)
    assert np.abs(ref - ortho).max() > 1e-2
    p = vr.default_params(W, H, S, flags=vr.VR_FLAG_CONIC)
    p.real_screen_width, p.real_screen_height = rsw, rsh
    exact = r152.render(p, cam)
    assert_bitwise(exact, ref)
    p.flags = vr.VR_FLAG_CONIC | vr.VR_FLAG_ESS
    assert np.array_equal(r152.render(p, cam), exact)
    p.flags = vr.VR_FLAG_CONIC | vr.VR_FLAG_ESS | vr.VR_FLAG_ERT
    assert np.abs(r152.render(p, cam) - ref).max() <= TOL
    p.flags = vr.VR_FLAG_CONIC
    assert r152.count_samples(p, cam) == avg152_octree.count_in_samples(op, ocam)
    with pytest.raises(vr.VRError):
        r152.render(vr.default_params(W, H, S, mode=vr.VR_MODE_TEST, flags=vr.VR_FLAG_CONIC), cam)


def test_point_cloud_matches_oracle(r152, avg152, oracle_mod):
    """POINT mode vertex array (prepareVolumeColors, myApp.cu:1280-1316), bit for bit."""
    import torch
    vol, cal = avg152
    out = torch.empty((vol.size, 7), dtype=torch.float32, device="cuda:0")
    r152.point_cloud_device(out.data_ptr())
    assert np.array_equal(out.cpu().numpy(), oracle_mod.point_cloud(vol, cal))
    odd = np.random.default_rng(5).integers(0, 300, size=(13, 7, 29)).astype(np.float32)
    r = vr.VolumeRenderer(odd, 255.0, device=0)
    out = torch.empty((odd.size, 7), dtype=torch.float32, device="cuda:0")
    r.point_cloud_device(out.data_ptr())
    assert np.array_equal(out.cpu().numpy(), oracle_mod.point_cloud(odd, 255.0))
    r.close()


def test_point_cloud_colours_on_the_screenshot_hull(r152, avg152, oracle_mod):
    """POINT mode pinned to the reference's own POINT screenshots (image_100x100_a0,
    image_300x300_a0, image_700x700_a0, myOutputIsAwesome: 100 % of their foreground within 2/255 of
    the hull of {background, the TF's colours}, tests/test_oracle_pin.py).  The GPU's vertex array
    (vr_point_cloud) carries exactly the TF's RGBA per voxel, and its points drawn the way the
    reference's GL path blends them (GL_SRC_ALPHA, GL_ONE_MINUS_SRC_ALPHA over the 0.2 background,
    myApp.cu:159-160, :977; one pixel per voxel column along z, in vertex order) give a frame whose
    8-bit foreground lies 100 % on that same hull."""
    import os
    import sys
    import torch
    from conftest import ROOT
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import screenshot_pin as SP
    vol, cal = avg152
    d1, d2, d3 = vol.shape
    out = torch.empty((vol.size, 7), dtype=torch.float32, device="cuda:0")
    r152.point_cloud_device(out.data_ptr())
    v = out.cpu().numpy()
    arr, n = oracle_mod.default_tf()
    rows = {tuple(np.float32(c) for c in arr[i].rgba) for i in range(n)}
    assert {tuple(np.float32(c) for c in x) for x in np.unique(v[:, 3:7], axis=0)} <= rows
    rgba = v[:, 3:7].reshape(d1, d2, d3, 4)
    img = np.full((d1, d2, 3), 0.2, np.float64)
    for z in range(d3):   # vertex order within a column is z ascending
        a = rgba[:, :, z, 3:4].astype(np.float64)
        img = rgba[:, :, z, :3] * a + img * (1.0 - a)
    img8 = np.clip(np.round(img * 255), 0, 255).astype(np.uint8)
    assert SP.fg_mask(img8).mean() > 0.2
    assert SP.palette_fraction(img8, SP.PALETTE_REF) == 1.0


def test_view_table_reuse_is_exact(avg152):
    """The axis-aligned view table published by one launch and staged by the next launches of the
    same view gives bitwise the frames of a context that rebuilds it in every launch, across view,
    flag, S and launch-kind changes (view_table_reuse = 0 is the rebuild-always context)."""
    import os
    import torch
    vol, cal = avg152
    ref_r = vr.VolumeRenderer(vol, cal, device=0, options=vr.default_options(view_table_reuse=0))
    r = vr.VolumeRenderer(vol, cal, device=0)
    try:
        EE, E = vr.VR_FLAG_ESS | vr.VR_FLAG_ERT, vr.VR_FLAG_ESS
        seq = [(100, 100, 100, EE), (100, 100, 100, EE), (100, 100, 100, 0), (100, 100, 100, 0),
               (100, 100, 257, E), (100, 100, 100, EE), (64, 48, 64, E), (64, 48, 64, E), (64, 48, 64, EE),
               (100, 100, 100, EE), (100, 100, 100, vr.VR_FLAG_ERT), (100, 100, 100, EE)]
        for i, (W, H, S, flags) in enumerate(seq):
            p = vr.default_params(W, H, S, flags=flags)
            cam = vr.default_camera(W, H)
            assert np.array_equal(r.render(p, cam), ref_r.render(p, cam)), (i, W, H, S, flags)
            if i == 6:   # a tile launch of the current view in between
                tiles = torch.zeros((8, 32 * 32, 4), dtype=torch.float32, device="cuda:0")
                r.render_tiles(p, cam, 32, 32, 0, 1, tiles.data_ptr())
                tref = torch.zeros_like(tiles)
                ref_r.render_tiles(p, cam, 32, 32, 0, 1, tref.data_ptr())
                assert torch.equal(tiles, tref)
        # the copies are kept per stream: alternate two streams and the context's own
        p = vr.default_params(96, 80, 200, flags=EE)
        cam = vr.default_camera(96, 80)
        want = ref_r.render(p, cam)
        s1, s2 = torch.cuda.Stream(device=0), torch.cuda.Stream(device=0)
        for st in (s1, s2, s1, None, s2, s1):
            r.set_stream(st.cuda_stream if st is not None else 0)
            assert np.array_equal(r.render(p, cam), want)
        r.set_stream(0)
        # an oblique view (no table) and back
        p = vr.default_params(100, 100, 100, flags=EE)
        assert np.array_equal(r.render(p, vr.reset_camera()), ref_r.render(p, vr.reset_camera()))
        assert np.array_equal(r.render(p, vr.default_camera(100, 100)), ref_r.render(p, vr.default_camera(100, 100)))
    finally:
        r.close()
        ref_r.close()


@pytest.mark.parametrize("volume", ["avg152", "cube_filling"])
def test_leaf_map_pad_is_exact(avg152, volume):
    """General orthographic views (every flag combination): the padded-leaf-map batches (no
    per-sample clamps, the padding's kMapOut as the out-of-cube test) give bitwise the frames of the clamped lookups
    (leaf_map_pad = 0), over orbit views, rays cut at S inside the dataset (the tail batches), a
    sample count whose pad would exceed the cap (padding off), a cube-filling volume (clip margins
    outside the cube) and tile launches."""
    import math
    import torch
    if volume == "avg152":
        vol, cal = avg152
    else:
        rng = np.random.default_rng(11)
        vol = rng.integers(0, 256, size=(64, 40, 64)).astype(np.float32)
        vol[vol < 110] = 0
        cal = 255.0
    a = vr.VolumeRenderer(vol, cal, device=0)
    b = vr.VolumeRenderer(vol, cal, device=0, options=vr.default_options(leaf_map_pad=0))
    try:
        W, H = 160, 120
        up = tuple(vr.default_camera(W, H).up)
        cams = [vr.reset_camera()]
        for i in range(5):
            t = 2 * math.pi * (i + 0.21) / 5
            p0 = vr.default_params(W, H, 300)
            cams.append(vr.derive_camera((math.sin(t), 0.4 * math.cos(2 * t), math.cos(t)), up,
                                         p0.real_screen_width, p0.real_screen_height))
        E, T = vr.VR_FLAG_ESS, vr.VR_FLAG_ERT
        for S, cut in ((300, None), (301, 61), (100, 37), (517, None), (9, None)):
            for flags in (E | T, 0, E, T):   # front to back; exact / ESS-only back to front; ERT alone
                p = vr.default_params(W, H, S, flags=flags)
                if cut is not None:
                    p.samples_per_ray = cut   # same sample distance, rays end inside the volume
                for i, cam in enumerate(cams):
                    assert np.array_equal(a.render(p, cam), b.render(p, cam)), (S, cut, flags, i)
        p = vr.default_params(W, H, 300, flags=vr.VR_FLAG_ESS | vr.VR_FLAG_ERT)
        ta = torch.zeros((20, 32 * 32, 4), dtype=torch.float32, device="cuda:0")
        tb = torch.zeros_like(ta)
        a.render_tiles(p, cams[1], 32, 32, 0, 1, ta.data_ptr())
        b.render_tiles(p, cams[1], 32, 32, 0, 1, tb.data_ptr())
        assert torch.equal(ta, tb)
    finally:
        a.close()
        b.close()


@pytest.mark.parametrize("kind", ["axis", "orbit"])
def test_visible_tiles_occupancy_culls_are_conservative(mni_standin, kind):
    """Every tile vr_visible_tiles drops is exactly the background, for the occupancy-based culls
    beyond the projected box (cull = 2): axis-parallel views (each volume axis, both directions,
    rolled, zoomed in) drop tiles over empty cell columns only; general orthographic views (orbit,
    zoomed, oblique) keep only the tiles an occupied super cell's projection reaches.  Both drop
    tiles the box tests (cull = 1) keep."""
    import math
    vol, cal = mni_standin
    W, H, S = 480, 270, 200
    dropped_beyond_box = 0
    with vr.VolumeRenderer(vol, cal, device=0) as r, \
            vr.VolumeRenderer(vol, cal, device=0, options=vr.default_options(cull=1)) as r1:
        p0 = vr.default_params(W, H, S)
        views = []
        if kind == "axis":
            for pos, up in [((1.0, 0, 0), (0, 1.0, 0)), ((-1.0, 0, 0), (0, 0, 1.0)), ((0, 1.0, 0), (0, 0, 1.0)),
                            ((0, -0.6, 0), (1.0, 0, 0)), ((0, 0, 1.0), (0, 1.0, 0)), ((0, 0, -0.3), (0.6, 0.8, 0))]:
                views.append(vr.derive_camera(pos, up, p0.real_screen_width, p0.real_screen_height))
            views.append(vr.default_camera(W, H))
        else:
            up = tuple(vr.default_camera(W, H).up)
            for i in range(5):
                t = 2 * math.pi * (i + 0.13) / 5
                for rad in (1.0, 0.4):
                    pos = (rad * math.sin(t), rad * 0.45 * math.cos(2 * t), rad * math.cos(t))
                    views.append(vr.derive_camera(pos, up, p0.real_screen_width, p0.real_screen_height))
            views.append(vr.reset_camera())
        for i, cam in enumerate(views):
            n_axes = sum(1 for a in range(3) if cam.front[a] != 0.0)
            assert (n_axes == 1) == (kind == "axis"), i
            for flags in (vr.VR_FLAG_ESS | vr.VR_FLAG_ERT, 0):
                p = vr.default_params(W, H, S, flags=flags)
                full = r.render(p, cam)
                bg = np.array(list(p.background), np.float32)
                for tw, th in [(64, 64), (16, 32), (32, 16)]:
                    ids = set(r.visible_tiles(p, cam, tw, th).tolist())
                    ids1 = set(r1.visible_tiles(p, cam, tw, th).tolist())
                    assert ids <= ids1
                    dropped_beyond_box += len(ids1 - ids)
                    ntx, nty = -(-W // tw), -(-H // th)
                    for t in range(ntx * nty):
                        if t not in ids:
                            tx, ty = divmod(t, nty)
                            assert np.all(full[tx * tw:(tx + 1) * tw, ty * th:(ty + 1) * th] == bg), (i, t, tw, th)
    assert dropped_beyond_box > 0


@pytest.mark.parametrize("volume", ["avg152", "mni"])
def test_hull_cull_is_exact(avg152, mni_standin, volume):
    """The march's workgroup cull of the work tiles off the projected box's hull (vr_options.cull =
    2, the default) gives bitwise the frames of the rectangle cull alone (cull = 1) and of no
    culling (cull = 0): orbit views, the oblique reset camera, zoomed-in views whose box overfills
    the screen, a conic camera, non-multiple-of-16 frame sizes, every flag combination."""
    import math
    vol, cal = avg152 if volume == "avg152" else mni_standin
    rs = [vr.VolumeRenderer(vol, cal, device=0, options=vr.default_options(cull=c)) for c in (2, 1, 0)]
    try:
        E, T = vr.VR_FLAG_ESS, vr.VR_FLAG_ERT
        for W, H in ((480, 270), (203, 157)):
            p0 = vr.default_params(W, H, 300)
            up = tuple(vr.default_camera(W, H).up)
            views = [(vr.reset_camera(), 0)]
            for i in range(6):
                t = 2 * math.pi * (i + 0.37) / 6
                for rad in (1.0, 0.35):   # 0.35: the box overfills the screen
                    pos = (rad * math.sin(t), rad * 0.5 * math.cos(2 * t), rad * math.cos(t))
                    views.append((vr.derive_camera(pos, up, p0.real_screen_width, p0.real_screen_height), 0))
            vpd = 2.0
            rsw = float(np.float32(np.float32(2 * math.tan(np.float32(math.pi / 4))) * np.float32(vpd)))
            rsh = float(np.float32(np.float32(rsw) * np.float32(H) / np.float32(W)))
            views.append((vr.derive_camera_conic((0.3, 0.2, 1.2), up, rsw, rsh, vpd), vr.VR_FLAG_CONIC))
            for flags in (E | T, 0, E, T):
                for i, (cam, extra) in enumerate(views):
                    p = vr.default_params(W, H, 300, flags=flags | extra)
                    if extra:
                        p.real_screen_width, p.real_screen_height = rsw, rsh
                    ref = rs[2].render(p, cam)
                    for r in rs[:2]:
                        assert np.array_equal(r.render(p, cam), ref), (W, H, flags, i)
    finally:
        for r in rs:
            r.close()


@pytest.mark.parametrize("volume", ["avg152", "mni"])
def test_column_cull_is_exact(avg152, mni_standin, volume):
    """Axis-parallel whole frames: worklist_kernel marks the work tiles whose rays' cell columns are
    all empty (vr_options.cull = 2, the default) -- bitwise the frames of no culling, for views
    along every axis in both directions, rolled, panned and zoomed in (the box overfilling the
    screen), non-multiple-of-16 sizes, every flag combination; and batches of moving axis-parallel
    cameras (a dolly and a pan: the device list is keyed by the camera) equal single frames."""
    import torch
    vol, cal = avg152 if volume == "avg152" else mni_standin
    rs = [vr.VolumeRenderer(vol, cal, device=0, options=vr.default_options(cull=c)) for c in (2, 0)]
    try:
        E, T = vr.VR_FLAG_ESS, vr.VR_FLAG_ERT
        for W, H in ((480, 270), (203, 157)):
            rsw, rsh = 2.0, 2.0 * H / W
            views = []
            for ax in range(3):
                for sgn in (1.0, -1.0):
                    pos = [0.0, 0.0, 0.0]
                    pos[ax] = sgn * 1.3
                    up = (0.0, 0.0, 1.0) if ax == 1 else (0.0, 1.0, 0.0)
                    views.append(vr.derive_camera(tuple(pos), up, rsw, rsh))
            views.append(vr.derive_camera((0.0, 0.0, 0.3), (0.0, 1.0, 0.0), rsw, rsh))    # zoomed in
            views.append(vr.derive_camera((0.0, 0.0, 1.0), (1.0, 0.0, 0.0), rsw, rsh))    # rolled 90 degrees
            pan = vr.derive_camera((0.0, 0.0, 1.0), (0.0, 1.0, 0.0), rsw, rsh)
            for a in range(3):
                pan.top_left[a] += 0.17 * pan.right[a] - 0.11 * pan.up[a]                  # panned
            views.append(pan)
            for flags in (E | T, 0, E, T):
                p = vr.default_params(W, H, 300, flags=flags)
                for i, cam in enumerate(views):
                    assert np.array_equal(rs[0].render(p, cam), rs[1].render(p, cam)), (W, H, flags, i)
        # moving axis-parallel cameras through the batched path: the list is rebuilt per camera
        W, H = 480, 270
        p = vr.default_params(W, H, 300, flags=E | T)
        cams = []
        for k in range(6):
            c = vr.derive_camera((0.0, 0.0, 1.4 - 0.2 * k), (0.0, 1.0, 0.0), 2.0, 2.0 * H / W)
            for a in range(3):
                c.top_left[a] += 0.03 * k * c.right[a]
            cams.append(c)
        out = torch.empty((len(cams), W, H, 4), dtype=torch.float32, device="cuda:0")
        rs[0].render_batch_device(p, cams, out.data_ptr())
        got = out.cpu().numpy()
        for k, c in enumerate(cams):
            assert np.array_equal(got[k], rs[1].render(p, c)), k
    finally:
        for r in rs:
            r.close()


def test_exact_skip_is_exact(avg152, avg152_octree, oracle_mod, mni_standin):
    """Exact orthographic frames march with empty-space skipping by default (vr_options.exact_skip):
    bitwise the frames of the plain march (exact_skip = 0) along each volume axis, in both
    directions, and for general views, for several S, and bitwise the oracle's."""
    vol, cal = avg152
    W, H = 120, 90
    a = vr.VolumeRenderer(vol, cal, device=0)
    b = vr.VolumeRenderer(vol, cal, device=0, options=vr.default_options(exact_skip=0))
    try:
        p0 = vr.default_params(W, H, 100)
        rsw, rsh = p0.real_screen_width, p0.real_screen_height
        cams = [vr.default_camera(W, H),
                vr.derive_camera((1.0, 0.0, 0.0), (0.0, 1.0, 0.0), rsw, rsh),
                vr.derive_camera((0.0, -1.0, 0.0), (0.0, 0.0, 1.0), rsw, rsh),
                vr.derive_camera((0.0, 0.0, -1.0), (0.0, 1.0, 0.0), rsw, rsh),
                vr.reset_camera(),                                            # general views
                vr.derive_camera((0.6, 0.3, 0.74), (0.0, 1.0, 0.0), rsw, rsh)]
        for S in (100, 257, 33):
            p = vr.default_params(W, H, S)
            for i, cam in enumerate(cams):
                assert np.array_equal(a.render(p, cam), b.render(p, cam)), (S, i)
        O = oracle_mod
        ref = avg152_octree.render_vrc(cal, O.default_tf(), O.params(W, H, 100), O.camera_default(W, H))
        assert_bitwise(a.render(vr.default_params(W, H, 100), cams[0]), ref)
    finally:
        a.close()
        b.close()
    vol, cal = mni_standin
    with vr.VolumeRenderer(vol, cal, device=0) as a, \
            vr.VolumeRenderer(vol, cal, device=0, options=vr.default_options(exact_skip=0)) as b:
        p = vr.default_params(700, 700, 500)
        cam = vr.default_camera(700, 700)
        assert np.array_equal(a.render(p, cam), b.render(p, cam))


def test_nonzero_class_of_zero(avg152, avg152_octree, oracle_mod):
    """A TF whose interval for value 0 is not interval 0 (class of TF(0) = 1, still alpha 0): the
    select-based gather paths (VRC axis-aligned march and TEST corners) instead of the class-0
    shortcuts, against the oracle."""
    vol, cal = avg152
    tf = [(0.3, 0.6, (0.9, 0.8, 0.7, 0.4)), (0.0, 0.05, (0.0, 0.0, 0.0, 0.0)), (0.05, 0.3, (0.2, 0.5, 0.3, 0.2))]
    W, H, S = 80, 64, 120
    O = oracle_mod
    ref = avg152_octree.render_vrc(cal, O.tf_array(tf), O.params(W, H, S), O.camera_default(W, H))
    reft = O.render_test(vol, cal, O.tf_array(tf), O.params(W, H, S), O.camera_default(W, H))
    with vr.VolumeRenderer(vol, cal, tf=tf) as r:
        assert r.info.zero_transparent == 1
        cam = vr.default_camera(W, H)
        exact = r.render(vr.default_params(W, H, S), cam)
        assert_bitwise(exact, ref)
        assert np.array_equal(r.render(vr.default_params(W, H, S, flags=vr.VR_FLAG_ESS), cam), exact)
        for _ in range(2):   # the second frame stages the published view table
            got = r.render(vr.default_params(W, H, S, flags=vr.VR_FLAG_ESS | vr.VR_FLAG_ERT), cam)
            assert np.abs(got - ref).max() <= TOL
        for flags in (0, vr.VR_FLAG_ERT, vr.VR_FLAG_ESS | vr.VR_FLAG_ERT):
            got = r.render(vr.default_params(W, H, S, mode=vr.VR_MODE_TEST, flags=flags), cam)
            assert np.abs(got - reft).max() <= TOL, flags


@pytest.mark.parametrize("camera", ["default", "oblique"])
@pytest.mark.parametrize("W,H,S", [(1, 1, 1), (1, 130, 2), (257, 3, 1), (3, 2, 700), (17, 250, 9)])
def test_degenerate_frame_shapes(r152, avg152, avg152_octree, oracle_mod, W, H, S, camera):
    """Single-pixel, single-sample, one-column/one-row and ragged frames (partial 8x8 waves and
    16x16 workgroups, a march shorter than one K-batch, a march of many batches on a tiny frame):
    VRC exact and ESS bitwise, ERT within TOL, TEST within TOL, all against the oracle."""
    vol, cal = avg152
    cam = cam_of(W, H, camera)
    ref = oracle_vrc(oracle_mod, avg152_octree, cal, W, H, S, camera)
    exact = r152.render(vr.default_params(W, H, S), cam)
    assert exact.shape == ref.shape
    assert_bitwise(exact, ref)
    assert np.array_equal(r152.render(vr.default_params(W, H, S, flags=vr.VR_FLAG_ESS), cam), exact)
    got = r152.render(vr.default_params(W, H, S, flags=vr.VR_FLAG_ESS | vr.VR_FLAG_ERT), cam)
    assert np.abs(got - ref).max() <= TOL
    reft = oracle_test(oracle_mod, vol, cal, W, H, S, camera)
    for flags in (0, vr.VR_FLAG_ESS | vr.VR_FLAG_ERT):
        got = r152.render(vr.default_params(W, H, S, mode=vr.VR_MODE_TEST, flags=flags), cam)
        assert np.abs(got - reft).max() <= TOL, flags


@pytest.mark.parametrize("W,H,S,mode,flags", [
    (0, 10, 10, vr.VR_MODE_VRC, 0), (10, 0, 10, vr.VR_MODE_VRC, 0), (10, 10, 0, vr.VR_MODE_VRC, 0),
    (-4, 10, 10, vr.VR_MODE_VRC, 0), (65536, 1, 1, vr.VR_MODE_VRC, 0), (10, 10, 10, 3, 0),
    (10, 10, 10, vr.VR_MODE_TEST, vr.VR_FLAG_SHADE), (10, 10, 10, vr.VR_MODE_VRC, 1 << 12)])
def test_bad_render_arguments_raise_einval(r152, W, H, S, mode, flags):
    """Bad sizes / modes / flags are refused with VR_EINVAL before any launch (the reference
    would index out of bounds or silently render nothing), and the context stays usable."""
    p = vr.default_params(max(W, 1), max(H, 1), max(S, 1), mode=mode, flags=flags)
    p.width, p.height, p.samples_per_ray = W, H, S
    out = np.zeros(65536 * 10 * 4, np.float32)      # host buffer larger than any frame above
    cam = vr.default_camera(10, 10)
    rc = vr.lib().vr_render(r152._ctx, ctypes.byref(p), ctypes.byref(cam), out.ctypes.data_as(ctypes.c_void_p), 0)
    assert rc == VR_EINVAL
    assert not out.any()                              # refused before anything was written
    ok = r152.render(vr.default_params(8, 8, 8), vr.default_camera(8, 8))
    assert ok.shape[:2] in ((8, 8),) and np.all(ok[..., 3] == 1.0)


def _tf_n(n, seed=3):
    """n intervals over [0, 1]: interval 0 transparent (TF(0)), the rest coloured, some transparent."""
    rng = np.random.default_rng(seed)
    edges = np.linspace(0.0, 1.0, n + 1)
    tf = [(0.0, float(edges[1]) * 0.5, (0.0, 0.0, 0.0, 0.0))]
    for i in range(1, n):
        a = 0.0 if i % 5 == 0 else float(rng.uniform(0.05, 0.8))
        tf.append((float(edges[i]), float(edges[i + 1]), tuple(float(x) for x in rng.uniform(0, 1, 3)) + (a,)))
    return tf


@pytest.mark.parametrize("n_tf", [4, 10, 20])
def test_class_bits_are_exact(avg152, oracle_mod, n_tf):
    """Compact class volumes (vr_options.class_bits: 2 / 4 / 8 bits per class, bit-addressed in 128-B
    bricks) hold exactly the classes of the 8-bit volume: every width the TF allows renders the same
    frames bit for bit -- axis-aligned views on the compact volume, oblique and orbit views on its
    byte copy (or, with 64-bit offsets, on the compact volume too), exact / ESS / ERT / shading --
    and the exact frames equal the oracle's."""
    vol, cal = avg152
    O = oracle_mod
    tf = _tf_n(n_tf)
    widths = [w for w in (2, 4, 8) if (1 << w) >= n_tf] + [0]
    rs = {w: vr.VolumeRenderer(vol, cal, tf=tf, device=0, options=vr.default_options(class_bits=w)) for w in widths}
    # compact classes with 64-bit offsets (general views then gather bits too: no byte copy)
    rs["x64"] = vr.VolumeRenderer(vol, cal, tf=tf, device=0, options=vr.default_options(class_bits=0, force_idx64=1))
    W, H, S = 120, 90, 150
    up = tuple(vr.default_camera(W, H).up)
    cams = {"default": vr.default_camera(W, H), "oblique": vr.reset_camera(),
            "orbit": vr.derive_camera((0.6, 0.3, 0.74), up, 2.0, 2.0 * H / W)}
    ref = {}
    for name, cam in cams.items():
        for flags in (0, vr.VR_FLAG_ESS, vr.VR_FLAG_ERT | vr.VR_FLAG_ESS, vr.VR_FLAG_SHADE):
            p = vr.default_params(W, H, S, flags=flags)
            frames = {w: r.render(p, cam) for w, r in rs.items()}
            for w in list(widths[1:]) + ["x64"]:
                assert_bitwise(frames[w], frames[widths[0]])
            if flags == 0:
                ref[name] = frames[widths[0]]
    octree = O.OracleOctree(vol)
    ocams = {"default": O.camera_default(W, H), "oblique": O.camera_oblique(W, H),
             "orbit": O.camera_derive((0.6, 0.3, 0.74), up, 2.0, 2.0 * H / W)}
    for name in cams:
        assert_bitwise(ref[name], octree.render_vrc(cal, O.tf_array(tf), O.params(W, H, S), ocams[name]))
    for r in rs.values():
        r.close()


def test_class_bits_follow_tf_updates(avg152, avg152_octree, oracle_mod):
    """A context with 2-bit classes (the default TF) given a TF of 10 and then 20 classes re-lays its
    class volume (4, then 8 bits) and back; every frame equals the oracle's bitwise."""
    vol, cal = avg152
    O = oracle_mod
    W, H, S = 100, 80, 120
    with vr.VolumeRenderer(vol, cal, device=0) as r:
        for tf in (_tf_n(10), _tf_n(20, seed=5), vr.default_transfer_function(), _tf_n(16, seed=9)):
            r.set_transfer_function(tf)
            for cam, ocam in ((vr.default_camera(W, H), O.camera_default(W, H)), (vr.reset_camera(), O.camera_oblique(W, H))):
                got = r.render(vr.default_params(W, H, S), cam)
                assert_bitwise(got, avg152_octree.render_vrc(cal, O.tf_array(tf), O.params(W, H, S), ocam))
                fast = r.render(vr.default_params(W, H, S, flags=vr.VR_FLAG_ESS | vr.VR_FLAG_ERT), cam)
                assert np.abs(fast - got).max() <= TOL


@pytest.mark.parametrize("camera", ["default", "oblique"])
def test_count_marched_is_the_work_done(avg152, camera):
    """vr_count_marched (the bench's roofline numerator) counts the class gathers the march issues:
    with nothing skipped (exact mode, exact_skip = 0, and cull = 0: the occupancy cull of axis views
    drops whole tiles of empty columns) that is every in-dataset sample -- N_in of vr_count_samples
     -- and empty-space skipping / early termination only remove gathers.  The counting pass renders the same frame as vr_render."""
    vol, cal = avg152
    W, H, S = 160, 120, 200
    cam = cam_of(W, H, camera)
    plain = vr.VolumeRenderer(vol, cal, device=0, options=vr.default_options(exact_skip=0, cull=0))
    r = vr.VolumeRenderer(vol, cal, device=0)
    p0 = vr.default_params(W, H, S)
    n_in = plain.count_samples(p0, cam)
    g0, e0 = plain.count_marched(p0, cam)
    assert g0 == n_in and e0 >= n_in
    prev = g0
    for flags in (0, vr.VR_FLAG_ESS, vr.VR_FLAG_ESS | vr.VR_FLAG_ERT):
        g, e = r.count_marched(vr.default_params(W, H, S, flags=flags), cam)
        assert 0 < g <= n_in and g <= e
        if flags & vr.VR_FLAG_ERT:
            assert g < prev            # termination removes gathers on this volume
        prev = g
    plain.close()
    r.close()


@pytest.mark.parametrize("n_tf", [4, 10, 20])
def test_run_words_are_exact(avg152, oracle_mod, n_tf):
    """Run-word gathers (vr_options.run_words = 2: a batch's classes from the two aligned 8-byte words
    of its first and last samples, per-sample loads when a lane's batch spans more) and the split
    {byte, bit} view table (table_split = 1) render the frames of per-sample gathers of summed bit
    offsets (run_words = 1, table_split = 0) bit for bit: views along +z and -z, 2 / 4 / 8-bit classes,
    32- and 64-bit offsets, exact / ESS / ESS+ERT / ERT, coarse (batches past two runs), normal and
    dense sampling; the exact frames equal the oracle's."""
    vol, cal = avg152
    O = oracle_mod
    tf = _tf_n(n_tf)
    W, H = 112, 96
    cam = vr.default_camera(W, H)
    back = vr.derive_camera(tuple(-x for x in cam.pos), tuple(cam.up), 2.0, 2.0 * H / W)
    for idx64 in (0, 1):
        mk = lambda rw, ts: vr.VolumeRenderer(vol, cal, tf=tf, device=0,
                                              options=vr.default_options(run_words=rw, table_split=ts,
                                                                         force_idx64=idx64))
        # reference: per-sample gathers of summed bit offsets; then the split {byte, bit} view table
        # (the default along z) and run words
        with mk(1, 0) as r1, mk(1, 1) as r3, mk(2, 1) as r2:
            for S in (40, 150, 600):
                for c in (cam, back):
                    for flags in (0, vr.VR_FLAG_ESS, vr.VR_FLAG_ESS | vr.VR_FLAG_ERT, vr.VR_FLAG_ERT):
                        p = vr.default_params(W, H, S, flags=flags)
                        a = r1.render(p, c)
                        assert_bitwise(r2.render(p, c), a)
                        assert_bitwise(r3.render(p, c), a)
                        if flags == 0 and S == 150 and c is cam:
                            octree = O.OracleOctree(vol)
                            assert_bitwise(a, octree.render_vrc(cal, O.tf_array(tf), O.params(W, H, S),
                                                                O.camera_default(W, H)))


@pytest.mark.parametrize("brick,class_bits", [((4, 4, 16), 8), ((4, 4, 6), 2), ((4, 4, 5), 4), ((2, 4, 3), 8),
                                              ((4, 4, 32), 4)])
def test_run_words_odd_bricks_are_exact(avg152, brick, class_bits):
    """Run words with bricks whose z-run does not tile an aligned 8-byte word (bz * cbits not a
    divisor of 64: a run straddles two words, or spans several): the batches that span two bricks
    must keep the per-sample miss test (the zspan2 shortcut assumed one word per run).
    64-bit offsets (the run-word default), views along +z and -z, dense and coarse sampling: bitwise
    the frames of per-sample gathers (run_words = 1)."""
    vol, cal = avg152
    W, H = 96, 80
    cam = vr.default_camera(W, H)
    back = vr.derive_camera(tuple(-x for x in cam.pos), tuple(cam.up), 2.0, 2.0 * H / W)
    mk = lambda rw: vr.VolumeRenderer(vol, cal, device=0, options=vr.default_options(
        run_words=rw, force_idx64=1, brick=list(brick), class_bits=class_bits))
    with mk(1) as r1, mk(2) as r2:
        for S in (60, 220, 700):
            for c in (cam, back):
                for flags in (0, vr.VR_FLAG_ESS | vr.VR_FLAG_ERT):
                    p = vr.default_params(W, H, S, flags=flags)
                    assert_bitwise(r2.render(p, c), r1.render(p, c))


@pytest.mark.parametrize("field,value", [("run_words", 3), ("run_words", -1), ("table_split", 2),
                                         ("frames_in_flight", 4), ("frames_in_flight", -1), ("batch", 5),
                                         ("work_order", 3)])
def test_bad_render_options_raise_einval(r152, field, value):
    """Out-of-range render options are refused by vr_set_options with VR_EINVAL and leave the
    context's options and frames unchanged."""
    p, cam = vr.default_params(64, 48, 60), vr.default_camera(64, 48)
    before = r152.render(p, cam)
    with pytest.raises(vr.VRError) as e:
        r152.set_options(vr.default_options(**{field: value}))
    assert e.value.code == VR_EINVAL
    assert_bitwise(r152.render(p, cam), before)


@pytest.mark.parametrize("volume", ["avg152", "sparse"])
def test_leaf_columns_are_exact(avg152, volume):
    """Axis-aligned ESS marches with the empty-cell mask of the ray's own leaf column
    (vr_options.leaf_columns = 1, default) against the 4 x 4-leaf cell-column mask (0): back to front
    (ESS alone) bitwise the same frames and the exact frame; front to back (ESS + ERT) within the ERT
    tolerance of the exact frame (the jumps land elsewhere, so ERT is checked at other batch ends).
    Views along x, y and z in both directions, a zoomed view, tile output, and a sparse random volume
    (many leaf columns empty inside occupied cells)."""
    import torch
    if volume == "avg152":
        vol, cal = avg152
    else:
        rng = np.random.default_rng(3)
        vol = rng.integers(0, 256, size=(70, 53, 61)).astype(np.float32)
        vol[vol < 235] = 0
        cal = 255.0
    a = vr.VolumeRenderer(vol, cal, device=0)
    b = vr.VolumeRenderer(vol, cal, device=0, options=vr.default_options(leaf_columns=0))
    try:
        W, H, S = 120, 96, 180
        up = tuple(vr.default_camera(W, H).up)
        rsw, rsh = 2.0, 2.0 * H / W
        cams = [vr.default_camera(W, H),
                vr.derive_camera((0.0, 0.0, -1.0), up, rsw, rsh),
                vr.derive_camera((0.0, 0.0, 0.45), up, rsw, rsh),
                vr.derive_camera((1.0, 0.0, 0.0), (0.0, 1.0, 0.0), rsw, rsh),
                vr.derive_camera((-1.0, 0.0, 0.0), (0.0, 1.0, 0.0), rsw, rsh),
                vr.derive_camera((0.0, 1.0, 0.0), (0.0, 0.0, 1.0), rsw, rsh),
                vr.derive_camera((0.0, -1.0, 0.0), (0.0, 0.0, 1.0), rsw, rsh)]
        E, T = vr.VR_FLAG_ESS, vr.VR_FLAG_ERT
        for i, cam in enumerate(cams):
            exact = a.render(vr.default_params(W, H, S), cam)
            pe = vr.default_params(W, H, S, flags=E)
            fa = a.render(pe, cam)
            assert np.array_equal(fa, b.render(pe, cam)), i
            assert np.array_equal(fa, exact), i
            pf = vr.default_params(W, H, S, flags=E | T)
            assert np.abs(a.render(pf, cam) - exact).max() <= 1e-4, i
            assert np.abs(b.render(pf, cam) - exact).max() <= 1e-4, i
        # tile output of the default view, ESS alone: the same tiles as the cell-column context
        p = vr.default_params(W, H, S, flags=E)
        ta = torch.zeros((4, 32 * 32, 4), dtype=torch.float32, device="cuda:0")
        tb = torch.zeros_like(ta)
        a.render_tiles(p, cams[0], 32, 32, 1, 3, ta.data_ptr())
        b.render_tiles(p, cams[0], 32, 32, 1, 3, tb.data_ptr())
        assert torch.equal(ta, tb)
    finally:
        a.close()
        b.close()
