"""Pinning the oracle (the CPU restatement in oracle/) to the reference itself, on CPU.

What of the reference can be checked here ("Oracle and parity pinning"):
  1. glm arithmetic: oracle/_ref/glm_probe is compiled against the reference's own vendored glm
     (/root/reference/glm, compiled as-is) and evaluates the hot path's camera / sample-position /
     TEST-matrix expressions; tests/golden/glm_vectors.json is its output.  The oracle and libvr's
     host math must reproduce every value bit for bit (tests/test_host.py), and the fixture must be
     what the probe prints (this file, when the reference is mounted).
  2. rendered frames: the reference ships screenshots (image_output/*.png, 8-bit, GL-rasterised,
     undocumented code revisions and cameras, made from MNI152_T1_1mm, which the reference does not
     ship).  Values: every foreground colour of every a1 / a5 / a0 screenshot lies within 2/255 of
     the convex hull of the background and the reference TF's colours -- the only colours
     compositing can form from them -- while the TF variant commented out in the reference cannot
     produce them.  Silhouettes: the 300x300 VRC and TEST ones match the oracle's at the default
     camera.  The per-screenshot characterisation (tools/screenshot_pin.py ->
     tests/golden/screenshot_pin.json) records what does not match and why.
  3. regression: the committed golden frames are the oracle's own output (tools/make_golden.py).
The reference's Octree/TransferFunction/BinaryLoader classes cannot be compiled here (they include
CUDA and GL headers this image lacks); their semantics are restated and cross-checked instead
(leaf grid == restated recursive octree on every leaf, tests/test_host.py).
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import GOLDEN, ROOT

PROBE = os.path.join(ROOT, "oracle", "_ref", "glm_probe")


@pytest.mark.skipif(not os.path.exists(PROBE), reason="oracle/_ref not built (reference not mounted)")
def test_glm_fixture_is_reference_glm_output():
    out = subprocess.run([PROBE], capture_output=True, text=True, check=True).stdout
    assert json.loads(out) == json.load(open(os.path.join(GOLDEN, "glm_vectors.json")))


def test_oracle_reproduces_golden_frames(avg152, avg152_octree, oracle_mod):
    O = oracle_mod
    vol, cal = avg152
    g = np.load(os.path.join(GOLDEN, "frames_avg152.npz"))
    tf = O.default_tf()
    for (W, H, S) in [(100, 100, 100), (64, 48, 64)]:
        for camn in ["default", "oblique"]:
            cam = O.camera_default(W, H) if camn == "default" else O.camera_oblique(W, H)
            p = O.params(W, H, S)
            assert np.array_equal(avg152_octree.render_vrc(cal, tf, p, cam), g[f"vrc_{W}x{H}x{S}_{camn}"])
            assert np.array_equal(O.render_test(vol, cal, tf, p, cam), g[f"test_{W}x{H}x{S}_{camn}"])
            assert avg152_octree.count_in_samples(p, cam) == int(g[f"nin_{W}x{H}x{S}_{camn}"])
    # the survey's exact replay of the C1 geometry: 88,200 in-dataset samples
    assert int(g["nin_100x100x100_default"]) == 88200
    p = O.params(100, 100, 100)
    cam = O.camera_default(100, 100)
    for (x, y), ref in zip(g["ray_pixels"], g["ray_samples"]):
        assert np.array_equal(avg152_octree.ray_samples(cal, tf, p, cam, int(x), int(y)), ref)


def display_like_reference(frame, rotate180):
    """myApp.cu:1661-1688 + GL: pixel (x, y) drawn at NDC (2x/W-1, 2y/H-1), VRC rotated 180 deg
    about z (myApp.cu:933), read back bottom-up and flipped by stbi (myApp.cu:1954)."""
    W, H = frame.shape[:2]
    img = np.zeros((H, W, 3))
    xs, ys = np.meshgrid(np.arange(W), np.arange(H), indexing="ij")
    nx, ny = (W - 1 - xs, H - 1 - ys) if rotate180 else (xs, ys)
    img[H - 1 - ny, nx] = frame[xs, ys, :3]
    return np.clip(np.round(img * 255), 0, 255).astype(np.uint8)


def silhouette_iou(a, b):
    ma = np.abs(a.astype(int) - a[0, 0].astype(int)).max(2) > 3
    mb = np.abs(b.astype(int) - b[0, 0].astype(int)).max(2) > 3
    return (ma & mb).sum() / max(1, (ma | mb).sum())


def test_vrc_matches_reference_screenshot_silhouette(avg152, avg152_octree, oracle_mod):
    """image_300x300_a1_spr300.png (VRC, 300x300, 300 samples/ray, default camera)."""
    from PIL import Image
    O = oracle_mod
    vol, cal = avg152
    fr = avg152_octree.render_vrc(cal, O.default_tf(), O.params(300, 300, 300), O.camera_default(300, 300))
    ref = np.asarray(Image.open(os.path.join(GOLDEN, "ref_screens", "image_300x300_a1_spr300.png")).convert("RGB"))
    ours = display_like_reference(fr, rotate180=True)
    assert tuple(ref[0, 0]) == (51, 51, 51) == tuple(ours[0, 0])      # background (.2,.2,.2) -> 51
    assert silhouette_iou(ours, ref) >= 0.90
    assert silhouette_iou(ours[:, ::-1], ref) < 0.80                  # orientation is pinned too


def test_test_mode_screenshot_silhouette(avg152, oracle_mod):
    """image_300x300_a5_spr300.png (TEST).  It matches our TEST frame mirrored left-right: the
    screenshot predates the shipped TEST display path (its revision is undocumented), so only the
    silhouette is pinned, and the mirror is recorded rather than hidden."""
    from PIL import Image
    O = oracle_mod
    vol, cal = avg152
    fr = O.render_test(vol, cal, O.default_tf(), O.params(300, 300, 300), O.camera_default(300, 300))
    ref = np.asarray(Image.open(os.path.join(GOLDEN, "ref_screens", "image_300x300_a5_spr300.png")).convert("RGB"))
    ours = display_like_reference(fr, rotate180=False)
    assert silhouette_iou(ours[:, ::-1], ref) >= 0.90


def _pin():
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import screenshot_pin
    return screenshot_pin


SCREENS = sorted(os.listdir(os.path.join(GOLDEN, "ref_screens")))


@pytest.mark.parametrize("name", SCREENS)
def test_screenshot_colours_are_the_reference_tf_palette(name):
    """Value-level pin of the TF colours (TransferFunction.cu:19-23, Material.cpp:28-42): 100 % of the
    screenshot's foreground within 2/255 of the hull of {background, empty, bone, muscle, brain};
    the commented-out variant (TransferFunction.cu:12-15: glass instead of brain) misses most of
    the screenshots made at the default camera."""
    from PIL import Image
    SP = _pin()
    ref = np.asarray(Image.open(os.path.join(GOLDEN, "ref_screens", name)).convert("RGB"))
    fixture = json.load(open(os.path.join(GOLDEN, "screenshot_pin.json")))[name]
    got = round(SP.palette_fraction(ref, SP.PALETTE_REF), 4)
    assert got == fixture["palette_ref_tf"] == 1.0
    alt = round(SP.palette_fraction(ref, SP.PALETTE_ALT), 4)
    assert alt == fixture["palette_alt_tf"]
    # default-camera ray-cast screenshots (the two zoomed ones are mostly black); POINT mode (a0 and
    # myOutputIsAwesome) blends many points per pixel, whose mixtures of bone and muscle the
    # alternative hull also covers, so only the reference TF's 100 % discriminates there
    if SP.fg_mask(ref).mean() < 0.5 and ("_a1_" in name or "_a5_" in name):
        assert alt < 0.7


def test_screenshot_silhouettes_match_fixture(avg152, avg152_octree, oracle_mod):
    """The 300x300 VRC / TEST silhouettes recomputed equal the recorded characterisation; VRC
    matches unmirrored, TEST matches mirrored -- equivalently the camera at (0, 0, -1): orthographic
    views from opposite sides have mirror-image silhouettes (measured IoU 0.938 both ways)."""
    from PIL import Image
    SP = _pin()
    vol, cal = avg152
    fixture = json.load(open(os.path.join(GOLDEN, "screenshot_pin.json")))
    for name in ("image_300x300_a1_spr300.png", "image_300x300_a5_spr300.png"):
        fr, alg = SP.oracle_frame(name, vol, cal, avg152_octree, oracle_mod)
        ref = np.asarray(Image.open(os.path.join(GOLDEN, "ref_screens", name)).convert("RGB"))
        sil = SP.silhouette(SP.display_like_reference(fr, rotate180=alg == 1), ref)
        assert sil == fixture[name]["oracle_default_camera"]
        assert round(SP.frame_palette_fraction(fr, SP.PALETTE_REF), 4) == 1.0
    assert fixture["image_300x300_a1_spr300.png"]["oracle_default_camera"]["plain"]["iou"] >= 0.93
    assert fixture["image_300x300_a5_spr300.png"]["oracle_default_camera"]["mirrored"]["iou"] >= 0.93


def test_contraction_model_sensitivity(avg152, avg152_octree, oracle_mod):
    """One FP model, contraction off.  Under the other model -- every a*b + c of
    the position arithmetic fused, as nvcc's default -fmad=true may compile the reference -- no C1
    sample changes leaf (VRC) or voxels (TEST) at the default camera (its products are exact), and
    3 of 87,339 VRC samples change at the oblique camera; 300^3: 15 VRC, 6 TEST of 2.35 M."""
    O = oracle_mod
    vol, cal = avg152
    for (W, H, S), cam, vrc, test in [((100, 100, 100), "default", (0, 88200), (0, 84050)),
                                      ((100, 100, 100), "oblique", (3, 87339), (0, 87123)),
                                      ((300, 300, 300), "oblique", (15, 2358423), (6, 2352365))]:
        p = O.params(W, H, S)
        c = O.camera_default(W, H) if cam == "default" else O.camera_oblique(W, H)
        assert O.vrc_contraction_flips(avg152_octree, p, c) == vrc
        assert O.test_contraction_flips(vol.shape, p, c) == test
