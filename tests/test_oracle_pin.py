"""Pinning the oracle (the CPU restatement in oracle/) to the reference itself, on CPU.

What of the reference can be checked here ("Oracle and parity pinning"):
  1. glm arithmetic: oracle/_ref/glm_probe is compiled against the reference's own vendored glm
     (/root/reference/glm, compiled as-is) and evaluates the hot path's camera / sample-position /
     TEST-matrix expressions; tests/golden/glm_vectors.json is its output.  The oracle and libvr's
     host math must reproduce every value bit for bit (tests/test_host.py), and the fixture must be
     what the probe prints (this file, when the reference is mounted).
  2. rendered frames: the reference ships screenshots (image_output/*.png, 8-bit, GL-rasterised,
     undocumented code revision).  The 300x300 ones match the oracle's silhouette.
  3. regression: the committed golden frames are the oracle's own output (tools/make_golden.py).
The reference's Octree/TransferFunction/BinaryLoader classes cannot be compiled here (they include
CUDA and GL headers this image lacks); their semantics are restated and cross-checked instead
(leaf grid == restated recursive octree on every leaf, tests/test_host.py).
"""
import json
import os
import subprocess

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
