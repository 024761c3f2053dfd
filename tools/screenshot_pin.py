#!/usr/bin/env python3
"""Characterise the oracle against the reference's own screenshots (image_output/*.png, committed as
fixtures under tests/golden/ref_screens/) -> tests/golden/screenshot_pin.json.

Per screenshot (algorithm a1 = VRC, a5 = TEST, a0 = POINT; W x H, samples per ray from the name;
myOutputIsAwesome.png, a 700 x 700 POINT-mode capture, carries neither):
  * silhouette IoU of the oracle frame at the steady default camera, displayed as the reference's
    window shows it (VRC rotated 180 deg, myApp.cu:933; TEST unrotated, :1033; stbi flip :1954),
    plain and left-right mirrored, and the foreground fractions;
  * on the common foreground, the median per-channel 8-bit difference and the fraction within 2;
  * the palette pin: the fraction of foreground colours within 2 (8-bit, Euclidean) of the convex
    hull of {background, TF colours (the empty material's black included)}.  Compositing -- back-to-front blends, TEST's trilinear lerps,
    GL's point blending -- only forms convex combinations of the background and the classified
    colours, so every pixel the reference TF (TransferFunction.cu:19-23, Material.cpp:28-42) can
    produce lies in that hull, whatever the volume or camera.  The same fraction is given for the
    TF variant commented out at TransferFunction.cu:12-15 (empty / glass / muscle / bone: no brain
    colour), as the counter-hypothesis.

The screenshots were made with MNI152_T1_1mm (myApp.cu:240), which the reference does not ship
(.MISSING_LARGE_BLOBS:1), under undocumented code revisions and cameras; the oracle renders the
avg152 volume that ships.  So interiors are not expected to match value for value -- the palette
and the silhouettes are what the screenshots can pin.

usage: python tools/screenshot_pin.py [--out tests/golden/screenshot_pin.json]
"""
import argparse
import json
import os
import re
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
SCREENS = os.path.join(ROOT, "tests", "golden", "ref_screens")

BG = (51, 51, 51)
# the classified colours include the empty material (0, 0, 0), alpha 0 (Material.cpp:32-34): it
# enters TEST's colour lerps (classify-then-interpolate, kernel.cu:162-175) at reduced alpha
PALETTE_REF = [BG, (0, 0, 0), (241, 218, 202), (124, 9, 42), (223, 155, 141)]   # bg, empty, bone, muscle, brain
PALETTE_ALT = [BG, (0, 0, 0), (51, 51, 51), (124, 9, 42), (241, 218, 202)]      # bg, empty, glass, muscle, bone


def display_like_reference(frame, rotate180):
    """myApp.cu:1661-1688 + GL: pixel (x, y) drawn at NDC (2x/W-1, 2y/H-1), VRC rotated 180 deg
    about z (myApp.cu:933), read back bottom-up and flipped by stbi (myApp.cu:1954)."""
    W, H = frame.shape[:2]
    img = np.zeros((H, W, 3))
    xs, ys = np.meshgrid(np.arange(W), np.arange(H), indexing="ij")
    nx, ny = (W - 1 - xs, H - 1 - ys) if rotate180 else (xs, ys)
    img[H - 1 - ny, nx] = frame[xs, ys, :3]
    return np.clip(np.round(img * 255), 0, 255).astype(np.uint8)


def fg_mask(a):
    return np.abs(a.astype(int) - a[0, 0].astype(int)).max(2) > 3


def hull_distance(colours, palette):
    """Euclidean distance (8-bit units) of each colour to the convex hull of the palette: min over
    convex weights w >= 0, sum w = 1 of |P^T w - c| (NNLS with a heavily weighted sum row)."""
    from scipy.optimize import nnls
    P = np.asarray(palette, float)
    A = np.vstack([P.T, 1e4 * np.ones(len(P))])
    out = np.empty(len(colours))
    for i, c in enumerate(colours):
        w, _ = nnls(A, np.concatenate([np.asarray(c, float), [1e4]]))
        out[i] = np.linalg.norm(P.T @ w - c)
    return out


def palette_fraction(img, palette, tol=2.0):
    m = fg_mask(img)
    px = img[m].reshape(-1, 3)
    cols, counts = np.unique(px, axis=0, return_counts=True)
    d = hull_distance(cols, palette)
    return float(counts[d <= tol].sum() / max(1, counts.sum()))


def silhouette(ours, ref):
    res = {}
    for name, o in (("plain", ours), ("mirrored", ours[:, ::-1])):
        ma, mb = fg_mask(o), fg_mask(ref)
        both = ma & mb
        d = np.abs(o.astype(int)[both] - ref.astype(int)[both])
        res[name] = {"iou": round(float((ma & mb).sum() / max(1, (ma | mb).sum())), 4),
                     "median_diff": [int(v) for v in np.median(d, axis=0)],
                     "within_2": round(float((d.max(1) <= 2).mean()), 4)}
    res["fg_ours"] = round(float(fg_mask(ours).mean()), 4)
    res["fg_ref"] = round(float(fg_mask(ref).mean()), 4)
    return res


def oracle_frame(name, vol, cal, octree, O):
    m = re.match(r"image_(\d+)x(\d+)_a(\d)_spr(\d+)\.png", name)
    if m is None:   # (myOutputIsAwesome.png: a POINT-mode capture without size / mode in its name)
        return None, 0
    W, H, alg, S = int(m.group(1)), int(m.group(2)), int(m.group(3)), int(m.group(4))
    if alg not in (1, 5):
        return None, alg
    p, cam = O.params(W, H, S), O.camera_default(W, H)
    if alg == 1:
        return octree.render_vrc(cal, O.default_tf(), p, cam), alg
    return O.render_test(vol, cal, O.default_tf(), p, cam), alg


def frame_palette_fraction(fr, palette, tol=2.0):
    """palette_fraction of a float frame (0..1), before any 8-bit rounding."""
    m = np.abs(fr[..., :3] - fr[0, 0, :3]).max(-1) > 1e-6
    cols, counts = np.unique((fr[m][:, :3] * 255.0).round(3), axis=0, return_counts=True)
    d = hull_distance(cols, palette)
    return float(counts[d <= tol].sum() / max(1, counts.sum()))


def oracle_display(name, vol, cal, octree, O):
    m = re.match(r"image_(\d+)x(\d+)_a(\d)_spr(\d+)\.png", name)
    W, H, alg, S = int(m.group(1)), int(m.group(2)), int(m.group(3)), int(m.group(4))
    if alg not in (1, 5):
        return None
    p, cam = O.params(W, H, S), O.camera_default(W, H)
    if alg == 1:
        fr = octree.render_vrc(cal, O.default_tf(), p, cam)
    else:
        fr = O.render_test(vol, cal, O.default_tf(), p, cam)
    return display_like_reference(fr, rotate180=alg == 1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "tests", "golden", "screenshot_pin.json"))
    a = ap.parse_args()
    from PIL import Image
    import oracle as O
    from volumerenderingproject_amd import volumes
    vol, hdr = volumes.avg152()
    cal = hdr["cal_max"]
    octree = O.OracleOctree(vol)
    res = {}
    for name in sorted(os.listdir(SCREENS)):
        ref = np.asarray(Image.open(os.path.join(SCREENS, name)).convert("RGB"))
        e = {"palette_ref_tf": round(palette_fraction(ref, PALETTE_REF), 4),
             "palette_alt_tf": round(palette_fraction(ref, PALETTE_ALT), 4)}
        fr, alg = oracle_frame(name, vol, cal, octree, O)
        if fr is not None:
            ours = display_like_reference(fr, rotate180=alg == 1)
            if ours.shape == ref.shape:
                e["oracle_default_camera"] = silhouette(ours, ref)
                e["palette_ref_tf_oracle_frame"] = round(frame_palette_fraction(fr, PALETTE_REF), 4)
        res[name] = e
        print(name, json.dumps(e), flush=True)
    json.dump(res, open(a.out, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
