"""A/B timing sweep of the march kernel: variants (vr_options fields given at vr_create_ex) x configs,
timed in ONE process with interleaved rounds; HIP-event kernel time on the ctx stream.

usage: python tools/sweep.py [--rounds 5] [--volume mni] [--variants "brick=1x1x1;brick=4x4x8,batch=8"]
       [--configs c3,c3ess,...]
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

ALL = {
    "c3": ("C3 ess+ert", 1920, 1080, 500, "ess,ert", "vrc", "default"),
    "c3sh": ("C3 ess+ert+shade", 1920, 1080, 500, "ess,ert,shade", "vrc", "default"),
    "c3shobl": ("C3 ess+ert+shade oblique", 1920, 1080, 500, "ess,ert,shade", "vrc", "oblique"),
    "c3ess": ("C3 ess", 1920, 1080, 500, "ess", "vrc", "default"),
    "c3ert": ("C3 ert", 1920, 1080, 500, "ert", "vrc", "default"),
    "c3exact": ("C3 exact", 1920, 1080, 500, "", "vrc", "default"),
    "c3obl": ("C3 ess+ert oblique", 1920, 1080, 500, "ess,ert", "vrc", "oblique"),
    "c3oblx": ("C3 exact oblique", 1920, 1080, 500, "", "vrc", "oblique"),
    "c3obls": ("C3 ess oblique", 1920, 1080, 500, "ess", "vrc", "oblique"),
    "c2x": ("C2 exact", 700, 700, 500, "", "vrc", "default"),
    "c4": ("C4-size ess+ert S=1024", 1920, 1080, 1024, "ess,ert", "vrc", "default"),
    "c4x": ("C4-size exact S=1024", 1920, 1080, 1024, "", "vrc", "default"),
    "c3s250": ("C3 ess+ert S=250", 1920, 1080, 250, "ess,ert", "vrc", "default"),
    "c2": ("C2 exact", 700, 700, 500, "", "vrc", "default"),
    "c3s1": ("C3 S=1 overhead", 1920, 1080, 1, "ess,ert", "vrc", "default"),
    "s1q": ("960x540 S=1", 960, 540, 1, "ess,ert", "vrc", "default"),
    "s1x4": ("3840x2160 S=1", 3840, 2160, 1, "ess,ert", "vrc", "default"),
    "s1x": ("1920x1080 S=1 exact", 1920, 1080, 1, "", "vrc", "default"),
    "c3s8": ("C3 S=8 overhead", 1920, 1080, 8, "ess,ert", "vrc", "default"),
    "c2f": ("C2 ess+ert", 700, 700, 500, "ess,ert", "vrc", "default"),
    "t3": ("C3 TEST ert", 1920, 1080, 500, "ert", "test", "default"),
    "t3e": ("C3 TEST ess+ert", 1920, 1080, 500, "ess,ert", "test", "default"),
    "t3eo": ("C3 TEST ess+ert oblique", 1920, 1080, 500, "ess,ert", "test", "oblique"),
    "t3x": ("C3 TEST exact", 1920, 1080, 500, "", "test", "default"),
    "t3ro": ("C3 TEST ert oblique", 1920, 1080, 500, "ert", "test", "oblique"),
    "t3s": ("C3 TEST ess", 1920, 1080, 500, "ess", "test", "default"),
    "t3xo": ("C3 TEST exact oblique", 1920, 1080, 500, "", "test", "oblique"),
    "t3so": ("C3 TEST ess oblique", 1920, 1080, 500, "ess", "test", "oblique"),
    "c3con": ("C3 ess+ert conic", 1920, 1080, 500, "ess,ert,conic", "vrc", "conic"),
    "c3conx": ("C3 exact conic", 1920, 1080, 500, "conic", "vrc", "conic"),
}


def conic_params_camera(vr, W, H, p):
    """Perspective camera at (0, 0, 1) with the conic screen of utils.h:57 (rsw = 2 tan(pi/4) vpd)."""
    import math
    import numpy as np
    vpd = 2.0
    rsw = float(np.float32(np.float32(2 * math.tan(np.float32(math.pi / 4))) * np.float32(vpd)))
    rsh = float(np.float32(np.float32(rsw) * np.float32(H) / np.float32(W)))
    p.real_screen_width, p.real_screen_height = rsw, rsh
    return vr.derive_camera_conic((0.0, 0.0, 1.0), tuple(vr.default_camera(W, H).up), rsw, rsh, vpd)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--volume", default="mni")
    ap.add_argument("--variants", default="")
    ap.add_argument("--configs", default="c3,c3ess,c3ert,c3exact,c3obl,c2,c2f,t3")
    a = ap.parse_args()
    import torch
    import volumerenderingproject_amd as vr
    from volumerenderingproject_amd import volumes
    if a.volume == "mni":
        vol, cal = volumes.mni152_standin()
    elif a.volume == "avg152":
        vol, h = volumes.avg152()
        cal = h["cal_max"]
    elif a.volume == "tiny":   # every 10th voxel of the MNI stand-in (19 x 22 x 19): a class volume that fits LDS
        import numpy as np
        v0, cal = volumes.mni152_standin()
        vol = np.ascontiguousarray(v0[::10, ::10, ::10])
    else:
        vol, cal = volumes.resample_512(volumes.mni152_standin()[0]), 255.0
    variants = [v for v in a.variants.split(";")] if a.variants else [""]
    rend = []
    for v in variants:
        fields = {}
        for kv in filter(None, v.split(",")):
            k, val = kv.split("=")
            fields[k] = [int(x) for x in val.split("x")] if k == "brick" else int(val)
        rend.append(vr.VolumeRenderer(vol, cal, options=vr.default_options(**fields)))
    cfgs = [ALL[c] for c in a.configs.split(",")]
    outs = {c[0]: torch.empty((c[1], c[2], 4), dtype=torch.float32, device="cuda:0") for c in cfgs}
    res = {}
    ref = {}
    for r in rend:
        r.timing_enable(True)
    for rnd in range(a.rounds):
        for vi, r in enumerate(rend):
            for name, W, H, S, fl, mode, camn in cfgs:
                flags = ((vr.VR_FLAG_ESS if "ess" in fl else 0) | (vr.VR_FLAG_ERT if "ert" in fl else 0)
                         | (vr.VR_FLAG_SHADE if "shade" in fl else 0) | (vr.VR_FLAG_CONIC if "conic" in fl else 0))
                p = vr.default_params(W, H, S, mode=vr.VR_MODE_VRC if mode == "vrc" else vr.VR_MODE_TEST, flags=flags)
                if camn == "conic":
                    cam = conic_params_camera(vr, W, H, p)
                else:
                    cam = vr.default_camera(W, H) if camn == "default" else vr.reset_camera()
                for _ in range(2):
                    r.render_device(p, cam, outs[name].data_ptr(), asynchronous=True)
                r.timing_read(reset=True)
                for _ in range(a.iters):
                    r.render_device(p, cam, outs[name].data_ptr(), asynchronous=True)
                t = r.timing_read(reset=True)
                res.setdefault((vi, name), []).append(t.total_ms / t.launches)
                if rnd == 0:   # every variant must produce the same frame
                    img = outs[name].cpu()
                    if vi == 0:   # (across libraries: compare these digests between runs)
                        import hashlib
                        print(f"frame digest {name}: {hashlib.sha1(img.numpy().tobytes()).hexdigest()[:16]}", flush=True)
                    if name in ref:
                        d = float((img - ref[name]).abs().max())
                        if d > 0:
                            print(f"~~ variant {variants[vi]!r} not bitwise on {name}: max |d| {d}", flush=True)
                        if d > 1e-4:
                            print(f"!! variant {variants[vi]!r} differs on {name}: {d}", flush=True)
                    else:
                        ref[name] = img
    out = {}
    for vi, v in enumerate(variants):
        for name, W, H, S, fl, mode, camn in cfgs:
            ms = res[(vi, name)]
            med = statistics.median(ms)
            out[f"{v}|{name}"] = {"ms_median": round(med, 4), "ms_min": round(min(ms), 4),
                                  "mrays": round(W * H / med / 1e3, 1)}
            print(f"{v:34s} {name:22s} median {med:8.4f} ms  min {min(ms):8.4f}  {W * H / med / 1e3:9.1f} Mrays/s",
                  flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
