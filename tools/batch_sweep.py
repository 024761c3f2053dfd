"""Throughput of vr_render_batch (frames in flight) for vr_options variants, in one process,
interleaved rounds: C3 default / oblique / orbit views, ESS + ERT and exact.

usage: python tools/batch_sweep.py [--variants "batch=8;batch=16"] [--frames 64] [--rounds 3]
"""
import argparse
import math
import os
import statistics
import sys
import time

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="batch=8;batch=16")
    ap.add_argument("--frames", type=int, default=64)
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    import torch
    import volumerenderingproject_amd as vr
    from volumerenderingproject_amd import volumes
    vol, cal = volumes.mni152_standin()
    W, H, S = 1920, 1080, 500
    variants = a.variants.split(";")
    rend = []
    for v in variants:
        fields = {k: int(x) for k, x in (kv.split("=") for kv in filter(None, v.split(",")))}
        rend.append(vr.VolumeRenderer(vol, cal, options=vr.default_options(**fields)))
    up = tuple(vr.default_camera(W, H).up)
    p0 = vr.default_params(W, H, S)
    n = a.frames
    views = {"default": [vr.default_camera(W, H)] * n, "oblique": [vr.reset_camera()] * n,
             "orbit": [vr.derive_camera((math.sin(2 * math.pi * i / n), 0.0, math.cos(2 * math.pi * i / n)), up,
                                        p0.real_screen_width, p0.real_screen_height) for i in range(n)]}
    out = torch.empty((a.batch, W, H, 4), dtype=torch.float32, device="cuda")
    res = {}
    for _ in range(a.rounds):
        for vi, r in enumerate(rend):
            for fl in (3, 0):
                p = vr.default_params(W, H, S, flags=fl)
                for name, cams in views.items():
                    arr = (vr.Camera * n)(*cams)
                    r.render_batch_device(p, arr[:a.batch], out.data_ptr(), asynchronous=True)
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    for i in range(0, n, a.batch):
                        r.render_batch_device(p, arr[i:i + a.batch], out.data_ptr(), asynchronous=True)
                    torch.cuda.synchronize()
                    res.setdefault((vi, fl, name), []).append(W * H * n / (time.perf_counter() - t0) / 1e6)
    for (vi, fl, name), v in sorted(res.items()):
        print(f"{variants[vi]:24s} flags {fl} {name:8s} {statistics.median(v):10.1f} Mrays/s")


if __name__ == "__main__":
    main()
