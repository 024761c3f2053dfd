"""Frames in flight: consecutive frames on one stream vs alternating over two or three HIP streams
(the tail of one frame's march overlapping the start of the next).  Prints Mrays/s per variant for
the default steady camera, the oblique camera and an orbit (a new view every frame).

usage: python tools/overlap_probe.py [--frames 64]
"""
import argparse
import math
import os
import sys
import time

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=64)
    a = ap.parse_args()
    import torch
    import volumerenderingproject_amd as vr
    from volumerenderingproject_amd import volumes
    vol, cal = volumes.mni152_standin()
    W, H, S = 1920, 1080, 500
    r = vr.VolumeRenderer(vol, cal)
    p = vr.default_params(W, H, S, flags=3)
    up = tuple(vr.default_camera(W, H).up)
    n = a.frames
    views = {
        "default": [vr.default_camera(W, H)] * n,
        "oblique": [vr.reset_camera()] * n,
        "orbit": [vr.derive_camera((math.sin(2 * math.pi * i / n), 0.0, math.cos(2 * math.pi * i / n)), up,
                                   p.real_screen_width, p.real_screen_height) for i in range(n)],
    }
    frames = [torch.empty((W, H, 4), dtype=torch.float32, device="cuda") for _ in range(3)]
    streams = [torch.cuda.Stream() for _ in range(3)]
    for name, cams in views.items():
        for k in (1, 2, 3):
            for rep in range(2):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for i, c in enumerate(cams):
                    j = i % k
                    r.set_stream(streams[j].cuda_stream)
                    r.render_device(p, c, frames[j].data_ptr(), asynchronous=True)
                torch.cuda.synchronize()
                dt = time.perf_counter() - t0
            print(f"{name:8s} streams {k}: {W * H * n / dt / 1e6:10.1f} Mrays/s  ({dt / n * 1e6:.1f} us/frame)",
                  flush=True)
    r.set_stream(0)
    r.close()


if __name__ == "__main__":
    main()
