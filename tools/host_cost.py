"""Host cost of queuing frames: wall time of asynchronous vr_render_batch / vr_render calls while the
stream is held busy (torch.cuda._sleep), so no call waits on the GPU.  Prints one JSON line.

usage: python tools/host_cost.py [--frames 32] [--reps 5]
"""
import argparse
import json
import math
import os
import statistics
import sys
import time

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=32)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    import torch
    import volumerenderingproject_amd as vr
    from volumerenderingproject_amd import volumes
    vol, cal = volumes.mni152_standin()
    W, H, S = 1920, 1080, 500
    r = vr.VolumeRenderer(vol, cal, device=0)
    stream = torch.cuda.Stream(device=0)
    torch.cuda.set_stream(stream)
    r.set_stream(stream.cuda_stream)
    p = vr.default_params(W, H, S, flags=vr.VR_FLAG_ESS | vr.VR_FLAG_ERT)
    n = a.frames
    frames = torch.empty((n, W, H, 4), dtype=torch.float32, device="cuda:0")
    up = tuple(vr.default_camera(W, H).up)
    steady = (vr.Camera * n)(*([vr.default_camera(W, H)] * n))
    orbit = (vr.Camera * n)(*[vr.derive_camera((math.sin(2 * math.pi * i / n), 0.3, math.cos(2 * math.pi * i / n)),
                                               up, 2.0, 2.0 * H / W) for i in range(n)])
    out = {}
    for name, cams in (("steady", steady), ("orbit", orbit)):
        for _ in range(2):   # warm: plans, lists, tables
            r.render_batch_device(p, cams, frames.data_ptr())
        torch.cuda.synchronize()
        batch, single, one = [], [], []
        for _ in range(a.reps):
            torch.cuda._sleep(200_000_000)   # keep the stream busy well past the calls below
            t0 = time.perf_counter()
            r.render_batch_device(p, cams, frames.data_ptr(), asynchronous=True)
            batch.append((time.perf_counter() - t0) / n * 1e6)
            # a one-frame call (bench.py's --lead call: the first frame of a timed region)
            for i in range(8):
                t0 = time.perf_counter()
                r.render_batch_device(p, cams, frames.data_ptr(), asynchronous=True, n=1)
                one.append((time.perf_counter() - t0) * 1e6)
            t0 = time.perf_counter()
            for i in range(n):
                r.render_device(p, cams[i], frames[i].data_ptr(), asynchronous=True)
            single.append((time.perf_counter() - t0) / n * 1e6)
            torch.cuda.synchronize()
        out[name] = {"batch_us_per_frame": round(statistics.median(batch), 2),
                     "one_frame_call_us": round(statistics.median(one), 2),
                     "render_us_per_frame": round(statistics.median(single), 2)}
    print(json.dumps({"host_cost": out, "frames_per_call": n}))
    r.close()


if __name__ == "__main__":
    main()
