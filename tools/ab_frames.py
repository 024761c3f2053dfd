"""A/B of two libvr builds on the same frames: per-camera SHA-256 of the frame bytes and the median
kernel time (HIP events, libvr's per-launch timing).  Run once per build (VR_LIB=<build>.so) and
diff the printed JSON: equal hashes = bitwise equal frames.

usage: VR_LIB=build_ab/b.so python tools/ab_frames.py [--reps 5] [--flags 3] [--volume mni|avg152]
"""
import argparse
import hashlib
import json
import math
import os
import sys

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--flags", type=int, default=3)
    ap.add_argument("--volume", default="mni")
    ap.add_argument("--size", default="1920x1080x500")
    a = ap.parse_args()
    import numpy as np
    import torch
    import volumerenderingproject_amd as vr
    from volumerenderingproject_amd import volumes
    if a.volume == "mni":
        vol, cal = volumes.mni152_standin()
    else:
        vol, h = volumes.avg152()
        cal = h["cal_max"]
    W, H, S = (int(x) for x in a.size.split("x"))
    r = vr.VolumeRenderer(vol, cal)
    st = torch.cuda.Stream()
    torch.cuda.set_stream(st)
    r.set_stream(st.cuda_stream)
    p = vr.default_params(W, H, S, flags=a.flags)
    up = tuple(vr.default_camera(W, H).up)
    cams = {"default": vr.default_camera(W, H), "oblique": vr.reset_camera()}
    for i in range(8):
        t = 2 * math.pi * (i + 0.37) / 8
        cams[f"orbit{i}"] = vr.derive_camera((math.sin(t), 0.3 * math.cos(3 * t), math.cos(t)), up,
                                             p.real_screen_width, p.real_screen_height)
    cams["dolly"] = vr.derive_camera((0.05, -0.1, 0.8), up, p.real_screen_width, p.real_screen_height)
    frame = torch.empty((W, H, 4), dtype=torch.float32, device="cuda")
    res = {}
    for name, c in cams.items():
        for _ in range(2):
            r.render_device(p, c, frame.data_ptr(), True)
        torch.cuda.synchronize()
        got = frame.cpu().numpy()
        h = hashlib.sha256(got.tobytes()).hexdigest()[:16]
        # the same view in the exact back-to-front mode (bitwise the oracle): ERT's deviation from it
        exact = r.render(vr.default_params(W, H, S, flags=0), c) if a.flags & vr.VR_FLAG_ERT else got
        dev = float(np.abs(got - exact).max())
        r.timing_enable(True)
        ts = []
        for _ in range(a.reps):
            r.timing_read(reset=True)
            r.render_device(p, c, frame.data_ptr(), True)
            ts.append(r.timing_read(reset=True).total_ms * 1e3)
        r.timing_enable(False)
        res[name] = {"sha": h, "us": round(float(np.median(ts)), 2), "maxdiff_vs_exact": dev}
    print(json.dumps({"lib": os.environ.get("VR_LIB", "libvr.so"), "size": a.size, "flags": a.flags, "frames": res}))
    r.close()


if __name__ == "__main__":
    main()
