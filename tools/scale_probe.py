"""Inputs of DESIGN section 7's multi-GPU prediction (tools/scale_model.py), measured on ONE GPU.

For C3 (MNI stand-in, 1920x1080, S = 500), C4 (512^3 resample, 1920x1080, S = 1024) and C5 (the
synthetic 2048^3 volume, 3840x2160, S = 4096), ESS + ERT, the default camera:
  * the visible 64 x 64 farm tiles (vr_visible_tiles: what an N-GPU context deals out; every peer
    tile crosses xGMI as 64 x 64 x 12 B of compact RGB),
  * the device time of one frame, one vr_render at a time (HIP events on the context's stream),
  * the same at S = 1: the per-frame cost that stays on rank 0 whatever the split (prologue, the
    background and the frame store).
usage: python tools/scale_probe.py [--iters 20] > profiles/r6_scale/probe.json
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def frame_ms(r, p, cam, out, iters):
    for _ in range(3):
        r.render_device(p, cam, out.data_ptr(), asynchronous=True)
    r.timing_enable(True)
    r.timing_read(reset=True)
    ms = []
    for _ in range(iters):
        r.render_device(p, cam, out.data_ptr(), asynchronous=True)
        t = r.timing_read(reset=True)
        ms.append(t.total_ms / max(1, t.launches))
    r.timing_enable(False)
    return statistics.median(ms)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--configs", default="c3,c4,c5")
    a = ap.parse_args()
    import torch
    import volumerenderingproject_amd as vr
    from volumerenderingproject_amd import volumes
    res = {}
    for name in a.configs.split(","):
        if name == "c3":
            vol, cal = volumes.mni152_standin()
            r = vr.VolumeRenderer(vol, cal, device=0)
            W, H, S = 1920, 1080, 500
        elif name == "c4":
            r = vr.VolumeRenderer(volumes.resample_512(volumes.mni152_standin()[0]), 255.0, device=0)
            W, H, S = 1920, 1080, 1024
        else:
            n = 2048
            dvol = torch.empty((n, n, n), dtype=torch.float32, device="cuda:0")
            vr.renderer.synthetic_volume(dvol.data_ptr(), n, device=0,
                                         stream=torch.cuda.current_stream(0).cuda_stream)
            torch.cuda.synchronize()
            r = vr.VolumeRenderer(device_ptr=dvol.data_ptr(), shape=(n, n, n), cal_max=255.0, device=0)
            del dvol
            torch.cuda.empty_cache()
            W, H, S = 3840, 2160, 4096
        flags = vr.VR_FLAG_ESS | vr.VR_FLAG_ERT
        cam = vr.default_camera(W, H)
        out = torch.empty((W, H, 4), dtype=torch.float32, device="cuda:0")
        p = vr.default_params(W, H, S, flags=flags)
        p1 = vr.default_params(W, H, 1, flags=flags)
        tiles = r.visible_tiles(p, cam, 64, 64)
        res[name] = {"W": W, "H": H, "S": S, "visible_tiles_64": int(len(tiles)),
                     "all_tiles_64": int(((W + 63) // 64) * ((H + 63) // 64)),
                     "frame_ms_one_launch": round(frame_ms(r, p, cam, out, a.iters), 5),
                     "frame_ms_S1_one_launch": round(frame_ms(r, p1, cam, out, a.iters), 5)}
        print(name, json.dumps(res[name]), file=sys.stderr, flush=True)
        r.close()
        del out
        torch.cuda.empty_cache()
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
