"""Per-rank share of the multi-GPU tile farm, timed on one GPU: rank 0's tile-list render at
stride N (the list entries 0, N, 2N, ...) for N = 1, 2, 4, 8, and the rank-0 assembly of a whole
gathered buffer.  HIP-event kernel time on the ctx stream (median of rounds).  This is the compute
side of the N-GPU frame; the RCCL gather between them is not measurable on a one-GPU box.

usage: python tools/farm_probe.py [--tile 64] [--rgb 1]
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tile", type=int, default=64)
    ap.add_argument("--rgb", type=int, default=1)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    import torch
    import volumerenderingproject_amd as vr
    from volumerenderingproject_amd import volumes
    vol, cal = volumes.mni152_standin()
    W, H, S, T = 1920, 1080, 500, a.tile
    r = vr.VolumeRenderer(vol, cal, device=0)
    s = torch.cuda.Stream()
    torch.cuda.set_stream(s)
    r.set_stream(s.cuda_stream)
    p = vr.default_params(W, H, S, flags=vr.VR_FLAG_ESS | vr.VR_FLAG_ERT)
    cam = vr.default_camera(W, H)
    ids = r.visible_tiles(p, cam, T, T)
    ch = 3 if a.rgb else 4
    res = {"tiles_farmed": int(len(ids)), "tile": T, "channels": ch}

    def timed(fn):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        out = []
        for _ in range(a.rounds):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(a.iters):
                fn()
            e1.record(s)
            torch.cuda.synchronize()
            out.append(e0.elapsed_time(e1) / a.iters * 1e3)
        return round(statistics.median(out), 2)

    frame = torch.empty((W, H, 4), dtype=torch.float32, device="cuda:0")
    res["whole_frame_us"] = timed(lambda: r.render_device(p, cam, frame.data_ptr(), asynchronous=True))
    for n in (1, 2, 4, 8):
        mt = -(-len(ids) // n)
        buf = torch.empty((mt, T * T, ch), dtype=torch.float32, device="cuda:0")
        res[f"rank0_render_us_n{n}"] = timed(
            lambda: r.render_tile_list(p, cam, T, T, ids, 0, n, buf.data_ptr(), asynchronous=True, rgb=bool(a.rgb)))
        allt = torch.zeros((n, mt, T * T, ch), dtype=torch.float32, device="cuda:0")
        res[f"assemble_us_n{n}"] = timed(
            lambda: r.assemble_tile_list(W, H, T, T, ids, n, mt, allt.data_ptr(), list(p.background),
                                         frame.data_ptr(), asynchronous=True, rgb=bool(a.rgb)))
        res[f"gather_bytes_into_rank0_n{n}"] = int((n - 1) * mt * T * T * ch * 4)
    res["VR_BATCH"] = os.environ.get("VR_BATCH")
    print(json.dumps(res))


if __name__ == "__main__":
    main()
