"""DESIGN section 7's prediction of the N-GPU screen-tile split (C3 / C4 / C5, N = 1, 2, 4, 8), from
one-GPU measurements (tools/scale_probe.py -> profiles/r6_scale/probe.json, and the driver-style
bench's steady frame time) and a link model.  Printed as a markdown table and JSON so the driver's
first SCALE line can be checked against it, field by field (bench.py's `peer_traffic`).

Model, per frame, rank-0 weight w (the bench tunes w over its --rank0-weights list; the best is
taken here), each of the N - 1 peers marching a share f = 1 / (N - 1 + w) of the V visible 64 x 64
tiles and rank 0 the share w f:
  * M = F1 - F0: the march work that scales with the tiles (F1 = the one-GPU frame, F0 = the
    S = 1 frame of the same size: prologue, background and the 16 B/pixel frame store, which stay on
    rank 0 whatever the split -- F0 / F1 from the one-launch probe, applied to the steady F1);
  * rank 0: F0 + w f M + scatter of the peers' tiles ((N - 1) f B bytes of compact RGB read, 16/12 of
    it written, at HBM_EFF);
  * a peer: F0_PEER + f M (its own launch and prologue, tiles into a compact buffer);
  * a link: f B / LINK, every peer on its own xGMI link into rank 0 (B = V x 64 x 64 x 12 B);
  * the frame: the largest of the three (batches double-buffer the transfer against the next march).
LINK = 64 GB/s one way per link is an assumption (no xGMI figure in the guides; the bench's
peer_traffic and march_ms_per_frame_by_rank let the run correct it); 50 and 76.8 GB/s are shown as
the range.
usage: python tools/scale_model.py [--probe profiles/r6_scale/probe.json]
"""
import argparse
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WEIGHTS = [1, 1.5, 2, 3, 4, 6, 8, 12, 16, 1e6]   # bench.py --rank0-weights default
TILE_BYTES = 64 * 64 * 12
HBM_EFF = 5.0e12      # B/s, scatter (read + write) -- the store-only floor measured ~5 TB/s
F0_PEER = 3.0e-6      # s, a peer's launch + prologue for its compact tile buffer
# steady one-GPU frame times (driver protocol, 20 steps, two frames in flight): round-6 bench lines
STEADY_MS = {"c3": 0.0178, "c4": 0.0244, "c5": 0.1779}


def predict(cfg, steady_ms, n, link):
    W, H, V = cfg["W"], cfg["H"], cfg["visible_tiles_64"]
    phi = cfg["frame_ms_S1_one_launch"] / cfg["frame_ms_one_launch"]
    F1 = steady_ms * 1e-3
    F0 = phi * F1
    M = F1 - F0
    B = V * TILE_BYTES
    if n == 1:
        return {"ms": F1 * 1e3, "mrays": W * H / F1 / 1e6, "w": None, "bytes_into_rank0": 0, "bound": "one GPU"}
    best = None
    for w in WEIGHTS:
        f = 1.0 / (n - 1 + w)
        peer_bytes = f * B
        r0 = F0 + w * f * M + (n - 1) * peer_bytes * (28.0 / 12.0) / HBM_EFF
        peer = F0_PEER + f * M
        lk = peer_bytes / link
        t = max(r0, peer, lk)
        bound = "rank 0" if t == r0 else ("peer march" if t == peer else "xGMI link")
        if best is None or t < best[0]:
            best = (t, w, int((n - 1) * peer_bytes), bound)
    t, w, into0, bound = best
    return {"ms": t * 1e3, "mrays": W * H / t / 1e6, "w": w, "bytes_into_rank0": into0, "bound": bound}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--probe", default=os.path.join(ROOT, "profiles", "r6_scale", "probe.json"))
    a = ap.parse_args()
    probe = json.load(open(a.probe))
    out = {}
    print("| Config | N | rank-0 weight | tiles into rank 0 per frame (MB) | frame (ms) | Mrays/s | x one GPU | bound | Mrays/s at 50 / 76.8 GB/s |")
    print("|---|---|---|---|---|---|---|---|---|")
    for name in ("c3", "c4", "c5"):
        cfg = probe[name]
        base = predict(cfg, STEADY_MS[name], 1, 64e9)
        for n in (1, 2, 4, 8):
            p = predict(cfg, STEADY_MS[name], n, 64e9)
            lo = predict(cfg, STEADY_MS[name], n, 50e9)["mrays"]
            hi = predict(cfg, STEADY_MS[name], n, 76.8e9)["mrays"]
            out[f"{name}_n{n}"] = dict(p, mrays_link50=lo, mrays_link76=hi)
            print(f"| {name.upper()} | {n} | {p['w'] if p['w'] is not None else '-'} | {p['bytes_into_rank0'] / 1e6:.2f} | "
                  f"{p['ms']:.4f} | {p['mrays']:,.0f} | {p['mrays'] / base['mrays']:.2f} | {p['bound']} | "
                  f"{lo:,.0f} / {hi:,.0f} |")
    print()
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
