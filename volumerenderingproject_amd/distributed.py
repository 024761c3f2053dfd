"""Screen-tile farming across GPUs: one process per GPU, torch.distributed over RCCL.

Plan for a W x H frame cut into tile_w x tile_h tiles numbered x-major (t = tx * ntiles_y + ty):
only the tiles that can hold a non-background pixel are farmed -- the list vr_visible_tiles derives
on every rank from the camera (the projected dataset box).  The list is dealt to the ranks
interleaved (so the centre-heavy head is spread over all GPUs) with a weight for rank 0
(weighted_lists): every peer's tiles cross an xGMI link into rank 0, which also stitches the
frame, so rank 0 keeps a larger share when the links, not the march, bound the frame rate.  Each
rank renders its tiles into a compact buffer [k][tile_w * tile_h][C] (pixel (i, j) of a tile at
i * tile_h + j -- the layout vr_render_tile_list writes; C = 3 with VR_OUT_RGB, the farm's
default: alpha is 1 by construction, kernel.cu:213, so only r, g, b travel).  The peers send their
buffers to rank 0 (RCCL point-to-point, one xGMI link each, only the tiles they hold), and
vr_assemble_tile_slots scatters them into the [x*H + y] frame, writing the exact background
everywhere else.

The numpy functions here are the host-side statement of that layout; tests/test_distributed_cpu.py
runs the whole plan over gloo on CPU with them, and tests/test_gpu_parity.py checks that the HIP
kernels produce exactly this layout.
"""
from __future__ import annotations

import numpy as np


def grid(W, H, tw, th):
    return (W + tw - 1) // tw, (H + th - 1) // th


def tiles_per_rank(W, H, tw, th, rank, world):
    ntx, nty = grid(W, H, tw, th)
    nt = ntx * nty
    return 0 if rank >= nt else (nt - 1 - rank) // world + 1


def max_tiles(W, H, tw, th, world):
    return max(tiles_per_rank(W, H, tw, th, r, world) for r in range(world))


def tiles_from_frame(frame: np.ndarray, tw, th, rank, world, slots=None, tiles=None, channels=4) -> np.ndarray:
    """The compact tile buffer rank `rank` produces for a full (W, H, 4) frame (vr_render_tiles;
    with `tiles`, vr_render_tile_list over that id list; channels=3: VR_OUT_RGB, r g b only)."""
    W, H = frame.shape[:2]
    ntx, nty = grid(W, H, tw, th)
    ids = list(range(ntx * nty)) if tiles is None else [int(t) for t in tiles]
    mine = ids[rank::world]
    n = len(mine)
    out = np.zeros((slots if slots is not None else n, tw * th, channels), np.float32)
    for k in range(n):
        t = mine[k]
        tx, ty = divmod(t, nty)
        x0, y0 = tx * tw, ty * th
        blk = frame[x0:x0 + tw, y0:y0 + th]
        tile = np.zeros((tw, th, channels), np.float32)
        tile[:blk.shape[0], :blk.shape[1]] = blk[..., :channels]
        out[k] = tile.reshape(tw * th, channels)
    return out


def assemble_frame(all_tiles: np.ndarray, W, H, tw, th, tiles=None, background=None) -> np.ndarray:
    """Inverse of tiles_from_frame over all ranks (vr_assemble_tiles; with `tiles`,
    vr_assemble_tile_list: pixels of unlisted tiles are `background`).  all_tiles: [N][mt][tw*th][C]
    with C = 4, or C = 3 (VR_OUT_RGB: alpha written as 1)."""
    world, mt = all_tiles.shape[:2]
    ch = all_tiles.shape[-1]
    ntx, nty = grid(W, H, tw, th)
    ids = list(range(ntx * nty)) if tiles is None else [int(t) for t in tiles]
    frame = np.zeros((W, H, 4), np.float32)
    if tiles is not None:
        frame[:] = np.asarray(background, np.float32)
    for rank in range(world):
        for k in range(mt):
            i = rank + k * world
            if i >= len(ids):
                continue
            t = ids[i]
            tx, ty = divmod(t, nty)
            x0, y0 = tx * tw, ty * th
            tile = all_tiles[rank, k].reshape(tw, th, ch)
            w, h = min(tw, W - x0), min(th, H - y0)
            frame[x0:x0 + w, y0:y0 + h, :ch] = tile[:w, :h]
            if ch == 3:
                frame[x0:x0 + w, y0:y0 + h, 3] = 1.0
    return frame


def weighted_lists(ids, world, w0=1.0):
    """Deal the tile ids to `world` ranks, rank 0 with weight w0 and every other rank weight 1,
    interleaved: tile i goes to the rank furthest below its target share of the first i + 1 tiles
    (ties: lowest rank).  w0 = 1 is an even interleave; a large w0 keeps (almost) every tile on
    rank 0.  Deterministic, so every rank derives the same plan."""
    ids = [int(t) for t in ids]
    wts = [float(w0)] + [1.0] * (world - 1)
    tot = sum(wts)
    lists = [[] for _ in range(world)]
    for i, t in enumerate(ids):
        best, bd = 0, None
        for r in range(world):
            d = wts[r] / tot * (i + 1) - len(lists[r])
            if bd is None or d > bd + 1e-12:
                best, bd = r, d
        lists[best].append(t)
    return lists


def plan_slots(lists):
    """(tiles, slots, mt): tile lists[r][k] sits in block r * mt + k of the [world][mt] buffer."""
    mt = max(1, max(len(L) for L in lists))
    tiles, slots = [], []
    for r, L in enumerate(lists):
        for k, t in enumerate(L):
            tiles.append(t)
            slots.append(r * mt + k)
    return tiles, slots, mt


def tiles_of_list(frame: np.ndarray, tw, th, ids, slots=None, channels=3) -> np.ndarray:
    """Compact buffer of an explicit tile list (vr_render_tile_list with first 0, stride 1)."""
    W, H = frame.shape[:2]
    nty = grid(W, H, tw, th)[1]
    out = np.zeros((slots if slots is not None else len(ids), tw * th, channels), np.float32)
    for k, t in enumerate(ids):
        tx, ty = divmod(int(t), nty)
        blk = frame[tx * tw:(tx + 1) * tw, ty * th:(ty + 1) * th]
        tile = np.zeros((tw, th, channels), np.float32)
        tile[:blk.shape[0], :blk.shape[1]] = blk[..., :channels]
        out[k] = tile.reshape(tw * th, channels)
    return out


def assemble_slots(blocks: np.ndarray, W, H, tw, th, tiles, slots, background) -> np.ndarray:
    """Numpy statement of vr_assemble_tile_slots: blocks [n_blocks][tw*th][C]; tile tiles[i] from
    block slots[i]; unlisted tiles are the background; C = 3 writes alpha = 1."""
    ch = blocks.shape[-1]
    nty = grid(W, H, tw, th)[1]
    frame = np.empty((W, H, 4), np.float32)
    frame[:] = np.asarray(background, np.float32)
    for t, sl in zip(tiles, slots):
        tx, ty = divmod(int(t), nty)
        x0, y0 = tx * tw, ty * th
        w, h = min(tw, W - x0), min(th, H - y0)
        tile = blocks[sl].reshape(tw, th, ch)
        frame[x0:x0 + w, y0:y0 + h, :ch] = tile[:w, :h]
        if ch == 3:
            frame[x0:x0 + w, y0:y0 + h, 3] = 1.0
    return frame


class TileFarm:
    """One rank's share of the multi-GPU frame: render own tiles, send them to rank 0, assemble there.

    render(buf, ids) fills a compact tile buffer with the tiles `ids`; assemble(blocks, frame,
    tiles, slots) scatters the [world * mt][tw*th][C] blocks into the frame (vr_render_tile_list /
    vr_assemble_tile_slots for libvr via `for_renderer`; tests pass host implementations).

    Transport: the peers' buffers go to rank 0 with point-to-point sends (torch.distributed
    batch_isend_irecv: RCCL over xGMI, or gloo), each of exactly the tiles that peer holds; rank 0
    renders its own share straight into its slot of the receive buffer.  Pipelined (RCCL, or gloo
    on host tensors): step i renders frame i and posts its transfers, then finishes frame i-1
    (rank 0: the assembly waits for the receives on a second stream, so it overlaps the next
    render).  Buffers are double-buffered; a buffer is reused only after the assembly (rank 0) or
    the send (peers) of the frame two steps back has completed.  Every step yields one whole frame
    on rank 0; drain() completes the last one.
    """

    def __init__(self, render, assemble, W, H, rank, world, tile=64, device="cuda:0", pipelined=True, ids=None,
                 channels=4, w0=1.0):
        import torch
        import torch.distributed as dist
        self.render, self.assemble = render, assemble
        self.W, self.H, self.rank, self.world, self.tile = W, H, rank, world, tile
        self.device = device
        self.channels = channels
        ntx, nty = grid(W, H, tile, tile)
        self.tile_ids = list(range(ntx * nty)) if ids is None else [int(t) for t in ids]
        self.on_gpu = str(device).startswith("cuda")
        # gloo cannot move device tensors: rehearsal runs stage tiles through host memory
        self.stage_host = dist.get_backend() == "gloo" and self.on_gpu and world > 1
        self.pipelined = pipelined and not self.stage_host
        self.asm_stream = torch.cuda.Stream(device=device) if (self.on_gpu and rank == 0 and self.pipelined) else None
        self.frame = torch.zeros((W, H, 4), dtype=torch.float32, device=device) if rank == 0 else None
        self.set_weight(w0)

    def set_weight(self, w0):
        """(Re)build the plan for rank-0 weight w0; drains any frame in flight first."""
        import torch
        if getattr(self, "pending", None) is not None:
            self.drain()
        self.w0 = float(w0)
        self.lists = weighted_lists(self.tile_ids, self.world, self.w0)
        self.tiles, self.slots, self.mt = plan_slots(self.lists)
        self.mine_ids = self.lists[self.rank]
        nbuf = 2 if self.pipelined else 1
        T2, ch, dev = self.tile * self.tile, self.channels, self.device
        if self.rank == 0:
            self.all = [torch.zeros((self.world * self.mt, T2, ch), dtype=torch.float32, device=dev)
                        for _ in range(nbuf)]
            self.mine = [a[:max(1, len(self.mine_ids))] for a in self.all]   # rank 0 renders in place
        else:
            self.all = None
            self.mine = [torch.zeros((max(1, len(self.mine_ids)), T2, ch), dtype=torch.float32, device=dev)
                         for _ in range(nbuf)]
        self.i = 0
        self.pending = None              # (requests, buffer index) of the frame in flight
        self.free_evt = [None] * nbuf    # rank 0: assembly of the buffer's last frame done
        self.rendered = [None] * nbuf    # rank 0: its own render of the buffer's frame done
        self.sends = [[] for _ in range(nbuf)]   # peers: send requests of the buffer's last frame

    @classmethod
    def for_renderer(cls, r, W, H, rank, world, params, camera, tile=64, device=0, pipelined=True, cull=True,
                     rgb=True, w0=1.0):
        """TileFarm over a libvr VolumeRenderer (device memory, asynchronous launches).

        rgb: tiles travel as 3 floats per pixel (VR_OUT_RGB; alpha is 1 by construction), a quarter
        fewer bytes over xGMI than float4 -- the transfers into rank 0 are the scaling limit.

        cull: render and send only the tiles vr_visible_tiles keeps (the projected dataset box);
        rank 0's assembly writes the exact background everywhere else.  Every rank derives the same
        list on the host from the same params and camera, so no exchange is needed for it.

        The renders and transfers share one stream: libvr is bound to torch's current stream,
        replaced first by a dedicated stream if it is the null stream (handle 0 would select
        libvr's own non-blocking stream, unordered against RCCL's work).  Rank 0's assembly runs on
        the farm's second stream (libvr is re-bound around that call)."""
        import torch
        s = torch.cuda.current_stream(device)
        if s.cuda_stream == 0:
            s = torch.cuda.Stream(device=device)
            torch.cuda.set_stream(s)
        r.set_stream(s.cuda_stream)
        ch = 3 if rgb else 4
        if cull:
            ids = [int(t) for t in r.visible_tiles(params, camera, tile, tile)]
        else:
            ntx, nty = grid(W, H, tile, tile)
            ids = list(range(ntx * nty))
        bg = [float(v) for v in params.background]
        main = s.cuda_stream

        def render(buf, my_ids):
            if my_ids:
                r.render_tile_list(params, camera, tile, tile, my_ids, 0, 1, buf.data_ptr(), asynchronous=True,
                                   rgb=rgb)

        def assemble(blocks, frame, tiles, slots):
            cur = torch.cuda.current_stream(device).cuda_stream
            if cur != main:
                r.set_stream(cur)
            try:
                r.assemble_tile_slots(W, H, tile, tile, tiles, slots, blocks.shape[0], blocks.data_ptr(), bg,
                                      frame.data_ptr(), asynchronous=True, rgb=rgb)
            finally:
                if cur != main:
                    r.set_stream(main)
        return cls(render, assemble, W, H, rank, world, tile=tile, device=f"cuda:{device}", pipelined=pipelined,
                   ids=ids, channels=ch, w0=w0)

    def _post(self, b):
        """Post frame b's transfers: peers send their tiles, rank 0 receives every peer's."""
        import torch.distributed as dist
        ops = []
        if self.rank == 0:
            for src in range(1, self.world):
                n = len(self.lists[src])
                if n:
                    ops.append(dist.P2POp(dist.irecv, self.all[b][src * self.mt:src * self.mt + n], src))
        elif self.mine_ids:
            ops.append(dist.P2POp(dist.isend, self.mine[b][:len(self.mine_ids)], 0))
        return dist.batch_isend_irecv(ops) if ops else []

    def _finish(self, reqs, b):
        import torch
        if self.rank != 0:
            self.sends[b] = reqs     # waited before the buffer is rendered into again
            return
        if self.asm_stream is not None:
            with torch.cuda.stream(self.asm_stream):
                if self.rendered[b] is not None:
                    self.asm_stream.wait_event(self.rendered[b])   # rank 0's own tiles (no receive orders them)
                for q in reqs:
                    q.wait()         # RCCL: the assembly stream waits for the receives (no host block)
                self.assemble(self.all[b], self.frame, self.tiles, self.slots)
                ev = torch.cuda.Event()
                ev.record(self.asm_stream)
                self.free_evt[b] = ev
        else:
            for q in reqs:
                q.wait()
            self.assemble(self.all[b], self.frame, self.tiles, self.slots)

    def step(self):
        import torch
        import torch.distributed as dist
        nbuf = len(self.mine)
        b = self.i % nbuf
        self.i += 1
        if self.stage_host:
            self.render(self.mine[b], self.mine_ids)
            torch.cuda.current_stream().synchronize()
            if self.rank == 0:
                host = self.all[b].cpu()
                for src in range(1, self.world):
                    n = len(self.lists[src])
                    if n:
                        dist.recv(host[src * self.mt:src * self.mt + n], src=src)
                self.all[b].copy_(host)
                self.assemble(self.all[b], self.frame, self.tiles, self.slots)
            elif self.mine_ids:
                dist.send(self.mine[b][:len(self.mine_ids)].cpu(), dst=0)
            return self.frame
        # the buffer's previous frame (two steps back) must be consumed before it is overwritten
        if self.free_evt[b] is not None:
            torch.cuda.current_stream().wait_event(self.free_evt[b])
            self.free_evt[b] = None
        for q in self.sends[b]:
            q.wait()
        self.sends[b] = []
        self.render(self.mine[b], self.mine_ids)
        if self.asm_stream is not None:
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream())
            self.rendered[b] = ev
        reqs = self._post(b)
        if not self.pipelined:
            for q in reqs:
                q.wait()
            self._finish([], b)
            if self.rank != 0:
                self.sends[b] = []
            return self.frame
        prev, self.pending = self.pending, (reqs, b)
        if prev is not None:
            self._finish(*prev)
        return self.frame

    def drain(self):
        if self.pending is not None:
            self._finish(*self.pending)
            self.pending = None
        if self.rank != 0:
            for b in range(len(self.sends)):
                for q in self.sends[b]:
                    q.wait()
                self.sends[b] = []
        return self.frame

    def tune(self, weights, frames=6, timer=None):
        """Pick rank 0's weight by measurement: for each candidate, run `frames` pipelined frames
        (outside any timed region) and take the max over ranks of the wall time; every rank gets
        the same all-reduced times, so all choose the same weight.  Returns {weight: seconds}."""
        import time
        import torch
        import torch.distributed as dist
        res = {}
        for w in weights:
            self.set_weight(w)
            for _ in range(2):
                self.step()
            self.drain()
            if self.on_gpu:
                torch.cuda.synchronize()
            dist.barrier()
            t0 = time.perf_counter()
            for _ in range(frames):
                self.step()
            self.drain()
            if self.on_gpu:
                torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            t = torch.tensor([dt], dtype=torch.float64,
                             device=self.device if (self.on_gpu and not self.stage_host) else "cpu")
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            res[float(w)] = float(t.item())
        best = min(res, key=lambda k: (res[k], k))
        self.set_weight(best)
        return res
