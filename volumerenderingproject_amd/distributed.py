"""Screen-tile farming across GPUs: one process per GPU, torch.distributed over RCCL.

Plan for a W x H frame cut into tile_w x tile_h tiles numbered x-major (t = tx * ntiles_y + ty):
only the tiles that can hold a non-background pixel are farmed -- the list vr_visible_tiles derives
on every rank from the camera (the projected dataset box).  The list is dealt to the ranks
interleaved (so the centre-heavy head is spread over all GPUs) with a weight for rank 0
(weighted_lists): every peer's tiles cross an xGMI link into rank 0, which also stitches the
frame, so rank 0 keeps a larger share when the links, not the march, bound the frame rate.  Each
rank renders its tiles into a compact buffer [k][tile_w * tile_h][C] (pixel (i, j) of a tile at
i * tile_h + j -- the layout vr_render_tile_list writes; C = 3 with VR_OUT_RGB, the farm's
default: alpha is 1 by construction, kernel.cu:213, so only r, g, b travel).  The buffers of a
batch of frames reach rank 0 in one RCCL gather (each peer over its own xGMI link), and
vr_assemble_tile_slots scatters each frame's tiles into its [x*H + y] frame, writing the exact
background everywhere else.  One transfer per batch keeps the host's per-frame work (a gather
costs ~20 us of host time through torch.distributed) below the GPU's.

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
    """One rank's share of the multi-GPU frames: render own tiles, gather to rank 0, assemble there.

    render(buf, ids) fills the first len(ids) tiles of a compact buffer with the tiles `ids` (ids
    may repeat a tile); assemble(blocks, frames, tiles, slots, nf) writes frames[f], f < nf, taking
    tile tiles[i] from blocks[slots[f * len(tiles) + i]] (vr_render_tile_list /
    vr_assemble_tile_slots_multi for libvr via `for_renderer`; tests pass host implementations).

    Plan: weighted_lists deals the tiles (rank 0 weight w0).  Per frame every rank contributes a
    block of mt tiles to the gather (mt = the largest peer share; a shorter share repeats its first
    tile as padding); rank 0's tiles beyond mt stay in a local extra region.

    Batches: the farm's camera is fixed, so B consecutive frames are B renders of the same tile
    list.  A batch is rendered by ONE launch over the list repeated B times (B x the workgroups of
    one frame: a rank's share of one frame is too small to fill the GPU at N = 8), its blocks reach
    rank 0 in ONE gather (the ~20 us host cost of a collective is paid once per batch) and rank 0
    assembles its B frames in ONE launch into a ring of B output frames, on a second stream that
    overlaps the next batch's render.  Every frame is rendered and assembled in full; step()
    accounts one frame, and the batch's work is enqueued by its last step.  Two buffer sets
    alternate, each with its own ring of B output frames; a set is reused only after its previous
    batch has been assembled (rank 0) or sent (peers).  drain() completes a partial batch and
    everything in flight.  The frame step() / drain() return is ordered on the caller's current
    stream (it waits for the assembly event), and stays valid until its set is reused two batches
    later.
    """

    def __init__(self, render, assemble, W, H, rank, world, tile=64, device="cuda:0", pipelined=True, ids=None,
                 channels=4, w0=1.0, batch=8):
        import torch
        import torch.distributed as dist
        self.render, self.assemble = render, assemble
        self.W, self.H, self.rank, self.world, self.tile = W, H, rank, world, tile
        self.device = device
        self.channels = channels
        ntx, nty = grid(W, H, tile, tile)
        self.tile_ids = list(range(ntx * nty)) if ids is None else [int(t) for t in ids]
        self.on_gpu = str(device).startswith("cuda")
        # gloo cannot move device tensors: multi-rank rehearsals stage tiles through host memory
        self.stage_host = dist.get_backend() == "gloo" and self.on_gpu and world > 1
        self.pipelined = pipelined and not self.stage_host
        self.asm_stream = torch.cuda.Stream(device=device) if (self.on_gpu and rank == 0 and self.pipelined) else None
        self.pending = None
        self.set_plan(w0, batch)

    def set_plan(self, w0, batch=None):
        """(Re)build the plan for rank-0 weight w0 and batch size; drains any batch in flight."""
        import torch
        if self.pending is not None or getattr(self, "i", 0) % getattr(self, "B", 1):
            self.drain()
        self.w0 = float(w0)
        if batch is not None:
            self.B = max(1, int(batch))
        B, world, rank = self.B, self.world, self.rank
        self.lists = weighted_lists(self.tile_ids, world, self.w0)
        n = [len(L) for L in self.lists]
        self.mt = max(1, max(n[1:]) if world > 1 else n[0])
        self.ex = max(0, n[0] - self.mt)                # rank 0's tiles outside the gathered block
        mt, ex = self.mt, self.ex
        head = self.lists[rank][:mt]
        self.head = head + head[:1] * (mt - len(head)) if head else []   # padded to mt (one block per frame)
        self.tail = self.lists[0][mt:] if rank == 0 else []
        self._rep = {}                                  # nf -> (head list, tail list) repeated nf times
        # slots of frame f in rank 0's blocks: [world][B][mt] gathered, then [B][ex] extra
        self.tiles = [t for L in self.lists for t in L]
        self.slots = []
        for f in range(B):
            for r, L in enumerate(self.lists):
                for k in range(len(L)):
                    self.slots.append(world * B * mt + f * ex + (k - mt) if k >= mt else (r * B + f) * mt + k)
        T2, ch, dev = self.tile * self.tile, self.channels, self.device
        nsets = 2 if self.pipelined else 1
        mk = lambda m: torch.zeros((m, T2, ch), dtype=torch.float32, device=dev)  # noqa: E731
        if rank == 0:
            self.blocks = [mk(world * B * mt + B * ex) for _ in range(nsets)]
            self.gout = [[b[r * B * mt:(r + 1) * B * mt] for r in range(world)] for b in self.blocks]
            self.extra = [b[world * B * mt:] for b in self.blocks]
            # one rank: its block is the gathered block itself (nothing to send)
            self.send = [self.gout[k][0] for k in range(nsets)] if world == 1 else [mk(B * mt) for _ in range(nsets)]
            # one frame ring per buffer set: the frames of a batch stay valid until their set is
            # reused two batches later (the next batch assembles into the other ring)
            self.frame_sets = [torch.zeros((B, self.W, self.H, 4), dtype=torch.float32, device=dev)
                               for _ in range(nsets)]
            self.frames = self.frame_sets[0]
        else:
            self.blocks = self.gout = self.extra = self.frames = self.frame_sets = None
            self.send = [mk(B * mt) for _ in range(nsets)]
        self.frame = self.frames[0] if rank == 0 else None
        self.frame_evt = None                     # rank 0: assembly event of self.frame (second stream)
        self.i = 0
        self.pending = None                       # (work, set, frames) of the batch in flight
        self.free_evt = [None] * nsets            # rank 0: the set's last batch assembled
        self.sends = [None] * nsets               # peers: the set's last gather
        self.rendered = [None] * nsets            # rank 0: its renders of the set's batch done

    @classmethod
    def for_renderer(cls, r, W, H, rank, world, params, camera, tile=64, device=0, pipelined=True, cull=True,
                     rgb=True, w0=1.0, batch=8, ids=None):
        """TileFarm over a libvr VolumeRenderer (device memory, asynchronous launches).

        rgb: tiles travel as 3 floats per pixel (VR_OUT_RGB; alpha is 1 by construction), a quarter
        fewer bytes over xGMI than float4.

        cull: render and send only the tiles vr_visible_tiles keeps (the projected dataset box);
        rank 0's assembly writes the exact background everywhere else.  Every rank derives the same
        list on the host from the same params and camera, so no exchange is needed for it.  ids:
        an explicit tile list instead (tools).

        The renders and the gathers share one stream: libvr is bound to torch's current stream,
        replaced first by a dedicated stream if it is the null stream (handle 0 would select
        libvr's own non-blocking stream, unordered against RCCL's work).  Rank 0's assembly runs on
        the farm's second stream (libvr is re-bound around that call).  The C-ABI calls are
        prepared once per tile list (ctypes arrays)."""
        import ctypes as C
        import torch
        from . import renderer as R
        s = torch.cuda.current_stream(device)
        if s.cuda_stream == 0:
            s = torch.cuda.Stream(device=device)
            torch.cuda.set_stream(s)
        r.set_stream(s.cuda_stream)
        ch = 3 if rgb else 4
        if ids is not None:
            ids = [int(t) for t in ids]
        elif cull:
            ids = [int(t) for t in r.visible_tiles(params, camera, tile, tile)]
        else:
            ntx, nty = grid(W, H, tile, tile)
            ids = list(range(ntx * nty))
        L = R.lib()
        ctx = r._ctx
        bg = (C.c_float * 4)(*[float(v) for v in params.background])
        flags = R.VR_OUT_ASYNC | (R.VR_OUT_RGB if rgb else 0)
        main = s.cuda_stream
        pp, pc = C.byref(params), C.byref(camera)
        nout = C.c_int32(0)
        arrays = {}

        def carr(v):
            key = (id(v), len(v))
            a = arrays.get(key)
            if a is None or a[0] is not v:
                a = (v, (C.c_int32 * max(1, len(v)))(*v))
                arrays[key] = a
            return a[1]

        def render(buf, my_ids):
            if my_ids:
                R._check(L.vr_render_tile_list(ctx, pp, pc, tile, tile, carr(my_ids), len(my_ids), 0, 1,
                                               C.c_void_p(buf.data_ptr()), C.byref(nout), flags),
                         "vr_render_tile_list")

        def assemble(blocks, frames, tiles, slots, nf):
            cur = torch.cuda.current_stream(device).cuda_stream
            if cur != main:
                r.set_stream(cur)
            try:
                R._check(L.vr_assemble_tile_slots_multi(ctx, W, H, tile, tile, carr(tiles), carr(slots), len(tiles),
                                                        nf, blocks.shape[0], C.c_void_p(blocks.data_ptr()), bg,
                                                        C.c_void_p(frames.data_ptr()), flags),
                         "vr_assemble_tile_slots_multi")
            finally:
                if cur != main:
                    r.set_stream(main)
        return cls(render, assemble, W, H, rank, world, tile=tile, device=f"cuda:{device}", pipelined=pipelined,
                   ids=ids, channels=ch, w0=w0, batch=batch)

    def _acquire(self, k):
        """Before buffer set k takes a new batch: its previous batch must be consumed."""
        import torch
        if self.free_evt[k] is not None:
            torch.cuda.current_stream().wait_event(self.free_evt[k])
            self.free_evt[k] = None
        if self.sends[k] is not None:
            self.sends[k].wait()
            self.sends[k] = None

    def _batch(self, k, nf):
        """Render frames 0..nf-1 of set k (one launch per region), gather them, finish the previous batch."""
        import torch
        import torch.distributed as dist
        self._acquire(k)
        rep = self._rep.get(nf)
        if rep is None:
            rep = self._rep[nf] = (self.head * nf, self.tail * nf)
        self.render(self.send[k], rep[0])
        if rep[1]:
            self.render(self.extra[k], rep[1])
        if self.stage_host:
            torch.cuda.current_stream().synchronize()
            host = self.send[k].cpu()
            glist = [torch.empty_like(host) for _ in range(self.world)] if self.rank == 0 else None
            dist.gather(host, glist, dst=0)
            if self.rank == 0:
                for r in range(self.world):
                    self.gout[k][r].copy_(glist[r])
                self._finish(None, k, nf)
            return
        work = None
        if self.world > 1:
            work = dist.gather(self.send[k], self.gout[k] if self.rank == 0 else None, dst=0,
                               async_op=self.pipelined)
        if self.asm_stream is not None:
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream())
            self.rendered[k] = ev
        if not self.pipelined:
            if work is not None:
                work.wait()
            self._finish(None, k, nf)
            return
        prev, self.pending = self.pending, (work, k, nf)
        if prev is not None:
            self._finish(*prev)

    def _finish(self, work, k, nf):
        import torch
        if self.rank != 0:
            self.sends[k] = work
            return
        frames = self.frame_sets[k]
        if self.asm_stream is not None:
            with torch.cuda.stream(self.asm_stream):
                if self.rendered[k] is not None:
                    self.asm_stream.wait_event(self.rendered[k])   # rank 0's own tiles
                if work is not None:
                    work.wait()       # RCCL: the assembly stream waits for the gather (no host block)
                self.assemble(self.blocks[k], frames, self.tiles, self.slots, nf)
                ev = torch.cuda.Event()
                ev.record(self.asm_stream)
                self.free_evt[k] = ev
                self.frame_evt = ev
        else:
            if work is not None:
                work.wait()
            self.assemble(self.blocks[k], frames, self.tiles, self.slots, nf)
        self.frames = frames
        self.frame = frames[nf - 1]

    def _ordered_frame(self):
        """self.frame, with the caller's stream ordered after the assembly that wrote it (that runs
        on the farm's second stream): reading it on the current stream needs no device-wide sync."""
        import torch
        if self.frame_evt is not None:
            torch.cuda.current_stream().wait_event(self.frame_evt)
        return self.frame

    def step(self):
        """One frame.  The last frame of a batch enqueues the batch's render, gather and assembly."""
        self.i += 1
        if self.i % self.B == 0:
            self._batch((self.i // self.B - 1) % len(self.send), self.B)
        return self._ordered_frame() if self.rank == 0 else None

    def drain(self):
        """Complete the partial batch (if any) and everything in flight; the next step starts a
        fresh batch."""
        f = self.i % self.B
        if f:
            self._batch((self.i // self.B) % len(self.send), f)
            self.i += self.B - f
        if self.pending is not None:
            self._finish(*self.pending)
            self.pending = None
        for k in range(len(self.send)):
            if self.sends[k] is not None:
                self.sends[k].wait()
                self.sends[k] = None
        return self._ordered_frame() if self.rank == 0 else None

    def tune(self, weights, frames=None):
        """Pick rank 0's weight by measurement: for each candidate, run a few batches (outside any
        timed region) and take the max over ranks of the wall time; every rank gets the same
        all-reduced times, so all choose the same weight.  Returns {weight: seconds}."""
        import time
        import torch
        import torch.distributed as dist
        frames = frames or 3 * self.B
        res = {}
        for w in weights:
            self.set_plan(w)
            for _ in range(self.B):
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
        self.set_plan(best)
        return res
