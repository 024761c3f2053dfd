"""Screen-tile farming across GPUs: one process per GPU, torch.distributed over RCCL.

Plan for a W x H frame cut into tile_w x tile_h tiles numbered x-major (t = tx * ntiles_y + ty):
only the tiles that can hold a non-background pixel are farmed -- the list vr_visible_tiles derives
on every rank from the camera (the projected dataset box).  Rank r of N renders list entries
r, r + N, r + 2N, ... (interleaved, so the centre-heavy head is spread over all GPUs) into a
compact buffer [k][tile_w * tile_h][C] (pixel (i, j) of a tile at i * tile_h + j -- the layout
vr_render_tile_list writes; C = 3 with VR_OUT_RGB, the farm's default: alpha is 1 by construction,
kernel.cu:213, so only r, g, b travel and the gathered bytes drop by a quarter).  Rank 0 gathers
the N buffers (RCCL gather, each peer over its own xGMI link) and vr_assemble_tile_list scatters them into the [x*H + y] frame, writing the exact
background everywhere else.  Without culling the list is every tile (vr_render_tiles /
vr_assemble_tiles).

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


class TileFarm:
    """One rank's share of the multi-GPU frame: render own tiles, RCCL-gather, assemble on rank 0.

    Double-buffered when the gather can run asynchronously (RCCL, or gloo on host tensors): step i
    enqueues the render of frame i and the gather of frame i, then finishes frame i-1 (wait for its
    gather, assemble on rank 0).  So the render of frame i overlaps the xGMI transfer of frame i-1;
    `drain()` completes the last frame.  Every step still produces exactly one whole frame on rank 0.

    render(buf) fills this rank's compact tile buffer; assemble(all_tiles, frame) scatters the
    gathered [N][mt][tw*th][C] tiles (C = `channels`: 3 for VR_OUT_RGB buffers) into the frame.
    For libvr these wrap vr_render_tiles / vr_assemble_tiles (`for_renderer`); tests pass host
    implementations.
    """

    def __init__(self, render, assemble, W, H, rank, world, tile=64, device="cuda:0", pipelined=True, n_tiles=None,
                 channels=4):
        import torch
        import torch.distributed as dist
        self.render, self.assemble = render, assemble
        self.W, self.H, self.rank, self.world, self.tile = W, H, rank, world, tile
        # n_tiles: length of the tile-id list when only listed tiles are rendered and gathered
        self.mt = max_tiles(W, H, tile, tile, world) if n_tiles is None else max(1, -(-n_tiles // world))
        on_gpu = str(device).startswith("cuda")
        # gloo cannot move device tensors: rehearsal runs stage tiles through host memory
        self.stage_host = dist.get_backend() == "gloo" and on_gpu
        self.pipelined = pipelined and not self.stage_host
        nbuf = 2 if self.pipelined else 1
        self.channels = channels
        self.mine = [torch.zeros((self.mt, tile * tile, channels), dtype=torch.float32, device=device)
                     for _ in range(nbuf)]
        if rank == 0:
            self.all = [torch.empty((world, self.mt, tile * tile, channels), dtype=torch.float32, device=device)
                        for _ in range(nbuf)]
            self.frame = torch.zeros((W, H, 4), dtype=torch.float32, device=device)
        else:
            self.all = None
            self.frame = None
        self.i = 0
        self.pending = None     # (work handle, buffer index) of the frame still being gathered

    @classmethod
    def for_renderer(cls, r, W, H, rank, world, params, camera, tile=64, device=0, pipelined=True, cull=True,
                     rgb=True):
        """TileFarm over a libvr VolumeRenderer (device memory, asynchronous launches).

        rgb: tiles travel as 3 floats per pixel (VR_OUT_RGB; alpha is 1 by construction), a quarter
        fewer bytes through the gather than float4 -- the gather is the multi-GPU scaling limit.

        cull: render and gather only the tiles vr_visible_tiles keeps (the projected dataset box);
        rank 0's assembly writes the exact background everywhere else.  Every rank derives the same
        list on the host from the same params and camera, so no exchange is needed for it.

        The renders, the gather and the assembly must share one stream: libvr is bound to torch's
        current stream, replaced first by a dedicated stream if it is the null stream (handle 0
        would select libvr's own non-blocking stream, unordered against RCCL's work)."""
        import torch
        s = torch.cuda.current_stream(device)
        if s.cuda_stream == 0:
            s = torch.cuda.Stream(device=device)
            torch.cuda.set_stream(s)
        r.set_stream(s.cuda_stream)
        ch = 3 if rgb else 4
        if not cull:
            def render(buf):
                r.render_tiles(params, camera, tile, tile, rank, world, buf.data_ptr(), asynchronous=True, rgb=rgb)

            def assemble(all_tiles, frame):
                r.assemble_tiles(W, H, tile, tile, world, all_tiles.shape[1], all_tiles.data_ptr(), frame.data_ptr(),
                                 asynchronous=True, rgb=rgb)
            return cls(render, assemble, W, H, rank, world, tile=tile, device=f"cuda:{device}", pipelined=pipelined,
                       channels=ch)
        ids = r.visible_tiles(params, camera, tile, tile)
        bg = [float(v) for v in params.background]

        def render(buf):
            r.render_tile_list(params, camera, tile, tile, ids, rank, world, buf.data_ptr(), asynchronous=True,
                               rgb=rgb)

        def assemble(all_tiles, frame):
            r.assemble_tile_list(W, H, tile, tile, ids, world, all_tiles.shape[1], all_tiles.data_ptr(), bg,
                                 frame.data_ptr(), asynchronous=True, rgb=rgb)
        farm = cls(render, assemble, W, H, rank, world, tile=tile, device=f"cuda:{device}", pipelined=pipelined,
                   n_tiles=len(ids), channels=ch)
        farm.tile_ids = ids
        return farm

    def _finish(self, work, b):
        if work is not None:
            work.wait()          # RCCL: the current stream waits for RCCL's stream (no host block)
        if self.rank == 0:
            self.assemble(self.all[b], self.frame)

    def step(self):
        import torch
        import torch.distributed as dist
        b = self.i % len(self.mine)
        self.i += 1
        self.render(self.mine[b])
        if self.stage_host:
            torch.cuda.current_stream().synchronize()
            host = self.mine[b].cpu()
            glist = [torch.empty_like(host) for _ in range(self.world)] if self.rank == 0 else None
            dist.gather(host, glist, dst=0)
            if self.rank == 0:
                self.all[b].copy_(torch.stack(glist))
            self._finish(None, b)
            return self.frame
        glist = list(self.all[b].unbind(0)) if self.rank == 0 else None
        work = dist.gather(self.mine[b], glist, dst=0, async_op=self.pipelined)
        if not self.pipelined:
            self._finish(None, b)
            return self.frame
        prev, self.pending = self.pending, (work, b)
        if prev is not None:
            self._finish(*prev)
        return self.frame

    def drain(self):
        if self.pending is not None:
            self._finish(*self.pending)
            self.pending = None
        return self.frame
