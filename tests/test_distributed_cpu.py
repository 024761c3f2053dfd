"""The multi-GPU plan (screen tiles -> gather -> assemble) on CPU with gloo, world size 2 and 3.

Each rank receives the volume by broadcast from rank 0 (as bench.py does over RCCL), cuts its
interleaved tiles out of the oracle frame with the layout vr_render_tiles writes
(volumerenderingproject_amd.distributed.tiles_from_frame; the GPU test checks the kernel against
it), rank 0 gathers and assembles, and the result must equal the single-process frame bitwise.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import GOLDEN


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def worker(rank, world, port, tw, th, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from volumerenderingproject_amd import distributed as D
        from volumerenderingproject_amd import volumes
        vol = torch.empty((91, 109, 91), dtype=torch.float32)
        if rank == 0:
            vol.copy_(torch.from_numpy(volumes.avg152()[0]))
        dist.broadcast(vol, src=0)
        assert np.array_equal(vol.numpy(), volumes.avg152()[0])
        frame = np.load(os.path.join(GOLDEN, "frames_avg152.npz"))["vrc_100x100x100_default"]
        W, H = frame.shape[:2]
        mt = D.max_tiles(W, H, tw, th, world)
        mine = torch.from_numpy(D.tiles_from_frame(frame, tw, th, rank, world, slots=mt))
        gathered = [torch.empty_like(mine) for _ in range(world)] if rank == 0 else None
        dist.gather(mine, gathered, dst=0)
        if rank == 0:
            allt = torch.stack(gathered).numpy()
            out = D.assemble_frame(allt, W, H, tw, th)
            q.put(bool(np.array_equal(out, frame)))
    finally:
        dist.destroy_process_group()


def farm_list_worker(rank, world, port, w0, batch, q):
    """TileFarm over a culled tile list (only listed tiles rendered and gathered; the rest of the
    frame is the background) with 3-float (VR_OUT_RGB) tile pixels and batched gathers, as
    TileFarm.for_renderer sets it up for libvr: every frame comes out on rank 0 whole, in order."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from volumerenderingproject_amd import distributed as D
        W, H, tw = 100, 70, 16
        bg = np.array([0.2, 0.2, 0.2, 1.0], np.float32)
        ntx, nty = D.grid(W, H, tw, tw)
        ids = [t for t in range(ntx * nty) if (t // nty) in (1, 2, 4) and (t % nty) in (0, 2, 3)]
        frames = []
        for i in range(11):
            f = np.broadcast_to(bg, (W, H, 4)).copy()
            rnd = np.random.default_rng(i).random((W, H, 4), dtype=np.float32)
            rnd[..., 3] = 1.0     # the renderer's alpha
            for t in ids:
                tx, ty = divmod(t, nty)
                f[tx * tw:(tx + 1) * tw, ty * tw:(ty + 1) * tw] = rnd[tx * tw:(tx + 1) * tw, ty * tw:(ty + 1) * tw]
            frames.append(f)
        cur = {"i": 0}
        got = []

        def render(buf, my_ids):
            # a batch renders its frames' lists back to back; this rank's frame f is batch frame f
            per = len(my_ids) // cur["nf"]
            for f in range(cur["nf"]):
                part = my_ids[f * per:(f + 1) * per]
                buf[f * per:(f + 1) * per].copy_(torch.from_numpy(
                    D.tiles_of_list(frames[cur["base"] + f], tw, tw, part, channels=3)))

        def assemble(blocks, frames_out, tiles, slots, nf):
            for f in range(nf):
                frames_out[f].copy_(torch.from_numpy(D.assemble_slots(
                    blocks.numpy(), W, H, tw, tw, tiles, slots[f * len(tiles):(f + 1) * len(tiles)], bg)))
                got.append(frames_out[f].numpy().copy())

        farm = D.TileFarm(render, assemble, W, H, rank, world, tile=tw, device="cpu", ids=ids, channels=3, w0=w0,
                          batch=batch)
        assert farm.send[0].shape[-1] == 3
        assert sorted(sum(farm.lists, [])) == sorted(ids)
        # the render callback learns which frames a batch holds from the step count
        orig_batch = farm._batch

        def batch_hook(k, nf):
            cur["nf"], cur["base"] = nf, cur["done"]
            cur["done"] += nf
            orig_batch(k, nf)
        farm._batch = batch_hook
        cur["done"] = 0
        for i in range(7):          # one full batch of 4 (or 7 of 1) + a partial one, then drain
            farm.step()
        farm.drain()
        for i in range(7, 11):      # after a drain the farm starts a fresh batch
            farm.step()
        farm.drain()
        if rank == 0:
            ok = len(got) == len(frames) and all(np.array_equal(a, b) for a, b in zip(got, frames))
            q.put(ok)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,w0,batch", [(2, 1.0, 4), (3, 1.0, 4), (2, 3.0, 4), (3, 1e6, 4), (2, 2.0, 1)])
def test_tile_farm_culled_list_gloo(world, w0, batch):
    """Weighted plans (rank 0 keeps w0 shares) with batched gathers: every tile reaches rank 0 once,
    frames whole and in order; w0 = 1e6 leaves the peers nothing but empty blocks."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=farm_list_worker, args=(r, world, port, w0, batch, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    assert q.get(timeout=10) is True


def farm_worker(rank, world, port, tw, th, pipelined, q):
    """TileFarm itself (double-buffered sets, async batched gather) over gloo on host tensors: a
    sequence of different frames must come out on rank 0 whole and in order."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from volumerenderingproject_amd import distributed as D
        W, H = 100, 37
        frames = [np.random.default_rng(i).random((W, H, 4), dtype=np.float32) for i in range(9)]
        cur = {"done": 0}
        got = []

        def render(buf, my_ids):
            per = len(my_ids) // cur["nf"]
            for f in range(cur["nf"]):
                part = my_ids[f * per:(f + 1) * per]
                buf[f * per:(f + 1) * per].copy_(torch.from_numpy(
                    D.tiles_of_list(frames[cur["base"] + f], tw, th, part, channels=4)))

        def assemble(blocks, frames_out, tiles, slots, nf):
            for f in range(nf):
                frames_out[f].copy_(torch.from_numpy(D.assemble_slots(
                    blocks.numpy(), W, H, tw, th, tiles, slots[f * len(tiles):(f + 1) * len(tiles)], [0, 0, 0, 0])))
                got.append(frames_out[f].numpy().copy())

        farm = D.TileFarm(render, assemble, W, H, rank, world, tile=tw, device="cpu", pipelined=pipelined, batch=2)
        orig_batch = farm._batch

        def batch_hook(k, nf):
            cur["nf"], cur["base"] = nf, cur["done"]
            cur["done"] += nf
            orig_batch(k, nf)
        farm._batch = batch_hook
        for i in range(len(frames)):
            farm.step()
        farm.drain()
        if rank == 0:
            q.put(len(got) == len(frames) and all(np.array_equal(a, b) for a, b in zip(got, frames)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,pipelined", [(2, True), (3, True), (2, False)])
def test_tile_farm_pipeline_gloo(world, pipelined):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=farm_worker, args=(r, world, port, 16, 16, pipelined, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    assert q.get(timeout=10) is True


@pytest.mark.parametrize("world,tw,th", [(2, 64, 64), (3, 32, 48), (2, 16, 16)])
def test_tile_farm_gather_assemble_gloo(world, tw, th):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=worker, args=(r, world, port, tw, th, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    assert q.get(timeout=10) is True


def test_tile_plan_partitions_every_tile_once():
    from volumerenderingproject_amd import distributed as D
    for (W, H, tw, th, world) in [(1920, 1080, 64, 64, 8), (700, 700, 64, 64, 3), (100, 37, 16, 16, 5)]:
        ntx, nty = D.grid(W, H, tw, th)
        seen = []
        for r in range(world):
            seen += [r + k * world for k in range(D.tiles_per_rank(W, H, tw, th, r, world))]
        assert sorted(seen) == list(range(ntx * nty))
        # interleaving balances the centre-heavy frame: tile counts differ by at most one
        counts = [D.tiles_per_rank(W, H, tw, th, r, world) for r in range(world)]
        assert max(counts) - min(counts) <= 1
    rng = np.random.default_rng(1)
    f = rng.random((100, 37, 4), dtype=np.float32)
    for world in (1, 2, 4):
        mt = D.max_tiles(100, 37, 16, 16, world)
        allt = np.stack([D.tiles_from_frame(f, 16, 16, r, world, slots=mt) for r in range(world)])
        assert np.array_equal(D.assemble_frame(allt, 100, 37, 16, 16), f)
        # VR_OUT_RGB transport: r g b travel, alpha comes back as 1 (the renderer's alpha)
        f1 = f.copy()
        f1[..., 3] = 1.0
        rgb = np.stack([D.tiles_from_frame(f1, 16, 16, r, world, slots=mt, channels=3) for r in range(world)])
        assert rgb.shape[-1] == 3 and rgb.nbytes * 4 == allt.nbytes * 3
        assert np.array_equal(D.assemble_frame(rgb, 100, 37, 16, 16), f1)


def test_weighted_lists_plan():
    from volumerenderingproject_amd import distributed as D
    ids = list(range(3, 230, 1))
    for world in (1, 2, 3, 8):
        for w0 in (1.0, 1.5, 3.0, 1e6):
            lists = D.weighted_lists(ids, world, w0)
            assert sorted(sum(lists, [])) == ids                    # every tile exactly once
            n = [len(L) for L in lists]
            share0 = w0 / (w0 + world - 1)
            assert abs(n[0] - share0 * len(ids)) <= 1.0 + 1e-9
            if world > 1:
                assert max(n[1:]) - min(n[1:]) <= 1                  # peers even
            for L in lists:                                          # interleaved, ascending
                assert L == sorted(L)
            tiles, slots, mt = D.plan_slots(lists)
            assert mt == max(1, max(n)) and len(set(slots)) == len(ids)
    assert D.weighted_lists(ids, 4, 1e6)[1:] == [[], [], []]
    # even plan == the plain interleave the uniform entry points use
    assert D.weighted_lists(list(range(10)), 3, 1.0) == [[0, 3, 6, 9], [1, 4, 7], [2, 5, 8]]
    # numpy statements agree: list buffers + slot assembly rebuild the frame
    rng = np.random.default_rng(3)
    f = rng.random((100, 37, 4), dtype=np.float32)
    f[..., 3] = 1.0
    lists = D.weighted_lists(list(range(7 * 3)), 3, 2.0)
    tiles, slots, mt = D.plan_slots(lists)
    blocks = np.concatenate([D.tiles_of_list(f, 16, 16, L, slots=mt, channels=3) for L in lists])
    assert np.array_equal(D.assemble_slots(blocks, 100, 37, 16, 16, tiles, slots, [0, 0, 0, 1]), f)
