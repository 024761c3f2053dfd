"""One rank of the multi-rank RCCL check (tests/test_gpu_multi.py::test_rccl_ranks_equal_one_gpu):
torchrun, one process per GPU, the RCCL id handed over with gloo.  Every rank renders the same
moving-camera batches through vr_create_rank; rank 0 compares each frame with a one-GPU vr_render
bitwise and prints RCCL_RANKS_OK."""
import math
import os
import sys

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.dirname(
    os.path.abspath(__file__))))))


def main():
    import numpy as np
    import torch
    import torch.distributed as dist
    import volumerenderingproject_amd as vr
    from volumerenderingproject_amd import renderer, volumes
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dev = int(os.environ.get("LOCAL_RANK", rank))
    dist.init_process_group("gloo")
    vol, cal = volumes.mni152_standin()
    cid = [renderer.comm_unique_id() if rank == 0 else None]
    dist.broadcast_object_list(cid, src=0)
    W, H, S = 640, 360, 500
    r = vr.VolumeRenderer(vol if rank == 0 else None, cal, shape=vol.shape, device=dev, rank=rank, n_ranks=world,
                          comm_id=cid[0], options=vr.default_options(farm_tile=64, farm_rank0_weight=1.0))
    up = tuple(vr.default_camera(W, H).up)
    cams = [vr.default_camera(W, H), vr.reset_camera()] + [
        vr.derive_camera((math.sin(0.7 * i), 0.3, math.cos(0.7 * i)), up, 2.0, 2.0 * H / W) for i in range(6)]
    ok = True
    ref = vr.VolumeRenderer(vol, cal, device=dev) if rank == 0 else None
    for flags in (vr.VR_FLAG_ESS | vr.VR_FLAG_ERT, 0):
        p = vr.default_params(W, H, S, flags=flags)
        n = len(cams)
        out = torch.empty((n, W, H, 4), dtype=torch.float32, device=f"cuda:{dev}") if rank == 0 else None
        for rep in range(3):   # batches back to back, asynchronous: double-buffered transfers
            r.render_batch_device(p, cams, out.data_ptr() if out is not None else None, asynchronous=True)
        r.synchronize()
        if rank == 0:
            got = out.cpu().numpy()
            for f in range(n):
                want = ref.render(p, cams[f])
                if not np.array_equal(got[f], want):
                    ok = False
                    print(f"frame {f} flags {flags}: max |d| {float(np.abs(got[f] - want).max())}", flush=True)
            tiles = [len(r.group_tiles(q)) for q in range(world)]
            print("tiles per rank", tiles, flush=True)
    t = torch.tensor([1 if ok else 0], dtype=torch.int32)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    r.close()
    if ref is not None:
        ref.close()
    dist.destroy_process_group()
    if rank == 0 and int(t.item()) == 1:
        print("RCCL_RANKS_OK", flush=True)
    return 0 if int(t.item()) == 1 else 1


if __name__ == "__main__":
    sys.exit(main())
