#!/usr/bin/env python3
"""Benchmark of the hot path: Mrays/s of the fused HIP ray march (BASELINE.json metric).

Step = one frame of the configured workload, inputs (volume, classes, occupancy) resident in HBM.
  N = 1 : C3 -- MNI152_T1_1mm stand-in (182x218x182) at 1920x1080, 500 samples/ray, ESS + ERT,
          default steady camera, one MI355X.  (C2 700x700 and C1 100x100 are parity-test cases.)
          Frames are issued --farm-batch at a time through vr_render_batch, two in flight (the tail
          of one frame's march overlaps the next one's start); extra.single_frame_mrays is one
          vr_render per frame.
  N > 1 : the same frame farmed over N GPUs in 64x64 screen tiles (tile t -> rank t mod N); each
          rank renders its tiles, the tiles are gathered to rank 0 over RCCL and assembled there.
          Total work per step is one frame regardless of N ("scaling": "strong").
value = W*H*steps / (max over ranks of the timed-region wall time), in Mrays/s.
roofline.achieved = HBM bytes per march launch from the PMC counters (profiles/traffic_*.json, made
by tools/pmc_traffic.py on the same workload: FETCH_SIZE x 2 + WRITE_SIZE) / the march kernel's
mean duration, timed live with HIP events on the stream the kernel runs on; frac = achieved / 8 TB/s.
Without a matching counter file, achieved counts only the 16 B/ray frame write the launch must make
(a lower bound on its HBM traffic, labelled as such in bytes_source).  SURVEY 8(d)'s exact-march
model (4 B * N_in + 16 B * W*H) is reported beside it as `model_*` -- with ESS + ERT the kernel
skips most of those samples, so that model exceeds the HBM peak and is never the fraction.
cpu_baseline = the reference's CPU ray-cast path (myApp.cu:1401-1495, restated in oracle/) on a
bounded column subset of the same frame, one host thread (the reference's own threading).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # a C3 frame takes ~21 us: 2000 frames make a ~45 ms timed region, so its fixed cost (the
    # barrier and synchronize on both sides, ~0.3 ms) stays small; 96 frames read ~10 % low
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=200)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--samples", type=int, default=500)
    ap.add_argument("--flags", default="ess,ert", help="comma list of ess,ert or 'exact'")
    ap.add_argument("--mode", default="vrc", choices=["vrc", "test"])
    ap.add_argument("--volume", default="mni", choices=["mni", "avg152", "r512", "c5"],
                    help="c5: synthetic 2048^3 float32 generated on the device (SURVEY 8(d) C5)")
    ap.add_argument("--camera", default="default", choices=["default", "oblique"],
                    help="oblique: the reset camera of key X (utils.h:77-81)")
    ap.add_argument("--tile", type=int, default=64)
    ap.add_argument("--rank0-weights", default="1,1.5,2,3,4,6,8,12,16,1e6",
                    help="N > 1: candidate weights of rank 0's tile share, tuned before the timed region")
    ap.add_argument("--farm", default="capi", choices=["capi", "torch", "capi1"],
                    help="N > 1: capi = libvr's multi-GPU context (vr_create_rank: RCCL broadcast + per-frame "
                         "ncclSend/ncclRecv of tiles inside libvr, one frame per step); torch = the Python "
                         "TileFarm over torch.distributed (batched gathers); capi1 = the capi path on a "
                         "one-rank group (rehearses the N > 1 code on one GPU)")
    # frames per vr_render_batch call: every call ends by joining the second in-flight stream into the
    # caller's (an idle gap of ~18 us between calls, profiles/r3_timeline), so larger batches waste less
    ap.add_argument("--farm-batch", type=int, default=32,
                    help="frames per vr_render_batch call (N > 1: per gather -- the host cost of a collective "
                         "is paid once per batch)")
    ap.add_argument("--devices", default=None,
                    help="N > 1 in one process: comma list of the GPUs of the group (default 0..N-1).  A list "
                         "that repeats a GPU (e.g. 0,0) rehearses the N-part plan on fewer GPUs (peer-copy "
                         "transport); it is labelled as a rehearsal in config.parallelism")
    ap.add_argument("--lead", type=int, default=1,
                    help="frames the first vr_render_batch call of a region issues at once, so the GPU starts "
                         "while the host gathers the rest of the batch (0: wait for a full batch)")
    ap.add_argument("--options", default="",
                    help="vr_options overrides for A/B runs, e.g. persist_wgs=6,cull=1 (default: none)")
    ap.add_argument("--cpu-baseline", type=int, default=1, help="0 to skip the CPU baseline leg")
    ap.add_argument("--cpu-columns", type=int, default=240, help="columns of the frame the CPU baseline renders")
    ap.add_argument("--extra", type=int, default=1, help="also time exact mode and the oblique camera (N=1)")
    ap.add_argument("--extra-configs", default=None,
                    help="comma list of c4,c5: also time BASELINE configs[3] (512^3, 1920x1080, S=1024) and "
                         "configs[4] (2048^3, 3840x2160, S=4096), ESS + ERT, under the same kind of context as "
                         "the headline (one GPU, vr_create_multi group or vr_create_rank ranks), on every "
                         "rank -- where the screen-tile split can pay (DESIGN section 7).  Default: c4,c5 "
                         "(none with --extra 0)")
    ap.add_argument("--check-extras", type=int, default=1,
                    help="compare one frame of each extra config with a fresh one-GPU context, bitwise "
                         "(1: C4; 2: C4 and C5)")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic_latest.json"),
                    help="PMC traffic summary (tools/pmc_traffic.py) to attach when it matches this workload")
    return ap.parse_args()


def fail(msg):
    print(f"bench.py: {msg}", file=sys.stderr, flush=True)
    raise SystemExit(2)


def group_devices(a, world):
    """The GPUs of a one-process group (--gpus N > 1 without torchrun), checked before any GPU work:
    --devices, else 0..N-1, which must exist.  None for the one-GPU and one-process-per-GPU runs."""
    if a.gpus < 1:
        fail(f"--gpus must be >= 1 (got {a.gpus})")
    if world > 1:
        # torchrun: one rank per GPU; the group size is the number of ranks
        if world != a.gpus:
            fail(f"launched with WORLD_SIZE={world} ranks but --gpus {a.gpus}: one rank per GPU, they must match")
        if a.devices:
            fail("--devices is for one-process groups (no torchrun)")
        return None
    if a.devices:
        devs = [int(x) for x in a.devices.split(",") if x.strip()]
        if len(devs) != a.gpus:
            fail(f"--devices lists {len(devs)} GPUs but --gpus is {a.gpus}")
    else:
        devs = list(range(a.gpus))
    import torch
    n = torch.cuda.device_count()   # (counting devices does not initialise the GPU)
    if n < max(devs) + 1:
        fail(f"--gpus {a.gpus} needs GPUs {sorted(set(devs))} but this machine has {n}; refusing to report an "
             f"N-GPU line from fewer GPUs (pass --devices to rehearse the plan on fewer GPUs)")
    return devs if (a.devices or a.gpus > 1) else None


def main():
    a = parse()
    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    devices = group_devices(a, world_env)
    # stdout carries exactly one JSON line: RCCL's version banner and gloo's peer announcements go
    # to fd 1 from native code, so fd 1 points at stderr and the line goes to a private copy
    result_out = os.fdopen(os.dup(1), "w")
    sys.stdout.flush()
    os.dup2(2, 1)
    import numpy as np
    import torch
    import volumerenderingproject_amd as vr
    from volumerenderingproject_amd import volumes

    world = world_env
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    # VR_DIST_BACKEND=gloo rehearses N ranks on fewer GPUs (ranks share devices round-robin, tiles
    # gathered through host memory); the real multi-GPU path is RCCL ("nccl"), one rank per GPU.
    backend = os.environ.get("VR_DIST_BACKEND", "nccl")
    device = local_rank % max(1, torch.cuda.device_count()) if backend == "gloo" else local_rank
    # one process driving N GPUs (python bench.py --gpus N, SURVEY 7.7: vr_create_multi, one
    # ncclCommInitAll, the volume broadcast and the per-batch tile gather all inside libvr)
    group = devices is not None
    if group:
        device = devices[0]
    n_gpus = len(devices) if group else world
    if world > 1 or a.farm == "capi1":
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29517")
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
        torch.cuda.set_device(device)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", device))
        else:
            dist.init_process_group("gloo")
    torch.cuda.set_device(device)

    cfg_name = {"avg152": "C1", "mni": "C2" if (a.width, a.height) == (700, 700) else "C3", "r512": "C4",
                "c5": "C5"}[a.volume]
    vol = None
    if a.volume == "mni":
        vol, cal = volumes.mni152_standin()
        vname = "MNI152_T1_1mm stand-in 182x218x182 (avg152T1_LR 2x nearest-replicate)"
    elif a.volume == "avg152":
        vol, h = volumes.avg152()
        cal = h["cal_max"]
        vname = "avg152T1_LR 91x109x91"
    elif a.volume == "r512":
        vol = volumes.resample_512(volumes.mni152_standin()[0])
        cal = 255.0
        vname = "MNI stand-in trilinear-resampled to 512^3"
    else:
        cal = 255.0
        vname = "synthetic 2048^3 float32 (SURVEY 8(d) C5, seed 0x5EED, generated on device)"
    shape = vol.shape if vol is not None else (2048, 2048, 2048)

    capi = (world > 1 and a.farm == "capi" and backend == "nccl") or a.farm == "capi1" or group
    # volume: rank 0 owns it and RCCL-broadcasts it to the other GPUs; with the C-ABI
    # farm libvr broadcasts it (vr_create_rank), otherwise torch.distributed does
    dvol = torch.empty(shape if (rank == 0 or not capi) else (1,), dtype=torch.float32, device=f"cuda:{device}")
    if vol is not None:
        if rank == 0:
            dvol.copy_(torch.from_numpy(vol))
    elif rank == 0 or backend != "nccl":
        # C5 is generated in place (34.4 GB); gloo rehearsals generate per rank (no 34 GB host staging)
        vr.renderer.synthetic_volume(dvol.data_ptr(), shape[0], device=device,
                                     stream=torch.cuda.current_stream(device).cuda_stream)
    def torch_broadcast(dvol):
        if backend == "nccl":
            flat = dvol.view(-1)
            chunk = 1 << 28      # 1 GiB pieces: bounded RCCL messages for the 34.4 GB C5 replica
            for i in range(0, flat.numel(), chunk):
                dist.broadcast(flat[i:i + chunk], src=0)
        elif vol is not None:
            hv = dvol.cpu()
            dist.broadcast(hv, src=0)
            dvol.copy_(hv)

    if dist is not None and not capi:
        torch_broadcast(dvol)
    torch.cuda.synchronize()
    farm_fallback = None
    r = None
    if group:
        # every GPU of the group gets the volume by ncclBroadcast from devices[0] (peer copies when
        # the list repeats a GPU); a failure here is a failure of the run, not a fallback
        r = vr.VolumeRenderer(device_ptr=dvol.data_ptr(), shape=shape, cal_max=cal, devices=devices,
                              options=bench_options(a, farm_tile=a.tile))
    elif capi:
        ok = 1
        try:
            cid = [vr.renderer.comm_unique_id() if rank == 0 else None]
            dist.broadcast_object_list(cid, src=0)
            r = vr.VolumeRenderer(device_ptr=dvol.data_ptr() if rank == 0 else None, shape=shape, cal_max=cal,
                                  device=device, rank=rank, n_ranks=world, comm_id=cid[0],
                                  options=bench_options(a, farm_tile=a.tile))
        except vr.VRError as e:
            if world == 1:   # (capi1: the one-rank rehearsal has nothing to fall back to)
                raise
            print(f"bench: libvr multi-GPU context failed on rank {rank}: {e}", file=sys.stderr, flush=True)
            farm_fallback = f"vr_create_rank failed ({e}); torch.distributed TileFarm used"
            ok = 0
        if world > 1:
            # every rank takes the same path: the libvr group only if it came up everywhere
            t = torch.tensor([ok], dtype=torch.int32, device=f"cuda:{device}")
            dist.all_reduce(t, op=dist.ReduceOp.MIN)
            if int(t.item()) == 0:
                if r is not None:
                    r.close()
                    r = None
                farm_fallback = farm_fallback or "vr_create_rank failed on another rank; torch.distributed TileFarm used"
                capi = False
                a.farm = "torch"
                if rank != 0:
                    dvol = torch.empty(shape, dtype=torch.float32, device=f"cuda:{device}")
                torch_broadcast(dvol)
                torch.cuda.synchronize()
    if r is None:
        r = vr.VolumeRenderer(device_ptr=dvol.data_ptr(), shape=shape, cal_max=cal, device=device,
                              options=bench_options(a))
    if vol is None and rank == 0 and a.cpu_baseline and n_gpus == 1:
        vol = dvol.cpu().numpy()     # host copy for the CPU baseline's oracle (C5: 34.4 GB of RAM)
    del dvol
    torch.cuda.empty_cache()

    flags = 0
    for f in a.flags.split(","):
        f = f.strip().lower()
        if f == "ess":
            flags |= vr.VR_FLAG_ESS
        elif f == "ert":
            flags |= vr.VR_FLAG_ERT
        elif f == "shade":
            flags |= vr.VR_FLAG_SHADE
    mode = vr.VR_MODE_VRC if a.mode == "vrc" else vr.VR_MODE_TEST
    W, H, S = a.width, a.height, a.samples
    p = vr.default_params(W, H, S, mode=mode, flags=flags)
    cam = vr.default_camera(W, H) if a.camera == "default" else vr.reset_camera()

    # one explicit (non-null) stream shared by libvr, torch events and RCCL: vr_set_stream(NULL)
    # would mean libvr's own stream, which torch's null-stream events do not order against
    stream = torch.cuda.Stream(device=device)
    torch.cuda.set_stream(stream)
    r.set_stream(stream.cuda_stream)
    drain = lambda: None  # noqa: E731
    sub = None
    tuning = None
    farm_info = None
    weights = [float(x) for x in a.rank0_weights.split(",")] if a.rank0_weights else [1.0]
    B = max(1, a.farm_batch)   # frames per vr_render_batch call
    if n_gpus == 1 and not capi:
        # one GPU: every --farm-batch steps one vr_render_batch call renders that many frames into
        # consecutive device frames, two frames in flight (vr_options.frames_in_flight); a step is one
        # frame.  extra.single_frame_mrays is the same view one vr_render per frame.
        frames_dev = torch.empty((B, W, H, 4), dtype=torch.float32, device=f"cuda:{device}")
        frame = frames_dev[0]
        sub = Submitter(r, p, cam, frames_dev.data_ptr(), W * H * 16, B, a.lead)
        step, drain = sub.step, sub.drain
    elif capi:
        # libvr's multi-GPU context (one process driving N GPUs, or one process per GPU): vr_render_batch
        # once per --farm-batch frames (one RCCL group and one scatter per batch); rank 0 gets the frames.
        # A step is one frame.
        frames_dev = torch.empty((B, W, H, 4), dtype=torch.float32, device=f"cuda:{device}") if rank == 0 else None
        fptr = frames_dev.data_ptr() if frames_dev is not None else None
        frame = frames_dev[0] if frames_dev is not None else None
        sub = Submitter(r, p, cam, fptr, W * H * 16, B, a.lead)
        step, drain = sub.step, sub.drain

        tuning = (capi_tune(r, weights, step, drain, a.tile, dist, device, frames=2 * B,
                            mkopt=lambda **k: bench_options(a, **k)) if len(weights) > 1 else None)
        if tuning is None:
            r.set_options(bench_options(a, farm_tile=a.tile, farm_rank0_weight=weights[0]))
        r.render_device(p, cam, fptr, asynchronous=True)
        r.synchronize()
        transport = {vr.renderer.VR_TRANSPORT_NONE: "none (one GPU)", vr.renderer.VR_TRANSPORT_RCCL: "RCCL ncclSend/ncclRecv",
                     vr.renderer.VR_TRANSPORT_PEER_COPY: "hipMemcpyPeerAsync (repeated devices)"}[r.group[2]]
        farm_info = {"tiles_farmed": len(r.visible_tiles(p, cam, a.tile, a.tile)),
                     "rank0_weight": float(r.options.farm_rank0_weight), "rank0_tiles": len(r.group_tiles(0)),
                     "frames_per_gather": B,
                     "tiles_per_rank": [len(r.group_tiles(q)) for q in range(n_gpus)],
                     "transport": (f"libvr vr_create_multi(devices={devices}) + vr_render_batch, {transport}, one group "
                                   "per batch" if group else
                                   "libvr vr_create_rank + vr_render_batch (one RCCL ncclSend/ncclRecv group per batch)")}
    else:
        from volumerenderingproject_amd.distributed import TileFarm
        farm = TileFarm.for_renderer(r, W, H, rank, world, p, cam, tile=a.tile, device=device, batch=a.farm_batch)
        # rank 0's share of the tiles, chosen by measurement before the timed region (every peer
        # tile crosses an xGMI link into rank 0; a very large weight keeps the frame on rank 0)
        tuning = farm.tune(weights) if len(weights) > 1 else None
        if tuning is None:
            farm.set_plan(weights[0])

        def step():
            farm.step()

        drain = farm.drain
        farm_info = {"tiles_farmed": len(farm.tile_ids), "rank0_weight": farm.w0, "rank0_tiles": len(farm.lists[0]),
                     "frames_per_gather": farm.B, "tiles_per_rank": [len(x) for x in farm.lists],
                     "transport": "python TileFarm (torch.distributed gather)"}

    for _ in range(a.warmup):
        step()
    drain()
    if sub is not None:
        sub.begin()
    if capi:
        # libvr's polled wait (vr_options.comm_timeout_ms): a peer that never sends its tiles fails
        # the run with VR_ECOMM -- communicators aborted, exit 3 -- instead of hanging in a sync
        r.synchronize()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    # Device time of the timed region: one HIP event pair on the launch stream around all K steps
    # (ev1 after the drain, so the window holds every one of the K frames whatever K mod the batch;
    # frames_in_flight forks from and joins back into this stream).  / K = device time per frame.
    # N > 1: libvr's per-launch event pairs on every part isolate the march from gather + assembly.
    per_launch_events = n_gpus > 1
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if per_launch_events:
        r.timing_enable(True)
        r.timing_read(reset=True)
    traffic_parts = (list(range(n_gpus)) if group else [rank]) if (capi and n_gpus > 1) else []
    for q in traffic_parts:   # the transport's posted bytes over the timed steps (vr_group_traffic_read)
        r.group_traffic(q, reset=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(a.steps):
        step()
    drain()     # the frames of a last, partial batch (K mod --farm-batch): still inside the K steps
    ev1.record(stream)
    if capi:
        r.synchronize()   # (bounded: see the warm-up)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    frame_ms_device = ev0.elapsed_time(ev1) / a.steps
    if per_launch_events:
        # march time per frame and launches on this process's GPU(s): one-process groups report every
        # part (the max is the slowest GPU), torchrun ranks their own
        parts = range(n_gpus) if group else [None]
        kts = [r.timing_read(reset=True, rank=q) for q in parts]
        r.timing_enable(False)
        # summed march-launch durations per frame, per GPU (launches of frames in flight overlap, so
        # a sum can exceed the step: a per-GPU load figure, not a per-step cost)
        march_ms_by_rank = [k.total_ms / a.steps for k in kts]
        launches_rank0 = kts[0].launches
        t_launch_rank0 = kts[0].total_ms / max(1, kts[0].launches)
    else:
        march_ms_by_rank = None
        launches_rank0 = a.steps
        t_launch_rank0 = None
    # per frame: the tile bytes each rank posted to rank 0 and rank 0's total ingress, to set beside
    # DESIGN section 7's predicted table (the driver's SCALE line has no other view of the link)
    peer_traffic = read_peer_traffic(r, traffic_parts, n_gpus, group, dist, device, backend, world)
    kernel_ms_local = frame_ms_device
    if n_gpus == 1:
        # the march kernel's own mean launch duration (what rocprofv3 --kernel-trace reports): libvr's
        # per-launch HIP event pairs on each launch's stream, in an untimed pass of the same batches
        # (with two frames in flight launches overlap: a launch lasts longer than a frame's share)
        r.timing_enable(True)
        r.timing_read(reset=True)
        for _ in range(a.steps):
            step()
        drain()
        torch.cuda.synchronize()
        kt1 = r.timing_read(reset=True)
        r.timing_enable(False)
        t_launch_rank0 = kt1.total_ms / max(1, kt1.launches)
    if dist is not None:
        rdev = f"cuda:{device}" if backend == "nccl" else "cpu"
        t = torch.tensor([elapsed], dtype=torch.float64, device=rdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        k = torch.tensor([kernel_ms_local], dtype=torch.float64, device=rdev)
        dist.all_reduce(k, op=dist.ReduceOp.MAX)
        kernel_ms = float(k.item())
    else:
        kernel_ms = kernel_ms_local

    # BASELINE configs[3] / [4] under the same kind of context (every rank takes part)
    ex_cfgs = a.extra_configs if a.extra_configs is not None else ("c4,c5" if a.extra else "")
    cfg_extras = {}
    for cname in filter(None, (x.strip() for x in ex_cfgs.split(","))):
        cfg_extras[cname] = extra_config(cname, a, vr, group, capi, dist, rank, world, device, devices, n_gpus,
                                         stream, weights, backend)
    torch.cuda.set_stream(stream)
    r.set_stream(stream.cuda_stream)

    if rank == 0:
        ms_per_step = elapsed / a.steps * 1e3
        mrays = W * H * a.steps / elapsed / 1e6
        n_in = r.count_samples(p, cam)
        # the work the march actually did (roofline numerator): class gathers that touched memory
        # (1 B each) and samples evaluated, from the counting instantiation of the same kernel
        # variant over the same frame (vr_count_marched; outside the timed region)
        # (vr_count_work: VRC or TEST, the bytes at each gather's own width)
        work = r.count_work(p, cam)
        gathers, evaluated, gbytes = work["gathers"], work["samples"], work["bytes"]
        model_frame = 4 * n_in + 16 * W * H                           # SURVEY 8(d), exact march
        frame_write = 16 * W * H   # the launch's one certain HBM traffic (lower bound)
        # rank 0's march launches per frame (N > 1: its share of the frame's tiles)
        lpf = launches_rank0 / a.steps
        share = 1.0 if n_gpus == 1 else farm_info["rank0_tiles"] / max(1, farm_info["tiles_farmed"])
        traffic = None
        traffic_src = None
        try:
            tj = json.load(open(a.traffic_json))
            if tj.get("workload_key") == workload_key(a.volume, W, H, S, a.mode, flags, n_gpus, a.camera):
                traffic = tj.get("hbm_bytes_per_launch")
                traffic_src = os.path.relpath(a.traffic_json, ROOT)
        except Exception:
            pass
        bytes_launch = traffic if traffic else frame_write * share / max(lpf, 1e-9)
        bytes_frame = bytes_launch * lpf            # rank 0's march bytes per frame
        # step basis: rank 0's march bytes per frame over the device time per frame of the timed region
        achieved = bytes_frame / (frame_ms_device * 1e-3) / 1e9
        frac = achieved / HBM_PEAK_GBS
        if frac > 1.0:       # a byte model above the peak is not a fraction: never report it as one
            frac = None
        achieved_launch = bytes_launch / (t_launch_rank0 * 1e-3) / 1e9 if t_launch_rank0 else None
        # step basis like frac: the bytes the march needed for its work (1 B per class gather + the
        # 16 B/ray frame write) per frame over the device time per frame.  One GPU only (the count
        # is a whole frame; at N > 1 rank 0 marches a share of it)
        marched_bytes = gbytes + frame_write if gathers is not None else None
        achieved_marched = (marched_bytes / (frame_ms_device * 1e-3) / 1e9
                            if marched_bytes is not None and n_gpus == 1 else None)
        extra = None
        if n_gpus == 1 and a.extra:
            # the same frame under the reference's exact back-to-front blend (no ESS/ERT) and under
            # the oblique reset camera (utils.h:77-81), for transparency next to the headline value
            # (round 6: the Python TileFarm's one-GPU rate is no longer in the line -- VERDICT r5: it is
            # not the C-ABI path the N > 1 runs take; `--farm torch` still runs that farm)
            extra = {}
            # the headline view one vr_render per frame (no frames in flight: per-frame latency)
            for _ in range(3):
                r.render_device(p, cam, frame.data_ptr(), asynchronous=True)
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            for _ in range(a.steps):
                r.render_device(p, cam, frame.data_ptr(), asynchronous=True)
            torch.cuda.synchronize()
            extra["single_frame_mrays"] = round(W * H * a.steps / (time.perf_counter() - t1) / 1e6, 1)
            # the exact mode and the oblique camera through the same batched calls as the headline
            for name, pp, cc in [("exact_mode", vr.default_params(W, H, S, mode=mode, flags=0), cam),
                                 ("oblique_camera", p, vr.reset_camera())]:
                extra[name + "_mrays"] = batched_mrays(r, W, H, pp, [cc] * a.steps, frames_dev, B)
            if mode == vr.VR_MODE_VRC:
                extra.update(moving_camera(r, W, H, p, frames_dev, B, a.steps))
        cpu = None
        if a.cpu_baseline and n_gpus == 1:
            # the host cores this process may run on (os.sched_getaffinity: the GPU box's lease pins one
            # GPU's share of the machine, 16 cores, while os.cpu_count() is the whole machine's), capped
            # by OMP_NUM_THREADS when set (16 there)
            mt = cpu_cores()
            cpu = cpu_baseline(vol, cal, W, H, S, a.cpu_columns, implicit=a.volume in ("r512", "c5"), threads_mt=mt)
        rehearsal = group and len(set(devices)) < len(devices)
        if n_gpus == 1:
            parallelism = "screen-tiles1-capi-group" if capi else "single-gpu"
        elif group:
            parallelism = f"screen-tiles{n_gpus}-one-process" + ("-peer-copy-rehearsal" if rehearsal else "")
        else:
            parallelism = f"screen-tiles{n_gpus}" + ("" if backend == "nccl" else f"-{backend}-rehearsal")
        line = {
            "metric": "Mrays/sec + achieved-HBM-% on MNI152 1mm @ 1920x1080, 1/2/4/8 GPU",
            "value": round(mrays, 3),
            "unit": "Mrays/s",
            "n_gpus": n_gpus,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic stand-in volume (reference blob MNI152_T1_1mm missing); no network",
            "config": {
                "workload": f"{cfg_name}: {vname}, {W}x{H}, {S} samples/ray, mode {a.mode.upper()}, "
                            f"flags {a.flags}, " + ("default steady camera" if a.camera == "default" else
                                                    "oblique reset camera (utils.h:77-81)"),
                "width": W, "height": H, "samples_per_ray": S, "volume": vname,
                "parallelism": parallelism,
                **({"options": a.options} if a.options else {}),
                "submission": (f"vr_render_batch calls of up to {B} frames into a ring of {B} device frames; the first "
                               f"call of the timed region issues {a.lead} frames at once") if sub is not None and sub.lead
                              else (f"vr_render_batch calls of {B} frames" if sub is not None else None),
                "devices": devices,
                "tile": a.tile if n_gpus > 1 else None,
                "tiles_farmed": farm_info["tiles_farmed"] if farm_info else None,
                "rank0_weight": farm_info["rank0_weight"] if farm_info else None,
                "rank0_tiles": farm_info["rank0_tiles"] if farm_info else None,
                "rank0_weight_tuning_s": tuning if n_gpus > 1 else None,
                "frames_per_gather": farm_info["frames_per_gather"] if farm_info else None,
                "farm_transport": farm_info["transport"] if farm_info else None,
                "farm_fallback": farm_fallback,
                "tiles_per_rank": farm_info["tiles_per_rank"] if farm_info else None,
                # the rank-0 weight is tuned by measurement; when it keeps every tile on rank 0 the
                # other GPUs render nothing and the line is a one-GPU frame rate
                "ranks_rendering": (sum(1 for n in farm_info["tiles_per_rank"] if n) if farm_info else 1),
                "peer_traffic": peer_traffic,
                "design7_prediction": design7_prediction(
                    "c3" if (a.volume == "mni" and (W, H, S) == (1920, 1080, 500) and a.mode == "vrc"
                             and a.camera == "default" and a.flags == "ess,ert") else None, n_gpus),
                "n_in_dataset_samples": n_in,
            },
            "roofline": {
                "bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(frac, 5) if frac is not None else None, "traffic": traffic,
                "basis": "step: rank 0's march HBM bytes per frame / device time per frame (one HIP event pair "
                         "on the launch stream around the K timed steps, / K)",
                "bytes_per_launch": int(bytes_launch),
                "bytes_per_frame": int(bytes_frame),
                "bytes_source": f"PMC counters ({traffic_src})" if traffic else
                                "lower bound (no PMC file for this workload): the 16 B/ray frame write only",
                # (TEST views along the volume's z axis -- the default camera -- march plane by plane)
                "kernel": "vrc_march_kernel" if a.mode == "vrc" else
                          ("test_axis_kernel" if a.camera == "default" else "test_march_kernel"),
                "frame_ms_device": round(frame_ms_device, 5),
                "frame_ms_device_x_steps": round(frame_ms_device * a.steps, 5),
                "frame_ms_device_max_ranks": round(kernel_ms, 5),   # frame_ms_device, max over ranks
                "march_ms_per_frame_by_rank": ([round(x, 5) for x in march_ms_by_rank]
                                               if march_ms_by_rank else None),
                "launches_per_frame_rank0": round(lpf, 4),
                # secondary: the march kernel's mean launch duration (libvr's per-launch event pairs in an
                # untimed pass; what rocprofv3 --kernel-trace reports).  With frames in flight launches
                # overlap, so a launch lasts longer than a frame's share of the device time.
                "kernel_ms_mean": round(t_launch_rank0, 5) if t_launch_rank0 else None,
                "achieved_per_launch": round(achieved_launch, 2) if achieved_launch else None,
                "frac_per_launch": round(achieved_launch / HBM_PEAK_GBS, 5) if achieved_launch else None,
                "samples_marched": gathers,
                "samples_evaluated": evaluated,
                "gather_bytes": gbytes,
                "marched_bytes_per_frame": marched_bytes,
                "achieved_marched": round(achieved_marched, 2) if achieved_marched is not None else None,
                "frac_marched": round(achieved_marched / HBM_PEAK_GBS, 5) if achieved_marched is not None else None,
                "model_bytes_per_frame": int(model_frame * share),
                "model_gbs": round(model_frame * share / (frame_ms_device * 1e-3) / 1e9, 1),
                "note": "frac = achieved / peak on the step basis (the counters' bytes of rank 0's march launches "
                        "in one frame over the frame's device time), so every figure follows from the timed "
                        "run; kernel_ms_mean / frac_per_launch are per-launch secondaries.  frac_marched is the "
                        "work measure: marched_bytes_per_frame = the bytes of the class gathers the march issued "
                        "to memory at their own widths (gather_bytes: VRC 1 B per class byte; TEST 2 B per corner-"
                        "volume entry at the default TF, 4 B per corner-row dword; samples_marched = the gathers, "
                        "vr_count_work: ESS / ERT applied) + 16 B per ray, over the same "
                        "device time per frame.  model_* is SURVEY "
                        "8(d)'s exact-march byte model (4 B per in-dataset sample + 16 B per ray): ESS + ERT "
                        "skip most of those samples and the 1-B class gathers hit L1/L2, so it is reported for "
                        "reference only and exceeds the peak.",
            },
            "cpu_baseline": cpu,
            "extra": extra,
        }
        if cfg_extras:
            line["extra"] = dict(line["extra"] or {})
            for cname, res in cfg_extras.items():
                line["extra"][cname] = res
                if res.get("mrays") is not None:
                    line["extra"][f"{cname}_mrays"] = res["mrays"]
        print(json.dumps(line), file=result_out, flush=True)
    r.close()
    if dist is not None:
        dist.destroy_process_group()


class Submitter:
    """Steps -> vr_render_batch calls.  Frames go into a ring of B device frames, each call a run
    of consecutive ring slots (never wrapping), issued when the run reaches the ring's end or, for
    the first call of a region (begin()), when `lead` frames are pending: the GPU starts on the
    first frame while the host gathers the rest of the batch."""

    def __init__(self, r, p, cam, fptr, frame_bytes, B, lead):
        import volumerenderingproject_amd as vr
        self.r, self.p, self.fptr, self.fb, self.B = r, p, fptr, frame_bytes, B
        self.lead = lead if 0 < lead < B else 0
        self.cams = (vr.Camera * B)(*([cam] * B))
        self.pos = self.pending = 0
        # warm-up frames go in full calls (both streams of frames_in_flight see work before the
        # timed region); the lead call is for the timed region only (begin())
        self.started = True

    def begin(self):
        self.started = False

    def step(self):
        self.pending += 1
        if self.pos + self.pending == self.B or (not self.started and self.pending == self.lead):
            self.drain()

    def drain(self):
        if self.pending:
            out = None if self.fptr is None else self.fptr + self.pos * self.fb
            self.r.render_batch_device(self.p, self.cams, out, asynchronous=True, n=self.pending)
            self.pos = (self.pos + self.pending) % self.B
            self.pending = 0
            self.started = True


EXTRA_CONFIGS = {
    # name: (BASELINE.json configs index, volume, W, H, S)
    "c4": (3, "r512", 1920, 1080, 1024),
    "c5": (4, "c5", 3840, 2160, 4096),
}


def design7_prediction(name, n_gpus):
    """DESIGN section 7's predicted Mrays/s, rank-0 weight and tile bytes into rank 0 per frame for this
    config at this N (tools/scale_model.py over profiles/r6_scale/probe.json), for the SCALE line to
    be read against; None when the config has no prediction."""
    if name not in ("c3", "c4", "c5"):
        return None
    try:
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        import scale_model
        probe = json.load(open(os.path.join(ROOT, "profiles", "r6_scale", "probe.json")))
        p = scale_model.predict(probe[name], scale_model.STEADY_MS[name], n_gpus, 64e9)
        return {"mrays": round(p["mrays"], 1), "rank0_weight": p["w"], "bytes_into_rank0_per_frame": p["bytes_into_rank0"],
                "bound": p["bound"], "link_gbs_assumed": 64}
    except Exception as e:   # (the prediction never fails a bench line)
        return {"error": f"{type(e).__name__}: {e}"}


def read_peer_traffic(r, parts, n_gpus, group, dist, device, backend, world):
    """vr_group_traffic_read over the parts this process holds (reset): per frame, the tile bytes every
    rank posted to rank 0 and rank 0's ingress; torchrun ranks sum their own.  None on one GPU."""
    import torch
    if not parts:
        return None
    tr = {q: r.group_traffic(q, reset=True) for q in parts}
    frames = max(1, max(t[2] for t in tr.values()))
    sent = [0.0] * n_gpus
    for q, (tx, _rx, _fr) in tr.items():
        sent[q] = float(tx)
    into0 = float(tr[0][1]) if 0 in tr else 0.0
    if dist is not None and not group:
        v = torch.tensor(sent + [into0, float(frames)], dtype=torch.float64,
                         device=f"cuda:{device}" if backend == "nccl" else "cpu")
        dist.all_reduce(v, op=dist.ReduceOp.SUM)
        vals = [float(x) for x in v.cpu()]
        sent, into0 = vals[:n_gpus], vals[n_gpus]
        frames = max(1, int(round(vals[n_gpus + 1] / world)))
    return {"frames": frames, "bytes_into_rank0_per_frame": int(into0 / frames),
            "bytes_sent_per_frame_by_rank": [int(x / frames) for x in sent],
            "note": "tile bytes posted to the transport per frame (compact RGB: 12 B per pixel of every peer "
                    "tile); compare DESIGN section 7's predicted table"}


def extra_config(cname, a, vr, group, capi, dist, rank, world, device, devices, n_gpus, stream, weights, backend):
    """One BASELINE config beyond the headline (C4: the MNI stand-in resampled to 512^3 at 1920x1080,
    S = 1024; C5: the synthetic 2048^3 volume at 3840x2160, S = 4096; ESS + ERT, default camera),
    rendered through the same kind of context as the headline -- a one-GPU context, a one-process
    vr_create_multi group, or vr_create_rank ranks under torchrun -- with its own rank-0 weight
    tuning, warm-up and timed region (--steps / --warmup, barrier + synchronize on both sides, the
    max over ranks).  These are the configs where the screen-tile split can pay.
    --check-extras: one frame of the context against a fresh one-GPU context of the same volume,
    bitwise (N > 1: the farmed frame; C4 by default, C5 with --check-extras 2).
    Returns the result dict on rank 0 (every rank must call it)."""
    import torch
    from volumerenderingproject_amd import volumes
    cfg_i, volname, W, H, S = EXTRA_CONFIGS[cname]
    out = {"config": f"BASELINE configs[{cfg_i}]: {volname}, {W}x{H}, {S} samples/ray, ESS+ERT, default camera"}
    if n_gpus > 1 and not capi:
        out["skipped"] = "torch.distributed TileFarm fallback (libvr group not up)"
        return out
    shape = (512,) * 3 if volname == "r512" else (2048,) * 3

    def any_rank(flag):
        """True on every rank when it is true on one (a skip or an error decided on one rank
        alone let the others walk into the config's collectives, which then paired up wrongly)."""
        if dist is None or world <= 1:
            return bool(flag)
        t = torch.tensor([1.0 if flag else 0.0], dtype=torch.float64,
                         device=f"cuda:{device}" if backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return bool(t.item() > 0)

    why = None
    try:
        free, _ = torch.cuda.mem_get_info(device)
        # volume + context copy + classes + frames, and the axis views' leaf-column masks (up to
        # kLeafColsMax = 2048 leaves per axis): a one-bit-per-leaf occupancy, transient, and 3 nleaf^2
        # 64-bit masks (C5: 1 GiB + 100 MB)
        nleaf = 1 << max(0, (shape[0] - 1).bit_length())
        leafcols = (nleaf ** 3 / 8 + 3 * nleaf ** 2 * 8) if nleaf <= 2048 else 0
        need = 4 * shape[0] ** 3 * 2.6 + leafcols + 16 * W * H * (a.farm_batch + 2)
        if need > free:
            why = f"needs ~{need / 2**30:.1f} GiB, {free / 2**30:.1f} GiB free"
    except Exception as e:
        why = f"{type(e).__name__}: {e}"
    if any_rank(why is not None):
        out["skipped"] = why or "skipped: another rank lacks the memory"
        return out if rank == 0 else None
    why = None
    try:
        dvol = torch.empty(shape if (rank == 0 or not capi or group) else (1,), dtype=torch.float32,
                           device=f"cuda:{device}")
        if rank == 0:
            if volname == "r512":
                dvol.copy_(torch.from_numpy(volumes.resample_512(volumes.mni152_standin()[0])))
            else:
                vr.renderer.synthetic_volume(dvol.data_ptr(), shape[0], device=device,
                                             stream=torch.cuda.current_stream(device).cuda_stream)
        torch.cuda.synchronize()
    except Exception as e:
        why = f"{type(e).__name__}: {e}"
    if any_rank(why is not None):   # (before the id broadcast and vr_create_rank: every rank or none)
        out["error"] = why or "error on another rank while preparing the volume"
        return out if rank == 0 else None
    try:
        opts = bench_options(a, farm_tile=a.tile)
        if group:
            r = vr.VolumeRenderer(device_ptr=dvol.data_ptr(), shape=shape, cal_max=255.0, devices=devices, options=opts)
        elif capi and world > 1:
            cid = [vr.renderer.comm_unique_id() if rank == 0 else None]
            dist.broadcast_object_list(cid, src=0)
            r = vr.VolumeRenderer(device_ptr=dvol.data_ptr() if rank == 0 else None, shape=shape, cal_max=255.0,
                                  device=device, rank=rank, n_ranks=world, comm_id=cid[0], options=opts)
        else:
            r = vr.VolumeRenderer(device_ptr=dvol.data_ptr(), shape=shape, cal_max=255.0, device=device,
                                  options=bench_options(a))
        # (the check holds the volume and builds a second context: C4 by default, C5 with --check-extras 2)
        check = a.check_extras >= (2 if volname == "c5" else 1)
        ref_vol = dvol if (check and rank == 0) else None
        del dvol
        torch.cuda.empty_cache()
        r.set_stream(stream.cuda_stream)
        torch.cuda.set_stream(stream)
        p = vr.default_params(W, H, S, flags=vr.VR_FLAG_ESS | vr.VR_FLAG_ERT)
        cam = vr.default_camera(W, H)
        B = max(1, a.farm_batch)
        frames = torch.empty((B, W, H, 4), dtype=torch.float32, device=f"cuda:{device}") if rank == 0 else None
        fptr = frames.data_ptr() if frames is not None else None
        sub = Submitter(r, p, cam, fptr, W * H * 16, B, a.lead)
        tuning = None
        if n_gpus > 1:
            tuning = capi_tune(r, weights, sub.step, sub.drain, a.tile, dist, device, frames=B,
                               mkopt=lambda **k: bench_options(a, **k)) if len(weights) > 1 else None
            if tuning is None:
                r.set_options(bench_options(a, farm_tile=a.tile, farm_rank0_weight=weights[0]))
        for _ in range(max(1, a.warmup)):
            sub.step()
        sub.drain()
        r.synchronize()
        sub.begin()
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()
        if n_gpus > 1:
            r.timing_enable(True)
            r.timing_read(reset=True)
        tparts = (list(range(n_gpus)) if group else [rank]) if n_gpus > 1 else []
        for q in tparts:
            r.group_traffic(q, reset=True)
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        ev0.record(stream)
        for _ in range(a.steps):
            sub.step()
        sub.drain()
        ev1.record(stream)
        r.synchronize()
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0
        march = None
        if n_gpus > 1:
            parts = range(n_gpus) if group else [None]
            march = [r.timing_read(reset=True, rank=q).total_ms / a.steps for q in parts]
            r.timing_enable(False)
        if dist is not None:
            rdev = f"cuda:{device}" if backend == "nccl" else "cpu"
            t = torch.tensor([elapsed], dtype=torch.float64, device=rdev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            elapsed = float(t.item())
            if march is not None and not group:   # one process per GPU: every rank's own march time
                mt = torch.zeros(world, dtype=torch.float64, device=rdev)
                mt[rank] = march[0]
                dist.all_reduce(mt, op=dist.ReduceOp.SUM)
                march = [float(x) for x in mt.cpu()]
        peer_traffic = read_peer_traffic(r, tparts, n_gpus, group, dist, device, backend, world)
        tiles = [len(r.group_tiles(q)) for q in range(n_gpus)] if n_gpus > 1 else None
        out.update({
            "mrays": round(W * H * a.steps / elapsed / 1e6, 3),
            "ms_per_step": round(elapsed / a.steps * 1e3, 4),
            "frame_ms_device": round(ev0.elapsed_time(ev1) / a.steps, 5),
            "steps": a.steps, "warmup": max(1, a.warmup),
            "tiles_farmed": len(r.visible_tiles(p, cam, a.tile, a.tile)) if n_gpus > 1 else None,
            "tiles_per_rank": tiles,
            "ranks_rendering": sum(1 for n in tiles if n) if tiles else 1,
            "rank0_weight": float(r.options.farm_rank0_weight) if n_gpus > 1 else None,
            "rank0_weight_tuning_s": tuning,
            "march_ms_per_frame_by_rank": [round(x, 5) for x in march] if march else None,
            "peer_traffic": peer_traffic,
            "design7_prediction": design7_prediction(cname, n_gpus),
        })
        if ref_vol is not None:
            # the farmed frame against a one-GPU context of the same volume (rays are independent:
            # the split must not change a bit)
            r.render_device(p, cam, fptr, asynchronous=False)
            one = vr.VolumeRenderer(device_ptr=ref_vol.data_ptr(), shape=shape, cal_max=255.0, device=device,
                                    options=bench_options(a))
            one.set_stream(stream.cuda_stream)
            ref = torch.empty((W, H, 4), dtype=torch.float32, device=f"cuda:{device}")
            one.render_device(p, cam, ref.data_ptr(), asynchronous=False)
            torch.cuda.synchronize()
            out["bitwise_vs_one_gpu"] = bool(torch.equal(frames[0], ref))
            one.close()
            del ref
        elif check and capi and not group and rank != 0:
            r.render_device(p, cam, None, asynchronous=False)   # (the check's frame: every rank takes part)
        del ref_vol
        r.close()
        del frames
        torch.cuda.empty_cache()
    except Exception as e:   # an extra config never fails the headline line; say why it is missing
        if getattr(e, "code", None) == VR_ECOMM_STATUS:
            raise
        out["error"] = f"{type(e).__name__}: {e}"
    return out if rank == 0 else None


def bench_options(a, **kw):
    """vr_options_default, then --options overrides (A/B runs), then the bench's own fields."""
    import volumerenderingproject_amd as vr
    over = {}
    for item in filter(None, (x.strip() for x in a.options.split(","))):
        k, v = item.split("=")
        k = k.strip()
        over[k] = (float(v) if k == "farm_rank0_weight" else
                   [int(x) for x in v.split("x")] if k == "brick" else int(v))   # brick=4x4x8
    over.update(kw)
    return vr.default_options(**over)


def capi_tune(r, weights, step, drain, tile, dist, device, frames=12, mkopt=None):
    """Rank 0's tile share for libvr's multi-GPU context, chosen by measurement before the timed
    region: a few frames per candidate weight, the max over ranks of the wall time (all-reduced, so
    every rank picks the same weight).  Returns {weight: seconds}."""
    import torch
    import volumerenderingproject_amd as vr
    res = {}
    for w in weights:
        r.set_options(mkopt(farm_tile=tile, farm_rank0_weight=w))
        for _ in range(3):
            step()
        drain()
        r.synchronize()
        if dist is not None:
            dist.barrier()
        t0 = time.perf_counter()
        for _ in range(frames):
            step()
        drain()
        r.synchronize()
        dt = time.perf_counter() - t0
        if dist is not None:
            t = torch.tensor([dt], dtype=torch.float64, device=f"cuda:{device}")
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dt = float(t.item())
        res[float(w)] = dt
    best = min(res, key=lambda k: (res[k], k))
    r.set_options(mkopt(farm_tile=tile, farm_rank0_weight=best))
    return res


def workload_key(volume, W, H, S, mode, flags, world, camera="default"):
    """Key of a PMC traffic file (tools/pmc_traffic.py) for this workload."""
    return f"{volume}:{W}x{H}x{S}:{mode}:{flags}:n{world}" + ("" if camera == "default" else f":{camera}")


def batched_mrays(r, W, H, p, cams, frames_dev, B):
    """Mrays/s of rendering `cams` (one frame each) in vr_render_batch calls of B frames (after one
    untimed call)."""
    import torch
    import volumerenderingproject_amd as vr
    arr = (vr.Camera * len(cams))(*cams)
    r.render_batch_device(p, arr[:min(B, len(cams))], frames_dev.data_ptr(), asynchronous=True)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for i in range(0, len(cams), B):
        r.render_batch_device(p, arr[i:i + B], frames_dev.data_ptr(), asynchronous=True)
    torch.cuda.synchronize()
    return round(W * H * len(cams) / (time.perf_counter() - t1) / 1e6, 1)


def moving_camera(r, W, H, p, frames_dev, B, steps):
    """Frames the reference renders: it re-renders only when the camera moves (myApp.cu:879,
    pointMoved), so every frame is a new view.  Each step re-derives the camera with processInput's
    formulas (vr_camera_derive, myApp.cu:1106-1112) from a new position:
      orbit -- around the y axis in 360/steps-degree steps (mostly oblique views, general march);
      dolly -- along the z axis towards the volume (axis-aligned views, the per-view sample table
               rebuilt by every launch).
    No view repeats, so no per-view table is reused; the class volume stays resident in HBM."""
    import math
    import torch
    import volumerenderingproject_amd as vr
    cam0 = vr.default_camera(W, H)
    up = tuple(cam0.up)
    rsw, rsh = p.real_screen_width, p.real_screen_height
    out = {}
    for name, n in (("orbit", steps), ("dolly", steps)):
        cams = []
        for i in range(n + 3):
            if name == "orbit":
                t = 2 * math.pi * i / (n + 3)
                pos = (math.sin(t), 0.0, math.cos(t))
            else:
                pos = (0.0, 0.0, 1.0 - 0.2 * i / (n + 3))
            cams.append(vr.derive_camera(pos, up, rsw, rsh))
        out[f"moving_camera_{name}_mrays"] = batched_mrays(r, W, H, p, cams[3:], frames_dev, B)
    return out


def cpu_baseline(vol, cal, W, H, S, columns, implicit=False, threads_mt=0):
    """The reference CPU ray-cast path (myApp.cu:1401-1495) restated in oracle/, 1 thread, on
    `columns` evenly strided screen columns of the same W x H x S frame.  implicit: C4/C5, whose
    node pool (5.5 GB / 353 GB) the reference could not build; the closed-form lookup is used and
    the sample is bounded to about the same number of samples as at C3."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    oct_ = oracle.OracleOctree(vol, implicit=implicit)
    if implicit:
        columns = max(1, min(columns, int(columns * 1080 * 500 / (H * S))))
    tf = oracle.default_tf()
    p = oracle.params(W, H, S)
    cam = oracle.camera_default(W, H)
    xs = [int(i * W / columns) for i in range(columns)]
    rays = len(xs) * H
    res = {}
    for threads in (1, threads_mt):
        if threads == 1 or threads_mt > 1:
            t0 = time.perf_counter()
            oct_.render_cpu_path_columns(cal, tf, p, cam, xs, threads=threads)
            res[threads] = time.perf_counter() - t0
    dt = res[1]
    out = {"value": round(rays / dt / 1e6, 5), "unit": "Mrays/s", "cores": 1, "kind": "port",
           "sample": f"{len(xs)} strided columns x {H} rows ({rays} rays, {S} samples/ray) of the same frame, "
                     f"{dt:.1f} s, myApp.cu:1401-1495 semantics with the restated Octree.cu lookup"
                     + (" (closed form, no node pool)" if implicit else "")}
    if threads_mt > 1:   # the same sample on threads_mt host cores (OpenMP over columns)
        out["openmp"] = {"value": round(rays / res[threads_mt] / 1e6, 5), "cores": threads_mt,
                         "cores_source": "min(len(os.sched_getaffinity(0)), OMP_NUM_THREADS)",
                         "affinity_cores": len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else None,
                         "cpu": cpu_model()}
        if not implicit:
            # one full frame (every column) on the same threads_mt cores;
            # about 64 s on one core at C3, a few seconds on 16
            t0 = time.perf_counter()
            oct_.render_cpu_path_columns(cal, tf, p, cam, list(range(W)), threads=threads_mt)
            dt_full = time.perf_counter() - t0
            out["openmp"]["full_frame"] = {"value": round(W * H / dt_full / 1e6, 5), "seconds": round(dt_full, 2),
                                           "rays": W * H, "cores": threads_mt}
    return out


def cpu_cores():
    """Threads for the OpenMP CPU baseline and where the number comes from."""
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = os.cpu_count() or 1
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return min(aff, omp) if omp > 0 else aff


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def run():
    """main(), with a failed multi-GPU context (VR_ECOMM: an RCCL error or a wait past
    vr_options.comm_timeout_ms, communicators aborted by libvr) reported and exit status 3 -- no
    JSON line, no hang, no re-exec."""
    try:
        main()
    except Exception as e:   # (the renderer's VRError; imported lazily inside main)
        if getattr(e, "code", None) == VR_ECOMM_STATUS:
            print(f"bench.py: multi-GPU failure on rank {os.environ.get('RANK', '0')}: {e}", file=sys.stderr, flush=True)
            sys.stdout.flush()
            os._exit(3)   # (torch.distributed / RCCL teardown could block on the aborted peers)
        raise


VR_ECOMM_STATUS = -8


if __name__ == "__main__":
    run()
