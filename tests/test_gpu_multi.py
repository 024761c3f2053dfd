"""Multi-GPU contexts behind the C-ABI (vr_create_multi / vr_create_rank).

On the one-GPU test box: a one-GPU group renders through the farmed path (visible tiles -> compact
RGB tiles -> assembly) and must equal vr_render bitwise; device lists that repeat the GPU rehearse
the N-rank plan (peer-copy transport: RCCL refuses two ranks on one device) with the same bitwise
bar; a one-rank RCCL communicator (vr_comm_unique_id + vr_create_rank) exercises the RCCL create /
broadcast path.  Rays are independent (kernel.cu:205-209), so any tile deal gives the one-GPU frame.
"""
import numpy as np
import pytest

import volumerenderingproject_amd as vr
from volumerenderingproject_amd import distributed, renderer

pytestmark = pytest.mark.gpu

E, T = vr.VR_FLAG_ESS, vr.VR_FLAG_ERT


def frames(r, cams, W, H, S, flags, mode=vr.VR_MODE_VRC):
    return [r.render(vr.default_params(W, H, S, mode=mode, flags=flags), c) for c in cams]


def cameras(W, H):
    return [vr.default_camera(W, H), vr.reset_camera(),
            vr.derive_camera((0.6, 0.3, 0.74), tuple(vr.default_camera(W, H).up), 2.0, 2.0 * H / W)]


@pytest.mark.parametrize("devices,w0", [([0], 1.0), ([0, 0], 1.0), ([0, 0, 0], 3.0), ([0, 0, 0, 0, 0, 0, 0, 0], 1.5)])
def test_group_equals_one_gpu(mni_standin, devices, w0):
    vol, cal = mni_standin
    W, H, S = 700, 500, 300
    one = vr.VolumeRenderer(vol, cal, device=0)
    g = vr.VolumeRenderer(vol, cal, devices=devices, options=vr.default_options(farm_rank0_weight=w0))
    n, rank, transport = g.group
    assert (n, rank) == (len(devices), 0)
    assert transport == (renderer.VR_TRANSPORT_NONE if len(devices) == 1 else renderer.VR_TRANSPORT_PEER_COPY)
    cams = cameras(W, H)
    for flags in (0, E, E | T):
        for mode in (vr.VR_MODE_VRC, vr.VR_MODE_TEST):
            a = frames(one, cams, W, H, S, flags, mode)
            b = frames(g, cams, W, H, S, flags, mode)
            for x, y in zip(a, b):
                assert np.array_equal(x, y), (flags, mode)
    # the deal: rank 0 weighted, interleaved, a partition of the visible tiles (distributed.py's statement)
    p = vr.default_params(W, H, S, flags=E | T)
    ids = one.visible_tiles(p, cams[1], 64, 64)
    g.render(p, cams[1])
    lists = distributed.weighted_lists(ids, len(devices), w0)
    for r in range(len(devices)):
        assert list(g.group_tiles(r)) == lists[r]
    one.close()
    g.close()


def test_group_async_frames_and_tf_update(mni_standin):
    """Back-to-back asynchronous frames of a moving camera into distinct device frames (buffers
    reused across frames must not race), then a TF change applied to every part of the group."""
    import torch
    vol, cal = mni_standin
    W, H, S = 640, 360, 400
    one = vr.VolumeRenderer(vol, cal, device=0)
    g = vr.VolumeRenderer(vol, cal, devices=[0, 0, 0])
    up = tuple(vr.default_camera(W, H).up)
    cams = [vr.derive_camera((np.sin(t), 0.0, np.cos(t)), up, 2.0, 2.0 * H / W) for t in np.linspace(0, 1.2, 6)]
    p = vr.default_params(W, H, S, flags=E | T)
    outs = [torch.empty((W, H, 4), dtype=torch.float32, device="cuda:0") for _ in cams]
    for c, o in zip(cams, outs):
        g.render_device(p, c, o.data_ptr(), asynchronous=True)
    g.synchronize()
    for c, o in zip(cams, outs):
        assert np.array_equal(o.cpu().numpy(), one.render(p, c))
    tf = [(0.0, 1.0, (0, 0, 0, 0)), (40 / 255, 90 / 255, (0.9, 0.8, 0.1, 0.5)), (100 / 255, 200 / 255, (0.1, 0.4, 0.9, 0.2))]
    one.set_transfer_function(tf)
    g.set_transfer_function(tf)
    for c in cams[:2]:
        assert np.array_equal(g.render(p, c), one.render(p, c))
    one.close()
    g.close()


def test_group_options_replan(avg152):
    vol, cal = avg152
    W, H, S = 300, 300, 200
    one = vr.VolumeRenderer(vol, cal, device=0)
    g = vr.VolumeRenderer(vol, cal, devices=[0, 0])
    p = vr.default_params(W, H, S, flags=E | T)
    cam = vr.default_camera(W, H)
    ref = one.render(p, cam)
    for tile, w0 in ((32, 1.0), (128, 4.0), (16, 1e6)):
        g.set_options(vr.default_options(farm_tile=tile, farm_rank0_weight=w0))
        assert np.array_equal(g.render(p, cam), ref)
        ids = one.visible_tiles(p, cam, tile, tile)
        assert sorted(list(g.group_tiles(0)) + list(g.group_tiles(1))) == list(ids)
    with pytest.raises(vr.VRError):
        g.set_options(vr.default_options(farm_tile=24))
    one.close()
    g.close()


def test_rank_context_rccl_one_rank(avg152):
    """vr_comm_unique_id + vr_create_rank with one rank: RCCL communicator init and the volume
    broadcast run for real; the frame equals vr_render's."""
    vol, cal = avg152
    W, H, S = 200, 150, 120
    cid = renderer.comm_unique_id()
    assert len(cid) == renderer.VR_COMM_ID_BYTES
    g = vr.VolumeRenderer(vol, cal, device=0, rank=0, n_ranks=1, comm_id=cid)
    assert g.group[:2] == (1, 0)
    one = vr.VolumeRenderer(vol, cal, device=0)
    for cam in (vr.default_camera(W, H), vr.reset_camera()):
        for flags in (0, E | T):
            p = vr.default_params(W, H, S, flags=flags)
            assert np.array_equal(g.render(p, cam), one.render(p, cam))
    g.close()
    one.close()


@pytest.mark.parametrize("kind", ["peer_copy", "rccl_one_rank"])
def test_group_wait_past_deadline_fails_loudly(avg152, kind):
    """Failure detection: a part whose stream stays busy past vr_options.comm_timeout_ms
    -- here a torch.cuda._sleep queued ahead of the march on rank 0's stream, standing in for a peer
    that never sends -- fails the call with VR_ECOMM (communicators aborted: the one-rank group has a
    real RCCL communicator) instead of blocking; later calls fail the same way, and the context is
    destroyable once the stream has drained."""
    import time
    import torch
    vol, cal = avg152
    W, H, S = 128, 96, 64
    opt = vr.default_options(comm_timeout_ms=300)
    if kind == "peer_copy":
        g = vr.VolumeRenderer(vol, cal, devices=[0, 0], options=opt)
    else:
        g = vr.VolumeRenderer(vol, cal, device=0, rank=0, n_ranks=1, comm_id=renderer.comm_unique_id(), options=opt)
    p = vr.default_params(W, H, S, flags=E | T)
    cam = vr.default_camera(W, H)
    out = torch.empty((W, H, 4), dtype=torch.float32, device="cuda:0")
    st = torch.cuda.Stream(device=0)
    g.set_stream(st.cuda_stream)
    g.render_device(p, cam, out.data_ptr())            # healthy first (and the stream's caches built)
    with torch.cuda.stream(st):
        torch.cuda._sleep(4_000_000_000)               # ~2 s of GPU cycles ahead of the march
    t0 = time.perf_counter()
    with pytest.raises(vr.VRError) as e:
        g.render_device(p, cam, out.data_ptr())
    waited = time.perf_counter() - t0
    assert e.value.code == -8 and "timed out" in str(e.value), str(e.value)
    # the deadline, not the sleep -- except that ncclCommAbort itself waits for the work already
    # queued on the communicator's stream (here the ~2 s sleep ahead of the march)
    assert 0.25 < waited < (1.5 if kind == "peer_copy" else 4.0), waited
    with pytest.raises(vr.VRError) as e2:
        g.render_device(p, cam, out.data_ptr())
    assert e2.value.code == -8 and "failed earlier" in str(e2.value)
    st.synchronize()
    g.set_stream(0)
    g.close()                                          # destroy drains and frees without error


def test_bad_group_arguments(avg152):
    vol, cal = avg152
    with pytest.raises(vr.VRError) as e:
        vr.VolumeRenderer(vol, cal, devices=[0, 99])
    assert e.value.code == -6
    with pytest.raises(vr.VRError):
        vr.VolumeRenderer(vol, cal, devices=[0], options=vr.default_options(farm_rank0_weight=0.0))


@pytest.mark.parametrize("devices", [None, [0], [0, 0, 0]])
def test_render_batch_equals_frames(mni_standin, devices):
    """vr_render_batch: n frames of a moving camera (each its own visible-tile list and deal), one
    RCCL group / peer-copy batch and one scatter per call, equal bitwise to n vr_render calls; host
    and device outputs, batches of different lengths reusing the double buffers back to back."""
    import torch
    vol, cal = mni_standin
    W, H, S = 640, 360, 400
    one = vr.VolumeRenderer(vol, cal, device=0)
    g = one if devices is None else vr.VolumeRenderer(vol, cal, devices=devices)
    up = tuple(vr.default_camera(W, H).up)
    cams = [vr.derive_camera((np.sin(t), 0.2 * t, np.cos(t)), up, 2.0, 2.0 * H / W) for t in np.linspace(0, 2.0, 7)]
    cams.append(vr.default_camera(W, H))
    for flags, mode in ((E | T, vr.VR_MODE_VRC), (0, vr.VR_MODE_VRC), (E, vr.VR_MODE_TEST)):
        p = vr.default_params(W, H, S, mode=mode, flags=flags)
        ref = [one.render(p, c) for c in cams]
        host = g.render_batch(p, cams)
        assert host.shape == (len(cams), W, H, 4)
        for i, r in enumerate(ref):
            assert np.array_equal(host[i], r), (flags, mode, i)
        dev = torch.empty((len(cams), W, H, 4), dtype=torch.float32, device="cuda:0")
        g.render_batch_device(p, cams[:3], dev.data_ptr(), asynchronous=True)
        g.render_batch_device(p, cams[3:], dev[3:].data_ptr(), asynchronous=True)
        g.synchronize()
        got = dev.cpu().numpy()
        for i, r in enumerate(ref):
            assert np.array_equal(got[i], r), (flags, mode, i)
    with pytest.raises(vr.VRError):
        g.render_batch(vr.default_params(W, H, S), [])
    if g is not one:
        g.close()
    one.close()


def test_render_batch_many_views_trims_plan_cache(avg152):
    """More distinct views than the group's plan cache holds (64), within one batch and across
    batches: every frame still equals its own vr_render bitwise (the cache is trimmed only between
    batches, never under a batch's plans)."""
    import math
    vol, cal = avg152
    W, H, S = 160, 120, 150
    one = vr.VolumeRenderer(vol, cal, device=0)
    g = vr.VolumeRenderer(vol, cal, devices=[0, 0, 0], options=vr.default_options(farm_tile=32))
    p = vr.default_params(W, H, S, flags=E | T)
    up = tuple(vr.default_camera(W, H).up)
    cams = [vr.derive_camera((math.sin(t), 0.25 * math.sin(3 * t), math.cos(t)), up, p.real_screen_width,
                             p.real_screen_height) for t in np.linspace(0.0, 2 * math.pi, 90, endpoint=False)]
    ref = [one.render(p, c) for c in cams]
    for lo, hi in ((0, 70), (70, 90), (10, 40), (0, 90)):
        got = g.render_batch(p, cams[lo:hi])
        for i in range(hi - lo):
            assert np.array_equal(got[i], ref[lo + i]), (lo, i)
    g.close()
    one.close()


@pytest.mark.parametrize("fif", [1, 3])
def test_frames_in_flight_join_the_callers_stream(mni_standin, fif):
    """vr_render_batch with 1 + fif streams in flight (frame f on stream f mod (1 + fif), the others
    libvr's auxiliary streams): work queued afterwards on the caller's stream sees every frame
    complete, without a device-wide sync; frames equal the one-stream batch (frames_in_flight = 0)
    bitwise."""
    import math
    import torch
    vol, cal = mni_standin
    W, H, S = 640, 360, 400
    a = vr.VolumeRenderer(vol, cal, device=0, options=vr.default_options(frames_in_flight=fif))
    b = vr.VolumeRenderer(vol, cal, device=0, options=vr.default_options(frames_in_flight=0))
    p = vr.default_params(W, H, S, flags=E | T)
    up = tuple(vr.default_camera(W, H).up)
    cams = [vr.derive_camera((math.sin(t), 0.0, math.cos(t)), up, p.real_screen_width, p.real_screen_height)
            for t in np.linspace(0.0, 1.5, 6)]
    st = torch.cuda.Stream(device=0)
    a.set_stream(st.cuda_stream)
    out = torch.zeros((len(cams), W, H, 4), dtype=torch.float32, device="cuda:0")
    a.render_batch_device(p, cams, out.data_ptr(), asynchronous=True)
    with torch.cuda.stream(st):
        sums = out.sum(dim=(1, 2, 3))   # ordered after the batch on the caller's stream only
        snap = out.clone()
    st.synchronize()
    ref = b.render_batch(p, cams)
    for i in range(len(cams)):
        assert np.array_equal(snap[i].cpu().numpy(), ref[i]), i
        assert abs(float(sums[i]) - float(ref[i].sum(dtype=np.float64))) < 1e-3 * W * H
    a.set_stream(0)
    a.close()
    b.close()


def test_moving_camera_group_planned_on_the_device(mni_standin):
    """A 64-view orbit through a devices=[0, 0, 0] group in asynchronous batches of 8 (the reference
    re-renders on every camera move, myApp.cu:879): frames bitwise equal to vr_render, and no host
    synchronisation per frame -- with the GPU held busy by a long kernel queued ahead on the group's
    stream, every batch call returns while that kernel still runs (the plan is uploaded
    asynchronously and expanded on the device, vr_multi.cpp group_render).  Host time per frame is
    printed for DESIGN section 7."""
    import math
    import time
    import torch
    vol, cal = mni_standin
    W, H, S = 640, 360, 300
    one = vr.VolumeRenderer(vol, cal, device=0)
    g = vr.VolumeRenderer(vol, cal, devices=[0, 0, 0])
    p = vr.default_params(W, H, S, flags=E | T)
    up = tuple(vr.default_camera(W, H).up)
    cams = [vr.derive_camera((math.sin(t), 0.3 * math.sin(2 * t), math.cos(t)), up, p.real_screen_width,
                             p.real_screen_height) for t in np.linspace(0.0, 2 * math.pi, 64, endpoint=False)]
    st = torch.cuda.Stream(device=0)
    g.set_stream(st.cuda_stream)
    out = torch.empty((64, W, H, 4), dtype=torch.float32, device="cuda:0")
    g.render_batch_device(p, cams[:8], out.data_ptr(), asynchronous=True)   # warm: buffers, events
    g.synchronize()
    with torch.cuda.stream(st):
        torch.cuda._sleep(2_000_000_000)   # ~1 s of spinning ahead of the batches on this stream
    for b in range(0, 64, 8):
        g.render_batch_device(p, cams[b:b + 8], out[b].data_ptr(), asynchronous=True)
    busy = not st.query()
    g.synchronize()
    assert busy, "a batch call waited for the GPU"
    got = out.cpu().numpy()
    # host time per frame with the GPU free (the planning arithmetic and the launches)
    t0 = time.perf_counter()
    for b in range(0, 64, 8):
        g.render_batch_device(p, cams[b:b + 8], out[b].data_ptr(), asynchronous=True)
    host = time.perf_counter() - t0
    g.synchronize()
    print(f"host time per frame (64 new views, 3 parts, batches of 8): {host / 64 * 1e6:.1f} us")
    for i, c in enumerate(cams):
        assert np.array_equal(got[i], one.render(p, c)), i
    g.set_stream(0)
    g.close()
    one.close()


def _n_gpus():
    import torch
    return torch.cuda.device_count()


@pytest.mark.parametrize("n", [2, 4, 8])
def test_rccl_group_distinct_gpus(mni_standin, n):
    """vr_create_multi over n distinct GPUs (ncclCommInitAll, ncclBroadcast, grouped ncclSend /
    ncclRecv into GPU 0): moving-camera batches equal one-GPU frames bitwise.  Needs n GPUs (the
    driver's 8-GPU node; skipped on the one-GPU box)."""
    import torch
    if _n_gpus() < n:
        pytest.skip(f"needs {n} GPUs")
    vol, cal = mni_standin
    W, H, S = 640, 360, 500
    one = vr.VolumeRenderer(vol, cal, device=0)
    g = vr.VolumeRenderer(vol, cal, devices=list(range(n)), options=vr.default_options(farm_rank0_weight=1.0))
    assert g.group[2] == renderer.VR_TRANSPORT_RCCL
    cams = cameras(W, H) * 3
    for flags in (E | T, 0):
        p = vr.default_params(W, H, S, flags=flags)
        out = torch.empty((len(cams), W, H, 4), dtype=torch.float32, device="cuda:0")
        for _ in range(3):
            g.render_batch_device(p, cams, out.data_ptr(), asynchronous=True)
        g.synchronize()
        got = out.cpu().numpy()
        for f, c in enumerate(cams):
            assert np.array_equal(got[f], one.render(p, c)), (flags, f)
    assert sum(len(g.group_tiles(q)) > 0 for q in range(n)) > 1   # the tiles really were farmed
    one.close()
    g.close()


@pytest.mark.parametrize("n", [2, 4])
def test_rccl_ranks_equal_one_gpu(n):
    """vr_create_rank with n one-GPU processes (torchrun; the RCCL id over gloo): moving-camera
    batches gathered into rank 0 equal one-GPU frames bitwise (tests/mgpu/rccl_ranks.py).  Needs n
    GPUs (skipped on the one-GPU box)."""
    import os
    import subprocess
    import sys
    if _n_gpus() < n:
        pytest.skip(f"needs {n} GPUs")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
                        "--master-addr", "127.0.0.1", "--master-port", str(29700 + n),
                        os.path.join(root, "tests", "mgpu", "rccl_ranks.py")],
                       capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0 and "RCCL_RANKS_OK" in r.stdout, r.stdout[-3000:] + r.stderr[-3000:]
