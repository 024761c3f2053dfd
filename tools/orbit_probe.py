"""Orbit frames: wall time per frame, host enqueue time, and per-view kernel time moving vs static (HIP events)."""
import math, time, sys, os
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import torch
import volumerenderingproject_amd as vr
from volumerenderingproject_amd import volumes
vol, cal = volumes.mni152_standin()
W, H, S = 1920, 1080, 500
r = vr.VolumeRenderer(vol, cal)
st = torch.cuda.Stream(); torch.cuda.set_stream(st); r.set_stream(st.cuda_stream)
p = vr.default_params(W, H, S, flags=3)
up = tuple(vr.default_camera(W, H).up)
frame = torch.empty((W, H, 4), device="cuda")
n = 60
cams = [vr.derive_camera((math.sin(2*math.pi*i/n), 0.0, math.cos(2*math.pi*i/n)), up, p.real_screen_width, p.real_screen_height) for i in range(n)]
for c in cams[:3]: r.render_device(p, c, frame.data_ptr(), True)
torch.cuda.synchronize()
# moving: wall
t0 = time.perf_counter()
for c in cams: r.render_device(p, c, frame.data_ptr(), True)
torch.cuda.synchronize(); wall = (time.perf_counter() - t0) / n
# host enqueue cost only (GPU may lag)
t0 = time.perf_counter()
for c in cams: r.render_device(p, c, frame.data_ptr(), True)
host = (time.perf_counter() - t0) / n
torch.cuda.synchronize()
# kernel times per view: static repeats with events
r.timing_enable(True); r.timing_read(reset=True)
for c in cams: r.render_device(p, c, frame.data_ptr(), True)
kt = r.timing_read(reset=True)
ks = []
for c in cams:
    for _ in range(3): r.render_device(p, c, frame.data_ptr(), True)
    r.timing_read(reset=True)
    for _ in range(3): r.render_device(p, c, frame.data_ptr(), True)
    ks.append(r.timing_read(reset=True).total_ms / 3)
print(f"moving wall {wall*1e6:.1f} us/frame, host enqueue {host*1e6:.1f} us/frame, moving kernel {kt.total_ms/kt.launches*1e3:.1f} us, static kernel mean {sum(ks)/len(ks)*1e3:.1f} us min {min(ks)*1e3:.1f} max {max(ks)*1e3:.1f}")
