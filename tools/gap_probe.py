import time, sys, os
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import torch
import volumerenderingproject_amd as vr
from volumerenderingproject_amd import volumes
vol, cal = volumes.mni152_standin()
r = vr.VolumeRenderer(vol, cal, device=0)
W, H, S = 1920, 1080, 500
p = vr.default_params(W, H, S, flags=vr.VR_FLAG_ESS | vr.VR_FLAG_ERT)
cam = vr.default_camera(W, H)
st = torch.cuda.current_stream()
r.set_stream(st.cuda_stream)
fr = torch.empty((W, H, 4), dtype=torch.float32, device="cuda:0")
def run(n, timing):
    r.timing_enable(timing)
    r.timing_read(reset=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        r.render_device(p, cam, fr.data_ptr(), asynchronous=True)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / n * 1e3
    kt = r.timing_read(reset=True) if timing else None
    return dt, (kt.total_ms / kt.launches if kt and kt.launches else None)
for _ in range(3):
    run(20, False)
for timing in (False, True, False, True):
    print("timing", timing, run(200, timing))
# host cost of one call (no GPU wait)
r.timing_enable(False)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(200):
    r.render_device(p, cam, fr.data_ptr(), asynchronous=True)
t1 = time.perf_counter()
torch.cuda.synchronize()
print("host us per call (enqueue only, may block)", (t1 - t0) / 200 * 1e6)
