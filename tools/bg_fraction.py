import sys, os
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import numpy as np
import volumerenderingproject_amd as vr
from volumerenderingproject_amd import volumes
vol, cal = volumes.mni152_standin()
W, H, S = 1920, 1080, 500
for cull, name, cam in [(c, n, cam) for c in (1, 2) for n, cam in (("default", vr.default_camera(W, H)),
                                                                 ("oblique", vr.reset_camera()))]:
    r = vr.VolumeRenderer(vol, cal, options=vr.default_options(cull=cull))
    p = vr.default_params(W, H, S, flags=3)
    fr = r.render(p, cam)
    bg = np.array(list(p.background), np.float32)[:3]
    isbg = np.all(fr[..., :3] == bg, axis=-1)
    T = 64
    ids = r.visible_tiles(p, cam, T, T)
    nty = -(-H // T)
    tot = bgc = 0
    for t in ids:
        tx, ty = divmod(int(t), nty)
        blk = isbg[tx*T:(tx+1)*T, ty*T:(ty+1)*T]
        tot += blk.size; bgc += blk.sum()
    print(f"cull={cull}", name, "visible tiles", len(ids), "pixels", tot, "background fraction in visible tiles", round(bgc/tot, 3), "frame bg fraction", round(isbg.mean(), 3))
    r.close()
