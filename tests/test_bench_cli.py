"""bench.py's GPU-count contract, checked before any GPU work (no GPU needed).

The driver runs `python bench.py --gpus N` (one process) and `torchrun --nproc-per-node N bench.py
--gpus N` (one rank per GPU).  An N-GPU line must come from N GPUs: a plain run on a machine with
fewer GPUs, a WORLD_SIZE that disagrees with --gpus, or a --devices list of the wrong length stops
with a message and exit status 2 instead of printing a line with the wrong n_gpus.  Also the
multi-GPU C-ABI's argument checks that need no GPU (mixed device lists, bad dims)."""
import ctypes as C
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT


def run_bench(args, env_extra=None):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                          env=env, timeout=120)


def gpu_count():
    import torch
    return torch.cuda.device_count()


def test_more_gpus_than_present_fails_loudly():
    n = gpu_count()
    r = run_bench(["--gpus", str(n + 1), "--steps", "1", "--warmup", "0"])
    assert r.returncode == 2, r.stderr
    assert "refusing to report an N-GPU line" in r.stderr
    assert r.stdout.strip() == ""   # no JSON line


def test_world_size_must_match_gpus():
    r = run_bench(["--gpus", "1"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2 and "WORLD_SIZE=2" in r.stderr
    r = run_bench(["--gpus", "2", "--devices", "0,0"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2 and "--devices is for one-process groups" in r.stderr


def test_devices_list_must_match_gpus():
    r = run_bench(["--gpus", "3", "--devices", "0,0"])
    assert r.returncode == 2 and "--devices lists 2 GPUs" in r.stderr
    r = run_bench(["--gpus", "0"])
    assert r.returncode == 2


def test_workload_keys_per_gpu_count():
    sys.path.insert(0, ROOT)
    import bench
    k1 = bench.workload_key("mni", 1920, 1080, 500, "vrc", 3, 1)
    k8 = bench.workload_key("mni", 1920, 1080, 500, "vrc", 3, 8)
    assert k1 != k8 and k1.endswith(":n1") and k8.endswith(":n8")


def test_mixed_device_list_rejected_before_any_gpu_work():
    """{0, 1, 1} would need RCCL between GPUs 0 and 1 and peer copies on GPU 1 at once: VR_EINVAL,
    decided from the list alone (the ADVICE r2 finding: its peer-copy events would sit on another
    GPU's stream)."""
    from volumerenderingproject_amd import renderer as R
    tf = R._tf_array(R.default_transfer_function())
    v = np.zeros((4, 4, 4), np.float32)
    ctx = C.c_void_p()
    for devs in ([0, 1, 1], [1, 0, 0, 2]):
        d = (C.c_int32 * len(devs))(*devs)
        rc = R.lib().vr_create_multi_ex(v.ctypes.data_as(C.c_void_p), 0, 4, 4, 4, 255.0, tf, 4, d, len(devs), None,
                                        C.byref(ctx))
        assert rc == -1 and not ctx.value, devs
        assert b"repeats one GPU" in R.lib().vr_strerror(rc)


@pytest.mark.parametrize("dims", [(0, 4, 4), (4, -1, 4), (1 << 40, 1 << 20, 1 << 10)])
def test_bad_dims_rejected_before_any_gpu_work(dims):
    from volumerenderingproject_amd import renderer as R
    tf = R._tf_array(R.default_transfer_function())
    v = np.zeros(8, np.float32)
    ctx = C.c_void_p()
    d = (C.c_int32 * 2)(0, 0)
    rc = R.lib().vr_create_multi_ex(v.ctypes.data_as(C.c_void_p), 0, *dims, 255.0, tf, 4, d, 2, None, C.byref(ctx))
    assert rc in (-1, -7) and not ctx.value
    cid = (C.c_uint8 * R.VR_COMM_ID_BYTES)()
    rc = R.lib().vr_create_rank(v.ctypes.data_as(C.c_void_p), 0, *dims, 255.0, tf, 4, 0, 0, 2, cid, None,
                                C.byref(ctx))
    assert rc in (-1, -7) and not ctx.value   # before ncclCommInitRank: no peer is left waiting


def test_design7_prediction_model():
    """DESIGN section 7's prediction (tools/scale_model.py over the committed one-GPU probe): N = 1 is
    the measured one-GPU rate, no config loses by adding GPUs (the tuner can keep every tile on rank
    0), C5 -- the longest march against its tile bytes -- gains the most, and the tile bytes into
    rank 0 per frame are whole 64 x 64 x 12 B tiles' worth or less."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import scale_model
    probe = json.load(open(os.path.join(ROOT, "profiles", "r6_scale", "probe.json")))
    gain = {}
    for name in ("c3", "c4", "c5"):
        one = scale_model.predict(probe[name], scale_model.STEADY_MS[name], 1, 64e9)
        assert abs(one["ms"] - scale_model.STEADY_MS[name]) < 1e-9
        prev = one["mrays"]
        for n in (2, 4, 8):
            p = scale_model.predict(probe[name], scale_model.STEADY_MS[name], n, 64e9)
            assert p["mrays"] >= prev * 0.999
            assert 0 <= p["bytes_into_rank0"] <= probe[name]["visible_tiles_64"] * 64 * 64 * 12
            prev = p["mrays"]
        gain[name] = prev / one["mrays"]
    assert gain["c5"] > gain["c4"] > gain["c3"] >= 1.0
