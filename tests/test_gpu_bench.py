"""bench.py end to end on the GPU: the one-process N-GPU path (vr_create_multi) and the accounting.

`python bench.py --gpus N` drives N GPUs from one process (one ncclCommInitAll, the
volume broadcast, one tile-gather group per batch, all inside libvr).  On the one-GPU test box the
N-part plan runs with --devices 0,0 (peer-copy transport, labelled a rehearsal); a plain --gpus 2
there must fail instead of printing a one-GPU line.  BASELINE.json metric: "1/2/4/8 GPU";
the reference renders on device 0 only (kernel.cu:885).
"""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def bench(args, timeout=300):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                       env=env, timeout=timeout)
    return r


def line_of(r):
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


def test_one_process_two_part_group_line():
    r = bench(["--gpus", "2", "--devices", "0,0", "--steps", "20", "--warmup", "4", "--cpu-baseline", "0",
               "--extra", "0", "--rank0-weights", "1,3"])
    L = line_of(r)
    c = L["config"]
    assert L["n_gpus"] == 2 and L["steps"] == 20
    assert c["parallelism"] == "screen-tiles2-one-process-peer-copy-rehearsal"
    assert c["devices"] == [0, 0]
    assert len(c["tiles_per_rank"]) == 2 and sum(c["tiles_per_rank"]) == c["tiles_farmed"] > 0
    assert c["ranks_rendering"] in (1, 2)
    assert "vr_create_multi" in c["farm_transport"] and "hipMemcpyPeerAsync" in c["farm_transport"]
    assert sorted(float(k) for k in c["rank0_weight_tuning_s"]) == [1.0, 3.0]
    rf = L["roofline"]
    assert rf["frame_ms_device"] > 0 and rf["frame_ms_device_max_ranks"] >= rf["frame_ms_device"] * 0.9999
    assert L["value"] > 0


def test_more_gpus_than_the_box_has_fails():
    import torch
    n = torch.cuda.device_count()
    r = bench(["--gpus", str(n + 1), "--steps", "4", "--warmup", "1", "--cpu-baseline", "0", "--extra", "0"])
    assert r.returncode == 2
    assert "refusing to report an N-GPU line" in r.stderr
    assert not [x for x in r.stdout.splitlines() if x.startswith("{")]


def test_one_gpu_accounting_follows_from_the_timed_run():
    """--steps 20 with batches of 8 (20 mod 8 != 0): the event window holds all 20 frames, the device
    time per step (one event pair inside the wall-clock window) is at most the wall time per step,
    frac is bytes per frame over that time, and frac_marched is the counted work over the same time."""
    r = bench(["--steps", "20", "--warmup", "5", "--cpu-baseline", "0", "--extra", "0"])
    L = line_of(r)
    rf = L["roofline"]
    assert L["n_gpus"] == 1 and L["config"]["parallelism"] == "single-gpu"
    assert rf["frame_ms_device"] <= L["ms_per_step"] * 1.0001
    W, H = L["config"]["width"], L["config"]["height"]
    assert 0 < rf["samples_marched"] <= rf["samples_evaluated"] <= W * H * L["config"]["samples_per_ray"]
    assert rf["samples_marched"] <= L["config"]["n_in_dataset_samples"]   # ESS + ERT skip, never add
    assert rf["marched_bytes_per_frame"] == rf["samples_marched"] + 16 * W * H
    assert 0 < rf["frac_marched"] <= 1.0
    assert abs(rf["frac_marched"] - rf["marched_bytes_per_frame"] / (rf["frame_ms_device"] * 1e-3) / 1e9
               / rf["peak"]) < 1e-3
    assert abs(rf["frame_ms_device_x_steps"] - rf["frame_ms_device"] * 20) < 1e-3
    assert rf["launches_per_frame_rank0"] == 1.0
    if rf["frac"] is not None:
        assert abs(rf["frac"] - rf["bytes_per_frame"] / (rf["frame_ms_device"] * 1e-3) / 1e9 / rf["peak"]) < 1e-3
    assert rf["kernel_ms_mean"] > 0   # the per-launch secondary (rocprof's mean)


def test_c4_extra_one_gpu():
    """BASELINE configs[3] (512^3, 1920x1080, S = 1024, ESS + ERT) rides the bench line as
    extra.c4 under the headline's kind of context: its own timed region, ranks_rendering, and one
    frame bitwise equal to a fresh one-GPU context's vr_render."""
    r = bench(["--steps", "6", "--warmup", "2", "--cpu-baseline", "0", "--extra", "0", "--extra-configs", "c4"])
    L = line_of(r)
    c4 = L["extra"]["c4"]
    assert "error" not in c4 and "skipped" not in c4, c4
    assert c4["mrays"] > 0 and L["extra"]["c4_mrays"] == c4["mrays"]
    assert c4["ranks_rendering"] == 1 and c4["steps"] == 6
    assert c4["bitwise_vs_one_gpu"] is True
    assert 0 < c4["frame_ms_device"] <= c4["ms_per_step"] * 1.0001


def test_c4_extra_two_part_group():
    """The same extra through a one-process two-part group (--devices 0,0: the N-part plan with the
    peer-copy transport): per-rank tiles and march times, the rank-0 weight tuned by measurement, and
    the farmed frame bitwise equal to a one-GPU context's."""
    r = bench(["--gpus", "2", "--devices", "0,0", "--steps", "6", "--warmup", "2", "--cpu-baseline", "0",
               "--extra", "0", "--extra-configs", "c4", "--rank0-weights", "1,3"])
    L = line_of(r)
    c4 = L["extra"]["c4"]
    assert "error" not in c4 and "skipped" not in c4, c4
    assert len(c4["tiles_per_rank"]) == 2 and sum(c4["tiles_per_rank"]) == c4["tiles_farmed"] > 0
    assert c4["ranks_rendering"] in (1, 2)
    assert sorted(float(k) for k in c4["rank0_weight_tuning_s"]) == [1.0, 3.0]
    assert len(c4["march_ms_per_frame_by_rank"]) == 2
    assert c4["bitwise_vs_one_gpu"] is True


def test_peer_traffic_fields_two_part_group():
    """the N > 1 line carries the tile bytes the transport moved per frame
    (vr_group_traffic_read), to compare with DESIGN section 7's prediction.  An even deal (weight 1,
    no tuning) over a two-part group: rank 1 sends its tiles' compact RGB, 64 x 64 x 12 B each, every
    frame; rank 0 sends nothing and receives exactly what rank 1 sent; the C4 extra carries the same."""
    r = bench(["--gpus", "2", "--devices", "0,0", "--steps", "8", "--warmup", "2", "--cpu-baseline", "0",
               "--extra", "0", "--extra-configs", "c4", "--rank0-weights", "1"])
    L = line_of(r)
    c = L["config"]
    for blk, tiles in ((c["peer_traffic"], c["tiles_per_rank"]), (L["extra"]["c4"]["peer_traffic"],
                                                                    L["extra"]["c4"]["tiles_per_rank"])):
        assert blk["frames"] >= 8
        sent = blk["bytes_sent_per_frame_by_rank"]
        assert sent[0] == 0 and tiles[1] > 0
        assert sent[1] == tiles[1] * 64 * 64 * 12
        assert blk["bytes_into_rank0_per_frame"] == sent[1]
