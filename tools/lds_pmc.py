#!/usr/bin/env python3
"""LDS pressure of the march kernel from one PMC pass (on the GPU box): LDS-array cycles
(SQ_LDS_IDX_ACTIVE), their bank-conflict part (SQ_LDS_BANK_CONFLICT), the LDS issue stall
(SQ_WAIT_INST_LDS, a part of SQ_WAIT_INST_ANY) and the LDS / VALU instruction counts, averaged over
the timed march launches of `bench.py <args>` (tools/pmc_traffic.py's pass runner).

Derived: conflict share = BANK_CONFLICT / IDX_ACTIVE; LDS-array busy share = IDX_ACTIVE /
(GRBM_GUI_ACTIVE x 256 CUs) -- assuming IDX_ACTIVE sums LDS-array cycles over every CU and
GRBM_GUI_ACTIVE counts GPU-busy cycles (units not calibrated in the guides; a relative figure for
A/Bs); the LDS issue stall as a share of SQ_WAVE_CYCLES (both quad-cycles).
usage: python tools/lds_pmc.py <out.json> [bench args ...]
"""
import json
import os
import shutil
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import pmc_traffic  # noqa: E402

LDS = ["SQ_LDS_IDX_ACTIVE", "SQ_LDS_BANK_CONFLICT", "SQ_WAIT_INST_LDS", "SQ_INSTS_LDS", "SQ_INSTS_VALU",
       "SQ_WAVE_CYCLES", "GRBM_GUI_ACTIVE"]


def main():
    out_json = sys.argv[1]
    bench_args = sys.argv[2:]
    tmp = tempfile.mkdtemp(prefix="vr_lds_", dir="/tmp")
    rows = []
    try:
        v, n, line = pmc_traffic.run_pass(LDS, bench_args, tmp, "lds", rows)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    res = {
        "bench_args": bench_args,
        "dispatches": n["SQ_LDS_IDX_ACTIVE"],
        "counters": v,
        "conflict_share": v["SQ_LDS_BANK_CONFLICT"] / max(1.0, v["SQ_LDS_IDX_ACTIVE"]),
        "lds_busy_share_est": v["SQ_LDS_IDX_ACTIVE"] / max(1.0, v["GRBM_GUI_ACTIVE"] * 256.0),
        "wait_inst_lds_share": v["SQ_WAIT_INST_LDS"] / max(1.0, v["SQ_WAVE_CYCLES"]),
        "lds_per_valu": v["SQ_INSTS_LDS"] / max(1.0, v["SQ_INSTS_VALU"]),
        "ms_per_step": line.get("ms_per_step"),
    }
    json.dump(res, open(out_json, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
