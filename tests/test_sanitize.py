"""ASan + UBSan CPU build of the host model and the oracle, fed a malformed-header corpus.

SURVEY section 5 asks for "an ASan/UBSan CPU build of the restatement".  tests/sanitize/Makefile
builds libvr's host model (csrc/host/scene.cpp: NiftiFile, OctreeHandler, TransferFunction, the
camera and TEST matrices) and the oracle (oracle/vr_oracle.c) with -fsanitize=address,undefined
-fno-sanitize-recover=all into tests/sanitize/_build/fuzz_host.  The loader parses untrusted
headers (BinaryLoader.cu:273-335 semantics, hardened: fail hard instead of continuing with an
uninitialised header, BinaryLoader.cu:333), so besides the real avg152 file it is fed a
deterministic corpus of malformed NIfTI-1/-2 files (truncations, bad sizes, hostile dims and
offsets, NaN / infinite fields, unknown datatypes, byte-swapped headers, seeded random byte flips):
each must load or be refused with vr::Error, with no sanitizer report.
"""
import gzip
import os
import struct
import subprocess

import numpy as np

from conftest import ROOT

SAN = os.path.join(ROOT, "tests", "sanitize")


def nifti2(dims, datatype=16, bitpix=32, vox_offset=544, cal_max=255.0, data=None, dim0=3, endian="<",
           pixdim=(1.0, 1.0, 1.0)):
    """A NIfTI-2 file (nifti2.h:59-98 field offsets: sizeof_hdr 0, datatype 12, bitpix 14, dim 16,
    pixdim 104, vox_offset 168, scl_slope 176, scl_inter 184, cal_max 192, cal_min 200)."""
    h = bytearray(540)
    struct.pack_into(endian + "i", h, 0, 540)
    struct.pack_into(endian + "hh", h, 12, datatype, bitpix)
    d = [dim0] + list(dims) + [1] * (7 - len(dims))
    struct.pack_into(endian + "8q", h, 16, *d)
    struct.pack_into(endian + "8d", h, 104, 0.0, *pixdim, 1.0, 1.0, 1.0, 1.0)
    struct.pack_into(endian + "q", h, 168, vox_offset)
    struct.pack_into(endian + "4d", h, 176, 1.0, 0.0, cal_max, 0.0)
    body = bytes(4) + (data if data is not None else b"")
    return bytes(h) + body


def nifti1(dims, datatype=16, bitpix=32, vox_offset=352.0, cal_max=255.0, data=None, dim0=3, endian="<"):
    """A NIfTI-1 file (nifti1.h: dim 40 (int16), datatype 70, bitpix 72, pixdim 76, vox_offset 108
    (float), scl_slope 112, scl_inter 116, cal_max 124, cal_min 128)."""
    h = bytearray(348)
    struct.pack_into(endian + "i", h, 0, 348)
    d = [dim0] + list(dims) + [1] * (7 - len(dims))
    struct.pack_into(endian + "8h", h, 40, *d)
    struct.pack_into(endian + "hh", h, 70, datatype, bitpix)
    struct.pack_into(endian + "8f", h, 76, 0.0, 1.0, 1.0, 1.0, 1.0, 1.0, 1.0, 1.0)
    struct.pack_into(endian + "f", h, 108, vox_offset)
    struct.pack_into(endian + "ff", h, 112, 1.0, 0.0)
    struct.pack_into(endian + "ff", h, 124, cal_max, 0.0)
    return bytes(h) + bytes(4) + (data if data is not None else b"")


def corpus():
    """(name, bytes) of the malformed / edge-case files, deterministic."""
    rng = np.random.default_rng(0x5A11)
    small = np.arange(5 * 4 * 3, dtype=np.float32).tobytes()
    v2 = nifti2((5, 4, 3), data=small)
    v1 = nifti1((5, 4, 3), data=small)
    out = [("empty", b""), ("ten_bytes", b"0123456789"), ("short347", bytes(347)), ("zeros348", bytes(348)),
           ("zeros540", bytes(540)), ("valid2_small", v2), ("valid1_small", v1),
           ("valid2_swapped", nifti2((5, 4, 3), endian=">", data=np.arange(60, dtype=">f4").tobytes())),
           ("truncated_data", v2[:-9]), ("header_only", v2[:540])]
    I64 = 2 ** 63 - 1
    for name, kw in [
        ("dim0_2", dict(dims=(5, 4, 3), dim0=2)), ("dim0_neg", dict(dims=(5, 4, 3), dim0=-1)),
        ("dim0_9", dict(dims=(5, 4, 3), dim0=9)), ("dim4d", dict(dims=(5, 4, 3, 2), dim0=4)),
        ("dim_zero", dict(dims=(0, 4, 3))), ("dim_neg", dict(dims=(5, -4, 3))),
        ("dim_2p31", dict(dims=(2 ** 31, 1, 1))), ("dim_2p40", dict(dims=(2 ** 40, 2 ** 40, 2 ** 40))),
        ("dim_max", dict(dims=(I64, I64, I64))), ("dim_overflow", dict(dims=(2 ** 21, 2 ** 21, 2 ** 22))),
        ("vox_neg", dict(dims=(5, 4, 3), vox_offset=-1)), ("vox_huge", dict(dims=(5, 4, 3), vox_offset=I64)),
        ("vox_past_end", dict(dims=(5, 4, 3), vox_offset=10 ** 6)),
        ("dt_0", dict(dims=(5, 4, 3), datatype=0)), ("dt_128", dict(dims=(5, 4, 3), datatype=128)),
        ("dt_2048", dict(dims=(5, 4, 3), datatype=2048)), ("dt_f64_short", dict(dims=(5, 4, 3), datatype=64)),
        ("calmax_nan", dict(dims=(5, 4, 3), cal_max=float("nan"))),
        ("calmax_inf", dict(dims=(5, 4, 3), cal_max=float("inf"))), ("calmax_0", dict(dims=(5, 4, 3), cal_max=0.0)),
    ]:
        out.append((name, nifti2(data=small, **kw)))
    for dt, bp in ((2, 8), (256, 8), (4, 16), (512, 16), (8, 32), (768, 32), (64, 64)):
        n = 5 * 4 * 3 * bp // 8
        out.append((f"dt{dt}_ok", nifti2((5, 4, 3), datatype=dt, bitpix=bp, data=rng.bytes(n))))
        out.append((f"dt{dt}_short", nifti2((5, 4, 3), datatype=dt, bitpix=bp, data=rng.bytes(n // 2))))
    for name, vo in [("n1_vox_nan", float("nan")), ("n1_vox_inf", float("inf")), ("n1_vox_ninf", float("-inf")),
                     ("n1_vox_1e30", 1e30), ("n1_vox_neg", -4.0), ("n1_vox_frac", 352.5), ("n1_vox_2p63", 2.0 ** 63)]:
        out.append((name, nifti1((5, 4, 3), vox_offset=vo, data=small)))
    out.append(("n1_dims_neg", nifti1((-5, 4, 3), data=small)))
    out.append(("n1_dims_max", nifti1((32767, 32767, 32767), data=small)))
    out.append(("n1_swapped", nifti1((5, 4, 3), endian=">", data=np.arange(60, dtype=">f4").tobytes())))
    for i in range(160):   # seeded byte flips in the header region of valid files
        base = bytearray(v2 if i % 2 == 0 else v1)
        hl = 540 if i % 2 == 0 else 348
        for _ in range(int(rng.integers(1, 9))):
            base[int(rng.integers(0, hl))] = int(rng.integers(0, 256))
        out.append((f"flip{i:03d}", bytes(base)))
    return out


def real_avg152(path):
    """The reference's avg152T1_LR_nifti2.nii rebuilt from the committed header + uint8 voxels."""
    hdr = open(os.path.join(ROOT, "data", "avg152T1_LR_nifti2.hdr"), "rb").read()
    vox = np.frombuffer(gzip.open(os.path.join(ROOT, "data", "avg152T1_LR.u8.gz")).read(), np.uint8)
    vo = struct.unpack_from("<q", hdr, 168)[0]
    with open(path, "wb") as f:
        f.write(hdr[:540].ljust(vo, b"\0"))
        f.write(vox.astype("<f4").tobytes())


def test_sanitized_host_model_and_oracle(tmp_path):
    # -B: always rebuild from the current sources (a stale binary would say nothing about them)
    r = subprocess.run(["make", "-B", "-s", "-C", SAN], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    valid = tmp_path / "avg152T1_LR_nifti2.nii"
    real_avg152(valid)
    files = []
    for name, data in corpus():
        p = tmp_path / (name + ".nii")
        p.write_bytes(data)
        files.append(str(p))
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:halt_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([os.path.join(SAN, "_build", "fuzz_host"), str(valid)] + files, capture_output=True,
                       text=True, env=env, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-6000:]
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-6000:]
    line = [x for x in r.stdout.splitlines() if x.startswith("fuzz_host:")][-1]
    n_loaded = int(line.split(": ")[2].split(" loaded")[0])
    assert f"corpus {len(files)} files" in line
    # the valid small files load; the hostile dims / offsets / datatypes are refused
    assert 10 <= n_loaded < len(files) - 30, line
