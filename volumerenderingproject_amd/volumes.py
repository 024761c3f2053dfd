"""Input volumes of the benchmark configs (BASELINE.json configs).

* avg152T1_LR -- the only volume the reference ships (NIfTI-2, float32, 91x109x91, cal_max 255,
  integer valued).  Kept in data/ as its 544-byte header + gzip'd uint8 payload (exact), and
  reconstructed here bit for bit (sha256 of the float32 payload is checked).
* MNI152_T1_1mm stand-in -- the reference hard-codes MNI152_T1_1mm_nifti2.nii (myApp.cu:240) but
  that blob is missing (.MISSING_LARGE_BLOBS:1).  avg152 is exactly the 2 mm version of the same
  template, so a 2x nearest-replicate per axis gives the 182x218x182 shape (same header fields).
"""
from __future__ import annotations

import gzip
import hashlib
import json
import os
import struct

import numpy as np

DATA = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "data")


def avg152():
    """(volume float32 [91,109,91] x-major, header dict) exactly as BinaryLoader.cu:273-335 reads it."""
    meta = json.load(open(os.path.join(DATA, "avg152T1_LR.json")))
    hdr = open(os.path.join(DATA, "avg152T1_LR_nifti2.hdr"), "rb").read()
    u8 = np.frombuffer(gzip.open(os.path.join(DATA, "avg152T1_LR.u8.gz")).read(), np.uint8)
    vol = u8.astype("<f4")
    if hashlib.sha256(vol.tobytes()).hexdigest() != meta["payload_f32_sha256"]:
        raise ValueError("avg152 fixture does not reconstruct the reference payload")
    h = parse_nifti2_header(hdr)
    return vol.reshape(h["dim"][1], h["dim"][2], h["dim"][3]), h


def avg152_nifti_bytes():
    """The reference's avg152T1_LR_nifti2.nii, byte for byte."""
    vol, _ = avg152()
    hdr = open(os.path.join(DATA, "avg152T1_LR_nifti2.hdr"), "rb").read()
    return hdr + vol.astype("<f4").tobytes()


def parse_nifti2_header(b: bytes):
    (sizeof_hdr,) = struct.unpack_from("<i", b, 0)
    datatype, bitpix = struct.unpack_from("<hh", b, 12)
    dim = list(struct.unpack_from("<8q", b, 16))
    pixdim = list(struct.unpack_from("<8d", b, 104))
    (vox_offset,) = struct.unpack_from("<q", b, 168)
    scl_slope, scl_inter, cal_max, cal_min = struct.unpack_from("<4d", b, 176)
    return dict(sizeof_hdr=sizeof_hdr, datatype=datatype, bitpix=bitpix, dim=dim, pixdim=pixdim,
                vox_offset=vox_offset, scl_slope=scl_slope, scl_inter=scl_inter, cal_max=cal_max, cal_min=cal_min)


def make_nifti2(vol: np.ndarray, cal_max: float, pixdim=(1.0, 1.0, 1.0)) -> bytes:
    """A NIfTI-2 file (datatype 16, vox_offset 544) holding an x-major float32 volume."""
    h = bytearray(544)
    struct.pack_into("<i", h, 0, 540)
    h[4:12] = b"n+2\x00\r\n\x1a\n"
    struct.pack_into("<hh", h, 12, 16, 32)
    d1, d2, d3 = vol.shape
    struct.pack_into("<8q", h, 16, 3, d1, d2, d3, 1, 1, 1, 1)
    struct.pack_into("<8d", h, 104, 0.0, pixdim[0], pixdim[1], pixdim[2], 1.0, 1.0, 1.0, 1.0)
    struct.pack_into("<q", h, 168, 544)
    struct.pack_into("<4d", h, 176, 0.0, 0.0, cal_max, 0.0)
    return bytes(h) + np.ascontiguousarray(vol, "<f4").tobytes()


def mni152_standin():
    """182x218x182 float32 stand-in for MNI152_T1_1mm (avg152 2x nearest-replicate), cal_max 255."""
    vol, h = avg152()
    big = np.repeat(np.repeat(np.repeat(vol, 2, 0), 2, 1), 2, 2)
    return np.ascontiguousarray(big), h["cal_max"]


def resample_512(vol: np.ndarray):
    """C4: stand-in trilinearly resampled (align-corners) to 512^3 and rounded to ints 0..255."""
    out_n = 512
    src = vol.astype(np.float32)
    coords = [np.linspace(0.0, s - 1.0, out_n, dtype=np.float64) for s in src.shape]
    # separable linear interpolation, axis by axis
    for axis, c in enumerate(coords):
        i0 = np.floor(c).astype(np.int64)
        i1 = np.minimum(i0 + 1, src.shape[axis] - 1)
        w = (c - i0).astype(np.float32)
        a = np.take(src, i0, axis=axis)
        b = np.take(src, i1, axis=axis)
        shape = [1, 1, 1]
        shape[axis] = out_n
        w = w.reshape(shape)
        src = a * (1 - w) + b * w
    return np.ascontiguousarray(np.clip(np.rint(src), 0, 255).astype(np.float32))
