"""Make data/avg152T1_LR.* from the reference's only shipped volume (run in the build container).

The reference ships avg152T1_LR_nifti2.nii (NIfTI-2, float32, 91x109x91, cal_max 255) whose
voxels are all integers 0..255, so a uint8 copy is exact.  We keep the 544-byte header verbatim
and the payload as gzip'd uint8, plus the sha256 of the original float32 payload so
volumerenderingproject_amd.volumes.avg152() can prove it reconstructs the file bit for bit.
"""
import gzip, hashlib, json, os, sys
import numpy as np

SRC = sys.argv[1] if len(sys.argv) > 1 else "/root/reference/avg152T1_LR_nifti2.nii"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "data")
raw = open(SRC, "rb").read()
hdr = raw[:544]
vox = np.frombuffer(raw, dtype="<f4", offset=544)
assert vox.size == 91 * 109 * 91 and np.all(vox == np.round(vox)) and vox.min() >= 0 and vox.max() <= 255
u8 = vox.astype(np.uint8)
assert np.array_equal(u8.astype("<f4"), vox)
open(os.path.join(OUT, "avg152T1_LR_nifti2.hdr"), "wb").write(hdr)
with gzip.GzipFile(os.path.join(OUT, "avg152T1_LR.u8.gz"), "wb", mtime=0) as f:
    f.write(u8.tobytes())
meta = {"source": "avg152T1_LR_nifti2.nii (reference repo root)", "shape": [91, 109, 91],
        "file_sha256": hashlib.sha256(raw).hexdigest(),
        "payload_f32_sha256": hashlib.sha256(vox.tobytes()).hexdigest()}
json.dump(meta, open(os.path.join(OUT, "avg152T1_LR.json"), "w"), indent=1)
print(meta)
