"""Host-side model (no GPU): NIfTI loader, OctreeHandler leaf maps, camera + TEST matrices,
transfer function -- all through libvr.so's C-ABI, checked against the oracle and the reference's
own glm (tests/golden/glm_vectors.json)."""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN
from volumerenderingproject_amd import renderer as R
from volumerenderingproject_amd import volumes as V


def hexf(s):
    return np.float32(float.fromhex(s))


def bits_equal(a, b_hex):
    a = np.asarray(a, np.float32).ravel()
    b = np.asarray([hexf(x) for x in b_hex], np.float32)
    return np.array_equal(a.view(np.uint32), b.view(np.uint32))


@pytest.fixture(scope="module")
def glm_vectors():
    return json.load(open(os.path.join(GOLDEN, "glm_vectors.json")))


# ------------------------------------------------------------------ NIfTI loader

def test_nifti_roundtrip_avg152(tmp_path):
    path = tmp_path / "avg152T1_LR_nifti2.nii"
    path.write_bytes(V.avg152_nifti_bytes())
    vol, cal = R.nifti_read(str(path))
    ref, hdr = V.avg152()
    assert vol.shape == (91, 109, 91) and cal == 255.0
    assert np.array_equal(vol, ref)


def test_nifti_missing_file_fails_hard(tmp_path):
    with pytest.raises(R.VRError) as e:
        R.nifti_read(str(tmp_path / "MNI152_T1_1mm_nifti2.nii"))
    assert e.value.code == -2


def test_nifti_garbage_and_truncated(tmp_path):
    bad = tmp_path / "bad.nii"
    bad.write_bytes(b"\x00" * 600)
    with pytest.raises(R.VRError):
        R.nifti_read(str(bad))
    vol, _ = V.avg152()
    trunc = tmp_path / "trunc.nii"
    trunc.write_bytes(V.make_nifti2(vol, 255.0)[:-100])
    with pytest.raises(R.VRError) as e:
        R.nifti_read(str(trunc))
    assert e.value.code == -2


def test_nifti_datatypes_and_nifti1(tmp_path):
    import struct
    rng = np.random.default_rng(0)
    v = rng.integers(0, 200, size=(5, 6, 7)).astype(np.float32)
    # int16 NIfTI-2
    b = bytearray(V.make_nifti2(v, 200.0))
    struct.pack_into("<hh", b, 12, 4, 16)
    b = bytes(b[:544]) + v.astype("<i2").tobytes()
    p = tmp_path / "i16.nii"
    p.write_bytes(b)
    got, cal = R.nifti_read(str(p))
    assert np.array_equal(got, v) and cal == 200.0
    # NIfTI-1, uint8, 352-byte offset
    h = bytearray(352)
    struct.pack_into("<i", h, 0, 348)
    struct.pack_into("<8h", h, 40, 3, 5, 6, 7, 1, 1, 1, 1)
    struct.pack_into("<hh", h, 70, 2, 8)
    struct.pack_into("<f", h, 108, 352.0)
    struct.pack_into("<f", h, 124, 199.0)
    p1 = tmp_path / "u8.nii"
    p1.write_bytes(bytes(h) + v.astype(np.uint8).tobytes())
    got, cal = R.nifti_read(str(p1))
    assert np.array_equal(got, v) and cal == 199.0
    # big-endian float32 NIfTI-2
    be = bytearray(544)
    struct.pack_into(">i", be, 0, 540)
    struct.pack_into(">hh", be, 12, 16, 32)
    struct.pack_into(">8q", be, 16, 3, 5, 6, 7, 1, 1, 1, 1)
    struct.pack_into(">q", be, 168, 544)
    struct.pack_into(">d", be, 192, 255.0)
    p2 = tmp_path / "be.nii"
    p2.write_bytes(bytes(be) + v.astype(">f4").tobytes())
    got, cal = R.nifti_read(str(p2))
    assert np.array_equal(got, v) and cal == 255.0


def test_nifti_4d_rejected(tmp_path):
    import struct
    v = np.zeros((2, 2, 2), np.float32)
    b = bytearray(V.make_nifti2(v, 1.0))
    struct.pack_into("<8q", b, 16, 4, 2, 2, 2, 3, 1, 1, 1)
    p = tmp_path / "4d.nii"
    p.write_bytes(bytes(b))
    with pytest.raises(R.VRError) as e:
        R.nifti_read(str(p))
    assert e.value.code == -3


# ------------------------------------------------------------------ octree leaf grid

@pytest.mark.parametrize("shape", [(91, 109, 91), (7, 5, 9), (64, 64, 64), (33, 17, 40), (1, 1, 1), (2, 3, 1)])
def test_leaf_maps_equal_reference_octree(shape, oracle_mod):
    """OctreeHandler's closed form == the restated Octree.cu build + recursive lookup, every leaf."""
    rng = np.random.default_rng(hash(shape) & 0xFFFF)
    vol = rng.integers(0, 256, size=shape).astype(np.float32) + 1.0   # > 0 so the clamp never hides a voxel
    oct_ = oracle_mod.OracleOctree(vol)
    maps, depth = R.octree_leaf_maps(*shape)
    assert depth == oct_.depth
    n = 1 << depth
    ref = oct_.leaf_values()
    mx, my, mz = maps
    inside = (mx[:, None, None] >= 0) & (my[None, :, None] >= 0) & (mz[None, None, :] >= 0)
    idx = (np.clip(mx, 0, None)[:, None, None] * shape[1] * shape[2] + np.clip(my, 0, None)[None, :, None] * shape[2]
           + np.clip(mz, 0, None)[None, None, :])
    got = np.where(inside, vol.ravel()[idx], 0.0).astype(np.float32)
    assert got.shape == (n, n, n)
    assert np.array_equal(got, ref)


def test_leaf_maps_mni_shape(mni_standin, oracle_mod):
    vol, _ = mni_standin
    maps, depth = R.octree_leaf_maps(*vol.shape)
    assert depth == 8
    # acceptance per axis: dataset centred in the 256^3 leaf grid, voxel monotone in leaf, steps <= 1
    for a, d in enumerate(vol.shape):
        m = maps[a]
        valid = m[m >= 0]
        assert valid[0] == 0 and valid[-1] == d - 1
        assert np.all(np.diff(valid) >= 0) and np.all(np.diff(valid) <= 1)


# ------------------------------------------------------------------ camera / matrices vs glm

def test_camera_and_positions_match_glm(glm_vectors, oracle_mod):
    for f in glm_vectors["frames"]:
        W, H, S = f["W"], f["H"], f["S"]
        p = R.default_params(W, H, S)
        assert bits_equal([p.real_screen_width], [f["rsw"]])
        assert bits_equal([p.real_screen_height], [f["rsh"]])
        assert bits_equal([p.sample_distance], [f["sd"]])
        cam = R.default_camera(W, H) if f["camera"] == "default" else R.reset_camera()
        for k, gk in [("pos", "pos"), ("front", "front"), ("right", "right"), ("up", "up"), ("top_left", "tlc")]:
            assert bits_equal(list(getattr(cam, k)), f[gk]), (W, H, f["camera"], k)
        # the oracle's sample points use the same camera
        ocam = oracle_mod.camera_default(W, H) if f["camera"] == "default" else oracle_mod.camera_oblique(W, H)
        op = oracle_mod.params(W, H, S)
        for x, y, s, q in f["vrc_points"]:
            assert bits_equal(oracle_mod.sample_point(op, ocam, x, y, s), q)


def test_oracle_glm_primitives(glm_vectors, oracle_mod):
    L = oracle_mod.lib()
    O = oracle_mod
    I = O.M4()
    for i in range(16):
        I.m[i] = 1.0 if i % 5 == 0 else 0.0

    def V3(a):
        return O.V3(*[hexf(x) for x in a])
    for p in glm_vectors["prims"]:
        a, b = V3(p["a"]), V3(p["b"])
        n = L.or_glm_normalize(a)
        assert bits_equal([n.x, n.y, n.z], p["normalize_a"])
        c = L.or_glm_cross(a, b)
        assert bits_equal([c.x, c.y, c.z], p["cross_ab"])
        eye = O.V3(np.float32(a.x) * np.float32(3), np.float32(a.y) * np.float32(3), np.float32(a.z) * np.float32(3))
        la = L.or_glm_lookat(eye, O.V3(0, 0, 0), b)
        assert bits_equal(la.m, p["lookat"])
        inv = L.or_glm_inverse(la)
        assert bits_equal(inv.m, p["inverse"])
        rot = L.or_glm_rotate(L.or_glm_translate(I, a), hexf(p["ang"]), b)
        assert bits_equal(rot.m, p["rotate"])
        sc = L.or_glm_scale(rot, b)
        assert bits_equal(sc.m, p["scale"])
        mm = L.or_glm_mul(inv, sc)
        assert bits_equal(mm.m, p["mul"])
        mv = L.or_glm_mulv(mm, O.V4(a.x, a.y, a.z, 1))
        assert bits_equal([mv.x, mv.y, mv.z, mv.w], p["mulv"])


def test_test_mode_matrices_match_glm(glm_vectors, oracle_mod):
    O = oracle_mod
    L = O.lib()
    for f in glm_vectors["frames"]:
        W, H, S = f["W"], f["H"], f["S"]
        p = O.params(W, H, S)
        cam = O.camera_default(W, H) if f["camera"] == "default" else O.camera_oblique(W, H)
        for t in f["test"]:
            mc, iv, tv = O.test_matrices(t["dim"], p, cam)
            assert bits_equal(mc, t["model_cam"]) and bits_equal(iv, t["inverse_view"]) and bits_equal(tv, t["to_volume"])
            M = [O.M4(), O.M4(), O.M4()]
            for m, src in zip(M, (mc, iv, tv)):
                for i, x in enumerate(src.ravel()):
                    m.m[i] = x
            for x, y, s, q in t["points"]:
                v = O.V4(float(x), float(y), float(s), 1.0)
                for m in M:
                    r = L.or_glm_mulv(m, v)
                    v = O.V4(r.x, r.y, r.z, 1.0)
                assert bits_equal([v.x, v.y, v.z], q)


def test_cpu_path_model_matrix_matches_glm(glm_vectors, oracle_mod):
    O = oracle_mod
    L = O.lib()
    I = O.M4()
    for i in range(16):
        I.m[i] = 1.0 if i % 5 == 0 else 0.0
    m = L.or_glm_translate(I, O.V3(0.5, 0.5, 0.5))
    r90 = np.float32(90.0) * np.float32(0.01745329251994329576923690768489)
    m = L.or_glm_rotate(m, r90, O.V3(0, 1, 0))
    m = L.or_glm_rotate(m, r90, O.V3(-1, 0, 0))
    assert bits_equal(m.m, glm_vectors["cpu_path_model"])


def test_derive_camera_is_processinput():
    p = R.default_params(300, 300, 300)
    c = R.derive_camera([0.0, 0.0, 1.0], [0.0, 1.0, 0.0], p.real_screen_width, p.real_screen_height)
    assert list(c.right) == [-1.0, 0.0, 0.0] and list(c.up) == [0.0, 1.0, 0.0]   # mirrored right
    assert list(c.top_left) == [1.0, 1.0, 1.0]


# ------------------------------------------------------------------ transfer function

def test_default_tf_and_classes(oracle_mod):
    tf = R.default_transfer_function()
    otf, n = oracle_mod.default_tf()
    assert len(tf) == n == 4
    for i in range(4):
        assert np.float32(tf[i][0]) == np.float32(otf[i].lo) and np.float32(tf[i][1]) == np.float32(otf[i].hi)
        assert np.array_equal(np.float32(tf[i][2]), np.float32(list(otf[i].rgba)))
    # last-match wins, closed bounds, default interval 0 (TransferFunction.cu:46-55)
    assert oracle_mod.tf_class(otf, n, np.float32(30.0 / 255.0)) == 1
    assert oracle_mod.tf_class(otf, n, np.float32(80.0) / np.float32(255.0)) == 1
    assert oracle_mod.tf_class(otf, n, 110.0 / 255.0) == 3
    assert oracle_mod.tf_class(otf, n, 2.0) == 0
    assert oracle_mod.tf_class(otf, n, -0.5) == 0
    assert oracle_mod.tf_class(otf, n, float("nan")) == 0
    # for integer intensities / 255 the classification is a 256-entry LUT
    lut = [oracle_mod.tf_class(otf, n, np.float32(i) / np.float32(255)) for i in range(256)]
    assert lut[29] == 0 and lut[30] == 1 and lut[80] == 1 and lut[81] == 0
    assert lut[105] == 3 and lut[120] == 3 and lut[140] == 2 and lut[160] == 2 and lut[161] == 0


def test_conic_camera_matches_oracle(oracle_mod):
    """vr_camera_derive_conic (utils.h:93-97) against the oracle restatement, bit for bit."""
    import math
    for pos, up in [((0.0, 0.0, 1.0), (0.0, 1.0, 0.0)), ((0.456607, 0.693644, -0.55711), (0.868199, -0.484147, 0.108777))]:
        rsw = np.float32(2 * math.tan(np.float32(math.pi / 4))) * np.float32(2.0)
        rsh = np.float32(rsw * np.float32(480) / np.float32(640))
        got = R.derive_camera_conic(pos, up, float(rsw), float(rsh), 2.0)
        ref = oracle_mod.camera_derive_conic(pos, up, float(rsw), float(rsh), 2.0)
        for k in ("pos", "front", "right", "up", "top_left"):
            assert list(getattr(got, k)) == list(getattr(ref, k)), k


def test_point_cloud_oracle_layout(avg152, oracle_mod):
    """or_point_cloud (prepareVolumeColors, myApp.cu:1280-1316) against a numpy statement."""
    vol, cal = avg152
    pc = oracle_mod.point_cloud(vol, cal)
    d1, d2, d3 = vol.shape
    L = max(vol.shape)
    x, y, z = np.meshgrid(np.arange(d1), np.arange(d2), np.arange(d3), indexing="ij")
    f32 = np.float32
    for a, (g, d) in enumerate([(x, d1), (y, d2), (z, d3)]):
        ref = ((g.astype(f32) + f32(L / 2.0)) - f32(d) / f32(2.0)) / f32(L)
        assert np.array_equal(pc[:, a], ref.reshape(-1).astype(f32))
    tf, n = oracle_mod.default_tf()
    rgba = np.array([list(tf[i].rgba) for i in range(n)], np.float32)
    cls = np.array([oracle_mod.tf_class(tf, n, float(np.float32(float(v) / float(cal)))) for v in np.unique(vol)])
    lut = dict(zip(np.unique(vol).tolist(), cls.tolist()))
    idx = np.vectorize(lut.get)(vol.reshape(-1))
    assert np.array_equal(pc[:, 3:], rgba[idx])


def test_nifti2_wrapping_dims_refused(tmp_path):
    """Untrusted NIfTI-2 int64 dims: a product that wraps 64 bits (2^21 x 2^21 x 2^22 = 2^64 -> 0) or
    a dim beyond the int32 row index is refused (VR_ERANGE) before any allocation or read, instead
    of passing the truncation check on a wrapped count."""
    import struct
    vol, _ = V.avg152()
    good = bytearray(V.make_nifti2(vol, 255.0))
    assert struct.unpack_from("<i", good, 0)[0] == 540
    for dims in [(1 << 21, 1 << 21, 1 << 22), (1 << 31, 1, 1), (3, 1 << 40, 5)]:
        b = bytearray(good)
        struct.pack_into("<3q", b, 16 + 8, *dims)
        p = tmp_path / "crafted.nii"
        p.write_bytes(bytes(b))
        with pytest.raises(R.VRError) as e:
            R.nifti_read(str(p))
        assert e.value.code == -7, dims   # VR_ERANGE
