"""ctypes front-end of the CPU oracle (liboracle.so) -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module, and only
as the checker / the timed CPU baseline.  The product path (volumerenderingproject_amd) never
imports it.  See oracle/vr_oracle.h for the reference file:line map.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


class Interval(C.Structure):
    _fields_ = [("lo", C.c_float), ("hi", C.c_float), ("rgba", C.c_float * 4)]


class Node(C.Structure):
    _fields_ = [("depth", C.c_int32), ("maximum_value", C.c_float), ("minimum_value", C.c_float),
                ("lower", C.c_float * 3), ("upper", C.c_float * 3)]


class Octree(C.Structure):
    _fields_ = [("nodes", C.POINTER(Node)), ("number_of_nodes", C.c_uint64),
                ("maximum_depth", C.c_uint32), ("longest_dimension", C.c_uint32),
                ("dim", C.c_int64 * 3), ("volume", C.POINTER(C.c_float))]


class Camera(C.Structure):
    _fields_ = [("pos", C.c_float * 3), ("front", C.c_float * 3), ("right", C.c_float * 3),
                ("up", C.c_float * 3), ("top_left", C.c_float * 3)]

    def as_dict(self):
        return {k: list(getattr(self, k)) for k, _ in self._fields_}


class Params(C.Structure):
    _fields_ = [("width", C.c_int32), ("height", C.c_int32), ("samples_per_ray", C.c_int32),
                ("real_screen_width", C.c_float), ("real_screen_height", C.c_float),
                ("viewplane_distance", C.c_float), ("front_clip_plane", C.c_float),
                ("sample_distance", C.c_float), ("background", C.c_float * 4), ("conic", C.c_int32)]


class M4(C.Structure):
    _fields_ = [("m", C.c_float * 16)]

    def np(self):
        return np.array(self.m, dtype=np.float32).reshape(4, 4)  # [column][row] like glm


class V3(C.Structure):
    _fields_ = [("x", C.c_float), ("y", C.c_float), ("z", C.c_float)]


class V4(C.Structure):
    _fields_ = [("x", C.c_float), ("y", C.c_float), ("z", C.c_float), ("w", C.c_float)]


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "liboracle.so")
        if not os.path.exists(path):
            subprocess.check_call(["make", "-s", "-C", _HERE])
        L = C.CDLL(path)
        fp = C.POINTER(C.c_float)
        L.or_default_tf.argtypes = [C.POINTER(Interval)]
        L.or_tf_class.argtypes = [C.POINTER(Interval), C.c_int, C.c_float]
        L.or_tf_class.restype = C.c_int
        L.or_octree_build.argtypes = [C.POINTER(Octree), fp, C.c_int64, C.c_int64, C.c_int64]
        L.or_octree_free.argtypes = [C.POINTER(Octree)]
        L.or_octree_init_implicit.argtypes = [C.POINTER(Octree), fp, C.c_int64, C.c_int64, C.c_int64]
        L.or_render_vrc_columns.argtypes = [C.POINTER(Octree), C.c_double, C.POINTER(Interval), C.c_int,
                                            C.POINTER(Params), C.POINTER(Camera), C.POINTER(C.c_int), C.c_int, fp,
                                            C.c_int]
        L.or_synthetic_voxel.argtypes = [C.c_int64, C.c_uint64, C.c_int64, C.c_int64, C.c_int64]
        L.or_synthetic_voxel.restype = C.c_float
        L.or_synthetic_slab.argtypes = [C.c_int64, C.c_uint64, C.c_int64, C.c_int64, fp, C.c_int]
        L.or_octree_intensity.argtypes = [C.POINTER(Octree), C.c_float, C.c_float, C.c_float]
        L.or_octree_intensity.restype = C.c_float
        L.or_octree_leaf_values.argtypes = [C.POINTER(Octree), fp, C.c_int]
        L.or_camera_derive.argtypes = [fp, fp, C.c_float, C.c_float, C.POINTER(Camera)]
        L.or_camera_derive_conic.argtypes = [fp, fp, C.c_float, C.c_float, C.c_float, C.POINTER(Camera)]
        L.or_point_cloud.argtypes = [fp, C.c_int64, C.c_int64, C.c_int64, C.c_double, C.POINTER(Interval), C.c_int,
                                     fp]
        L.or_camera_default.argtypes = [C.c_int, C.c_int, C.POINTER(Camera)]
        L.or_camera_oblique.argtypes = [C.c_int, C.c_int, C.POINTER(Camera)]
        L.or_params_default.argtypes = [C.c_int, C.c_int, C.c_int, C.POINTER(Params)]
        L.or_render_vrc.argtypes = [C.POINTER(Octree), C.c_double, C.POINTER(Interval), C.c_int,
                                    C.POINTER(Params), C.POINTER(Camera), fp, C.c_int]
        L.or_render_vrc_shaded.argtypes = [C.POINTER(Octree), C.c_double, C.POINTER(Interval), C.c_int,
                                           C.POINTER(Params), C.POINTER(Camera), fp, fp, C.c_int]
        L.or_vrc_ray_samples.argtypes = [C.POINTER(Octree), C.c_double, C.POINTER(Interval), C.c_int,
                                         C.POINTER(Params), C.POINTER(Camera), C.c_int, C.c_int, fp]
        L.or_vrc_sample_point.argtypes = [C.POINTER(Params), C.POINTER(Camera), C.c_int, C.c_int, C.c_int, fp]
        L.or_render_test.argtypes = [fp, C.c_int64, C.c_int64, C.c_int64, C.c_double, C.POINTER(Interval),
                                     C.c_int, C.POINTER(Params), C.POINTER(Camera), fp, C.c_int]
        L.or_render_test_columns.argtypes = [fp, C.c_int64, C.c_int64, C.c_int64, C.c_double, C.POINTER(Interval),
                                             C.c_int, C.POINTER(Params), C.POINTER(Camera), C.POINTER(C.c_int),
                                             C.c_int, fp, C.c_int]
        L.or_test_matrices.argtypes = [C.c_int64, C.c_int64, C.c_int64, C.POINTER(Params), C.POINTER(Camera),
                                       C.POINTER(M4), C.POINTER(M4), C.POINTER(M4)]
        L.or_render_cpu_path.argtypes = [C.POINTER(Octree), C.c_double, C.POINTER(Interval), C.c_int,
                                         C.POINTER(Params), C.POINTER(Camera), C.c_int, C.c_int, fp, C.c_int]
        L.or_render_cpu_path_columns.argtypes = [C.POINTER(Octree), C.c_double, C.POINTER(Interval), C.c_int,
                                                 C.POINTER(Params), C.POINTER(Camera), C.POINTER(C.c_int), C.c_int,
                                                 C.c_int, fp, C.c_int]
        L.or_count_in_samples.argtypes = [C.POINTER(Octree), C.POINTER(Params), C.POINTER(Camera), C.c_int]
        L.or_count_in_samples.restype = C.c_uint64
        L.or_vrc_contraction_flips.argtypes = [C.POINTER(Octree), C.POINTER(Params), C.POINTER(Camera),
                                               C.POINTER(C.c_uint64)]
        L.or_vrc_contraction_flips.restype = C.c_uint64
        L.or_test_contraction_flips.argtypes = [C.c_int64, C.c_int64, C.c_int64, C.POINTER(Params), C.POINTER(Camera),
                                                C.POINTER(C.c_uint64)]
        L.or_test_contraction_flips.restype = C.c_uint64
        for name, args, res in [
            ("or_glm_translate", [M4, V3], M4), ("or_glm_scale", [M4, V3], M4),
            ("or_glm_rotate", [M4, C.c_float, V3], M4), ("or_glm_lookat", [V3, V3, V3], M4),
            ("or_glm_inverse", [M4], M4), ("or_glm_mul", [M4, M4], M4), ("or_glm_mulv", [M4, V4], V4),
            ("or_glm_normalize", [V3], V3), ("or_glm_cross", [V3, V3], V3)]:
            f = getattr(L, name)
            f.argtypes = args
            f.restype = res
        _LIB = L
    return _LIB


def _fp(a):
    return a.ctypes.data_as(C.POINTER(C.c_float))


def default_tf():
    arr = (Interval * 4)()
    lib().or_default_tf(arr)
    return arr, 4


def tf_array(intervals):
    """intervals: list of (lo, hi, (r, g, b, a))."""
    arr = (Interval * len(intervals))()
    for i, (lo, hi, rgba) in enumerate(intervals):
        arr[i].lo, arr[i].hi = lo, hi
        for c in range(4):
            arr[i].rgba[c] = rgba[c]
    return arr, len(intervals)


def tf_class(tf, n, value):
    return lib().or_tf_class(tf, n, value)


def params(W, H, S):
    p = Params()
    lib().or_params_default(W, H, S, C.byref(p))
    return p


def camera_default(W, H):
    c = Camera()
    lib().or_camera_default(W, H, C.byref(c))
    return c


def camera_oblique(W, H):
    c = Camera()
    lib().or_camera_oblique(W, H, C.byref(c))
    return c


def camera_derive(pos, up, rsw, rsh):
    c = Camera()
    P = np.asarray(pos, np.float32)
    U = np.asarray(up, np.float32)
    lib().or_camera_derive(_fp(P), _fp(U), rsw, rsh, C.byref(c))
    return c


class OracleOctree:
    """The reference's implicit complete octree, built by the restated Octree.cu code.

    implicit=True keeps no node pool and evaluates the search in closed form (or_octree_init_implicit;
    pinned to the literal tree by tests/test_oracle_pin.py) -- for 512^3 / 2048^3 volumes."""

    def __init__(self, volume: np.ndarray, implicit=False):
        self.volume = np.ascontiguousarray(volume, dtype=np.float32)
        self.o = Octree()
        d1, d2, d3 = self.volume.shape
        init = lib().or_octree_init_implicit if implicit else lib().or_octree_build
        rc = init(C.byref(self.o), _fp(self.volume), d1, d2, d3)
        if rc != 0:
            raise MemoryError("octree build failed")

    def __del__(self):
        try:
            lib().or_octree_free(C.byref(self.o))
        except Exception:
            pass

    @property
    def depth(self):
        return self.o.maximum_depth

    @property
    def longest_dimension(self):
        return self.o.longest_dimension

    def intensity(self, q):
        return lib().or_octree_intensity(C.byref(self.o), float(q[0]), float(q[1]), float(q[2]))

    def leaf_values(self, threads=0):
        n = 1 << self.depth
        out = np.empty(n * n * n, np.float32)
        lib().or_octree_leaf_values(C.byref(self.o), _fp(out), threads)
        return out.reshape(n, n, n)

    def render_vrc(self, cal_max, tf, p, cam, threads=0):
        out = np.empty((p.width * p.height * 4,), np.float32)
        lib().or_render_vrc(C.byref(self.o), cal_max, tf[0], tf[1], C.byref(p), C.byref(cam), _fp(out), threads)
        return out.reshape(p.width, p.height, 4)

    def render_vrc_columns(self, cal_max, tf, p, cam, xs, threads=0):
        """Columns xs of the VRC frame: shape (len(xs), H, 4)."""
        xs = np.ascontiguousarray(xs, dtype=np.int32)
        out = np.empty((len(xs) * p.height * 4,), np.float32)
        lib().or_render_vrc_columns(C.byref(self.o), cal_max, tf[0], tf[1], C.byref(p), C.byref(cam),
                                    xs.ctypes.data_as(C.POINTER(C.c_int)), len(xs), _fp(out), threads)
        return out.reshape(len(xs), p.height, 4)

    def render_vrc_shaded(self, cal_max, tf, p, cam, shade, threads=0):
        sh = np.asarray(shade, np.float32)
        out = np.empty((p.width * p.height * 4,), np.float32)
        lib().or_render_vrc_shaded(C.byref(self.o), cal_max, tf[0], tf[1], C.byref(p), C.byref(cam), _fp(sh),
                                   _fp(out), threads)
        return out.reshape(p.width, p.height, 4)

    def ray_samples(self, cal_max, tf, p, cam, x, y):
        out = np.empty((p.samples_per_ray * 4,), np.float32)
        lib().or_vrc_ray_samples(C.byref(self.o), cal_max, tf[0], tf[1], C.byref(p), C.byref(cam), x, y, _fp(out))
        return out.reshape(-1, 4)

    def render_cpu_path(self, cal_max, tf, p, cam, x0, x1, threads=1):
        out = np.empty(((x1 - x0) * p.height * 4,), np.float32)
        lib().or_render_cpu_path(C.byref(self.o), cal_max, tf[0], tf[1], C.byref(p), C.byref(cam),
                                 x0, x1, _fp(out), threads)
        return out.reshape(x1 - x0, p.height, 4)

    def render_cpu_path_columns(self, cal_max, tf, p, cam, xs, threads=0):
        xs = np.ascontiguousarray(xs, dtype=np.int32)
        out = np.empty((len(xs) * p.height * 4,), np.float32)
        lib().or_render_cpu_path_columns(C.byref(self.o), cal_max, tf[0], tf[1], C.byref(p), C.byref(cam),
                                         xs.ctypes.data_as(C.POINTER(C.c_int)), 0, len(xs), _fp(out), threads)
        return out.reshape(len(xs), p.height, 4)

    def count_in_samples(self, p, cam, threads=0):
        return int(lib().or_count_in_samples(C.byref(self.o), C.byref(p), C.byref(cam), threads))


def vrc_contraction_flips(octree, p, cam):
    """(samples whose leaf changes under the fused model, samples in the dataset under either)."""
    n = C.c_uint64(0)
    f = lib().or_vrc_contraction_flips(C.byref(octree.o), C.byref(p), C.byref(cam), C.byref(n))
    return int(f), int(n.value)


def test_contraction_flips(shape, p, cam):
    n = C.c_uint64(0)
    f = lib().or_test_contraction_flips(shape[0], shape[1], shape[2], C.byref(p), C.byref(cam), C.byref(n))
    return int(f), int(n.value)


def sample_point(p, cam, x, y, s):
    q = np.empty(3, np.float32)
    lib().or_vrc_sample_point(C.byref(p), C.byref(cam), x, y, s, _fp(q))
    return q


def render_test(volume, cal_max, tf, p, cam, threads=0):
    v = np.ascontiguousarray(volume, dtype=np.float32)
    d1, d2, d3 = v.shape
    out = np.empty((p.width * p.height * 4,), np.float32)
    lib().or_render_test(_fp(v), d1, d2, d3, cal_max, tf[0], tf[1], C.byref(p), C.byref(cam), _fp(out), threads)
    return out.reshape(p.width, p.height, 4)


def render_test_columns(volume, cal_max, tf, p, cam, xs, threads=0):
    """Columns xs of the TEST frame: shape (len(xs), H, 4)."""
    v = np.ascontiguousarray(volume, dtype=np.float32)
    d1, d2, d3 = v.shape
    xs = np.ascontiguousarray(xs, dtype=np.int32)
    out = np.empty((len(xs) * p.height * 4,), np.float32)
    lib().or_render_test_columns(_fp(v), d1, d2, d3, cal_max, tf[0], tf[1], C.byref(p), C.byref(cam),
                                 xs.ctypes.data_as(C.POINTER(C.c_int)), len(xs), _fp(out), threads)
    return out.reshape(len(xs), p.height, 4)


def test_matrices(shape, p, cam):
    a, b, c = M4(), M4(), M4()
    lib().or_test_matrices(shape[0], shape[1], shape[2], C.byref(p), C.byref(cam), C.byref(a), C.byref(b), C.byref(c))
    return a.np(), b.np(), c.np()


def synthetic_slab(n, x0, nx, seed=0x5EED, threads=0):
    """Slab [x0, x0+nx) of the synthetic n^3 C5 volume (or_synthetic_slab), shape (nx, n, n)."""
    out = np.empty((nx * n * n,), np.float32)
    lib().or_synthetic_slab(n, seed, x0, nx, _fp(out), threads)
    return out.reshape(nx, n, n)


def camera_derive_conic(pos, up, rsw, rsh, vpd):
    c = Camera()
    P = np.asarray(pos, np.float32)
    U = np.asarray(up, np.float32)
    lib().or_camera_derive_conic(_fp(P), _fp(U), rsw, rsh, vpd, C.byref(c))
    return c


def point_cloud(volume, cal_max, tf=None):
    """POINT-mode vertex array (prepareVolumeColors): shape (d1*d2*d3, 7)."""
    v = np.ascontiguousarray(volume, dtype=np.float32)
    tf = tf or default_tf()
    out = np.empty((v.size * 7,), np.float32)
    lib().or_point_cloud(_fp(v), v.shape[0], v.shape[1], v.shape[2], cal_max, tf[0], tf[1], _fp(out))
    return out.reshape(v.size, 7)
