"""Python host mirror of the reference's render-path API over the C-ABI (include/vr_api.h).

The reference drives its renderer from C++ (myApp.cu renderLoop -> namespace myCUDAspace,
kernel.h:15-75).  This module is the thin ctypes layer tests and bench.py use to reach the same
C-ABI the C++ host would link against: `VolumeRenderer` owns a `vr_ctx` (one GPU), `RenderParams`
mirrors AppData's render fields (utils.h:36-74) and `Camera` its camera fields (utils.h:41-46,
68-70).  It never computes a frame itself: if libvr.so is missing or fails to load, every call
raises -- there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("VR_LIB") or os.path.join(_HERE, "libvr.so")   # VR_LIB: A/B builds only

VR_OK = 0
VR_MODE_VRC = 1
VR_MODE_TEST = 5
VR_FLAG_ESS = 1
VR_FLAG_ERT = 2
VR_FLAG_SHADE = 8
VR_FLAG_CONIC = 16
VR_OUT_DEVICE = 1
VR_OUT_ASYNC = 2
VR_OUT_RGB = 4      # tile buffers of 3 floats per pixel (alpha is 1 by construction)

# every symbol include/vr_api.h declares (checked by tests/test_abi.py)
EXPORTED = [
    "vr_create", "vr_create_from_device", "vr_create_from_nifti", "vr_set_transfer_function", "vr_destroy",
    "vr_render", "vr_render_tiles", "vr_assemble_tiles", "vr_count_samples", "vr_count_marched", "vr_synchronize", "vr_set_stream",
    "vr_params_default", "vr_camera_derive", "vr_camera_default", "vr_camera_reset",
    "vr_default_transfer_function", "vr_get_volume_info", "vr_timing_enable", "vr_timing_read", "vr_strerror",
    "vr_device_count", "vr_api_version", "vr_nifti_read", "vr_octree_leaf_maps",
    "vr_frame_to_rgb8", "vr_write_png", "vr_synthetic_volume", "vr_camera_derive_conic", "vr_point_cloud",
    "vr_visible_tiles", "vr_render_tile_list", "vr_assemble_tile_list", "vr_assemble_tile_slots",
    "vr_assemble_tile_slots_multi", "vr_options_default", "vr_create_ex", "vr_get_options", "vr_set_options",
    "vr_create_multi", "vr_comm_unique_id", "vr_create_rank", "vr_group_info", "vr_group_tiles", "vr_render_png",
    "vr_render_batch", "vr_create_multi_ex", "vr_group_timing_read", "vr_count_work", "vr_group_traffic_read",
]
VR_COMM_ID_BYTES = 128
VR_TRANSPORT_NONE, VR_TRANSPORT_RCCL, VR_TRANSPORT_PEER_COPY = 0, 1, 2

VR_ORIENT_RAW = 0
VR_ORIENT_VRC_DISPLAY = 1
VR_ORIENT_TEST_DISPLAY = 2
C5_SEED = 0x5EED


class VRError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"{msg} (status {code})")
        self.code = code


class Camera(C.Structure):
    """vr_camera: the AppData camera after processInput's re-derivation (myApp.cu:1106-1112)."""
    _fields_ = [("pos", C.c_float * 3), ("front", C.c_float * 3), ("right", C.c_float * 3),
                ("up", C.c_float * 3), ("top_left", C.c_float * 3)]

    def as_dict(self):
        return {k: [float(v) for v in getattr(self, k)] for k, _ in self._fields_}

    @classmethod
    def from_dict(cls, d):
        c = cls()
        for k, _ in cls._fields_:
            for i in range(3):
                getattr(c, k)[i] = d[k][i]
        return c


class TFInterval(C.Structure):
    _fields_ = [("lo", C.c_float), ("hi", C.c_float), ("rgba", C.c_float * 4)]


class RenderParams(C.Structure):
    """vr_params: AppData render fields (utils.h:36-74) made runtime."""
    _fields_ = [("width", C.c_int32), ("height", C.c_int32), ("samples_per_ray", C.c_int32),
                ("mode", C.c_int32), ("flags", C.c_int32),
                ("real_screen_width", C.c_float), ("real_screen_height", C.c_float),
                ("viewplane_distance", C.c_float), ("front_clip_plane", C.c_float),
                ("sample_distance", C.c_float), ("background", C.c_float * 4), ("ert_epsilon", C.c_float),
                ("shade_ambient", C.c_float), ("shade_diffuse", C.c_float), ("shade_specular", C.c_float),
                ("shade_shininess", C.c_float)]


class VolumeInfo(C.Structure):
    _fields_ = [("dim", C.c_int64 * 3), ("cal_max", C.c_double), ("longest_dimension", C.c_uint32),
                ("octree_depth", C.c_uint32), ("n_tf", C.c_int32), ("zero_transparent", C.c_int32),
                ("device_bytes", C.c_uint64), ("idx64", C.c_int32), ("reserved", C.c_int32),
                ("class_bytes", C.c_uint64)]


class Options(C.Structure):
    """vr_options: measured-default tuning knobs of a context (no environment variables)."""
    _fields_ = [("brick", C.c_int32 * 3), ("cell_shift", C.c_int32), ("force_idx64", C.c_int32),
                ("batch", C.c_int32), ("cull", C.c_int32), ("view_table_reuse", C.c_int32),
                ("work_order", C.c_int32), ("axis_table", C.c_int32), ("occ_lds", C.c_int32),
                ("persist_wgs", C.c_int32), ("farm_tile", C.c_int32), ("farm_rank0_weight", C.c_float),
                ("leaf_map_pad", C.c_int32), ("exact_skip", C.c_int32), ("frames_in_flight", C.c_int32),
                ("test_plane_march", C.c_int32),
                ("comm_timeout_ms", C.c_int32),
                ("class_bits", C.c_int32),
                ("run_words", C.c_int32),
                ("table_split", C.c_int32),
                ("test_corners", C.c_int32),
                ("leaf_columns", C.c_int32)]


class WorkCount(C.Structure):
    """vr_work_count: gathers, bytes and samples evaluated of one frame's march."""
    _fields_ = [("gathers", C.c_uint64), ("bytes", C.c_uint64), ("samples", C.c_uint64),
                ("reserved", C.c_uint64)]


_lib = None


def lib():
    """Load libvr.so (built in-tree by __graft_entry__.build()).  Raises if absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"libvr.so not built at {LIB_PATH}: run `python -c 'import __graft_entry__ as g; g.build()'`")
    # PyTorch-ROCm bundles its own libamdhip64 with the same soname (libamdhip64.so.7).  Load torch
    # first so libvr.so binds to THAT runtime: one HIP runtime per process, and device pointers and
    # streams from torch are valid in libvr (loading /opt/rocm's copy first hides the GPUs from torch).
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = C.CDLL(LIB_PATH)
    P = C.POINTER
    vp = C.c_void_p
    sig = {
        "vr_create": ([P(C.c_float), C.c_int64, C.c_int64, C.c_int64, C.c_double, P(TFInterval), C.c_int32,
                       C.c_int32, P(vp)], C.c_int),
        "vr_create_from_device": ([vp, C.c_int64, C.c_int64, C.c_int64, C.c_double, P(TFInterval), C.c_int32,
                                   C.c_int32, P(vp)], C.c_int),
        "vr_create_from_nifti": ([C.c_char_p, P(TFInterval), C.c_int32, C.c_int32, P(vp)], C.c_int),
        "vr_options_default": ([P(Options)], C.c_int),
        "vr_create_ex": ([vp, C.c_int32, C.c_int64, C.c_int64, C.c_int64, C.c_double, P(TFInterval), C.c_int32,
                          C.c_int32, P(Options), P(vp)], C.c_int),
        "vr_get_options": ([vp, P(Options)], C.c_int),
        "vr_create_multi": ([vp, C.c_int64, C.c_int64, C.c_int64, C.c_double, P(TFInterval), C.c_int32,
                             P(C.c_int32), C.c_int32, P(Options), P(vp)], C.c_int),
        "vr_create_multi_ex": ([vp, C.c_int32, C.c_int64, C.c_int64, C.c_int64, C.c_double, P(TFInterval), C.c_int32,
                                P(C.c_int32), C.c_int32, P(Options), P(vp)], C.c_int),
        "vr_group_timing_read": ([vp, C.c_int32, P(C.c_double), P(C.c_int64), C.c_int32], C.c_int),
        "vr_group_traffic_read": ([vp, C.c_int32, P(C.c_int64), P(C.c_int64), P(C.c_int64), C.c_int32], C.c_int),
        "vr_comm_unique_id": ([vp], C.c_int),
        "vr_create_rank": ([vp, C.c_int32, C.c_int64, C.c_int64, C.c_int64, C.c_double, P(TFInterval), C.c_int32,
                            C.c_int32, C.c_int32, C.c_int32, vp, P(Options), P(vp)], C.c_int),
        "vr_group_info": ([vp, P(C.c_int32), P(C.c_int32), P(C.c_int32)], C.c_int),
        "vr_render_png": ([vp, P(RenderParams), P(Camera), C.c_int32, C.c_char_p], C.c_int),
        "vr_render_batch": ([vp, P(RenderParams), P(Camera), C.c_int32, vp, C.c_int32], C.c_int),
        "vr_group_tiles": ([vp, C.c_int32, P(C.c_int32), C.c_int32, P(C.c_int32)], C.c_int),
        "vr_set_options": ([vp, P(Options)], C.c_int),
        "vr_set_transfer_function": ([vp, P(TFInterval), C.c_int32], C.c_int),
        "vr_destroy": ([vp], C.c_int),
        "vr_render": ([vp, P(RenderParams), P(Camera), vp, C.c_int32], C.c_int),
        "vr_render_tiles": ([vp, P(RenderParams), P(Camera), C.c_int32, C.c_int32, C.c_int32, C.c_int32, vp,
                             P(C.c_int32), C.c_int32], C.c_int),
        "vr_assemble_tiles": ([vp, C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_int32, vp, vp,
                               C.c_int32], C.c_int),
        "vr_count_samples": ([vp, P(RenderParams), P(Camera), P(C.c_uint64)], C.c_int),
        "vr_count_marched": ([vp, P(RenderParams), P(Camera), P(C.c_uint64), P(C.c_uint64)], C.c_int),
        "vr_count_work": ([vp, P(RenderParams), P(Camera), P(WorkCount)], C.c_int),
        "vr_synchronize": ([vp], C.c_int),
        "vr_set_stream": ([vp, vp], C.c_int),
        "vr_params_default": ([C.c_int32, C.c_int32, C.c_int32, P(RenderParams)], C.c_int),
        "vr_camera_derive": ([P(C.c_float), P(C.c_float), C.c_float, C.c_float, P(Camera)], C.c_int),
        "vr_camera_default": ([C.c_int32, C.c_int32, P(Camera)], C.c_int),
        "vr_camera_reset": ([P(Camera)], C.c_int),
        "vr_default_transfer_function": ([P(TFInterval), C.c_int32], C.c_int),
        "vr_get_volume_info": ([vp, P(VolumeInfo)], C.c_int),
        "vr_timing_enable": ([vp, C.c_int32], C.c_int),
        "vr_timing_read": ([vp, P(C.c_double), P(C.c_int64), C.c_int32], C.c_int),
        "vr_strerror": ([C.c_int], C.c_char_p),
        "vr_device_count": ([P(C.c_int32)], C.c_int),
        "vr_api_version": ([], C.c_int),
        "vr_nifti_read": ([C.c_char_p, P(C.c_int64), P(C.c_double), vp], C.c_int),
        "vr_octree_leaf_maps": ([C.c_int64, C.c_int64, C.c_int64, vp, C.c_int64, P(C.c_uint32)], C.c_int),
        "vr_frame_to_rgb8": ([vp, C.c_int32, C.c_int32, C.c_int32, vp, vp, C.c_int32], C.c_int),
        "vr_write_png": ([C.c_char_p, C.c_int32, C.c_int32, vp], C.c_int),
        "vr_synthetic_volume": ([vp, C.c_int64, C.c_int64, C.c_int64, C.c_uint64, C.c_int32, vp], C.c_int),
        "vr_camera_derive_conic": ([P(C.c_float), P(C.c_float), C.c_float, C.c_float, C.c_float, P(Camera)], C.c_int),
        "vr_point_cloud": ([vp, vp, C.c_int32], C.c_int),
        "vr_visible_tiles": ([vp, P(RenderParams), P(Camera), C.c_int32, C.c_int32, P(C.c_int32), C.c_int32,
                              P(C.c_int32)], C.c_int),
        "vr_render_tile_list": ([vp, P(RenderParams), P(Camera), C.c_int32, C.c_int32, P(C.c_int32), C.c_int32,
                                 C.c_int32, C.c_int32, vp, P(C.c_int32), C.c_int32], C.c_int),
        "vr_assemble_tile_list": ([vp, C.c_int32, C.c_int32, C.c_int32, C.c_int32, P(C.c_int32), C.c_int32,
                                   C.c_int32, C.c_int32, vp, P(C.c_float), vp, C.c_int32], C.c_int),
        "vr_assemble_tile_slots": ([vp, C.c_int32, C.c_int32, C.c_int32, C.c_int32, P(C.c_int32), P(C.c_int32),
                                    C.c_int32, C.c_int32, vp, P(C.c_float), vp, C.c_int32], C.c_int),
        "vr_assemble_tile_slots_multi": ([vp, C.c_int32, C.c_int32, C.c_int32, C.c_int32, P(C.c_int32),
                                          P(C.c_int32), C.c_int32, C.c_int32, C.c_int32, vp, P(C.c_float), vp,
                                          C.c_int32], C.c_int),
    }
    for name, (args, res) in sig.items():
        if os.environ.get("VR_LIB") and not hasattr(L, name):
            continue   # (an A/B build from an earlier revision: entry points it predates stay unbound)
        f = getattr(L, name)
        f.argtypes = args
        f.restype = res
    _lib = L
    return L


def _check(rc, what):
    if rc < 0:
        raise VRError(rc, f"{what}: {lib().vr_strerror(rc).decode()}")
    return rc


# ------------------------------------------------------------------------------------------------
# host helpers (AppData / processInput / TransferFunction restated in libvr.so)
# ------------------------------------------------------------------------------------------------

def _out_flags(asynchronous, rgb):
    """out_flags of the tile entry points: VR_OUT_ASYNC, VR_OUT_RGB (3-float tile pixels)."""
    return (VR_OUT_ASYNC if asynchronous else 0) | (VR_OUT_RGB if rgb else 0)


def default_options(**overrides) -> Options:
    """vr_options_default, then the given fields (e.g. cull=0, force_idx64=1, brick=(1, 1, 1))."""
    o = Options()
    _check(lib().vr_options_default(C.byref(o)), "vr_options_default")
    for k, v in overrides.items():
        if k == "brick":
            for i in range(3):
                o.brick[i] = int(v[i])
        elif k == "farm_rank0_weight":
            o.farm_rank0_weight = float(v)
        else:
            setattr(o, k, int(v))
    return o


def default_params(width, height, samples_per_ray, mode=VR_MODE_VRC, flags=0, ert_epsilon=1e-5) -> RenderParams:
    p = RenderParams()
    _check(lib().vr_params_default(width, height, samples_per_ray, C.byref(p)), "vr_params_default")
    p.mode, p.flags, p.ert_epsilon = mode, flags, ert_epsilon
    return p


def default_camera(width, height) -> Camera:
    c = Camera()
    _check(lib().vr_camera_default(width, height, C.byref(c)), "vr_camera_default")
    return c


def reset_camera() -> Camera:
    c = Camera()
    _check(lib().vr_camera_reset(C.byref(c)), "vr_camera_reset")
    return c


def derive_camera(pos, up, real_screen_width, real_screen_height) -> Camera:
    c = Camera()
    P = (C.c_float * 3)(*pos)
    U = (C.c_float * 3)(*up)
    _check(lib().vr_camera_derive(P, U, real_screen_width, real_screen_height, C.byref(c)), "vr_camera_derive")
    return c


def derive_camera_conic(pos, up, real_screen_width, real_screen_height, viewplane_distance) -> Camera:
    c = Camera()
    P = (C.c_float * 3)(*pos)
    U = (C.c_float * 3)(*up)
    _check(lib().vr_camera_derive_conic(P, U, real_screen_width, real_screen_height, viewplane_distance,
                                        C.byref(c)), "vr_camera_derive_conic")
    return c


def default_transfer_function():
    arr = (TFInterval * 16)()
    n = _check(lib().vr_default_transfer_function(arr, 16), "vr_default_transfer_function")
    return [(arr[i].lo, arr[i].hi, tuple(arr[i].rgba)) for i in range(n)]


def _tf_array(tf):
    arr = (TFInterval * len(tf))()
    for i, (lo, hi, rgba) in enumerate(tf):
        arr[i].lo, arr[i].hi = lo, hi
        for c in range(4):
            arr[i].rgba[c] = rgba[c]
    return arr


def nifti_read(path):
    """NiftiFile (BinaryLoader.cu:273-335, hardened) -> (volume float32 [d1,d2,d3], cal_max)."""
    dims = (C.c_int64 * 3)()
    cal = C.c_double(0)
    _check(lib().vr_nifti_read(path.encode(), dims, C.byref(cal), None), "vr_nifti_read")
    vol = np.empty((dims[0], dims[1], dims[2]), np.float32)
    _check(lib().vr_nifti_read(path.encode(), dims, C.byref(cal), vol.ctypes.data_as(C.c_void_p)), "vr_nifti_read")
    return vol, cal.value


def octree_leaf_maps(d1, d2, d3):
    """OctreeHandler's leaf -> voxel maps: (maps int32 [3, 2^D], depth D)."""
    depth = C.c_uint32(0)
    n = _check(lib().vr_octree_leaf_maps(d1, d2, d3, None, 0, C.byref(depth)), "vr_octree_leaf_maps")
    maps = np.empty(n, np.int32)
    _check(lib().vr_octree_leaf_maps(d1, d2, d3, maps.ctypes.data_as(C.c_void_p), n, C.byref(depth)),
           "vr_octree_leaf_maps")
    return maps.reshape(3, -1), depth.value


def device_count():
    n = C.c_int32(0)
    lib().vr_device_count(C.byref(n))
    return n.value


@dataclass
class Timing:
    total_ms: float
    launches: int


class VolumeRenderer:
    """One vr_ctx: a volume + transfer function resident on one GPU."""

    def __init__(self, volume=None, cal_max=None, tf=None, device=0, nifti_path=None, device_ptr=None, shape=None,
                 options: Options | None = None, devices=None, rank=None, n_ranks=None, comm_id=None):
        """One GPU (device), or a multi-GPU context: devices=[...] (one process drives them all,
        vr_create_multi) or rank/n_ranks/comm_id (one process per GPU, vr_create_rank; only rank 0
        passes the volume -- a host array, or with device_ptr a device pointer -- the others pass
        shape)."""
        self._ctx = C.c_void_p()
        if devices is not None or rank is not None:
            self._create_group(device_ptr if device_ptr is not None else volume, cal_max, tf, device, shape, options,
                               devices, rank, n_ranks, comm_id)
            return
        tf = tf if tf is not None else default_transfer_function()
        self._tf = _tf_array(tf)
        L = lib()
        opt = C.byref(options) if options is not None else None
        if options is not None and nifti_path is not None:
            raise ValueError("options: load the volume with nifti_read and pass it as volume=")
        if nifti_path is not None:
            _check(L.vr_create_from_nifti(nifti_path.encode(), self._tf, len(tf), device, C.byref(self._ctx)),
                   "vr_create_from_nifti")
        elif device_ptr is not None:
            d1, d2, d3 = shape
            _check(L.vr_create_ex(C.c_void_p(device_ptr), 1, d1, d2, d3, float(cal_max), self._tf, len(tf),
                                  device, opt, C.byref(self._ctx)), "vr_create_ex")
        else:
            v = np.ascontiguousarray(volume, dtype=np.float32)
            d1, d2, d3 = v.shape
            _check(L.vr_create_ex(v.ctypes.data_as(C.c_void_p), 0, d1, d2, d3, float(cal_max), self._tf,
                                  len(tf), device, opt, C.byref(self._ctx)), "vr_create_ex")
        self.device = device

    def _create_group(self, volume, cal_max, tf, device, shape, options, devices, rank, n_ranks, comm_id):
        tf = tf if tf is not None else default_transfer_function()
        self._tf = _tf_array(tf)
        L = lib()
        opt = C.byref(options) if options is not None else None
        on_dev = 0
        if isinstance(volume, int):          # a device pointer (devices[0] / rank 0's GPU)
            v, vp, on_dev = None, C.c_void_p(volume), 1
            d1, d2, d3 = shape
        else:
            v = None if volume is None else np.ascontiguousarray(volume, dtype=np.float32)
            d1, d2, d3 = v.shape if v is not None else shape
            vp = v.ctypes.data_as(C.c_void_p) if v is not None else None
        if devices is not None:
            devs = (C.c_int32 * len(devices))(*devices)
            _check(L.vr_create_multi_ex(vp, on_dev, d1, d2, d3, float(cal_max), self._tf, len(tf), devs, len(devices),
                                        opt, C.byref(self._ctx)), "vr_create_multi_ex")
            self.device = devices[0]
        else:
            cid = (C.c_uint8 * VR_COMM_ID_BYTES).from_buffer_copy(bytes(comm_id))
            _check(L.vr_create_rank(vp, on_dev, d1, d2, d3, float(cal_max), self._tf, len(tf), device, rank, n_ranks, cid, opt,
                                    C.byref(self._ctx)), "vr_create_rank")
            self.device = device

    @property
    def group(self):
        """(n_gpus, rank, transport) of this context (vr_group_info)."""
        n, r, t = C.c_int32(0), C.c_int32(0), C.c_int32(0)
        _check(lib().vr_group_info(self._ctx, C.byref(n), C.byref(r), C.byref(t)), "vr_group_info")
        return n.value, r.value, t.value

    def group_traffic(self, rank=0, reset=False):
        """(bytes_sent, bytes_received, frames) of part `rank` since the last reset
        (vr_group_traffic_read): tile bytes posted to rank 0 over the transport / posted to receive."""
        tx, rx, fr = C.c_int64(), C.c_int64(), C.c_int64()
        _check(lib().vr_group_traffic_read(self._ctx, rank, C.byref(tx), C.byref(rx), C.byref(fr), int(reset)),
               "vr_group_traffic_read")
        return tx.value, rx.value, fr.value

    def group_tiles(self, rank):
        """Tile ids rank `rank` rendered in the last multi-GPU frame."""
        n = C.c_int32(0)
        _check(lib().vr_group_tiles(self._ctx, rank, None, 0, C.byref(n)), "vr_group_tiles")
        out = np.zeros(max(1, n.value), np.int32)
        _check(lib().vr_group_tiles(self._ctx, rank, out.ctypes.data_as(C.POINTER(C.c_int32)), n.value, C.byref(n)),
               "vr_group_tiles")
        return out[:n.value]

    def close(self):
        if self._ctx:
            lib().vr_destroy(self._ctx)
            self._ctx = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    @property
    def info(self) -> VolumeInfo:
        i = VolumeInfo()
        _check(lib().vr_get_volume_info(self._ctx, C.byref(i)), "vr_get_volume_info")
        return i

    @property
    def options(self) -> Options:
        o = Options()
        _check(lib().vr_get_options(self._ctx, C.byref(o)), "vr_get_options")
        return o

    def set_options(self, options: Options):
        _check(lib().vr_set_options(self._ctx, C.byref(options)), "vr_set_options")

    def set_transfer_function(self, tf):
        self._tf = _tf_array(tf)
        _check(lib().vr_set_transfer_function(self._ctx, self._tf, len(tf)), "vr_set_transfer_function")

    def render(self, params: RenderParams, camera: Camera) -> np.ndarray:
        """Host frame, shape (W, H, 4), x-major like the reference's screen buffer."""
        out = np.empty((params.width, params.height, 4), np.float32)
        _check(lib().vr_render(self._ctx, C.byref(params), C.byref(camera), out.ctypes.data_as(C.c_void_p), 0),
               "vr_render")
        return out

    def render_device(self, params: RenderParams, camera: Camera, out_ptr, asynchronous=False):
        """Frame into device memory (out_ptr; None on the non-zero ranks of a one-process-per-GPU group)."""
        flags = VR_OUT_DEVICE | (VR_OUT_ASYNC if asynchronous else 0)
        _check(lib().vr_render(self._ctx, C.byref(params), C.byref(camera), C.c_void_p(out_ptr), flags), "vr_render")

    def render_batch_device(self, params: RenderParams, cameras, out_ptr, asynchronous=False, n=None):
        """vr_render_batch: len(cameras) frames (or the first n of a ctypes Camera array) into
        consecutive device frames at out_ptr (None on the non-zero ranks of a one-process-per-GPU group)."""
        cams = cameras if isinstance(cameras, C.Array) else (Camera * len(cameras))(*cameras)
        n = len(cams) if n is None else int(n)
        if not 0 <= n <= len(cams):
            raise ValueError("render_batch_device: n out of range")
        flags = VR_OUT_DEVICE | (VR_OUT_ASYNC if asynchronous else 0)
        _check(lib().vr_render_batch(self._ctx, C.byref(params), cams, n, C.c_void_p(out_ptr), flags),
               "vr_render_batch")

    def render_batch(self, params: RenderParams, cameras) -> np.ndarray:
        """Host frames, shape (n, W, H, 4)."""
        cams = (Camera * len(cameras))(*cameras)
        out = np.empty((len(cameras), params.width, params.height, 4), np.float32)
        _check(lib().vr_render_batch(self._ctx, C.byref(params), cams, len(cams), out.ctypes.data_as(C.c_void_p), 0),
               "vr_render_batch")
        return out

    def render_tiles(self, params, camera, tile_w, tile_h, first_tile, tile_stride, out_ptr, asynchronous=False,
                     rgb=False):
        n = C.c_int32(0)
        _check(lib().vr_render_tiles(self._ctx, C.byref(params), C.byref(camera), tile_w, tile_h, first_tile,
                                     tile_stride, C.c_void_p(out_ptr), C.byref(n), _out_flags(asynchronous, rgb)),
               "vr_render_tiles")
        return n.value

    def assemble_tiles(self, width, height, tile_w, tile_h, n_ranks, max_tiles, tiles_ptr, frame_ptr,
                       asynchronous=False, rgb=False):
        _check(lib().vr_assemble_tiles(self._ctx, width, height, tile_w, tile_h, n_ranks, max_tiles,
                                       C.c_void_p(tiles_ptr), C.c_void_p(frame_ptr), _out_flags(asynchronous, rgb)),
               "vr_assemble_tiles")

    def visible_tiles(self, params, camera, tile_w, tile_h) -> np.ndarray:
        """Tile ids that can hold a non-background pixel (vr_visible_tiles), ascending."""
        n = C.c_int32(0)
        _check(lib().vr_visible_tiles(self._ctx, C.byref(params), C.byref(camera), tile_w, tile_h, None, 0,
                                      C.byref(n)), "vr_visible_tiles")
        out = np.zeros(max(1, n.value), np.int32)
        _check(lib().vr_visible_tiles(self._ctx, C.byref(params), C.byref(camera), tile_w, tile_h,
                                      out.ctypes.data_as(C.POINTER(C.c_int32)), n.value, C.byref(n)),
               "vr_visible_tiles")
        return out[:n.value]

    def render_tile_list(self, params, camera, tile_w, tile_h, tiles, first, stride, out_ptr, asynchronous=False,
                         rgb=False):
        t = np.ascontiguousarray(tiles, dtype=np.int32)
        n = C.c_int32(0)
        _check(lib().vr_render_tile_list(self._ctx, C.byref(params), C.byref(camera), tile_w, tile_h,
                                         t.ctypes.data_as(C.POINTER(C.c_int32)), len(t), first, stride,
                                         C.c_void_p(out_ptr), C.byref(n), _out_flags(asynchronous, rgb)),
               "vr_render_tile_list")
        return n.value

    def assemble_tile_list(self, width, height, tile_w, tile_h, tiles, n_ranks, max_tiles, tiles_ptr, background,
                           frame_ptr, asynchronous=False, rgb=False):
        t = np.ascontiguousarray(tiles, dtype=np.int32)
        bg = (C.c_float * 4)(*background)
        _check(lib().vr_assemble_tile_list(self._ctx, width, height, tile_w, tile_h,
                                           t.ctypes.data_as(C.POINTER(C.c_int32)), len(t), n_ranks, max_tiles,
                                           C.c_void_p(tiles_ptr), bg, C.c_void_p(frame_ptr),
                                           _out_flags(asynchronous, rgb)), "vr_assemble_tile_list")

    def assemble_tile_slots(self, width, height, tile_w, tile_h, tiles, slots, n_blocks, tiles_ptr, background,
                            frame_ptr, asynchronous=False, rgb=False):
        """vr_assemble_tile_slots: tile tiles[i] is block slots[i] of the gathered buffer."""
        t = np.ascontiguousarray(tiles, dtype=np.int32)
        sl = np.ascontiguousarray(slots, dtype=np.int32)
        if len(t) != len(sl):
            raise ValueError("tiles and slots differ in length")
        bg = (C.c_float * 4)(*background)
        _check(lib().vr_assemble_tile_slots(self._ctx, width, height, tile_w, tile_h,
                                            t.ctypes.data_as(C.POINTER(C.c_int32)),
                                            sl.ctypes.data_as(C.POINTER(C.c_int32)), len(t), n_blocks,
                                            C.c_void_p(tiles_ptr), bg, C.c_void_p(frame_ptr),
                                            _out_flags(asynchronous, rgb)), "vr_assemble_tile_slots")

    def count_samples(self, params, camera) -> int:
        n = C.c_uint64(0)
        _check(lib().vr_count_samples(self._ctx, C.byref(params), C.byref(camera), C.byref(n)), "vr_count_samples")
        return int(n.value)

    def count_marched(self, params, camera):
        """(class gathers that touched memory, samples evaluated) of one frame as vr_render marches
        it (vr_count_marched: the counting instantiation of the same kernel variant)."""
        g, n = C.c_uint64(0), C.c_uint64(0)
        _check(lib().vr_count_marched(self._ctx, C.byref(params), C.byref(camera), C.byref(g), C.byref(n)),
               "vr_count_marched")
        return int(g.value), int(n.value)

    def count_work(self, params, camera) -> dict:
        """{gathers, bytes, samples} of one frame as vr_render marches it, VRC or TEST
        (vr_count_work: the counting instantiation of the same kernel variant)."""
        w = WorkCount()
        _check(lib().vr_count_work(self._ctx, C.byref(params), C.byref(camera), C.byref(w)), "vr_count_work")
        return {"gathers": int(w.gathers), "bytes": int(w.bytes), "samples": int(w.samples)}

    def synchronize(self):
        _check(lib().vr_synchronize(self._ctx), "vr_synchronize")

    def set_stream(self, stream_handle):
        _check(lib().vr_set_stream(self._ctx, C.c_void_p(stream_handle)), "vr_set_stream")

    def point_cloud_device(self, out_ptr, asynchronous=False):
        """POINT-mode vertex array (vr_point_cloud) into device memory: d1*d2*d3*7 floats."""
        _check(lib().vr_point_cloud(self._ctx, C.c_void_p(out_ptr), VR_OUT_ASYNC if asynchronous else 0),
               "vr_point_cloud")

    def frame_to_rgb8(self, width, height, frame_ptr, orientation=VR_ORIENT_VRC_DISPLAY) -> np.ndarray:
        """Display-ordered RGB8 image (H, W, 3) of a device frame (vr_frame_to_rgb8)."""
        img = np.empty((height, width, 3), np.uint8)
        _check(lib().vr_frame_to_rgb8(self._ctx, width, height, orientation, C.c_void_p(frame_ptr),
                                      img.ctypes.data_as(C.c_void_p), 0), "vr_frame_to_rgb8")
        return img

    def save_png(self, path, width, height, frame_ptr, orientation=VR_ORIENT_VRC_DISPLAY) -> np.ndarray:
        """saveImage for a headless box: device frame -> RGB8 on the GPU -> PNG file.  Returns the image."""
        img = self.frame_to_rgb8(width, height, frame_ptr, orientation)
        write_png(path, img)
        return img

    def timing_enable(self, on=True):
        _check(lib().vr_timing_enable(self._ctx, 1 if on else 0), "vr_timing_enable")

    def timing_read(self, reset=True, rank=None) -> Timing:
        """Summed march-kernel milliseconds and launches since the last reset; rank: one GPU of a
        multi-GPU context (vr_group_timing_read), None = this context's own GPU."""
        ms = C.c_double(0)
        n = C.c_int64(0)
        if rank is None:
            _check(lib().vr_timing_read(self._ctx, C.byref(ms), C.byref(n), 1 if reset else 0), "vr_timing_read")
        else:
            _check(lib().vr_group_timing_read(self._ctx, rank, C.byref(ms), C.byref(n), 1 if reset else 0),
                   "vr_group_timing_read")
        return Timing(ms.value, n.value)


def comm_unique_id() -> bytes:
    """An RCCL unique id for vr_create_rank (rank 0 makes it, every rank gets a copy)."""
    buf = (C.c_uint8 * VR_COMM_ID_BYTES)()
    _check(lib().vr_comm_unique_id(buf), "vr_comm_unique_id")
    return bytes(buf)


def write_png(path, img: np.ndarray):
    """vr_write_png of an (H, W, 3) uint8 image, top row first."""
    img = np.ascontiguousarray(img, dtype=np.uint8)
    if img.ndim != 3 or img.shape[2] != 3:
        raise ValueError("write_png: need an (H, W, 3) uint8 image")
    _check(lib().vr_write_png(os.fsencode(path), img.shape[1], img.shape[0], img.ctypes.data_as(C.c_void_p)),
           "vr_write_png")


def synthetic_volume(out_ptr, n, x0=0, nx=None, seed=C5_SEED, device=0, stream=0):
    """Fill device memory with the x-slab [x0, x0+nx) of the synthetic n^3 C5 volume (vr_synthetic_volume)."""
    nx = n - x0 if nx is None else nx
    _check(lib().vr_synthetic_volume(C.c_void_p(out_ptr), n, x0, nx, seed, device, C.c_void_p(stream)),
           "vr_synthetic_volume")


def tiles_per_rank(width, height, tile_w, tile_h, rank, world):
    ntx = (width + tile_w - 1) // tile_w
    nty = (height + tile_h - 1) // tile_h
    nt = ntx * nty
    return 0 if rank >= nt else (nt - 1 - rank) // world + 1
