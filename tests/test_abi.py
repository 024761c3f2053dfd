"""The C-ABI library builds, loads and exports every symbol include/vr_api.h declares (no GPU)."""
import os
import re
import subprocess

from conftest import ROOT


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "vr_api.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:int|const char\*|int32_t)\s+(vr_\w+)\s*\(", src, flags=re.M)))


def test_header_symbols_exported():
    from volumerenderingproject_amd import renderer
    L = renderer.lib()
    syms = declared_symbols()
    assert len(syms) >= 20
    for s in syms:
        assert hasattr(L, s), s
    assert sorted(renderer.EXPORTED) == syms
    out = subprocess.run(["nm", "-D", "--defined-only", renderer.LIB_PATH], capture_output=True, text=True).stdout
    for s in syms:
        assert re.search(rf"\bT {s}$", out, flags=re.M), f"{s} not exported as text symbol"


def test_library_is_gfx950_code_object():
    from volumerenderingproject_amd import renderer
    data = open(renderer.LIB_PATH, "rb").read()
    assert b"gfx950" in data


def test_header_compiles_as_c():
    # the boundary is plain C: no C++ or torch types
    r = subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-fsyntax-only", "-x", "c", "-I", os.path.join(ROOT, "include"),
                        "-"], input='#include "vr_api.h"\nint main(void){return vr_api_version();}\n',
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def test_no_gpu_paths_fail_cleanly():
    from volumerenderingproject_amd import renderer as R
    import ctypes as C
    ctx = C.c_void_p()
    tf = R._tf_array(R.default_transfer_function())
    import numpy as np
    v = np.zeros((4, 4, 4), np.float32)
    rc = R.lib().vr_create(v.ctypes.data_as(C.POINTER(C.c_float)), 4, 4, 4, 255.0, tf, 4, 0, C.byref(ctx))
    if R.device_count() == 0:
        assert rc == -6 and not ctx.value   # VR_ENODEV, nothing allocated
    else:
        assert rc == 0
        R.lib().vr_destroy(ctx)
    assert R.lib().vr_render(None, None, None, None, 0) == -1
    assert R.lib().vr_strerror(-6) == b"no such GPU"


def test_struct_layouts_match_ctypes(tmp_path):
    """Every C struct of the boundary has the size and field offsets of its ctypes mirror (the
    Python binding passes them by pointer)."""
    import ctypes as C
    from volumerenderingproject_amd import renderer as R
    pairs = [("vr_camera", R.Camera), ("vr_tf_interval", R.TFInterval), ("vr_params", R.RenderParams),
             ("vr_volume_info", R.VolumeInfo), ("vr_options", R.Options), ("vr_work_count", R.WorkCount)]
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "vr_api.h"', "int main(void) {"]
    for cname, py in pairs:
        lines.append(f'printf("{cname} size %zu\\n", sizeof({cname}));')
        for fname, _ in py._fields_:
            lines.append(f'printf("{cname} {fname} %zu\\n", offsetof({cname}, {fname}));')
    lines.append("return 0; }")
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines) + "\n")
    exe = tmp_path / "layout"
    r = subprocess.run(["gcc", "-std=c99", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    got = dict(line.rsplit(" ", 1) for line in subprocess.run([str(exe)], capture_output=True, text=True,
                                                                check=True).stdout.splitlines())
    for cname, py in pairs:
        assert int(got[f"{cname} size"]) == C.sizeof(py), cname
        for fname, _ in py._fields_:
            assert int(got[f"{cname} {fname}"]) == getattr(py, fname).offset, (cname, fname)


def test_options_defaults():
    """vr_options_default (no GPU needed) fills the measured defaults DESIGN.md documents: leaf-column
    ESS masks on, the x-major TEST corner volume (round 6), two frames in flight, automatic batch and class width."""
    from volumerenderingproject_amd import renderer as R
    o = R.default_options()
    assert o.leaf_columns == 1 and o.test_corners == 0 and o.frames_in_flight == 1
    assert o.batch == 0 and o.class_bits == 0 and o.cull == 2 and o.cell_shift == -1
    assert R.default_options(leaf_columns=0).leaf_columns == 0
