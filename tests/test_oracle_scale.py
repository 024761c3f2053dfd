"""CPU checks of the oracle pieces used at C4/C5 scale (no GPU):

* the node-pool-free octree (closed form of Octree.cu:158-183) equals the literal tree on every leaf
  and on whole frames, so it can stand in where the node pool cannot exist (512^3: 5.5 GB,
  2048^3: 353 GB);
* the column renderer equals the full-frame renderer on those columns;
* the synthetic C5 generator equals an independent numpy statement of the formula.
"""
import numpy as np
import pytest


@pytest.mark.parametrize("shape", [(91, 109, 91), (7, 5, 3), (16, 16, 16), (17, 9, 33)])
def test_implicit_octree_equals_literal_tree(oracle_mod, shape):
    rng = np.random.default_rng(sum(shape))
    vol = rng.integers(-20, 255, size=shape).astype(np.float32)
    lit = oracle_mod.OracleOctree(vol)
    imp = oracle_mod.OracleOctree(vol, implicit=True)
    assert imp.depth == lit.depth and imp.longest_dimension == lit.longest_dimension
    assert np.array_equal(imp.leaf_values(), lit.leaf_values())
    q = rng.uniform(-0.1, 1.1, size=(2000, 3)).astype(np.float32)
    assert all(imp.intensity(p) == lit.intensity(p) for p in q)


@pytest.mark.parametrize("camera", ["default", "oblique"])
def test_implicit_octree_frames_and_columns(avg152, avg152_octree, oracle_mod, camera):
    O = oracle_mod
    vol, cal = avg152
    W, H, S = 40, 30, 64
    cam = O.camera_default(W, H) if camera == "default" else O.camera_oblique(W, H)
    p = O.params(W, H, S)
    ref = avg152_octree.render_vrc(cal, O.default_tf(), p, cam)
    imp = O.OracleOctree(vol, implicit=True)
    assert np.array_equal(imp.render_vrc(cal, O.default_tf(), p, cam), ref)
    xs = [0, 7, 19, 20, 39]
    assert np.array_equal(imp.render_vrc_columns(cal, O.default_tf(), p, cam, xs), ref[xs])


def splitmix64(x):
    with np.errstate(over="ignore"):
        z = x + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def synthetic_numpy(n, x0, nx, seed=0x5EED):
    x, y, z = np.meshgrid(np.arange(x0, x0 + nx), np.arange(n), np.arange(n), indexing="ij")
    c = (n - 1) / 2.0
    r = np.sqrt((x - c) ** 2 + (y - c) ** 2 + (z - c) ** 2) / (n / 2.0)
    w = np.floor(127.5 + 127.5 * np.sin(16.0 * np.pi * r) + 0.5)        # round half away (w >= 0)
    idx = ((x * n + y) * n + z).astype(np.uint64)
    noise = (splitmix64(np.uint64(seed) ^ idx) % np.uint64(17)).astype(np.int64) - 8
    v = np.clip(w.astype(np.int64) + noise, 0, 255)
    return np.where(r < 0.95, v, 0).astype(np.float32)


@pytest.mark.parametrize("n,x0,nx", [(32, 0, 32), (2048, 1023, 2), (2048, 60, 1)])
def test_synthetic_generator_formula(oracle_mod, n, x0, nx):
    got = oracle_mod.synthetic_slab(n, x0, nx)
    ref = synthetic_numpy(n, x0, nx)
    assert np.array_equal(got, ref)
    if n == 2048 and x0 == 1023:
        assert got[:, 0, 0].max() == 0 and got.max() == 255     # corners outside r < 0.95; clamped range
