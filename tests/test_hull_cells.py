"""The MPR hull support's direction cells (so100_hull_cells, include/so100.h) against the exhaustive scan
the oracle does (oracle/so100_oracle.c mpr support; MuJoCo's mesh support): for every direction, the first
maximal vertex of the cell's candidate list, with fp32 scores as the kernel computes them, is the first
maximal vertex of the whole hull, so the lookup changes no result.  CPU only (a host function of the
C-ABI library)."""
import ctypes

import numpy as np
import pytest

from gym_so100 import _native
from gym_so100.model import NHULL_ALL as SO100_NHULL_ALL

G = _native.HULL_CELLG
NCELL = _native.HULL_NCELL


@pytest.fixture(scope="module")
def tables(model):
    lib = _native.load()
    n = lib.so100_hull_cells(ctypes.byref(model), None, None, 0)
    assert n > 0, lib.so100_last_error()
    cells = np.zeros(SO100_NHULL_ALL * NCELL, np.uint32)
    cand = np.zeros((n, 4), np.float32)
    assert lib.so100_hull_cells(ctypes.byref(model), ctypes.c_void_p(cells.ctypes.data),
                                ctypes.c_void_p(cand.ctypes.data), n) == n
    assert lib.so100_hull_cells(ctypes.byref(model), None, ctypes.c_void_p(cand.ctypes.data), n - 1) == -1
    return cells, cand


def hull_verts(model, k):
    s0, n = model.hull_start[k], model.hull_count[k]
    return np.array([[model.hull_vert[s0 + i][t] for t in range(3)] for i in range(n)], np.float32)


def cell_of(d):
    """The kernel's face / cell selection (so100_step.hip hull_support), fp32."""
    a = np.abs(d)
    fx = (a[:, 0] >= a[:, 1]) & (a[:, 0] >= a[:, 2])
    fy = ~fx & (a[:, 1] >= a[:, 2])
    am = np.where(fx, a[:, 0], np.where(fy, a[:, 1], a[:, 2]))
    na = np.where(fx, d[:, 0], np.where(fy, d[:, 1], d[:, 2]))
    nu = np.where(fx, d[:, 1], d[:, 0])
    nv = np.where(fx | fy, d[:, 2], d[:, 1])
    g = np.float32(0.5 * G) / am
    cu = np.clip(((nu + am) * g).astype(np.int64), 0, G - 1)
    cv = np.clip(((nv + am) * g).astype(np.int64), 0, G - 1)
    face = 2 * np.where(fx, 0, np.where(fy, 1, 2)) + (na < 0)
    return (face * G + cu) * G + cv


def scores(d, X, fma):
    d64, X64 = d.astype(np.float64), X.astype(np.float64)
    if fma:    # fma(n2, z, fma(n1, y, n0 * x)): each product exact in fp64, one rounding per step
        t = (d64[:, None, 0] * X64[None, :, 0]).astype(np.float32).astype(np.float64)
        t = (d64[:, None, 1] * X64[None, :, 1] + t).astype(np.float32).astype(np.float64)
        return (d64[:, None, 2] * X64[None, :, 2] + t).astype(np.float32)
    d32 = d.astype(np.float32)
    return (d32[:, None, 0] * X[None, :, 0] + d32[:, None, 1] * X[None, :, 1]) + d32[:, None, 2] * X[None, :, 2]


def directions(rng, X):
    d = [rng.standard_normal((6000, 3))]
    ax = np.eye(3)
    d.append(np.concatenate([ax, -ax]))                          # exact ties on axis-aligned flat faces
    d.append(np.concatenate([ax, -ax]).repeat(200, 0) + 1e-4 * rng.standard_normal((1200, 3)))
    # directions on and next to the cell boundaries of each face
    b = -1.0 + 2.0 * rng.integers(0, G + 1, (3000, 2)) / G + rng.choice([-1e-7, 0.0, 1e-7, 1e-4], (3000, 2))
    f = rng.integers(0, 6, 3000)
    e = np.zeros((3000, 3))
    for i in range(3000):
        axi, sg = f[i] // 2, (-1.0 if f[i] % 2 else 1.0)
        oth = [t for t in range(3) if t != axi]
        e[i, axi], e[i, oth[0]], e[i, oth[1]] = sg, b[i, 0], b[i, 1]
    d.append(e)
    # normals of the hull's faces through vertex triples (ties between coplanar vertices)
    i = rng.integers(0, len(X), (1500, 3))
    n = np.cross(X[i[:, 1]] - X[i[:, 0]], X[i[:, 2]] - X[i[:, 0]]).astype(np.float64)
    ok = np.linalg.norm(n, axis=1) > 1e-9
    d.append(n[ok] / np.linalg.norm(n[ok], axis=1, keepdims=True))
    d = np.concatenate(d)
    return (d / np.linalg.norm(d, axis=1, keepdims=True)).astype(np.float32)


@pytest.mark.parametrize("k", range(SO100_NHULL_ALL))
def test_cell_lists_give_the_scan_support(model, tables, k):
    cells, cand = tables
    X = hull_verts(model, k)
    rng = np.random.default_rng(100 + k)
    d = directions(rng, X)
    e = cells[k * NCELL + cell_of(d)]
    cnt, start = (e & 255).astype(np.int64), (e >> 8).astype(np.int64)
    assert (cnt > 0).mean() > 0.9, "most cells carry a list"
    for fma in (False, True):
        S = scores(d, X, fma)
        full = np.argmax(S, axis=1)                           # first maximal vertex
        for r in np.nonzero(cnt > 0)[0]:
            idx = cand[start[r]:start[r] + cnt[r], 3].view(np.int32)
            assert np.all(np.diff(idx) > 0), "candidates in vertex order"
            got = idx[np.argmax(S[r, idx])]
            assert got == full[r], (k, r, d[r], got, full[r])


def test_cell_candidates_are_hull_vertices(model, tables):
    cells, cand = tables
    sizes = []
    for k in range(SO100_NHULL_ALL):
        X = hull_verts(model, k)
        e = cells[k * NCELL:(k + 1) * NCELL]
        for c in e[(e & 255) > 0]:
            s, n = int(c >> 8), int(c & 255)
            idx = cand[s:s + n, 3].view(np.int32)
            assert np.all((idx >= 0) & (idx < len(X)))
            np.testing.assert_array_equal(cand[s:s + n, :3], X[idx])
            sizes.append(n)
    assert np.mean(sizes) < 16, "lists short enough to pay (one or two loads per lane)"
