"""Moller-Trumbore at a triangle's third edge (rt_device.h moller_trumbore_od, RT_MT_SURE): the kernels decide
(1 - b2) - b3 > 0 in float when RN(|b2n| + |b3n|) < RN(|den| (1 - 2^-20)) and |den| >= 2^-100, and take the
reference's double products only for lanes in the band around b2 + b3 = 1 (MC/TriangleMesh.h:19-45).  These
cases aim rays exactly at points of the edge b -> c (b2 + b3 = 1), a few ulps to either side of it, at the
other two edges, with grazing directions and at triangles small enough that den is subnormal, and compare
the device's verdict and t with the CPU restatement (oracle/rt_oracle.cpp or_mt, pinned to the reference's
mt_cases fixture in test_oracle_golden.py) bit for bit."""
import numpy as np
import pytest

import _oracle as O
from _rt import rt


def bits(a):
    return np.ascontiguousarray(a).view(np.uint64 if a.dtype == np.float64 else np.uint32)


def edge_cases(n=20000, seed=7):
    rng = np.random.default_rng(seed)
    a = rng.normal(size=(n, 3)).astype(np.float32)
    b = (a + rng.normal(size=(n, 3))).astype(np.float32)
    c = (a + rng.normal(size=(n, 3))).astype(np.float32)
    kind = rng.integers(0, 4, n)
    # a point on the edge b -> c (kind 0, 1), c -> a (2) or a -> b (3)
    s = rng.random(n)[:, None]
    p0, p1 = np.where(kind[:, None] <= 1, b, np.where(kind[:, None] == 2, c, a)), np.where(kind[:, None] <= 1, c, np.where(kind[:, None] == 2, a, b))
    p = p0.astype(np.float64) + s * (p1.astype(np.float64) - p0.astype(np.float64))
    o = (p + rng.normal(size=(n, 3)) * 3.0).astype(np.float32)
    d = (p - o.astype(np.float64))
    d /= np.linalg.norm(d, axis=1)[:, None]
    d = d.astype(np.float32)
    # kind 1: a few ulps off the exact direction, either way
    nud = rng.integers(-4, 5, (n, 3)).astype(np.int32)
    d = np.where((kind == 1)[:, None], (d.view(np.int32) + nud).view(np.float32), d)
    cases = np.concatenate([a, b, c, o, d], axis=1).astype(np.float32)
    # grazing rays: direction nearly in the triangle's plane
    m = n // 10
    nrm = np.cross(b[:m] - a[:m], c[:m] - a[:m])
    nrm /= np.linalg.norm(nrm, axis=1)[:, None]
    dg = cases[:m, 12:15] - (np.sum(cases[:m, 12:15] * nrm, axis=1)[:, None] * (1 - 1e-4 * rng.random(m)[:, None])) * nrm
    cases[:m, 12:15] = dg.astype(np.float32)
    # tiny triangles (den subnormal or near it): scale the geometry around the hit point by 2^-40 .. 2^-60
    t = n // 10
    sc = np.float32(2.0) ** -rng.integers(40, 61, t).astype(np.float32)
    tri = cases[m:m + t, 0:9].reshape(t, 3, 3)
    cases[m:m + t, 0:9] = (tri * sc[:, None, None]).reshape(t, 9)
    cases[m:m + t, 9:12] = cases[m:m + t, 9:12] * sc[:, None]
    return cases


def test_edge_cases_exercise_the_band():
    """The oracle sees hits and misses at the edges (the cases sit on the decision boundary)."""
    hit, _ = O.mt(edge_cases())
    assert 0.2 < hit.mean() < 0.8


@pytest.mark.gpu
def test_device_mt_at_the_edges_matches_oracle():
    cases = edge_cases()
    oh, ot = O.mt(cases)
    c = rt.Context(0)
    try:
        mh, mt, _ = c.debug_primitives(cases, np.zeros((1, 12), np.float32))
    finally:
        c.close()
    assert np.array_equal(mh, oh)
    hit = oh == 1
    assert np.array_equal(bits(mt[hit]), bits(ot[hit]))
