"""Statistical gate against the reference's SHIPPED random stream (last bullet).

The per-pixel parity tests pin every operation of the path with the counter-based Philox stream
injected into the reference.  This file checks that replacing the reference's
own generator -- one serial std::mt19937 seeded 5489 (WN/Random.cpp:5, WN/Random.h:27-48) -- by that
stream does not change the estimator: tests/golden/stat_mt19937.npz is the reference rendering the
Cornell box with its shipped stream (64x64, 1024 spp, RR 0.8; oracle/gen_golden.py `stat`).

Gate: RMSE(ours, shipped reference) <= 1.2 x the independent-seed noise floor RMSE(ours seed 0,
ours seed 1), and |mean(ours) - mean(reference)| < 0.5 % of the reference mean, on clamp(accum/spp)."""
import os

import numpy as np
import pytest

import _oracle as O
from _rt import rt

FLOOR_FACTOR = 1.2
MEAN_TOL = 0.005


@pytest.fixture(scope="module")
def shipped():
    z = np.load(os.path.join(O.GOLDEN, "stat_mt19937.npz"))
    return z["accum"], int(z["W"]), int(z["H"]), int(z["spp"]), float(z["rr"])


def img(acc, spp):
    return np.clip(acc[..., :3] / np.float32(spp), 0, 1).astype(np.float64)


def rmse(a, b):
    return float(np.sqrt(np.mean((a - b) ** 2)))


def gate(ref, a0, a1):
    err, floor = rmse(a0, ref), rmse(a0, a1)
    dmean = abs(a0.mean() - ref.mean()) / ref.mean()
    assert err <= FLOOR_FACTOR * floor, (err, floor)
    assert dmean < MEAN_TOL, dmean
    return err, floor, dmean


def test_oracle_counter_stream_matches_shipped_mt19937(shipped):
    acc, W, H, spp, rr = shipped
    sc = O.Scene()
    a0, _, _ = sc.render(W, H, spp, seed=0, rr=rr, threads=min(8, os.cpu_count() or 1))
    a1, _, _ = sc.render(W, H, spp, seed=1, rr=rr, threads=min(8, os.cpu_count() or 1))
    gate(img(acc, spp), img(a0, spp), img(a1, spp))


@pytest.mark.gpu
def test_gpu_matches_shipped_mt19937(shipped):
    acc, W, H, spp, rr = shipped
    ctx = rt.Context(0)
    try:
        ctx.upload(rt.Scene.cornell())
        ctx.resize(W, H)
        cam, _, _ = rt.camera_default(W, H)
        _, g0 = ctx.render(cam, spp, seed=0, rr=rr)
        _, g1 = ctx.render(cam, spp, seed=1, rr=rr)
        _, f0 = ctx.render(cam, spp, seed=0, rr=rr, exact=False)
    finally:
        ctx.close()
    ref = img(acc, spp)
    gate(ref, img(g0, spp), img(g1, spp))
    gate(ref, img(f0, spp), img(g1, spp))   # FAST (forward-accumulating) mode passes the same gate
