"""rt_device.h udiv24: x / d for x < 2^24 from the float reciprocal and one correction either way, as the path
kernel decodes its camera records (segment / n_tiles, tile / tiles_x, local row / band).  The device code uses
IEEE single operations only (u32 -> f32 conversion, a rounded multiply, truncation to u32, a 24-bit multiply),
so this numpy restatement of the same operations checks the algorithm on the CPU: every divisor up to 4096
and random large ones, against random and edge dividends below 2^24."""
import numpy as np


def udiv24(x, d):
    rd = np.float32(1.0 / float(d))   # the host's (float)(1.0 / (double)d)
    q = (x.astype(np.float32) * rd).astype(np.uint32)   # RN multiply, truncation
    r = x.astype(np.int64) - q.astype(np.int64) * d
    q = np.where(r < 0, q - 1, np.where(r >= d, q + 1, q))
    return q.astype(np.uint32)


def test_udiv24_matches_integer_division():
    rng = np.random.default_rng(0)
    top = (1 << 24) - 1
    edges = np.array([0, 1, 2, 3, top, top - 1, 1 << 23, (1 << 23) - 1, (1 << 23) + 1], np.uint32)
    ds = list(range(1, 4097)) + [int(v) for v in rng.integers(4097, 1 << 24, 300)] + [top, 1 << 23, (1 << 23) + 1]
    for d in ds:
        x = np.concatenate([edges, rng.integers(0, 1 << 24, 2000, dtype=np.uint32),
                            (np.arange(1, 200, dtype=np.uint64) * d).clip(0, top).astype(np.uint32),
                            ((np.arange(1, 200, dtype=np.uint64) * d).clip(1, top) - 1).astype(np.uint32)])
        assert np.array_equal(udiv24(x, d), x // np.uint32(d)), d
