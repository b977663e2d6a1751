#!/usr/bin/env python3
"""Exhaustive check of the kernels' cos/sin of the hemisphere angle (rt_device.h sincos_f, through
rt_math_selftest) against the host libm's cosf/sinf (glibc; oracle or_trig) for EVERY float in
[0, 2*PI] (MC/WhittedMaterial.h:80-81).  The GPU test (test_gpu_parity.py) sweeps a strided 3 % of
them; this tool covers all 1.09e9.

    python tools/verify_trig.py            # prints one JSON line
"""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
import _oracle as O  # noqa: E402
from _rt import rt  # noqa: E402


def main():
    ctx = rt.Context(0)
    top = int(np.float32(6.2831855).view(np.uint32))
    chunk = 1 << 24
    bad = 0
    n = 0
    for start in range(0, top + 1, chunk):
        b = np.arange(start, min(start + chunk, top + 1), dtype=np.uint32)
        x = b.view(np.float32)
        out = ctx.math_selftest(x)
        c, s = O.libm_trig(x)
        bad += int(np.count_nonzero(out[:, 2].view(np.uint32) != c.view(np.uint32)))
        bad += int(np.count_nonzero(out[:, 3].view(np.uint32) != s.view(np.uint32)))
        n += b.size
        print(f"{n} floats, {bad} mismatches", file=sys.stderr, flush=True)
    print(json.dumps({"floats": n, "range": "[0, 2*PI]", "mismatches": bad}))
    return 0 if bad == 0 else 1


if __name__ == "__main__":
    sys.exit(main())
