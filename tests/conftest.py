import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))

# The library reads its A/B and diagnostic knobs (RT_VERTEX, RT_SPLIT, RT_STACK_DEPTH, ...) only behind
# this gate (csrc/rt_knobs.h); the tests that set knobs rely on it.  test_knob_gate.py checks that
# without the gate a knob in the environment changes nothing.
os.environ["RT_DEBUG_KNOBS"] = "1"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run on the GPU box via gpurun)")
    config.addinivalue_line("markers", "slow: longer CPU-side checks")
