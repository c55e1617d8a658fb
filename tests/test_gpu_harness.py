"""The C ABI driven from a plain C++ program (tools/ono_harness.cpp) — no
Python or torch in the process — checked against the C oracle: a ring round
on host buckets, a three-worker TCP-edge ring, a BlockingStore + BarrierSync round."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HARNESS = os.path.join(ROOT, "tools", "ono_harness")

pytestmark = pytest.mark.gpu


def test_cpp_harness_bit_exact():
    if not os.path.exists(HARNESS):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tools"), "harness"], check=True)
    r = subprocess.run([HARNESS, "1000003"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.count("bit-exact") == 3, r.stdout  # ring n=1, TCP-edge ring, store
