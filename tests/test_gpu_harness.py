"""The C ABI driven from plain C++ programs (tests/native/ono_harness.cpp, tests/native/ono_xgmi_harness.cpp) — no
Python or torch in the process — checked against the C oracle: a ring round
on host buckets, a three-worker TCP-edge ring, a BlockingStore + BarrierSync round."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NATIVE = os.path.join(ROOT, "tests", "native")
HARNESS = os.path.join(NATIVE, "ono_harness")

pytestmark = pytest.mark.gpu


def test_cpp_harness_bit_exact():
    if not os.path.exists(HARNESS):
        subprocess.run(["make", "-s", "-C", NATIVE, "ono_harness"], check=True)
    r = subprocess.run([HARNESS, "1000003"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.count("bit-exact") == 3, r.stdout  # ring n=1, TCP-edge ring, store


XGMI_HARNESS = os.path.join(NATIVE, "ono_xgmi_harness")


@pytest.mark.parametrize("nranks,length", [(2, 109386), (4, 300007)])
def test_cpp_xgmi_harness_one_process_per_rank(nranks, length):
    """tests/native/ono_xgmi_harness.cpp: a C++ parent forks one worker process per
    rank (before any HIP call), relays the 128-byte handles over pipes, and
    every worker runs host-fed rounds of the xGMI ring for both wires through
    the C ABI, bit-exact with the C oracle (all ranks on device 0 here)."""
    if not os.path.exists(XGMI_HARNESS):
        subprocess.run(["make", "-s", "-C", NATIVE, "ono_xgmi_harness"], check=True)
    r = subprocess.run([XGMI_HARNESS, str(nranks), str(length), "0"], capture_output=True, text=True,
                       timeout=300, env=dict(os.environ, ONO_XGMI_TIMEOUT_S="10"))
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.count("6 rounds bit-exact") == nranks and "harness: " in r.stdout, r.stdout
