"""The xGMI exchange-region pool's bookkeeping on the CPU (no GPU): the
release order and the IPC-handle repeat guard of csrc/ono_xgmi_pool.{h,cpp},
driven by simulated processes over a simulated device
(tests/native/xgmi_pool_test.cpp; DESIGN.md §4 "Retention", §8 item 7).

What it pins: two-phase release (close imports everywhere, then free) frees
every region and never frees one while a simulated peer still has it imported;
a free that runs before a peer closes keeps the region (ONO_E_IO) and frees it
on the next call; a fresh allocation whose handle repeats an earlier one is
parked and never exported; an importer refuses a handle it opened before; a
failed allocation does not count as a live ring (round 4's g_live underflow);
quarantined regions are never freed or reused."""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
NATIVE = os.path.join(HERE, "native")


def test_xgmi_pool_bookkeeping():
    b = subprocess.run(["make", "-s", "xgmi_pool_test"], cwd=NATIVE, capture_output=True, text=True, timeout=300)
    assert b.returncode == 0, b.stderr[-3000:]
    r = subprocess.run([os.path.join(NATIVE, "xgmi_pool_test")], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr[-3000:]
    assert r.stdout.startswith("ok "), r.stdout
    assert int(r.stdout.split()[1]) >= 60
