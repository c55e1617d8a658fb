"""The C-ABI boundary on a CPU-only host: the library loads, exports every
symbol include/ono_reduce.h declares, and its host-only logic (argument
validation, DynBarrier, synchronizer reference counting) behaves like the
reference.  No compute call is made here (no GPU)."""
import ctypes as C
import threading
import time

import pytest

import ono_amd
from ono_amd import _lib


def test_library_exports_every_header_symbol():
    fns = ono_amd.header_functions()
    assert len(fns) >= 45
    missing = [f for f in fns if not hasattr(ono_amd.lib(), f)]
    assert missing == []
    # and the ctypes signature table covers the header exactly
    assert sorted(_lib._SIGS) == fns


def test_abi_version_and_device_count():
    L = ono_amd.lib()
    assert L.ono_abi_version() == 2
    c = C.c_int(-1)
    assert L.ono_device_count(C.byref(c)) == 0
    assert c.value >= 0


def test_argument_errors_without_gpu():
    h = C.c_void_p()
    with pytest.raises(ono_amd.InvalidArgument):
        _lib.call("ono_ring_create", C.byref(h), 0, 0, 10, 0, None, 0)
    with pytest.raises(ono_amd.InvalidArgument):
        _lib.call("ono_ring_create", C.byref(h), 3, 2, 10, 0, None, 0)
    # len < nranks: the reference panics on chunks[pos]; here SizeMismatch
    with pytest.raises(ono_amd.SizeMismatch):
        _lib.call("ono_ring_create", C.byref(h), 0, 4, 3, 0, b"\0" * 128, 0)
    with pytest.raises(ono_amd.InvalidArgument):
        _lib.call("ono_ring_create", C.byref(h), 0, 2, 10, 0, None, 0)  # uid required
    with pytest.raises(ono_amd.InvalidArgument):
        _lib.call("ono_sum_scale_f32", None, None, 0, 10, 1.0, None)
    with pytest.raises(ono_amd.InvalidArgument):
        _lib.call("ono_sum_scale_f32", None, None, 17, 10, 1.0, None)
    assert "k=17" in ono_amd.lib().ono_last_error().decode()


def test_dyn_barrier_one_leader_per_generation():
    b = ono_amd.DynBarrier(4)
    leaders = []
    lock = threading.Lock()

    def worker(i):
        for gen in range(5):
            def lead(i=i, gen=gen):
                with lock:
                    leaders.append((gen, i))
            b.wait_with(lead)

    ts = [threading.Thread(target=worker, args=(i,)) for i in range(4)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(10)
    assert all(not t.is_alive() for t in ts)
    assert sorted(g for g, _ in leaders) == [0, 1, 2, 3, 4]


def test_dyn_barrier_acquire_releases_waiters():
    """dyn_barrier.rs:72-81: a leaving worker shrinks the barrier; if it was
    the last one missing, the waiters are released and one of them leads."""
    b = ono_amd.DynBarrier(3)
    leaders = []
    ts = [threading.Thread(target=lambda: b.wait_with(lambda: leaders.append(1))) for _ in range(2)]
    for t in ts:
        t.start()
    time.sleep(0.2)
    assert all(t.is_alive() for t in ts)
    b.acquire()
    for t in ts:
        t.join(10)
    assert all(not t.is_alive() for t in ts)
    assert len(leaders) == 1
    # the barrier now has size 2
    ts = [threading.Thread(target=lambda: b.wait_with(lambda: leaders.append(2))) for _ in range(2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(10)
    assert leaders == [1, 2]


def test_sync_clone_release_refcount():
    s = ono_amd.BarrierSync(2)
    c = s.clone()
    c.drop()      # strong count 2 -> acquire() shrinks the barrier to 1
    s.drop()      # last clone frees the synchronizer
    nb = ono_amd.NoBlockingSync()
    nb.clone().drop()
    nb.drop()


def test_shard_size_for_matches_builder():
    # builder.rs:164-173: shards = min(nparams, 2*cores); size = ceil(nparams / shards)
    assert ono_amd.shard_size_for(109386, cores=8) == 6837
    assert ono_amd.shard_size_for(3, cores=8) == 1
    assert ono_amd.shard_size_for(0, cores=8) == 1
