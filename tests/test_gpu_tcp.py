"""GPU parity of the TCP edge (ono_ring_create_tcp).

The ring runs over the worker's own stream sockets and speaks the reference's
frames byte for byte ([u64 BE len][u32 BE kind=1][f16 LE], msg.rs:120-191),
with the hop arithmetic in HBM.  Several ranks share the one GPU of the box,
one Python thread each (the C ABI releases the GIL while it blocks on its
sockets):

* all-GPU rings over socket pairs: bit-exact with the oracle, device and
  host-fed forms, several rounds;
* mixed rings over loopback TCP: MI355X workers and reference-style CPU
  workers (oracle/ono_cpu_ring.c single mode, one process per rank) in ONE
  ring — wire compatibility with the reference;
* the bytes an MI355X worker puts on the wire equal the reference framing of
  the reference's f16 encoding of its chunk;
* the reference's failure behaviour: an invalid event is InvalidWorkerEvent
  (worker_ring.rs:136-138), a closed peer is an io error, abort() unblocks;
* the SparseCapable serializer (ono_ring_set_sparse): SparseGrad frames
  (kind 3, comms/src/protocol/msg.rs:175-178) when the stream is at most 2
  bytes per value, else the DenseGrad fallback (compressor.rs:79-89); the
  ring's branches per push (worker_ring.rs:126-133, 177-193: after a sparse
  gather push the owned residual is kept), and every worker accepting both
  gradient kinds (handles/worker.rs:102-108) — all-GPU and mixed rings with
  reference-style CPU workers of either serializer, bit-exact on grad and
  residual with the restatements (oracle ono_ref_ring_pull_grads_sparse and
  the independent numpy one, which agree);
* a scatter gradient of another length is added over the shorter length (the
  zip, :141-143); every non-gradient frame fails with recv_event's error class.
"""
import socket
import threading
import time

import numpy as np
import pytest
import torch

import ono_amd
from conftest import SEED, assert_bitexact
from oracle import oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def socketpair_links(n):
    """links[r] = (prev_sock, next_sock) of rank r; pair i carries i -> i+1."""
    pairs = [socket.socketpair() for _ in range(n)]
    return [(pairs[(r - 1) % n][1], pairs[r][0]) for r in range(n)], pairs


def close_all(socks):
    for s in socks:
        s.close()


def teardown(pairs, workers, test_ends=()):
    """Close the test's own socket ends first (the workers see the peer go
    away), let the workers finish, and only then close the workers' sockets:
    a socket closed under a thread still polling it frees its descriptor for
    the next test's sockets, which that thread would then read."""
    close_all(test_ends)
    for w in workers:
        w.join(60)
    close_all(s for p in pairs for s in p)


class GpuWorker(threading.Thread):
    """One MI355X ring worker on its own stream: per round, residual <- input,
    pull_grads (device or host-fed form); keeps the last round's results."""

    def __init__(self, rank, n, length, inputs, prev=None, nxt=None, connect=None, listener=None,
                 host_fed=False, sparse=None, sampler=None, reseed=None):
        super().__init__(daemon=True)
        self.sparse, self.sampler = sparse, sampler  # (ratio, seed) of SparseCapable; a sampler callback
        self.reseed = reseed or {}  # round -> (ratio, seed): ono_ring_set_sparse again before that round
        self.rank, self.n, self.length, self.inputs = rank, n, length, inputs
        self.prev, self.nxt, self.connect, self.listener = prev, nxt, connect, listener
        self.host_fed = host_fed
        self.err = None
        self.grad = self.residual = None
        self.ring = None
        self.ready = threading.Event()

    def run(self):
        try:
            torch.cuda.set_device(0)
            if self.connect is not None:  # builder.rs:272-311: connect to next, accept prev
                self.nxt = socket.create_connection(("127.0.0.1", self.connect()), timeout=60)
                self.nxt.settimeout(None)
                self.prev, _ = self.listener.accept()
            s = torch.cuda.Stream()
            with torch.cuda.stream(s):
                self.ring = ono_amd.WorkerRingManager.over_tcp(self.rank, self.n, self.length,
                                                               self.prev, self.nxt)
                if self.sparse is not None:
                    self.ring.set_sparse(*self.sparse)
                if self.sampler is not None:
                    self.ring.set_sampler(self.sampler)
                self.ready.set()
                for k, x in enumerate(self.inputs):
                    if k in self.reseed:
                        self.ring.set_sparse(*self.reseed[k])
                    if self.host_fed:
                        res = np.array(x, dtype=np.float32, copy=True)
                        grad = np.full_like(res, 7.0)
                        self.ring.pull_grads_host(res, grad)
                        self.grad, self.residual = grad, res
                    else:
                        self.ring.residual.copy_(torch.from_numpy(x).to(DEV))
                        self.ring.pull_grads(stream=s)
                        s.synchronize()
                        self.grad = self.ring.grad.cpu().numpy()
                        self.residual = self.ring.residual.cpu().numpy()
        except Exception as e:  # reported by the test thread
            self.err = e
        finally:
            self.ready.set()
            if self.ring is not None:
                self.ring.close()


def join_all(workers, timeout=300):
    for w in workers:
        w.join(timeout)
        assert not w.is_alive(), f"rank {w.rank} did not finish"
    for w in workers:
        if w.err is not None:
            raise w.err


def inputs_for(n, length, rounds, seed):
    return [[O.synth(length, seed + 100 * k, r) for r in range(n)] for k in range(rounds)]


@pytest.mark.parametrize("n", [2, 3, 4, 5])
@pytest.mark.parametrize("length", [109386, 4099, 2 ** 16 + 3])
@pytest.mark.parametrize("host_fed", [False, True])
@pytest.mark.parametrize("zero_copy", [True, False])
def test_tcp_ring_socketpairs_vs_oracle(n, length, host_fed, zero_copy, monkeypatch):
    """Frames of these sizes are small: by default the codec kernels read and
    write them in pinned host memory (zero-copy); ONO_TCP_ZEROCOPY=0 stages
    them through HBM wire buffers with D2H / H2D copies instead."""
    if not zero_copy:
        monkeypatch.setenv("ONO_TCP_ZEROCOPY", "0")
    rounds = 2
    ins = inputs_for(n, length, rounds, SEED + 21)
    links, pairs = socketpair_links(n)
    ws = [GpuWorker(r, n, length, [ins[k][r] for k in range(rounds)], *links[r], host_fed=host_fed)
          for r in range(n)]
    try:
        for w in ws:
            w.start()
        join_all(ws)
    finally:
        teardown(pairs, ws)
    eg, er = O.ring_pull_grads(ins[-1], "f16")
    for r in range(n):
        assert_bitexact(ws[r].grad, eg[r], f"grad rank {r}")
        assert_bitexact(ws[r].residual, er[r], f"residual rank {r}")


@pytest.mark.parametrize("n,length,piece_kib", [(2, 2 ** 20 + 7, 64), (3, 3 * 2 ** 19 + 5, 128),
                                                (4, 2 ** 21 + 3, 4096)])
@pytest.mark.parametrize("zero_copy", [False, True])
def test_tcp_ring_pipelined_pieces(n, length, piece_kib, zero_copy, monkeypatch):
    """Frames above the inline size go through the two-thread exchange: staged
    through HBM in pipelined D2H / H2D pieces (ONO_TCP_BLOCK_KIB, read at ring
    creation), or — with the zero-copy limit raised — read and written by the
    codec kernels in pinned host memory.  Bit-exact either way."""
    monkeypatch.setenv("ONO_TCP_BLOCK_KIB", str(piece_kib))
    monkeypatch.setenv("ONO_TCP_ZEROCOPY", "65536" if zero_copy else "0")
    ins = inputs_for(n, length, 2, SEED + 31)
    links, pairs = socketpair_links(n)
    ws = [GpuWorker(r, n, length, [ins[k][r] for k in range(2)], *links[r]) for r in range(n)]
    try:
        for w in ws:
            w.start()
        join_all(ws)
    finally:
        teardown(pairs, ws)
    eg, er = O.ring_pull_grads(ins[-1], "f16")
    for r in range(n):
        assert_bitexact(ws[r].grad, eg[r], f"grad rank {r}")
        assert_bitexact(ws[r].residual, er[r], f"residual rank {r}")


def test_tcp_ring_single_worker():
    """nranks == 1: no sockets; pull_grads = copy + zero (worker_ring.rs:82-94)."""
    x = O.synth(5000, SEED, 0)
    ring = ono_amd.WorkerRingManager.over_tcp(0, 1, x.size, None, None)
    try:
        ring.residual.copy_(torch.from_numpy(x).to(DEV))
        ring.pull_grads()
        torch.cuda.synchronize()
        assert_bitexact(ring.grad.cpu().numpy(), x, "grad")
        assert not ring.residual.cpu().numpy().view(np.uint32).any()
    finally:
        ring.close()


@pytest.mark.parametrize("n,cpu_ranks,length", [(2, (1,), 109386), (3, (1,), 10007),
                                                (4, (1, 3), 65539), (5, (2, 3), 4099)])
def test_tcp_ring_mixed_with_reference_workers(n, cpu_ranks, length):
    """MI355X workers and reference-style CPU workers in one loopback TCP ring:
    every rank's grad and residual are bit-exact with the oracle."""
    rounds, seed = 2, SEED + 7
    assert 0 not in cpu_ranks  # rank n-1 connects to rank 0, whose port must exist first
    listeners, ports = {}, {}
    for r in range(n):
        if r not in cpu_ranks:
            listeners[r] = socket.create_server(("127.0.0.1", 0))
            ports[r] = listeners[r].getsockname()[1]
    cpu, gpu = {}, []
    try:
        for r in sorted(cpu_ranks, reverse=True):  # a CPU rank's next is already listening
            cpu[r] = O.CpuRingWorker(r, n, length, ports[(r + 1) % n], rounds=rounds, seed=seed)
            ports[r] = cpu[r].port
        # the CPU workers feed the same input every round: synth(seed, rank)
        x = [O.synth(length, seed, r) for r in range(n)]
        gpu = [GpuWorker(r, n, length, [x[r]] * rounds, connect=lambda r=r: ports[(r + 1) % n],
                         listener=listeners[r]) for r in range(n) if r not in cpu_ranks]
        for w in gpu:
            w.start()
        join_all(gpu)
        got = {w.rank: (w.grad, w.residual) for w in gpu}
        for r, c in cpu.items():
            g, res, _ = c.result()
            got[r] = (g, res)
    finally:
        for c in cpu.values():
            c.close()
        close_all(listeners.values())
        for w in gpu:
            for s in (w.prev, w.nxt):
                if s is not None:
                    s.close()
    eg, er = O.ring_pull_grads(x, "f16")
    for r in range(n):
        assert_bitexact(got[r][0], eg[r], f"grad rank {r}")
        assert_bitexact(got[r][1], er[r], f"residual rank {r}")


def recv_frame(sock):
    head = b""
    while len(head) < 8:
        head += sock.recv(8 - len(head))
    ln = int.from_bytes(head, "big")
    body = b""
    while len(body) < ln:
        body += sock.recv(ln - len(body))
    return head + body


def start_two_rank(length, x):
    """Rank 0 on the GPU; rank 1 is the test itself on the other socket ends."""
    links, pairs = socketpair_links(2)
    w = GpuWorker(0, 2, length, [x], *links[0])
    w.start()
    links[1][0].settimeout(120)  # a frame that never comes fails the test instead of hanging it
    return w, links[1], pairs


def test_tcp_ring_wire_bytes():
    length = 10001
    x = O.synth(length, SEED + 1, 0)
    w, (from_gpu, to_gpu), pairs = start_two_rank(length, x)
    try:
        frame = recv_frame(from_gpu)
        (a, b) = O.split_chunks(length, 2)[0]
        assert frame == O.frame_dense(O.f16_encode(x[a:b]))  # byte for byte the reference's
        to_gpu.close()
        w.join(60)
    finally:
        teardown(pairs, [w], (from_gpu, to_gpu))


def frame(kind: int, payload: bytes) -> bytes:
    return (4 + len(payload)).to_bytes(8, "big") + kind.to_bytes(4, "big") + payload


# (kind, payload, error class, message) — WorkerHandle::recv_event
# (comms/src/handles/worker.rs:82-130) + the ring (worker_ring.rs:136-138)
EVENT_CASES = [
    (0, b'"upgraded"', "proto", "invalid worker event"),
    (0, b'"disconnect"', "proto", "invalid worker event"),
    (0, b'{"done": null}', "proto", "invalid worker event"),
    (0, b'{"report_loss": {"losses": [0.25, 1.5]}}', "proto", "invalid worker event"),
    (0, b'{"report_loss": {"losses": [0.25, null]}}', "io", "loss diverged"),
    (0, b'"ping"', "io", "Unexpected message"),
    (0, b'{"share_dataset_size": {"size": 3}}', "io", "Unexpected message"),
    (0, b'{"report_loss": {"losses": [1, }', "io", "control message"),
    (0, b'"no_such_command"', "io", "unknown variant"),
    (0, b'', "io", "control message"),
    (5, b"\0" * 16, "io", "Unexpected message"),
    (6, b"\0" * 16, "io", "Unexpected message"),
    (7, b"\0" * 16, "io", "invalid kind byte"),
    (200, b"", "io", "invalid kind byte"),
    (0x101, b"\0" * 10, "proto", "invalid worker event"),  # the kind is the header's low byte: 1, wrong length
]


@pytest.mark.parametrize("kind,payload,err,text", EVENT_CASES)
@pytest.mark.parametrize("phase", ["scatter", "gather"])
def test_tcp_ring_worker_event_classes(kind, payload, err, text, phase):
    """A frame that is not the expected gradient fails with the reference's
    error class and message: a worker event the ring rejects is
    InvalidWorkerEvent, everything recv_event itself refuses (the serde error,
    "loss diverged", "Unexpected message from worker", an invalid kind byte)
    is an io::Error.  Checked in both phases of the round."""
    if kind == 0x101 and phase == "scatter":
        pytest.skip("a shorter DenseGrad is the zip in the scatter (test_tcp_ring_scatter_zip)")
    length = 10001
    w, (from_gpu, to_gpu), pairs = start_two_rank(length, O.synth(length, SEED + 1, 0))
    (a, b), (c, d) = O.split_chunks(length, 2)
    try:
        recv_frame(from_gpu)
        if phase == "gather":  # a good scatter frame first, then the bad one in the gather
            to_gpu.sendall(O.frame_dense(O.f16_encode(O.synth(length, SEED + 1, 1)[c:d])))
            recv_frame(from_gpu)
        to_gpu.sendall(frame(kind, payload))
        w.join(60)
        want = ono_amd.InvalidWorkerEvent if err == "proto" else ono_amd.IoError
        assert isinstance(w.err, want), w.err
        assert text in str(w.err), w.err
    finally:
        teardown(pairs, [w], (from_gpu, to_gpu))


def test_worker_event_check_matches_the_ring():
    """The host-side verdict (ono_worker_event_check) is what the ring raises."""
    for kind, payload, err, text in EVENT_CASES:
        if kind == 0x101:
            continue
        want = ono_amd.InvalidWorkerEvent if err == "proto" else ono_amd.IoError
        with pytest.raises(want, match=text):
            ono_amd.worker_event_check(kind & 0xFF, payload)
    ono_amd.worker_event_check(1, b"\0\0")


def _sparse_with_far_run(stream: bytes, total: int, far: int, vals) -> bytes:
    """`stream` (a grad_drop of some prefix) with its total raised to `total`
    and one more record whose run starts at element `far`."""
    import struct
    body = bytearray(stream)
    body[:8] = total.to_bytes(8, "little")
    # the end of the last run in the stream: replay the parse
    gi, bi = 0, 8
    while bi < len(stream):
        off, ln = struct.unpack_from("<II", stream, bi)
        gi += off + ln
        bi += 8 + 2 * ln
    h = O.f16_encode(np.asarray(vals, dtype=np.float32))
    body += struct.pack("<II", far - gi, len(h)) + h.tobytes()
    return bytes(body)


@pytest.mark.parametrize("form,delta", [("dense", -3), ("dense", 5), ("sparse", -2), ("sparse", 4),
                                        ("sparse_far", 1 << 34)])
def test_tcp_ring_scatter_zip(form, delta):
    """A scatter gradient of another length than the hop's chunk is added over
    the shorter of the two (the zip of worker_ring.rs:141-143): the rest of the
    chunk keeps its value, values past the chunk are dropped.  sparse_far: a
    SparseGrad claiming 2^34 values with a run at 3 x 2^30 — the whole stream is
    validated but only the chunk's length is materialised (a frame's claimed
    total never sizes a device allocation)."""
    length = 10001
    x = O.synth(length, SEED + 11, 0)
    y = O.synth(length, SEED + 11, 1)
    w, (from_gpu, to_gpu), pairs = start_two_rank(length, x)
    (a, b), (c, d) = O.split_chunks(length, 2)
    far = form == "sparse_far"
    m = d - c + (4 if far else delta)
    peer = y[c:c + m] if m < d - c else np.concatenate([y[c:d], y[:m - (d - c)]])
    try:
        recv_frame(from_gpu)
        if form == "dense":
            to_gpu.sendall(O.frame_dense(O.f16_encode(peer)))
        elif far:
            st = O.grad_drop(peer, O.sparse_threshold(peer, 0.1))
            to_gpu.sendall(frame_sparse(_sparse_with_far_run(bytes(st), delta, 3 << 30, [1.5, -2.0, 3.25])))
        else:
            to_gpu.sendall(frame_sparse(O.grad_drop(peer, O.sparse_threshold(peer, 0.1))))
        g_frame = recv_frame(from_gpu)  # the owner's gather push of chunk 1
        to_gpu.sendall(O.frame_dense(O.f16_encode(y[a:b])))  # rank 1's gather push of chunk 0
        w.join(60)
        assert w.err is None, w.err
    finally:
        teardown(pairs, [w], (from_gpu, to_gpu))
    lifted = (O.f16_decode(O.f16_encode(peer)) if form == "dense"
              else O.grad_lift(O.grad_drop(peer, O.sparse_threshold(peer, 0.1)), m))
    k = min(m, d - c)
    own = x[c:d].copy()
    own[:k] = own[:k] + lifted[:k]
    assert g_frame == O.frame_dense(O.f16_encode(own))
    exp_grad = np.concatenate([O.f16_decode(O.f16_encode(y[a:b])), own]) / np.float32(2)
    assert_bitexact(w.grad, exp_grad.astype(np.float32), "grad")
    assert not w.residual.view(np.uint32).any()


def test_tcp_ring_wrong_length_is_invalid_event():
    """A gather DenseGrad of another length than the chunk: the reference's
    copy_from_slice (worker_ring.rs:200) panics; here InvalidWorkerEvent."""
    length = 10001
    w, (from_gpu, to_gpu), pairs = start_two_rank(length, O.synth(length, SEED, 0))
    (a, b), (c, d) = O.split_chunks(length, 2)
    try:
        recv_frame(from_gpu)
        to_gpu.sendall(O.frame_dense(O.f16_encode(np.zeros(d - c, np.float32))))
        recv_frame(from_gpu)
        to_gpu.sendall(O.frame_dense(np.zeros(7, np.uint16)))
        w.join(60)
        assert isinstance(w.err, ono_amd.InvalidWorkerEvent), w.err
    finally:
        teardown(pairs, [w], (from_gpu, to_gpu))


def test_tcp_ring_peer_closed_is_io_error():
    length = 10001
    w, (from_gpu, to_gpu), pairs = start_two_rank(length, O.synth(length, SEED, 0))
    try:
        recv_frame(from_gpu)
        to_gpu.close()
        w.join(60)
        assert isinstance(w.err, ono_amd.IoError), w.err
    finally:
        teardown(pairs, [w], (from_gpu, to_gpu))


def test_tcp_ring_abort_unblocks():
    length = 10001
    w, (from_gpu, to_gpu), pairs = start_two_rank(length, O.synth(length, SEED, 0))
    try:
        recv_frame(from_gpu)  # the peer never answers
        w.ready.wait(60)
        time.sleep(0.2)
        w.ring.abort()
        w.join(30)
        assert not w.is_alive()
        assert isinstance(w.err, ono_amd.Aborted), w.err
    finally:
        teardown(pairs, [w], (from_gpu, to_gpu))


# ------------------------------------------------------------ sparse mode
def frame_sparse(payload: bytes, kind: int = 3) -> bytes:
    return (4 + len(payload)).to_bytes(8, "big") + kind.to_bytes(4, "big") + payload


def oracle_rounds(x_rounds, ratios, seeds):
    """The restated rounds, the samplers' streams carried from round to round."""
    st = list(seeds)
    for x in x_rounds:
        g, res, st = O.ring_pull_grads_sparse(x, ratios, st)
    return g, res


@pytest.mark.parametrize("n,length,ratios", [(2, 10001, [0.4, 0.1]), (2, 70001, [0.1, 0.9]),
                                             (3, 40000, [0.05, 0.0, 0.6]), (4, 109386, [0.1, 0.3, 0.0, 1.0]),
                                             (5, 4099, [0.5, 0.0, 0.0, 0.1, 0.05]), (3, 60000, [0.1, 0.15, 0.05])])
@pytest.mark.parametrize("zero_copy", [True, False])
def test_tcp_ring_sparse_socketpairs_vs_oracle(n, length, ratios, zero_copy, monkeypatch):
    """All-GPU rings of SparseCapable and Base workers (chunks below and above
    the 16384-value sample), two rounds: bit-exact with the restatement."""
    if not zero_copy:
        monkeypatch.setenv("ONO_TCP_ZEROCOPY", "0")
    seeds = [77 + r for r in range(n)]
    ins = inputs_for(n, length, 2, SEED + 41)
    links, pairs = socketpair_links(n)
    ws = [GpuWorker(r, n, length, [ins[k][r] for k in range(2)], *links[r],
                    sparse=(ratios[r], seeds[r]) if ratios[r] else None) for r in range(n)]
    try:
        for w in ws:
            w.start()
        join_all(ws)
    finally:
        teardown(pairs, ws)
    eg, er = oracle_rounds(ins, ratios, seeds)
    for r in range(n):
        assert_bitexact(ws[r].grad, eg[r], f"grad rank {r}")
        assert_bitexact(ws[r].residual, er[r], f"residual rank {r}")


@pytest.mark.parametrize("n,length,ratios", [(2, 109386, [0.1, 0.1]), (3, 60000, [0.1, 0.15, 0.05])])
@pytest.mark.parametrize("refuse", [1, 3, 10 ** 6])
def test_tcp_ring_sparse_refused_lifts(n, length, ratios, refuse):
    """A received SparseGrad is lifted by the one-launch stream-ordered lift; a stream it refuses goes to the
    blocking device lift before the hop adds or copies it.  Lifts refused by the test hook (the first one,
    three, or every one of the rings'): the rings stay bit-exact with the restatement, and the refusals
    were taken."""
    seeds = [91 + r for r in range(n)]
    ins = inputs_for(n, length, 2, SEED + 45)
    links, pairs = socketpair_links(n)
    ws = [GpuWorker(r, n, length, [ins[k][r] for k in range(2)], *links[r], sparse=(ratios[r], seeds[r]))
          for r in range(n)]
    ono_amd.sparse.lift_debug_refuse(refuse)
    left = None
    try:
        for w in ws:
            w.start()
        join_all(ws)
    finally:
        left = ono_amd.sparse.lift_debug_refuse(0)
        teardown(pairs, ws)
    eg, er = oracle_rounds(ins, ratios, seeds)
    for r in range(n):
        assert_bitexact(ws[r].grad, eg[r], f"grad rank {r}")
        assert_bitexact(ws[r].residual, er[r], f"residual rank {r}")
    assert left < refuse and (refuse > 3 or left == 0), left  # (each ring round lifts at least 2 frames)


@pytest.mark.parametrize("n,length", [(2, 109386), (3, 60000)])
def test_tcp_ring_sparse_reseeded_between_rounds(n, length):
    """ono_ring_set_sparse between rounds restarts the default sampler's stream (and may change the ratio)
    while the sampler's helper threads are drawing the coming pushes ahead: the queue is re-planned, a draw
    still in flight is dropped, and no slot a stale draw is still writing is handed out again.  Five rounds,
    re-seeded before rounds 1, 2 (back to back) and 4 (new ratios): bit-exact with the restatement."""
    rounds = 5
    ratios0 = [0.1, 0.1, 0.05][:n]
    plan = {1: ([0.1, 0.1, 0.05][:n], [500 + r for r in range(n)]),
            2: ([0.1, 0.1, 0.05][:n], [600 + r for r in range(n)]),
            4: ([0.2, 0.05, 0.3][:n], [700 + r for r in range(n)])}
    seeds = [131 + r for r in range(n)]
    ins = inputs_for(n, length, rounds, SEED + 47)
    links, pairs = socketpair_links(n)
    ws = [GpuWorker(r, n, length, [ins[k][r] for k in range(rounds)], *links[r], sparse=(ratios0[r], seeds[r]),
                    reseed={k: (rs[r], sd[r]) for k, (rs, sd) in plan.items()}) for r in range(n)]
    try:
        for w in ws:
            w.start()
        join_all(ws)
    finally:
        teardown(pairs, ws)
    st, ratios = list(seeds), list(ratios0)
    for k, x in enumerate(ins):
        if k in plan:
            ratios, st = list(plan[k][0]), list(plan[k][1])
        g, res, st = O.ring_pull_grads_sparse(x, ratios, st)
    for r in range(n):
        assert_bitexact(ws[r].grad, g[r], f"grad rank {r}")
        assert_bitexact(ws[r].residual, res[r], f"residual rank {r}")


def test_tcp_ring_sparse_host_fed_and_sampler_callback():
    """The host-fed form, and a caller-installed sampler (the boundary a Rust
    integration uses to draw rand's index::sample): here a Python sampler that
    draws the stand-in stream, so the restatement still applies."""
    n, length, ratios = 3, 60000, [0.1, 0.3, 0.05]
    seeds = [5, 6, 7]
    ins = inputs_for(n, length, 2, SEED + 43)

    def sampler_for(seed):
        state = [seed]

        def draw(ln, amount):
            idx, state[0] = O.sample_default(state[0], ln, amount)
            return idx
        return draw
    links, pairs = socketpair_links(n)
    ws = [GpuWorker(r, n, length, [ins[k][r] for k in range(2)], *links[r], host_fed=(r == 1),
                    sparse=(ratios[r], 0), sampler=sampler_for(seeds[r])) for r in range(n)]
    try:
        for w in ws:
            w.start()
        join_all(ws)
    finally:
        teardown(pairs, ws)
    eg, er = oracle_rounds(ins, ratios, seeds)
    for r in range(n):
        assert_bitexact(ws[r].grad, eg[r], f"grad rank {r}")
        assert_bitexact(ws[r].residual, er[r], f"residual rank {r}")


@pytest.mark.parametrize("n,cpu_ranks,length,ratios", [(2, (1,), 109386, [0.1, 0.1]),
                                                       (2, (1,), 109386, [0.4, 0.05]),
                                                       (3, (1,), 40000, [0.0, 0.05, 0.5]),
                                                       (4, (1, 3), 65539, [0.3, 0.0, 0.1, 0.1]),
                                                       (5, (2, 3), 4099, [0.0, 0.9, 0.1, 0.0, 0.05])])
def test_tcp_ring_sparse_mixed_with_reference_workers(n, cpu_ranks, length, ratios):
    """MI355X workers and reference-style CPU workers, each with its own
    serializer (SparseCapable or Base), in one loopback ring: bit-exact."""
    rounds, seed = 2, SEED + 47
    seeds = [300 + r for r in range(n)]
    listeners, ports = {}, {}
    for r in range(n):
        if r not in cpu_ranks:
            listeners[r] = socket.create_server(("127.0.0.1", 0))
            ports[r] = listeners[r].getsockname()[1]
    cpu, gpu = {}, []
    try:
        for r in sorted(cpu_ranks, reverse=True):
            cpu[r] = O.CpuRingWorker(r, n, length, ports[(r + 1) % n], rounds=rounds, seed=seed, sparse=ratios[r],
                                     sparse_seed=seeds[r])
            ports[r] = cpu[r].port
        x = [O.synth(length, seed, r) for r in range(n)]
        gpu = [GpuWorker(r, n, length, [x[r]] * rounds, connect=lambda r=r: ports[(r + 1) % n],
                         listener=listeners[r], sparse=(ratios[r], seeds[r]) if ratios[r] else None)
               for r in range(n) if r not in cpu_ranks]
        for w in gpu:
            w.start()
        join_all(gpu)
        got = {w.rank: (w.grad, w.residual) for w in gpu}
        for r, c in cpu.items():
            g, res, _ = c.result()
            got[r] = (g, res)
    finally:
        for c in cpu.values():
            c.close()
        close_all(listeners.values())
        for w in gpu:
            for s in (w.prev, w.nxt):
                if s is not None:
                    s.close()
    eg, er = oracle_rounds([x] * rounds, ratios, seeds)
    for r in range(n):
        assert_bitexact(got[r][0], eg[r], f"grad rank {r}")
        assert_bitexact(got[r][1], er[r], f"residual rank {r}")


def expect_push(chunk, r, state=0):
    """The frame a SparseCapable{r} worker pushes for `chunk` (compressor.rs:71-98)."""
    sparse, t, state = O.sparse_push(chunk, r, state)
    if sparse:
        return frame_sparse(O.grad_drop(chunk, t)), t, state
    return O.frame_dense(O.f16_encode(chunk)), None, state


@pytest.mark.parametrize("r", [0.05, 0.1, 0.3, 0.9, 1.0])
def test_tcp_ring_sparse_wire_bytes_and_lift_of_peer_frame(r):
    """The frames of a SparseCapable MI355X worker are the reference's: the
    SparseGrad of grad_drop(chunk, calculate_threshold(chunk, r)) when that
    stream is at most 2 bytes per value, else the DenseGrad of f16(chunk)
    (compressor.rs:79-89) — r = 0.3 and above go dense on this distribution.
    A SparseGrad the peer sends back is lifted and added (scatter), and the
    owner's residual follows the push (worker_ring.rs:126-133, 177-193)."""
    length = 20000
    x = O.synth(length, SEED + 3, 0)
    links, pairs = socketpair_links(2)
    w = GpuWorker(0, 2, length, [x], *links[0], sparse=(r, 0))
    w.start()
    from_gpu, to_gpu = links[1]
    (a, b), (c, d) = O.split_chunks(length, 2)
    y = O.synth(length, SEED + 3, 1)
    ty = O.sparse_threshold(y[c:d], 0.1)
    try:
        f0 = recv_frame(from_gpu)
        exp0, t0, _ = expect_push(x[a:b], r)
        assert f0 == exp0
        assert f0[8:12] == ((3 if t0 is not None else 1)).to_bytes(4, "big")
        to_gpu.sendall(frame_sparse(O.grad_drop(y[c:d], ty)))  # rank 1's sparse chunk 1
        g_frame = recv_frame(from_gpu)  # rank 0's gather push of its owned chunk 1
        to_gpu.sendall(O.frame_dense(O.f16_encode(y[a:b])))
        w.join(60)
        assert w.err is None, w.err
    finally:
        teardown(pairs, [w], (from_gpu, to_gpu))
    owned = x[c:d] + O.grad_lift(O.grad_drop(y[c:d], ty), d - c)
    exp_g, t1, _ = expect_push(owned, r)
    assert g_frame == exp_g
    res0 = x[a:b].copy()
    if t0 is not None:
        res0[np.abs(res0) >= t0] = 0
    else:
        res0[:] = 0
    assert_bitexact(w.residual[a:b], res0, "scatter chunk residual")
    # the owned chunk: kept after a sparse gather push (:178-184), zeroed after a dense one (:191-193)
    assert_bitexact(w.residual[c:d], owned if t1 is not None else np.zeros_like(owned), "owned residual")
    g1 = owned.copy()
    if t1 is not None:
        g1[np.abs(g1) < t1] = 0
    assert_bitexact(w.grad[c:d], (g1 / np.float32(2)).astype(np.float32), "owned grad")


@pytest.mark.parametrize("payload,phase,err", [("short", "scatter", "io"), ("overrun", "scatter", "io"),
                                               ("tiny", "scatter", "io"), ("total", "gather", "proto"),
                                               ("short", "gather", "io")])
def test_tcp_ring_sparse_bad_frames(payload, phase, err):
    """A malformed sparse stream fails with the lift's io::Error
    (protocol.rs:96-144, recv_event's map_err); a well-formed one whose total
    is not the chunk length is fine in the scatter (the zip) but cannot be
    copied in the gather (copy_from_slice panics in the reference:
    InvalidWorkerEvent here)."""
    length = 10001
    w, (from_gpu, to_gpu), pairs = start_two_rank(length, O.synth(length, SEED, 0))
    (a, b), (c, d) = O.split_chunks(length, 2)
    m = (b - a) if phase == "gather" else (d - c)
    body = {"total": (m + 1).to_bytes(8, "little"),
            "short": m.to_bytes(8, "little") + b"\x00\x00\x00",
            "tiny": b"\x01\x02",
            "overrun": m.to_bytes(8, "little") + (m - 1).to_bytes(4, "little") + (5).to_bytes(4, "little") + b"\0" * 10,
            }[payload]
    try:
        recv_frame(from_gpu)
        if phase == "gather":
            to_gpu.sendall(O.frame_dense(O.f16_encode(np.zeros(d - c, np.float32))))
            recv_frame(from_gpu)
        to_gpu.sendall(frame_sparse(body))
        w.join(60)
        want = ono_amd.InvalidWorkerEvent if err == "proto" else ono_amd.IoError
        assert isinstance(w.err, want), w.err
    finally:
        teardown(pairs, [w], (from_gpu, to_gpu))


def test_tcp_ring_sparse_zero_length_runs_accepted():
    """A stream of many empty runs is valid for the reference (every record
    passes grad_lift_into's checks) whatever its length: the chunk lifts to
    zeros and the scatter adds them (x + 0: -0 becomes +0, as in Rust)."""
    length = 10001
    x = O.synth(length, SEED + 2, 0)
    w, (from_gpu, to_gpu), pairs = start_two_rank(length, x)
    (a, b), (c, d) = O.split_chunks(length, 2)
    m = d - c
    try:
        recv_frame(from_gpu)
        to_gpu.sendall(frame_sparse(m.to_bytes(8, "little") + b"\0" * (8 * m)))
        g_frame = recv_frame(from_gpu)
        to_gpu.sendall(O.frame_dense(O.f16_encode(np.zeros(b - a, np.float32))))
        w.join(60)
        assert w.err is None, w.err
    finally:
        teardown(pairs, [w], (from_gpu, to_gpu))
    assert g_frame == O.frame_dense(O.f16_encode(x[c:d] + np.zeros(m, np.float32)))
