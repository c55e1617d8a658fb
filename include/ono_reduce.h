/*
 * ono_reduce.h — C ABI of the MI355X-native gradient-bucket reduction path.
 *
 * Drop-in boundary for lminervino18/oxidized-neural-orchestra's data-parallel
 * hot path: the worker ring all-reduce and the parameter-server gradient
 * synchronizer/store.  The reference has no FFI for this path (it is pure
 * Rust); these entry points are what a Rust `extern "C"` block in worker/ and
 * parameter_server/ binds instead of the Rust types they replace (INTEGRATION.md
 * shows the binding).  Plain pointers and sizes only; `stream` is a
 * hipStream_t passed as void* (NULL = the legacy default stream).
 *
 * Conventions
 *   - every call returns an ono_status; on failure ono_last_error() returns a
 *     thread-local message (valid until the next failing call on that thread);
 *   - "_dev" pointers are device (HBM) pointers, "_host" pointers host memory;
 *   - the library owns every device buffer, stream and communicator it
 *     creates; caller host buffers are only used for the duration of a call;
 *   - numerics are bit-exact with the reference's CPU arithmetic (IEEE f32,
 *     no FMA contraction, correctly rounded division/sqrt, half-2.7.1 f16 RNE),
 *     except where a comment states a tolerance (RCCL summation order, n >= 3).
 */
#ifndef ONO_REDUCE_H
#define ONO_REDUCE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ONO_ABI_VERSION 2
#define ONO_UID_BYTES 128 /* sizeof(ncclUniqueId) */
#define ONO_MAX_INPUTS 16 /* max k of ono_sum_scale_f32 */

typedef enum {
    ONO_OK = 0,
    ONO_E_SIZE = 1,    /* ParamServerErr::SizeMismatch   parameter_server/src/storage/error.rs:13-17 */
    ONO_E_PROTO = 2,   /* "Received an invalid worker event"  worker/src/middlewares/worker_ring.rs:136-138 */
    ONO_E_HIP = 3,     /* HIP runtime failure */
    ONO_E_RCCL = 4,    /* RCCL failure (the TCP io::Error of the reference ring) */
    ONO_E_ABORTED = 5, /* ono_ring_abort() — the reference drops the ring future in select!
                          (worker/src/workers/all_reduce.rs:73-75) */
    ONO_E_ARG = 6,     /* invalid argument (NULL handle, bad enum, k out of range) */
    ONO_E_OTHER = 7,   /* ParamServerErr::Other */
    ONO_E_IO = 8       /* socket error on a TCP ring (the reference's io::Error from comms/) */
} ono_status;

/* Wire type of the ring.  F16 reproduces the reference exactly: gradients
 * travel as f16 (comms/src/protocol/msg.rs:26, handles/compressor.rs:106-118),
 * hop order c, c+1, ..., c+n-1, the chunk owner keeps f32 (worker_ring.rs:166)
 * while replicas hold f16 copies (:200).  F32 is RCCL's ring all-reduce over
 * xGMI (bit-exact with the f32-wire restatement for n <= 2; for n >= 3 within
 * |d| <= 2(n-1) 2^-24 sum|g| — summation order only).                        */
typedef enum { ONO_WIRE_F32 = 0, ONO_WIRE_F16 = 1 } ono_wire;

const char *ono_last_error(void);
int ono_abi_version(void);
/* number of visible HIP devices (0 when no GPU); never fails on a CPU host */
int ono_device_count(int *count);

/* ===================================================================== */
/* Elementwise kernels (HBM-bound, gfx950).  All pointers are device      */
/* pointers; any alignment is accepted.                                    */
/* ===================================================================== */

/* out[i] = (((ins[0][i] + ins[1][i]) + ...) + ins[k-1][i]) / divisor
 * — the per-chunk f32 sum-and-scale of the ring (worker_ring.rs:141-143 then
 * param_manager.rs:183-188).  divisor == 1 skips the division (the reference
 * only divides for n > 1).  1 <= k <= ONO_MAX_INPUTS; `ins` is a HOST array of
 * k device pointers; out may alias ins[0].                                   */
int ono_sum_scale_f32(float *out, const float *const *ins, int k, size_t n, float divisor,
                      void *stream);

/* acc[i] += in[i]   — ParamManager::acc_residual (param_manager.rs:191-197),
 * BlockingShard::accumulate (storage/blocking/shard.rs:61-66)              */
int ono_acc_f32(float *acc, const float *in, size_t n, void *stream);

/* dst[i] = src[i] / divisor (copy when divisor == 1); then zero[i] = 0 when
 * zero != NULL.  The tail of pull_grads(): normalize_gradient
 * (param_manager.rs:183-188) fused with the residual reset
 * (worker_ring.rs:168-171,191-193).  dst may equal src; zero may equal src. */
int ono_scale_zero_f32(float *dst, const float *src, size_t n, float divisor, float *zero,
                       void *stream);

/* dst[i] = src[i] and dst[i] = value: the library's own pure streams (the
 * kernels above minus the arithmetic).  The owner's `grad[own] =
 * residual[own]` copy and the residual reset of the gather (worker_ring.rs:
 * 166-171, 191-193) when they run alone, the plan interpreter's device copies
 * and zero fills, and the measured copy ceiling the path's kernels are read
 * against (bench.py copy_ceiling).  dst and src must not overlap.           */
int ono_copy_f32(float *dst, const float *src, size_t n, void *stream);
int ono_fill_f32(float *dst, float value, size_t n, void *stream);

/* f16 wire codec (crate half 2.7.1: RNE, overflow -> inf, subnormals kept,
 * NaN keeps payload + quiet bit).  compressor.rs:116 / handles/worker.rs:94  */
int ono_f16_encode(uint16_t *out, const float *in, size_t n, void *stream);
int ono_f16_decode(float *out, const uint16_t *in, size_t n, void *stream);
/* scatter send: out = f16(chunk); chunk = 0      (compressor.rs:116 + worker_ring.rs:133) */
int ono_f16_encode_zero(uint16_t *out, float *chunk, size_t n, void *stream);
/* scatter receive: acc += f32(in)                 (worker.rs:94 + worker_ring.rs:141-143) */
int ono_f16_decode_add(float *acc, const uint16_t *in, size_t n, void *stream);
/* fused receive-then-forward of one hop: x = acc + f32(in); out = f16(x); acc = 0
 * (a hop's :141-143 followed by the next hop's :122,:133 on the same chunk)   */
int ono_f16_add_encode_zero(uint16_t *out, float *acc, const uint16_t *in, size_t n,
                            void *stream);
/* gather receive: out = f32(in) / divisor         (worker_ring.rs:200 + :101-105) */
int ono_f16_decode_scale(float *out, const uint16_t *in, size_t n, float divisor, void *stream);

/* The chunk owner's reduction of the DIRECT / XGMI schedules (one fused
 * kernel per round): ins[j] = the slice of chunk c from rank c+j (HOST array
 * of k device pointers, the owner's own residual slice last).
 *   p = ins[0];  p = ins[j] + wire(p) for j = 1..k-1   (wire = f16 round trip
 *   or identity) — the reference hop chain worker_ring.rs:122-143;
 *   grad = p / divisor (:166 + param_manager.rs:183-188);
 *   out = f16(p) (f16 wire: the message the gather forwards, :177-193) or
 *   grad (f32 wire); out may be NULL;
 *   ins[k-1] = 0, or every ins[j] = 0 when zero_all (:133, :191-193).        */
int ono_direct_chain(float *grad, void *out, const float *const *ins, int k, size_t n, float divisor, int wire,
                     int zero_all, void *stream);

/* Sparse top-(1-r) gradient codec (comms/src/sparse/protocol.rs:33-144), the
 * SparseCapable serializer's wire format, byte-exact:
 *   [u64 LE total_len] { [u32 LE offset][u32 LE run_len][f16 LE x run_len] }*
 * The threshold is the caller's (the reference samples it with rand 0.9.4
 * StdRng, protocol.rs:33-49).  drop: g_dev -> buf_dev, *nbytes = encoded
 * length (blocking; ONO_E_SIZE if it exceeds cap; ono_sparse_max_bytes(n)
 * always suffices).  lift: host bytes (as received from comms/) -> g_dev of
 * *out_len = total_len values (zero-filled, then the runs); malformed input ->
 * ONO_E_PROTO with the reference's message.  mask: the ring's sparse
 * bookkeeping — zero_kept=1: g = 0 where |g| >= t (worker_ring.rs:128-131),
 * zero_kept=0: g = 0 where |g| < t (:183-187).                               */
size_t ono_sparse_max_bytes(size_t n);
/* calculate_threshold (protocol.rs:33-49) on the device: the k-th smallest
 * |g| of the sample in f32::total_cmp order, k = (m as f32 * (1 - r)) as
 * usize (at most m - 1), then f32::max with f16::MIN_POSITIVE.  The sample is
 * every value (idx_host NULL, m == n <= 16384) or the m <= 16384 indices the
 * caller drew (idx_host: the reference draws them with rand 0.9.4's
 * choose_multiple = rand::seq::index::sample(rng, n, 16384)).  Blocking.     */
int ono_sparse_threshold(float *t_out, const float *g_dev, size_t n, const uint32_t *idx_host, size_t m, float r,
                         void *stream);
/* The deterministic stand-in sampler (Floyd's algorithm over a splitmix64
 * stream at *state): `amount` distinct indices of [0, len) — all of them, with
 * no draws, when amount == len.  NOT rand 0.9.4's StdRng; used when no
 * sampler is installed, and restated by the CPU oracle.                     */
int ono_sparse_sample_default(uint64_t *state, size_t len, uint32_t *idx, size_t amount);
/* The drop keeps device scratch per (device, stream), grown to the largest
 * gradient seen and never shrunk: above 256 tiles of 2048 values about 2.1
 * bytes per value (the keep flags and a f16 slot per tile for the kept
 * values) plus 16 bytes per tile; up to 256 tiles 32 bytes per tile.
 * No writer stores past buf + cap: a tile whose range would pass it (only
 * possible with corrupt or stale scratch) stores nothing, and the call fails
 * with ONO_E_IO (blocking) or reports it through ono_sparse_drop_check and the
 * next drop on the stream (stream-ordered; its *nbytes_dev reads ~0 when the
 * totals pass cap).  The blocking drop cannot be captured into a HIP graph
 * (ONO_E_ARG: it waits for its result); ono_sparse_drop_async can (see there). */
int ono_sparse_drop(uint8_t *buf_dev, size_t cap, size_t *nbytes, const float *g_dev, size_t n,
                    float threshold, void *stream);
/* The stream-ordered drop: the same bytes, nothing waits on the host; the
 * wire length lands in *nbytes_dev (device or host-mapped u64) when the
 * stream reaches it.  cap must be ono_sparse_max_bytes(n) (ONO_E_SIZE
 * otherwise).  For a device-side consumer of the stream (an RCCL send of the
 * frame, a device lift) and for back-to-back timing.
 * It can be captured into a HIP graph once an uncaptured call on the same
 * stream has made its scratch for that size (else ONO_E_ARG; nothing is
 * allocated or zeroed under capture): captured, it always takes the two
 * launches, whose state between calls (the chunk aggregates' parity) lives on
 * the device.  The graph holds that stream's scratch: replay it ordered with
 * the stream's other drops (on the stream, or after it).                    */
int ono_sparse_drop_async(uint8_t *buf_dev, size_t cap, uint64_t *nbytes_dev, const float *g_dev, size_t n,
                          float threshold, void *stream);
/* Synchronizes the stream, then reports (and clears) an error a stream-ordered
 * drop on it left: ONO_E_IO when a writer found its range past the buffer or
 * the chunk aggregates disagreeing with the tile records; ONO_OK otherwise.  */
int ono_sparse_drop_check(void *stream);
/* Test hook: adds `add` to the kept-value and run counts of every chunk
 * aggregate that the stream's next two-launch drop will sum into — the
 * "aggregate not zero when the call began" fault — so that tests can show it
 * ends in ONO_E_IO, not an out-of-bounds store.  ONO_E_ARG before the first
 * two-launch drop on the stream.                                             */
int ono_sparse_drop_debug_stale(void *stream, uint32_t add);
int ono_sparse_lift(float *g_dev, size_t cap, size_t *out_len, const uint8_t *buf_host, size_t nbytes,
                    void *stream);
/* lift of a stream already in HBM (e.g. ono_sparse_drop's output or a frame
 * received into device memory); same results and errors as ono_sparse_lift.
 * Both parse on the device, in up to three tiers, each exact or refuted:
 * (1) the pattern path — in drop output with gaps and runs below 2^16 values
 * a record starts exactly where units k+1 and k+3 are zero; the candidates are
 * checked to be the sequential parse (head, every successor, the sum) in
 * parallel; (2) the walk path — speculative record starts per 128-B segment
 * and verified walks; (3) the reference's sequential host parse, when the walk
 * is refuted or the stream is malformed (and the source of its error
 * messages).  g[total, cap) is left untouched.                             */
int ono_sparse_lift_dev(float *g_dev, size_t cap, size_t *out_len, const uint8_t *buf_dev, size_t nbytes,
                        void *stream);
/* The stream-ordered lift (ono_sparse_drop_async's counterpart): the pattern
 * path alone, nothing waits on the host.  *ticket receives a nonzero value;
 * once the stream has passed the call, *status (device or host-mapped u64, one
 * per stream) equals *ticket iff the lift was refused — a stream outside the
 * pattern's shape, a malformed one, or total > cap — and g is then
 * unspecified: call ono_sparse_lift_dev (blocking), which parses any stream and
 * returns the reference's errors and ONO_E_SIZE.  Otherwise g[0, total) holds
 * the lift (total: the stream's first 8 bytes).  Scratch is per stream.
 * A refused call may already have written parts of g[0, total): check the
 * status before using g.  The one-launch form (an 8-B aligned stream of at
 * most 4096 tiles) needs its whole grid resident; when kernels of another
 * stream or process hold CU slots so that a waiting tile sees the words it
 * polls stand still for ~100 us, the call is refused rather than waiting for
 * them (tests/test_gpu_sparse_pattern.py: 3/4 of the CUs held by another
 * process — refused early, exact after the blocking lift).  */
int ono_sparse_lift_dev_async(float *g_dev, size_t cap, const uint8_t *buf_dev, size_t nbytes, uint64_t *status,
                              uint64_t *ticket, void *stream);
/* lifts so far (this process) that took the sequential host parse        */
size_t ono_sparse_lift_fallbacks(void);
/* test hook: the process's next `count` one-launch stream-ordered lifts are
 * refused (their status word set), whatever the stream — the path a caller
 * takes after a refusal (the blocking lift, as the TCP ring's hop does) is
 * then exercised on well-formed streams.  0 clears it.  Returns the count the
 * call replaced
 * (the refusals not yet taken).                                              */
int ono_sparse_lift_debug_refuse(uint32_t count);
/* lifts so far (this process) that the pattern path handed to the walk path */
size_t ono_sparse_lift_pattern_misses(void);
/* diagnostics: 0 (default) pattern path first; 1 walk path only            */
int ono_sparse_lift_set_mode(int mode);
int ono_sparse_mask(float *g_dev, size_t n, float threshold, int zero_kept, void *stream);

/* synthetic gradient bucket (SURVEY.md §8(d) distribution), bit-identical to
 * the CPU oracle's generator: out[j] = synth(seed, rank, offset + j)          */
int ono_synth_f32(float *out, size_t n, uint64_t seed, uint64_t rank, size_t offset, void *stream);

/* ===================================================================== */
/* Ring all-reduce — WorkerRingManager (worker/src/middlewares/worker_ring.rs) */
/* ===================================================================== */
typedef struct ono_ring ono_ring;

/* rank 0 generates the id; it travels to the other ranks out of band (over the
 * ring's existing TCP links, worker/src/builder.rs:272-311).               */
int ono_ring_unique_id(uint8_t uid[ONO_UID_BYTES]);

/* WorkerRingManager::new(pos, addrs, prev, next, size, layers) (:39-56).
 * Allocates the owned grad and residual buckets (size f32 each, zeroed) on
 * `device`.  nranks == 1 needs no uid (may be NULL).                        */
int ono_ring_create(ono_ring **out, int pos, int nranks, size_t size, int device,
                    const uint8_t *uid, int wire);
/* The TCP edge: the same manager over the worker's own sockets — fd_prev the
 * accepted connection from the previous worker, fd_next the connection to the
 * next (worker/src/builder.rs:272-311; the caller keeps ownership).  Frames
 * are the reference's byte for byte ([u64 BE len][u32 BE kind][payload],
 * comms/src/protocol/msg.rs:120-191): DenseGrad (kind 1/2, f16 LE) or, with
 * ono_ring_set_sparse, SparseGrad (kind 3/4), so MI355X workers and reference
 * Rust workers of either serializer form one ring.  A received gradient of
 * another length than the hop's chunk is added over the shorter length in the
 * scatter (the zip of worker_ring.rs:141-143) and refused in the gather
 * (ONO_E_PROTO; the reference's copy_from_slice at :200 panics).  Any other
 * frame fails as WorkerHandle::recv_event + the ring would
 * (ono_worker_event_check): ONO_E_PROTO "Received an invalid worker event" for
 * the worker events Upgraded / Disconnect / Done / ReportLoss, ONO_E_IO for a
 * kind byte >= 7 (msg.rs:187), "Unexpected message from worker" (params, data
 * chunks, other commands), "loss diverged", malformed JSON, a malformed sparse
 * stream and socket failures.  f16 wire, hop schedule; the hop arithmetic runs
 * in HBM (fused codec kernels), one D2H + H2D of the chunk per hop.          */
int ono_ring_create_tcp(ono_ring **out, int pos, int nranks, size_t size, int device, int fd_prev,
                        int fd_next);
/* The SparseCapable serializer of this worker (SerializerSpec sparse_capable{r};
 * Compressor::compress, comms/src/handles/compressor.rs:71-98): for every chunk
 * it pushes, t = calculate_threshold(chunk, r) and the grad_drop stream of the
 * values with |g| >= t; that stream goes out as a SparseGrad frame (kind 3)
 * when it is no longer than the chunk's f16 payload (2 bytes per value, :79),
 * else the chunk goes out as a DenseGrad of f16(chunk) (:84-89).  The ring
 * takes the branch push_grad's result selects (worker_ring.rs:125-134,
 * 177-193): after a SparseGrad the scatter zeroes only the sent values of the
 * residual and the gather keeps only the sent values in grad, leaving the
 * owned residual chunk as it is (the reset at :178-184 is commented out, so it
 * keeps the reduced sum into the next round); after a DenseGrad the scatter
 * zeroes the chunk and the gather zeroes the owned residual at j == 0.  ratio
 * in (0, 1]; 0 = the Base (dense f16) serializer.  TCP rings only (n > 1):
 * inside a node the dense schedules move fewer bytes than a sparse stream is
 * worth.  Every worker accepts both gradient kinds whatever its own serializer
 * (handles/worker.rs:102-108).  `seed` starts the default sampler's stream.  */
int ono_ring_set_sparse(ono_ring *ring, float ratio, uint64_t seed);
/* Draws the threshold sample of one push: `amount` = min(len, 16384) distinct
 * indices of [0, len) into idx; return 0 on success.  Called for every sparse
 * push (also when amount == len, so a caller-side RNG stays in step with the
 * reference's, which draws from its StdRng on every calculate_threshold).
 * A Rust integration installs rand::seq::index::sample over the Compressor's
 * StdRng — the reference's choose_multiple draws exactly those indices.
 * NULL restores the default (ono_sparse_sample_default).                     */
typedef int (*ono_sample_fn)(void *ctx, size_t len, uint32_t *idx, size_t amount);
int ono_ring_set_sampler(ono_ring *ring, ono_sample_fn fn, void *ctx);
/* WorkerHandle::recv_event's verdict on one received frame of this kind byte
 * (comms/src/handles/worker.rs:82-130, protocol/msg.rs:160-191) as the ring
 * sees it: ONO_OK for a gradient (kinds 1-4); kind 0 parses the JSON Command
 * (serde's externally tagged snake_case form) — Upgraded / Disconnect / Done /
 * a finite ReportLoss -> ONO_E_PROTO "Received an invalid worker event"
 * (worker_ring.rs:136-138), a ReportLoss with a null (NaN) loss -> ONO_E_IO
 * "loss diverged: NaN or Inf detected", another command -> ONO_E_IO
 * "Unexpected message from worker", malformed JSON or an unknown command ->
 * ONO_E_IO (the serde error); kinds 5 / 6 -> ONO_E_IO "Unexpected message from
 * worker"; kind >= 7 -> ONO_E_IO "Received an invalid kind byte".  Host only.  */
int ono_worker_event_check(uint32_t kind, const uint8_t *payload, size_t nbytes);
int ono_ring_destroy(ono_ring *ring);
/* the owned buckets (device pointers): grad = WorkerRingManager.grad,
 * residual = WorkerRingManager.residual                                      */
float *ono_ring_grad(ono_ring *ring);
float *ono_ring_residual(ono_ring *ring);
size_t ono_ring_size(const ono_ring *ring);
/* producer side: residual += grad_dev (ParamManager::acc_residual) */
int ono_ring_acc_residual(ono_ring *ring, const float *grad_dev, void *stream);
/* pull_grads (:82-94) on the owned buckets, device resident: on return
 * (stream-ordered) grad = averaged all-reduced bucket, residual = 0.        */
int ono_ring_pull_grads(ono_ring *ring, void *stream);
/* the same on caller device buffers of ono_ring_size() elements */
int ono_ring_pull_grads_dev(ono_ring *ring, float *residual_dev, float *grad_dev, size_t n,
                            void *stream);
/* host-fed form (the reference's buffers live in host memory and arrive on
 * TCP): chunked H2D -> reduce -> D2H pipeline on three streams; blocking.
 * The exact schedules (HOPS, DIRECT, XGMI) pipeline sub-rounds (a slice of
 * every chunk each, ono_plan_pull_grads_sub), so every element keeps its
 * owner and chain; a TCP ring and the sparse mode run whole buckets.        */
int ono_ring_pull_grads_host(ono_ring *ring, float *residual_host, float *grad_host, size_t n);
/* Page-lock long-lived caller buckets (the reference's WorkerRingManager
 * Vec<f32>s live as long as the manager) so pull_grads_host DMAs them in
 * place; unregistered buffers are staged through pinned bounce slots.       */
int ono_ring_register_host(ono_ring *ring, void *ptr, size_t bytes);
int ono_ring_unregister_host(ono_ring *ring, void *ptr);
/* Schedule of the n > 1 exchange (default AUTO: F32 -> ALLREDUCE, F16 -> DIRECT
 * for n <= ONO_MAX_INPUTS, else HOPS; a TCP ring always runs HOPS).
 *   ALLREDUCE  ncclAllReduce + fused ÷n / residual reset (f32 wire only)
 *   HOPS       the reference hop ring (n-1 scatter + n-1 gather hops) over
 *              ncclSend/ncclRecv, bit-exact for both wires
 *   DIRECT     all-to-all of chunk slices over every xGMI link at once, the
 *              owner replays the reference chain in one fused kernel, then an
 *              all-gather; bit-exact for both wires; n <= ONO_MAX_INPUTS     */
typedef enum {
    ONO_ALGO_AUTO = 0,
    ONO_ALGO_ALLREDUCE = 1,
    ONO_ALGO_HOPS = 2,
    ONO_ALGO_DIRECT = 3,
    ONO_ALGO_XGMI = 4
} ono_algo;
/*   XGMI       the direct schedule's arithmetic with no collective library in
 *              the data path: each rank maps its peers' exchange regions (IPC,
 *              uncached HBM) and the kernels push slices into the owners'
 *              receive slots and pull the owners' results over xGMI, with
 *              device-side flag barriers (timeout: ono_ring_set_xgmi_timeout,
 *              default 600 s -> ONO_E_IO).  Bit-exact for both wires; ranks of
 *              one node; n <= ONO_MAX_INPUTS.  On an RCCL ring the exchange
 *              regions are connected over the communicator on first use.
 *              One ring's rounds must run in issue order (one stream, or
 *              streams ordered by events): a barrier takes a peer's flag more
 *              than one epoch ahead as foreign and fails the round (ONO_E_IO),
 *              which two unordered rounds of one ring could produce.        */
int ono_ring_set_algo(ono_ring *ring, int algo);
/* A ring with no collective library at all (ONO_ALGO_XGMI only): create,
 * export this rank's handle, pass every rank's handle (nranks x
 * ONO_XGMI_HANDLE_BYTES, rank order) to connect.  The handles travel out of
 * band, like the RCCL id.  A handle is [IPC handle, 64 B][u64 ring id][u64
 * layout bytes][u64 region uid][u64 region alloc bytes], zero-padded to
 * ONO_XGMI_HANDLE_BYTES; connect maps every peer region, checks that every
 * page of each mapping shows that peer's ring id (a stale import -> ONO_E_IO),
 * and returns once every rank has connected (a device barrier).  Destroy is
 * collective: each rank marks every peer region it is done with; a region goes
 * back to the process's pool once all peers have marked it, and is
 * quarantined (never reused) when the timeout passed or the ring was aborted.
 * RETENTION: pooled regions and peer imports are kept for the life of the
 * process (a later ring reuses them) until released.  A fresh region whose
 * IPC handle repeats one this process obtained before is parked and another
 * allocated (re-importing a repeated handle handed out partly stale mappings on
 * this ROCm); an import of a handle this process opened before is ONO_E_IO.
 * RESIDUAL RISK: one wrong result seen in round 4 (a rank read stale lines of a
 * peer's result slot right after a pool release) was narrowed to the free and
 * re-import path, not proven; that path is now closed by the
 * rules above.  Round 6 saw it twice more in the host-fed form right after a
 * release, classified as one rank's copy-engine-written residual read back as
 * zeros at scattered lines; the host-fed round's residual is since written by
 * a kernel (ono_ring_pull_grads_host).  Not proven either: a caller that must
 * never see it can keep its rings (and the pool) for the process's life.    */
#define ONO_XGMI_HANDLE_BYTES 128
int ono_ring_create_xgmi(ono_ring **out, int pos, int nranks, size_t size, int device, int wire);
int ono_ring_xgmi_handle(ono_ring *ring, uint8_t handle[ONO_XGMI_HANDLE_BYTES]);
int ono_ring_xgmi_connect(ono_ring *ring, const uint8_t *handles);
/* Releasing the pool is two-phase, on every rank once all its xGMI rings are
 * destroyed (ONO_E_ARG while one is alive):
 *   1. ono_xgmi_pool_close_imports on every rank: each peer region this
 *      process maps is marked closed in the region itself (a system-scope add
 *      to its close counter), then its import is closed;
 *   2. a collective step (the caller's barrier over its control channel);
 *   3. ono_xgmi_pool_free_exports on every rank: each idle region is freed
 *      once its close counter has reached its open counter (each importer
 *      bumped the open counter when it mapped the region), waiting up to wait_s
 *      seconds (other pool calls are not held up meanwhile); a region some
 *      peer still maps is kept (ONO_E_IO, *kept > 0), never handed to a later
 *      ring, and freed by a later free_exports once its peers closed it.  So no
 *      region is freed while a peer still maps it.  Quarantined regions and
 *      parked allocations (fresh ones whose handle repeated an earlier one:
 *      freed, the allocator would return the same block and handle) stay.
 * Rings created afterwards export and import fresh regions (verified at
 * connect as always).  ono_xgmi_pool_release = phase 1 then phase 3 in one
 * call, waiting up to 30 s (env ONO_XGMI_RELEASE_WAIT_S) for the peers' phase 1:
 * the counters still order the frees after the peers' close marks, but the
 * mark precedes its import's close by one host call, so multi-process callers
 * should use the two phases with the collective step between.               */
int ono_xgmi_pool_close_imports(size_t *closed_imports);
int ono_xgmi_pool_free_exports(size_t *freed_bytes, size_t *kept, double wait_s);
int ono_xgmi_pool_release(size_t *freed_bytes, size_t *closed_imports);
/* regions pooled (and their bytes, of which quarantined), peer imports held */
int ono_xgmi_pool_stats(size_t *regions, size_t *region_bytes, size_t *quarantined, size_t *imports);
/* How long an xGMI barrier waits for a peer (seconds, > 0) before the round
 * fails with ONO_E_IO; 0 = env ONO_XGMI_TIMEOUT_S, else 600 s.  The reference
 * ring blocks while a peer is slow: set this above the longest time ranks may
 * drift apart between rounds (evaluation, checkpointing on one rank).
 * ono_ring_abort ends a waiting barrier at once.                            */
int ono_ring_set_xgmi_timeout(ono_ring *ring, double seconds);
/* Health of the rounds already enqueued: call after synchronizing the stream.
 * ONO_E_IO when an xGMI barrier timed out (that round's results are invalid,
 * and every later call fails the same way), ONO_E_ABORTED after
 * ono_ring_abort, else ONO_OK.                                               */
int ono_ring_check(const ono_ring *ring);
/* Segments of the f32 all-reduce schedule (ONO_ALGO_ALLREDUCE): with k > 1
 * the fused finaliser (÷n, residual = 0) of segment j overlaps the RCCL
 * all-reduce of segment j+1; 1 = one all-reduce then one finaliser; 0 = the
 * default (env ONO_AR_SEGMENTS, else 4).  At least 16 MiB per segment.  Results do
 * not depend on it beyond RCCL's own summation order.                       */
int ono_ring_set_pipeline(ono_ring *ring, int segments);
/* in-place averaged all-reduce of a device buffer (buf = sum_r buf_r / n) */
int ono_ring_allreduce_avg_dev(ono_ring *ring, float *buf_dev, size_t n, void *stream);
/* Cancellation: makes the in-flight and every later call fail with
 * ONO_E_ABORTED (RCCL communicator aborted).  Thread-safe.                   */
int ono_ring_abort(ono_ring *ring);
/* Device time of the library's own kernels inside pull_grads (HIP events on
 * the launch stream).  enable=1 starts recording; read returns the summed ms
 * and the launch count of the dominant local kernel since enabling.         */
int ono_ring_timing_enable(ono_ring *ring, int enable);
int ono_ring_timing_read(ono_ring *ring, double *kernel_ms, int64_t *launches,
                         double *collective_ms, int64_t *collectives);
/* The same split by phase (ms[ONO_PHASES], count[ONO_PHASES]): local kernels,
 * RCCL calls (on a TCP ring: the socket exchange of a hop), the xGMI
 * schedule's scatter (push), barriers and gather (pull, or owner chain +
 * remote stores with ONO_XGMI_GATHER=push), and on a TCP ring with the
 * SparseCapable serializer the sparse codec (threshold, drop, mask, lift of
 * a received SparseGrad).  The collective total of ono_ring_timing_read is
 * phases 1..4; the kernel total is phase 0.                                 */
typedef enum {
    ONO_PHASE_KERNEL = 0,
    ONO_PHASE_RCCL = 1,
    ONO_PHASE_XGMI_SCATTER = 2,
    ONO_PHASE_XGMI_BARRIER = 3,
    ONO_PHASE_XGMI_GATHER = 4,
    ONO_PHASE_SPARSE_CODEC = 5,
    ONO_PHASES = 6
} ono_phase;
int ono_ring_timing_phases(ono_ring *ring, double *ms, int64_t *count);

/* n virtual ranks co-resident on ONE device (the device analog of the
 * reference's loopback workers): residuals[r], grads[r] are device buckets of
 * n_elems; executes the exact hop schedule of worker_ring.rs with the wire
 * modelled by on-device f16/f32 message buffers.                            */
int ono_local_ring_pull_grads(float *const *residuals, float *const *grads, int nranks,
                              size_t n_elems, int wire, void *stream);
/* the same round with the DIRECT schedule's arithmetic (one fused owner kernel
 * per chunk reading every rank's slice); nranks <= ONO_MAX_INPUTS          */
int ono_local_direct_pull_grads(float *const *residuals, float *const *grads, int nranks,
                                size_t n_elems, int wire, void *stream);

/* ===================================================================== */
/* Parameter-server store & synchronizer — parameter_server/src/{storage,synchronization} */
/* ===================================================================== */
typedef enum { ONO_OPT_GD = 0, ONO_OPT_MOMENTUM = 1, ONO_OPT_ADAM = 2, ONO_OPT_ADD = 3 } ono_opt_kind;
typedef struct {
    int kind;       /* ono_opt_kind; ADD = the reference tests' AddOptimizer */
    float lr;       /* learning_rate (FloatPositive) */
    float momentum; /* GradientDescentWithMomentum::momentum */
    float beta1, beta2, eps; /* Adam */
} ono_opt_spec;

/* The all-reduce consumer (worker/src/workers/all_reduce.rs:126-132):
 * ParamManager::optimize (param_manager.rs:148-165) + zero_grad (:168-172) +
 * `optimization_params.copy_from_slice(&params)` as ONE fused kernel:
 * params = opt(params, grad); grad = 0; params_copy = params (when non-NULL).
 * The optimizer state (velocity / Adam moments and powers) lives in HBM.     */
typedef struct ono_optimizer ono_optimizer;
int ono_optimizer_create(ono_optimizer **out, const ono_opt_spec *opt, size_t n, int device);
int ono_optimizer_destroy(ono_optimizer *opt);
int ono_optimizer_step(ono_optimizer *opt, float *params_dev, float *grad_dev, float *params_copy_dev,
                       size_t n, void *stream);

typedef enum { ONO_STORE_BLOCKING = 0, ONO_STORE_WILD = 1 } ono_store_kind;
typedef struct ono_store ono_store;

/* BlockingStore::new / WildStore::new (blocking/store.rs:49-75, wild/store.rs:36-61):
 * init_params_host holds nparams initial values (the ParamGen output);
 * shard_size as ServerBuilder::resolve_store computes it (builder.rs:164-173)
 * bounds the per-shard optimizer state; nworkers = the barrier size.        */
int ono_store_create(ono_store **out, int kind, const float *init_params_host, size_t nparams,
                     size_t shard_size, size_t nworkers, const ono_opt_spec *opt, int device);
int ono_store_destroy(ono_store *store);
size_t ono_store_len(const ono_store *store);
/* Store::accumulate (store.rs:84-91): thread-safe; ONO_E_SIZE on length mismatch */
int ono_store_accumulate(ono_store *store, const float *grad_host, size_t n);
int ono_store_accumulate_dev(ono_store *store, const float *grad_dev, size_t n);
/* The same from the reference's wire form: the worker's f16 gradient payload
 * (ParamServerHandle::push_grad, comms/src/handles/parameter_server.rs:92-107)
 * crosses PCIe as f16 and is decoded inside the accumulate kernel — the
 * server's CPU decode (handles/worker.rs:82-101) + accumulate, fused.        */
int ono_store_accumulate_f16(ono_store *store, const uint16_t *grad_f16_host, size_t n);
int ono_store_accumulate_f16_dev(ono_store *store, const uint16_t *grad_f16_dev, size_t n);
/* Store::update_params (store.rs:93-108): CAS-guarded; a concurrent second
 * caller returns immediately without updating.                              */
int ono_store_update_params(ono_store *store);
/* Store::pull_params (store.rs:110-124) */
int ono_store_pull_params(ono_store *store, float *out_host, size_t n);
int ono_store_pull_params_dev(ono_store *store, float *out_dev, size_t n);
/* test hooks mirroring the reference unit tests' field access (store.rs:186-214) */
int ono_store_active_idx(const ono_store *store);
int ono_store_set_updating(ono_store *store, int updating);

typedef enum { ONO_SYNC_BARRIER = 0, ONO_SYNC_NONBLOCKING = 1 } ono_sync_kind;
typedef struct ono_sync ono_sync;
/* BarrierSync::new(size) / NoBlockingSync::new() */
int ono_sync_create(ono_sync **out, int kind, size_t barrier_size);
/* Clone: one handle per worker task (the Rust Arc clone) */
int ono_sync_clone(ono_sync *sync);
/* Drop of one clone: BarrierSync::drop shrinks the barrier when other clones
 * remain (barrier.rs:30-38); the last release frees the synchronizer.        */
int ono_sync_release(ono_sync *sync);
/* Synchronizer::step (synchronizer.rs:7-21; barrier.rs:41-50; non_blocking.rs:20-31):
 * accumulate(grad); [barrier: last arriver runs update_params]; pull_params(params) */
int ono_sync_step(ono_sync *sync, ono_store *store, const float *grad_host, float *params_host,
                  size_t n);
/* the same with the gradient as the f16 payload it arrives in (fused decode) */
int ono_sync_step_f16(ono_sync *sync, ono_store *store, const uint16_t *grad_f16_host, float *params_host,
                      size_t n);

/* DynBarrier (synchronization/dyn_barrier.rs:47-106), exposed for the host tests */
typedef struct ono_barrier ono_barrier;
typedef void (*ono_leader_fn)(void *ctx);
int ono_barrier_create(ono_barrier **out, size_t size);
int ono_barrier_destroy(ono_barrier *b);
int ono_barrier_wait_with(ono_barrier *b, ono_leader_fn leader, void *ctx);
int ono_barrier_acquire(ono_barrier *b);

/* ===================================================================== */
/* Multi-GPU parameter-server mode (BASELINE config 5): the sharded        */
/* synchronizer as reduce-scatter + fused (÷nworkers + optimizer) + all-gather */
/* over the ring's communicator.  Shards of ceil(n / nranks) parameters, the   */
/* last one zero-padded; rank r owns shard r (ono_plan_ps_step).            */
/* ===================================================================== */
typedef struct ono_ps ono_ps;
int ono_ps_create(ono_ps **out, ono_ring *ring, const float *init_params_host, size_t nparams,
                  const ono_opt_spec *opt);
int ono_ps_destroy(ono_ps *ps);
/* grad_dev: this worker's gradient (nparams); params_dev: receives the
 * updated full parameter vector.  Stream-ordered.                           */
int ono_ps_step(ono_ps *ps, const float *grad_dev, float *params_dev, void *stream);

/* ===================================================================== */
/* Exchange plans: the N > 1 schedules as data                             */
/* ===================================================================== */
/* Every collective schedule of pull_grads (ALLREDUCE incl. its segments,
 * HOPS, DIRECT; either wire) and of ono_ps_step is built as a list of steps by
 * a pure host function and executed by one interpreter (RCCL calls, HIP
 * kernels, memsets, copies, side-stream forks / joins).  The same lists are
 * exported here so a CPU test can check them for every rank count and bucket
 * length — matched sends / receives per group, offsets in bounds, chunks
 * tiling [0, N), no overlapping accesses across the two streams — and run
 * them with host copies against the oracle, without an 8-GPU node.
 * Operand i of a step is (buf[i], off[i]): an element offset into one of the
 * rank's buffers (ono_plan_buf; sizes from ono_plan_buffers).               */
typedef enum {
    ONO_PLAN_GROUP_BEGIN = 0, /* ncclGroupStart                                        */
    ONO_PLAN_SEND = 1,        /* ref0, count, dtype -> peer                              */
    ONO_PLAN_RECV = 2,        /* ref0, count, dtype <- peer                              */
    ONO_PLAN_GROUP_END = 3,   /* ncclGroupEnd                                          */
    ONO_PLAN_ALLREDUCE = 4,   /* ref1[0, count) = sum over ranks of ref0[0, count) (f32) */
    ONO_PLAN_REDUCE_SCATTER = 5, /* ref1[0, count) = sum over ranks of ref0[pos*count, +count) */
    ONO_PLAN_ALL_GATHER = 6,  /* ref1[q*count, +count) = rank q's ref0[0, count)         */
    ONO_PLAN_KERNEL = 7,      /* op over count elements                                  */
    ONO_PLAN_MEMSET = 8,      /* ref0[0, count) = 0                                      */
    ONO_PLAN_COPY = 9,        /* ref0[0, count) = ref1[0, count)                         */
    ONO_PLAN_FORK = 10,       /* the side stream waits for the main stream's work so far */
    ONO_PLAN_JOIN = 11        /* the main stream waits for the side stream's work so far */
} ono_plan_kind;
typedef enum {
    ONO_POP_ENCODE_ZERO = 0,     /* [out wire, chunk]: out = enc(chunk); chunk = 0          */
    ONO_POP_ADD_ENCODE_ZERO = 1, /* [out, acc, in]: x = acc + dec(in); out = enc(x); acc = 0 */
    ONO_POP_ADD_FINISH = 2,      /* [grad, out, acc, in]: x = acc + dec(in); grad = x / d;
                                    out = enc(x); acc = 0                                   */
    ONO_POP_DECODE_SCALE = 3,    /* [out f32, in wire]: out = dec(in) / d                   */
    ONO_POP_DIRECT = 4,          /* [grad, out | NONE, in_0 .. in_k-1]: p = in_0,
                                    p = in_j + wire(p); grad = p / d; out = enc(p) (f16) or
                                    grad (f32); zero in_k-1, or every in_j when flag      */
    ONO_POP_SCALE_ZERO = 5,      /* [dst, src, zero | NONE]: dst = src / d; zero = 0        */
    ONO_POP_OPT_UPDATE = 6       /* [g, w]: the store's fused (+0, / d, optimizer) update of
                                    a shard; flag = zero g afterwards                       */
} ono_plan_op;
typedef enum {
    ONO_PB_NONE = -1,
    ONO_PB_RESIDUAL = 0, ONO_PB_GRAD = 1, /* the buckets (f32, size)                       */
    ONO_PB_WIRE0 = 2, ONO_PB_WIRE1 = 3,   /* hop wire slots (wire dtype, maxchunk + 4)     */
    ONO_PB_RBUF = 4,                      /* direct receive slots (f32, n x (maxchunk + 4)) */
    ONO_PB_GSTAGE = 5,                    /* direct f16 all-gather staging (n x (maxchunk + 4)) */
    ONO_PB_MSG = 6,                       /* the owner's f16 message (maxchunk + 4)          */
    ONO_PB_GIN = 7, ONO_PB_GPAD = 8, ONO_PB_GSHARD = 9, /* PS: gradient in (nparams), padded
                                             copy (n x shard), reduced shard (shard)        */
    ONO_PB_PPAD = 10, ONO_PB_PARAMS = 11, /* PS: padded parameters, parameters out           */
    ONO_PB_COUNT = 12
} ono_plan_buf;
#define ONO_PLAN_REFS (ONO_MAX_INPUTS + 2)
typedef struct {
    int32_t kind;   /* ono_plan_kind */
    int32_t op;     /* ono_plan_op (KERNEL) */
    int32_t peer;   /* SEND / RECV */
    int32_t dtype;  /* ono_wire: element type of the step's data */
    int32_t stream; /* 0 = the caller's stream, 1 = the side stream */
    int32_t nref;
    int32_t flag;
    float divisor;
    uint64_t count;
    int32_t buf[ONO_PLAN_REFS];
    uint64_t off[ONO_PLAN_REFS];
} ono_plan_step;
/* pull_grads of rank pos: algo ALLREDUCE (f32 wire; `segments` as
 * ono_ring_set_pipeline resolves them, >= 1), HOPS or DIRECT.  Writes up to cap
 * steps; *count = the plan's length (call with cap 0 to size it).           */
int ono_plan_pull_grads(int algo, int wire, int pos, int nranks, size_t size, int segments, ono_plan_step *steps,
                        size_t cap, size_t *count);
/* sub-round sub_index of a host-fed HOPS / DIRECT round (what
 * ono_ring_pull_grads_host runs for those schedules): elements
 * [j sub, (j + 1) sub) of every chunk, sub = sub_elems rounded down to a
 * multiple of 64 (at least 64); steps over empty slices are left out on both
 * sides.  The sub-rounds in order equal the whole-bucket round bit for bit.  */
int ono_plan_pull_grads_sub(int algo, int wire, int pos, int nranks, size_t size, size_t sub_elems, size_t sub_index,
                            ono_plan_step *steps, size_t cap, size_t *count);
/* how many sub-rounds of sub_elems per chunk cover a bucket (0: no plan)    */
size_t ono_plan_sub_rounds(int nranks, size_t size, size_t sub_elems);
/* ono_ps_step of rank pos over the RCCL communicator (reduce-scatter, fused
 * update, all-gather; shards of ceil(nparams / nranks), zero-padded)        */
int ono_plan_ps_step(int pos, int nranks, size_t nparams, ono_plan_step *steps, size_t cap, size_t *count);
/* element counts of the plan buffers (ONO_PB_COUNT entries) for a ring of
 * nranks over `size` elements and a PS of nparams                           */
int ono_plan_buffers(int nranks, size_t size, size_t nparams, uint64_t *counts);
/* Every rank's plan executed by nranks co-resident ranks on ONE device, in
 * lockstep: local steps through the same kernel launcher the RCCL interpreter
 * uses; a group's sends matched with the peers' receives and carried out as
 * device copies; all-reduce / reduce-scatter as the sum over ranks in rank
 * order, all-gather as copies.  Runs the N > 1 schedules' device work on a
 * one-GPU box (RCCL refuses two ranks per device).  Blocking.
 * pull_grads: residuals[r], grads[r] are rank r's buckets of `size`.        */
int ono_plan_run_local(int algo, int wire, int nranks, size_t size, int segments, float *const *residuals,
                       float *const *grads, void *stream);
/* the host-fed sub-rounds of ono_plan_pull_grads_sub run one after another
 * by co-resident ranks, as ono_plan_run_local runs whole rounds (nranks >= 2) */
int ono_plan_run_local_sub(int algo, int wire, int nranks, size_t size, size_t sub_elems, float *const *residuals,
                           float *const *grads, void *stream);
/* ono_ps_step's plan: grads[r] (nparams) in, params[r] (nparams) out; shards[r]
 * is rank r's shard of the parameters (split at ceil(nparams / nranks)) and
 * its optimizer state v[r], s[r] (may be NULL for GD), updated in place;
 * step_size is Adam's lr sqrt(1 - b2^t) / (1 - b1^t) for this step.         */
int ono_plan_run_local_ps(int nranks, size_t nparams, const float *const *grads, float *const *params,
                          float *const *shards, float *const *v, float *const *s, const ono_opt_spec *opt,
                          float step_size, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* ONO_REDUCE_H */
