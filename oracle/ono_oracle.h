/*
 * ono_oracle.h — CPU ORACLE (TEST INFRASTRUCTURE ONLY).
 *
 * A plain-C restatement of the reference's gradient-bucket reduction path
 * (lminervino18/oxidized-neural-orchestra, Rust).  Only tests/, the smoke()
 * check in __graft_entry__.py and bench.py's cpu_baseline leg may load this;
 * the product (oxidized-neural-orchestra_amd/) never links or calls it.
 *
 * Parity pinning: the reference has no C/C++ source and no Rust toolchain is
 * present, so this is a restatement.  It is pinned by
 *   - the reference's byte KATs for the f16 wire (comms/src/sparse/protocol.rs:150-223,
 *     comms/src/sparse/tests.rs:13-59),
 *   - the BlockingShard / BlockingStore unit tests
 *     (parameter_server/src/storage/blocking/shard.rs:132-185, store.rs:156-243),
 *   - an independent numpy restatement (oracle/oracle_np.py) that generated the
 *     golden fixtures in tests/golden/ (tests/golden/make_golden.py).
 * The ring arithmetic itself is not covered by any reference test
 * (SURVEY.md §4): "parity pinned by restatement + numpy cross-check only".
 */
#ifndef ONO_ORACLE_H
#define ONO_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- f16 codec, crate `half` 2.7.1 semantics (IEEE binary16, RNE) ---------
 * call sites: comms/src/handles/compressor.rs:116 (encode),
 *             comms/src/handles/worker.rs:94 (decode)                       */
uint16_t ono_ref_f32_to_f16(float x);
float ono_ref_f16_to_f32(uint16_t h);
void ono_ref_f16_encode(uint16_t *out, const float *in, size_t n);
void ono_ref_f16_decode(float *out, const uint16_t *in, size_t n);

/* ---- chunking: worker/src/middlewares/mod.rs:15-59 -------------------------
 * Writes up to n+1 offsets; returns the number of chunks produced (which is
 * min(len, n) — the reference iterator stops at an empty slice).            */
size_t ono_ref_split_chunks(size_t len, size_t n, size_t *offsets);

/* ---- ring all-reduce: worker/src/middlewares/worker_ring.rs:82-204 ---------
 * Simulates all `nranks` workers of one pull_grads() round in lockstep.
 * residual[r], grad[r]: per-rank host buffers of `len` f32.
 * wire = 0: the reference f16 wire (compressor.rs:106-118)
 * wire = 1: an f32 wire (same hop order, no quantisation) — the RCCL model.
 * Returns 0, or -1 when the reference would panic (len < nranks, len == 0).  */
int ono_ref_ring_pull_grads(float *const *residual, float *const *grad, int nranks,
                            size_t len, int wire);
/* The same round with each worker's serializer: ratio[r] == 0 -> Base (dense
 * f16 DenseGrad), ratio[r] in (0, 1] -> SparseCapable{ratio[r]}
 * (Compressor::compress, comms/src/handles/compressor.rs:71-98): every push
 * computes t = calculate_threshold(chunk, ratio) (sample drawn with
 * ono_ref_sample_default at state[r] above 16384 values; state advanced) and
 * the grad_drop stream; the push is a SparseGrad only when that stream is no
 * longer than the chunk's f16 payload (len * 2 bytes, :79), else a DenseGrad.
 * The ring then takes the branch push_grad's result selects
 * (worker_ring.rs:125-134, 177-193):
 *   scatter: sparse -> zero the sent values (|g| >= t); dense -> zero the chunk;
 *   gather:  sparse -> grad keeps only the sent values (|g| < t -> 0) and the
 *            owned residual chunk is left as it is (:178-184 commented out);
 *            dense at j == 0 -> zero the owned residual chunk.
 * Receivers add (scatter) or copy (gather) the decoded / lifted chunk: a
 * SparseGrad lifts into a zero-filled buffer (handles/worker.rs:102-108).   */
int ono_ref_ring_pull_grads_sparse(float *const *residual, float *const *grad, int nranks, size_t len,
                                   const float *ratio, uint64_t *state);
/* One push of chunk ch by a worker of serializer `ratio`: 1 if it goes out as a
 * SparseGrad (threshold in *t), 0 if as a DenseGrad; the sampler state advances
 * as in the ring.                                                            */
int ono_ref_sparse_push_is_sparse(const float *ch, size_t cl, float ratio, uint64_t *state, float *t);

/* ---- sum-and-scale: out[i] = (((in0+in1)+in2)+...)/divisor ------------------
 * The f32-wire ring's per-chunk arithmetic (worker_ring.rs:141-143 then
 * param_manager.rs:183-188); divisor == 1 leaves the sum unscaled.          */
void ono_ref_sum_scale(float *out, const float *const *ins, int k, size_t n, float divisor);

/* ---- ParamManager: param_manager.rs:183-197 -------------------------------- */
void ono_ref_normalize(float *g, size_t n, size_t nworkers);       /* g /= n if n > 1 */
void ono_ref_acc_residual(float *res, const float *g, size_t n);   /* res += g       */

/* ---- optimizers: machine_learning/src/optimization/ (gd, momentum, adam) --------------------- */
enum { ONO_REF_OPT_GD = 0, ONO_REF_OPT_MOMENTUM = 1, ONO_REF_OPT_ADAM = 2, ONO_REF_OPT_ADD = 3 };
typedef struct {
    int kind;
    float lr, momentum, beta1, beta2, eps;
    float beta1_t, beta2_t; /* Adam running powers, start at 1 (adam.rs:39-40) */
    float *v, *s;           /* velocity / first moment, second moment */
    size_t len;
} ono_ref_opt;
int ono_ref_opt_init(ono_ref_opt *o, int kind, size_t len, float lr, float momentum,
                     float beta1, float beta2, float eps);
void ono_ref_opt_free(ono_ref_opt *o);
void ono_ref_opt_update(ono_ref_opt *o, const float *grad, float *params, size_t n);

/* ---- BlockingStore: parameter_server/src/storage/blocking/{store,shard}.rs -- */
typedef struct ono_ref_store ono_ref_store;
ono_ref_store *ono_ref_store_new(const float *init_params, size_t nparams, size_t shard_size,
                                 size_t nworkers, int opt_kind, float lr, float momentum,
                                 float beta1, float beta2, float eps);
void ono_ref_store_free(ono_ref_store *s);
int ono_ref_store_accumulate(ono_ref_store *s, const float *grad, size_t n); /* 0 ok, 1 size */
void ono_ref_store_update_params(ono_ref_store *s);
int ono_ref_store_pull_params(ono_ref_store *s, float *out, size_t n);
int ono_ref_store_active_idx(const ono_ref_store *s);
void ono_ref_store_set_updating(ono_ref_store *s, int updating);
size_t ono_ref_store_nshards(const ono_ref_store *s);

/* WildStore (wild/store.rs:77-91): optimizer applied per incoming gradient. */
typedef struct ono_ref_wild ono_ref_wild;
ono_ref_wild *ono_ref_wild_new(const float *init_params, size_t nparams, size_t shard_size,
                               int opt_kind, float lr, float momentum, float beta1,
                               float beta2, float eps);
void ono_ref_wild_free(ono_ref_wild *w);
int ono_ref_wild_accumulate(ono_ref_wild *w, const float *grad, size_t n);
int ono_ref_wild_pull_params(ono_ref_wild *w, float *out, size_t n);

/* ---- sparse codec: comms/src/sparse/protocol.rs:33-144 ----------------------
 * Threshold is only rng-independent when len <= 16384 (the sample is then the
 * whole gradient); returns NaN for longer inputs (rand 0.9.4 StdRng needed).  */
float ono_ref_sparse_threshold_full(const float *g, size_t n, float r);
/* calculate_threshold over a drawn sample (protocol.rs:33-49): idx = m sample
 * indices (NULL: every value, m == n).  f32::abs, select_nth_unstable_by
 * total_cmp at k = (m as f32 * (1 - r)) as usize (<= m - 1), f32::max with
 * f16::MIN_POSITIVE.                                                          */
float ono_ref_sparse_threshold_sample(const float *g, size_t n, const uint32_t *idx, size_t m, float r);
/* The stand-in sampler (NOT rand 0.9.4): Floyd's algorithm over splitmix64 at
 * *state; the identity with no draws when m == len.  Restated independently
 * of the product's ono_sparse_sample_default, which must equal it.          */
void ono_ref_sample_default(uint64_t *state, size_t len, uint32_t *idx, size_t m);
size_t ono_ref_grad_drop(uint8_t *buf, const float *g, size_t n, float threshold);
int ono_ref_grad_lift(float *g, size_t cap, size_t *out_len, const uint8_t *buf, size_t nbytes);

/* ---- wire framing: comms/src/protocol/msg.rs:120-191, codec/sink.rs:37-58 ---
 * [u64 BE len][u32 BE kind][payload]; kind 1/2 = dense f16 grad (is_last).   */
size_t ono_ref_frame_dense(uint8_t *out, const uint16_t *h, size_t n, int is_last);

/* ---- synthetic gradients; bit-identical to the device and
 *      numpy generators: integer hashing + one exact int->float + one f32 mul. */
void ono_ref_synth(float *out, size_t n, uint64_t seed, uint64_t rank, size_t offset);

#ifdef __cplusplus
}
#endif
#endif
