/*
 * ono_oracle.c — CPU ORACLE (TEST INFRASTRUCTURE ONLY; see ono_oracle.h).
 *
 * Plain scalar C, compiled with -ffp-contract=off so every f32 operation is
 * one IEEE-754 rounding, exactly as rustc emits for the reference (Rust never
 * contracts a*b+c into an FMA).  Each function cites the reference lines it
 * restates.  Nothing in here is used by the product library.
 */
#include "ono_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

static inline uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
static inline uint32_t f2u(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static inline float u2f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }

/* ------------------------------------------------------------------------- */
/* f16: `half` 2.7.1 f32_to_f16 / f16_to_f32 (IEEE binary16, round to nearest
 * even; NaN keeps its top payload bits and gets the quiet bit 0x0200).
 * Reference call sites: compressor.rs:116, worker.rs:94, protocol.rs:77,136. */
uint16_t ono_ref_f32_to_f16(float value) {
    uint32_t x = f2u(value);
    uint32_t sign = x & 0x80000000u, exp = x & 0x7F800000u, man = x & 0x007FFFFFu;
    if (exp == 0x7F800000u) {
        uint32_t nan_bit = man == 0 ? 0u : 0x0200u;
        return (uint16_t)((sign >> 16) | 0x7C00u | nan_bit | (man >> 13));
    }
    uint32_t half_sign = sign >> 16;
    int32_t half_exp = (int32_t)(exp >> 23) - 127 + 15;
    if (half_exp >= 0x1F) return (uint16_t)(half_sign | 0x7C00u);
    if (half_exp <= 0) {
        if (14 - half_exp > 24) return (uint16_t)half_sign;
        uint32_t m = man | 0x00800000u;
        uint32_t half_man = m >> (14 - half_exp);
        uint32_t round_bit = 1u << (13 - half_exp);
        /* round up iff round bit set and (sticky bits or result lsb) set */
        if ((m & round_bit) != 0 && (m & (3u * round_bit - 1u)) != 0) half_man += 1;
        return (uint16_t)(half_sign | half_man);
    }
    uint32_t half_exp_bits = (uint32_t)half_exp << 10;
    uint32_t half_man = man >> 13;
    uint32_t round_bit = 0x00001000u;
    uint32_t r = half_sign | half_exp_bits | half_man;
    if ((man & round_bit) != 0 && (man & (3u * round_bit - 1u)) != 0) r += 1; /* may carry into exp */
    return (uint16_t)r;
}

float ono_ref_f16_to_f32(uint16_t h) {
    uint32_t sign = (uint32_t)(h & 0x8000u) << 16;
    uint32_t e = h & 0x7C00u, m = h & 0x03FFu;
    if ((h & 0x7FFFu) == 0) return u2f(sign);
    if (e == 0x7C00u) {
        if (m == 0) return u2f(sign | 0x7F800000u);
        return u2f(sign | 0x7FC00000u | (m << 13));
    }
    if (e == 0) { /* subnormal: m * 2^-24, exact in f32 */
        float v = (float)m * 5.9604644775390625e-08f;
        return sign ? -v : v;
    }
    return u2f(sign | ((((e >> 10) - 15u + 127u) & 0xFFu) << 23) | (m << 13));
}

void ono_ref_f16_encode(uint16_t *out, const float *in, size_t n) {
    for (size_t i = 0; i < n; i++) out[i] = ono_ref_f32_to_f16(in[i]);
}
void ono_ref_f16_decode(float *out, const uint16_t *in, size_t n) {
    for (size_t i = 0; i < n; i++) out[i] = ono_ref_f16_to_f32(in[i]);
}

/* ------------------------------------------------------------------------- */
/* SplitChunks (worker/src/middlewares/mod.rs:15-59): len/n each, the first
 * len%n chunks one longer; iteration stops once the slice is empty.          */
size_t ono_ref_split_chunks(size_t len, size_t n, size_t *offsets) {
    size_t base = len / n, rem = len % n, pos = 0, k = 0;
    offsets[0] = 0;
    while (pos < len && k < n) {
        size_t l = base + (rem > 0 ? 1 : 0);
        if (rem > 0) rem--;
        pos += l;
        offsets[++k] = pos;
    }
    return k;
}

/* ------------------------------------------------------------------------- */
/* One pull_grads() round for every rank (worker_ring.rs:82-204), lockstep.
 * At scatter step s rank r pushes chunk i_r (f16-compressed, :122), zeroes it
 * (:133), receives prev's push into chunk i_r-1 (:140-143).  Gather copies
 * the owned chunk residual->grad (:166), forwards chunks, zeroes the owned
 * residual at j == 0 (:191-193), copies each received chunk (:200).  Then
 * grad /= n for n > 1 (:101-105, param_manager.rs:183-188).                  */
int ono_ref_ring_pull_grads(float *const *residual, float *const *grad, int n, size_t len,
                            int wire) {
    if (n <= 0) return -1;
    size_t *off = (size_t *)malloc(sizeof(size_t) * ((size_t)n + 1));
    size_t nch = ono_ref_split_chunks(len, (size_t)n, off);
    if (nch < (size_t)n) { free(off); return -1; } /* reference: chunks[pos] out of bounds */
    size_t maxc = off[1] - off[0];
    uint16_t *m16 = (uint16_t *)malloc(sizeof(uint16_t) * (size_t)n * (maxc ? maxc : 1));
    float *m32 = (float *)malloc(sizeof(float) * (size_t)n * (maxc ? maxc : 1));
    size_t *mlen = (size_t *)malloc(sizeof(size_t) * (size_t)n);
    int *idx = (int *)malloc(sizeof(int) * (size_t)n);

    /* scatter (reduce-scatter), worker_ring.rs:112-147 */
    for (int r = 0; r < n; r++) idx[r] = r;
    for (int s = 0; s < n - 1; s++) {
        for (int r = 0; r < n; r++) {
            int c = idx[r];
            float *ch = residual[r] + off[c];
            size_t cl = off[c + 1] - off[c];
            if (wire == 0) ono_ref_f16_encode(m16 + (size_t)r * maxc, ch, cl);
            else memcpy(m32 + (size_t)r * maxc, ch, cl * sizeof(float));
            mlen[r] = cl;
            memset(ch, 0, cl * sizeof(float)); /* dense: chunks[i].fill(0.0) */
        }
        for (int r = 0; r < n; r++) {
            int p = (r + n - 1) % n;
            idx[r] = (idx[r] + n - 1) % n;
            int c = idx[r];
            float *ch = residual[r] + off[c];
            size_t cl = off[c + 1] - off[c];
            size_t k = cl < mlen[p] ? cl : mlen[p]; /* zip() stops at the shorter */
            for (size_t i = 0; i < k; i++) {
                float g = wire == 0 ? ono_ref_f16_to_f32(m16[(size_t)p * maxc + i])
                                    : m32[(size_t)p * maxc + i];
                ch[i] += g;
            }
        }
    }

    /* gather (all-gather), worker_ring.rs:155-204 */
    for (int r = 0; r < n; r++) {
        idx[r] = (r + 1) % n;
        int c = idx[r];
        memcpy(grad[r] + off[c], residual[r] + off[c], (off[c + 1] - off[c]) * sizeof(float));
    }
    if (n == 1) {
        memset(residual[0] + off[idx[0]], 0, (off[idx[0] + 1] - off[idx[0]]) * sizeof(float));
    } else {
        for (int j = 0; j < n - 1; j++) {
            for (int r = 0; r < n; r++) {
                int c = idx[r];
                size_t cl = off[c + 1] - off[c];
                if (wire == 0) ono_ref_f16_encode(m16 + (size_t)r * maxc, grad[r] + off[c], cl);
                else memcpy(m32 + (size_t)r * maxc, grad[r] + off[c], cl * sizeof(float));
                mlen[r] = cl;
                if (j == 0) memset(residual[r] + off[c], 0, cl * sizeof(float));
            }
            for (int r = 0; r < n; r++) {
                int p = (r + n - 1) % n;
                idx[r] = (idx[r] + n - 1) % n;
                int c = idx[r];
                size_t cl = off[c + 1] - off[c];
                /* copy_from_slice panics on a length mismatch; never happens here */
                for (size_t i = 0; i < cl && i < mlen[p]; i++)
                    grad[r][off[c] + i] = wire == 0 ? ono_ref_f16_to_f32(m16[(size_t)p * maxc + i])
                                                    : m32[(size_t)p * maxc + i];
            }
        }
        for (int r = 0; r < n; r++) ono_ref_normalize(grad[r], len, (size_t)n);
    }
    free(off); free(m16); free(m32); free(mlen); free(idx);
    return 0;
}

/* Bytes grad_drop_into writes for `ch` at threshold t (protocol.rs:57-86):
 * the u64 total, then per run of |g| >= t an offset, a length and 2 B per value. */
static size_t drop_bytes(const float *ch, size_t cl, float t) {
    size_t nb = 8, i = 0;
    while (i < cl) {
        if (fabsf(ch[i]) >= t) {
            size_t s = i;
            while (i < cl && fabsf(ch[i]) >= t) i++;
            nb += 8 + 2 * (i - s);
        } else {
            i++;
        }
    }
    return nb;
}

/* One push_grad of chunk ch by a worker with serializer `ratio` (0 = Base),
 * handles/worker.rs:157-174 over Compressor::compress (compressor.rs:71-98):
 *   Base:            DenseGrad f16(ch)                              -> None
 *   SparseCapable:   t = calculate_threshold(ch, r) (the sampler state
 *                    advances whatever is sent); grad_drop_into(ch, t); if the
 *                    stream is no longer than the f16 payload, len * 2 bytes
 *                    (:79), a SparseGrad                            -> Some(t)
 *                    else the DenseGrad of f16(ch) (:84-89)         -> None
 * msg = the values the receiver's recv_event hands the ring: the decoded f16
 * payload, or the lift into a zero-filled buffer (worker.rs:84-108).
 * Returns 1 when the push was sparse (Some(t)), 0 when dense (None).        */
static int push_chunk(const float *ch, size_t cl, float ratio, uint64_t *state, float *msg, float *t) {
    *t = 0.0f;
    if (ratio > 0.0f) {
        const size_t m = cl < 16384 ? cl : 16384;
        uint32_t *idx = NULL;
        if (cl > 16384) {
            idx = (uint32_t *)malloc(m * sizeof(uint32_t));
            ono_ref_sample_default(state, cl, idx, m);
        }
        *t = ono_ref_sparse_threshold_sample(ch, cl, idx, m, ratio);
        free(idx);
        if (drop_bytes(ch, cl, *t) <= cl * 2) { /* compressor.rs:79 */
            for (size_t i = 0; i < cl; i++)
                msg[i] = fabsf(ch[i]) >= *t ? ono_ref_f16_to_f32(ono_ref_f32_to_f16(ch[i])) : 0.0f;
            return 1;
        }
    }
    for (size_t i = 0; i < cl; i++) msg[i] = ono_ref_f16_to_f32(ono_ref_f32_to_f16(ch[i]));
    return 0;
}

int ono_ref_sparse_push_is_sparse(const float *ch, size_t cl, float ratio, uint64_t *state, float *t) {
    float *msg = (float *)malloc(sizeof(float) * (cl ? cl : 1));
    int sp = push_chunk(ch, cl, ratio, state, msg, t);
    free(msg);
    return sp;
}

int ono_ref_ring_pull_grads_sparse(float *const *residual, float *const *grad, int n, size_t len,
                                   const float *ratio, uint64_t *state) {
    if (n <= 0) return -1;
    size_t *off = (size_t *)malloc(sizeof(size_t) * ((size_t)n + 1));
    size_t nch = ono_ref_split_chunks(len, (size_t)n, off);
    if (nch < (size_t)n) { free(off); return -1; }
    size_t maxc = off[1] - off[0];
    float *msg = (float *)malloc(sizeof(float) * (size_t)n * (maxc ? maxc : 1));
    float *thr = (float *)malloc(sizeof(float) * (size_t)n);
    int *idx = (int *)malloc(sizeof(int) * (size_t)n);
    /* scatter (worker_ring.rs:112-147) */
    for (int r = 0; r < n; r++) idx[r] = r;
    for (int s = 0; s < n - 1; s++) {
        for (int r = 0; r < n; r++) {
            int c = idx[r];
            float *ch = residual[r] + off[c];
            size_t cl = off[c + 1] - off[c];
            if (push_chunk(ch, cl, ratio[r], &state[r], msg + (size_t)r * maxc, &thr[r])) {
                for (size_t i = 0; i < cl; i++) if (fabsf(ch[i]) >= thr[r]) ch[i] = 0.0f; /* :126-132 */
            } else {
                memset(ch, 0, cl * sizeof(float)); /* :133 */
            }
        }
        for (int r = 0; r < n; r++) {
            int p = (r + n - 1) % n;
            idx[r] = (idx[r] + n - 1) % n;
            int c = idx[r];
            float *ch = residual[r] + off[c];
            size_t cl = off[c + 1] - off[c];
            for (size_t i = 0; i < cl; i++) ch[i] += msg[(size_t)p * maxc + i]; /* :140-143 */
        }
    }
    /* gather (worker_ring.rs:155-204) */
    for (int r = 0; r < n; r++) {
        idx[r] = (r + 1) % n;
        int c = idx[r];
        memcpy(grad[r] + off[c], residual[r] + off[c], (off[c + 1] - off[c]) * sizeof(float)); /* :166 */
    }
    if (n == 1) {
        memset(residual[0] + off[idx[0]], 0, (off[idx[0] + 1] - off[idx[0]]) * sizeof(float)); /* :168-171 */
    } else {
        for (int j = 0; j < n - 1; j++) {
            for (int r = 0; r < n; r++) {
                int c = idx[r];
                float *ch = grad[r] + off[c];
                size_t cl = off[c + 1] - off[c];
                if (push_chunk(ch, cl, ratio[r], &state[r], msg + (size_t)r * maxc, &thr[r])) {
                    /* :177-190 — the owned residual is NOT reset (the zeroing is
                     * commented out at :178-184): it keeps the reduced sum */
                    for (size_t i = 0; i < cl; i++) if (fabsf(ch[i]) < thr[r]) ch[i] = 0.0f;
                } else if (j == 0) {
                    memset(residual[r] + off[c], 0, cl * sizeof(float)); /* :191-193 */
                }
            }
            for (int r = 0; r < n; r++) {
                int p = (r + n - 1) % n;
                idx[r] = (idx[r] + n - 1) % n;
                int c = idx[r];
                memcpy(grad[r] + off[c], msg + (size_t)p * maxc, (off[c + 1] - off[c]) * sizeof(float)); /* :199-200 */
            }
        }
        for (int r = 0; r < n; r++) ono_ref_normalize(grad[r], len, (size_t)n); /* :101-105 */
    }
    free(off); free(msg); free(thr); free(idx);
    return 0;
}

void ono_ref_sum_scale(float *out, const float *const *ins, int k, size_t n, float divisor) {
    for (size_t i = 0; i < n; i++) {
        float acc = ins[0][i];
        for (int j = 1; j < k; j++) acc += ins[j][i];
        out[i] = divisor != 1.0f ? acc / divisor : acc;
    }
}

/* param_manager.rs:183-188: factor = n as f32; g /= factor (only called n > 1) */
void ono_ref_normalize(float *g, size_t n, size_t nworkers) {
    if (nworkers <= 1) return;
    float f = (float)nworkers;
    for (size_t i = 0; i < n; i++) g[i] /= f;
}

/* param_manager.rs:191-197 */
void ono_ref_acc_residual(float *res, const float *g, size_t n) {
    for (size_t i = 0; i < n; i++) res[i] += g[i];
}

/* ------------------------------------------------------------------------- */
int ono_ref_opt_init(ono_ref_opt *o, int kind, size_t len, float lr, float momentum,
                     float beta1, float beta2, float eps) {
    memset(o, 0, sizeof(*o));
    o->kind = kind; o->lr = lr; o->momentum = momentum;
    o->beta1 = beta1; o->beta2 = beta2; o->eps = eps;
    o->beta1_t = 1.0f; o->beta2_t = 1.0f; o->len = len;
    if (kind == ONO_REF_OPT_MOMENTUM || kind == ONO_REF_OPT_ADAM)
        o->v = (float *)calloc(len ? len : 1, sizeof(float));
    if (kind == ONO_REF_OPT_ADAM) o->s = (float *)calloc(len ? len : 1, sizeof(float));
    return 0;
}
void ono_ref_opt_free(ono_ref_opt *o) { free(o->v); free(o->s); o->v = o->s = NULL; }

void ono_ref_opt_update(ono_ref_opt *o, const float *g, float *w, size_t n) {
    switch (o->kind) {
    case ONO_REF_OPT_GD: /* gradient_descent.rs:44-47: w -= lr * g */
        for (size_t i = 0; i < n; i++) w[i] -= o->lr * g[i];
        break;
    case ONO_REF_OPT_MOMENTUM: /* gradient_descent_with_momentum.rs:56-62 */
        for (size_t i = 0; i < n; i++) {
            o->v[i] = (o->momentum * o->v[i]) + g[i];
            w[i] -= o->lr * o->v[i];
        }
        break;
    case ONO_REF_OPT_ADAM: { /* adam.rs:76-91 */
        o->beta1_t *= o->beta1;
        o->beta2_t *= o->beta2;
        float bc1 = 1.0f - o->beta1_t, bc2 = 1.0f - o->beta2_t;
        float step = o->lr * (sqrtf(bc2) / bc1);
        for (size_t i = 0; i < n; i++) {
            o->v[i] = o->beta1 * o->v[i] + (1.0f - o->beta1) * g[i];
            o->s[i] = o->beta2 * o->s[i] + (1.0f - o->beta2) * (g[i] * g[i]);
            w[i] -= step * o->v[i] / (sqrtf(o->s[i]) + o->eps);
        }
        break;
    }
    case ONO_REF_OPT_ADD: /* the AddOptimizer of blocking/shard.rs:117-128 tests */
        for (size_t i = 0; i < n; i++) w[i] += g[i];
        break;
    }
}

/* ------------------------------------------------------------------------- */
/* BlockingStore / BlockingShard (blocking/store.rs:49-124, shard.rs:56-109). */
struct ono_ref_store {
    size_t nparams, shard_size, nshards, nworkers;
    int active_idx, updating;
    float *grads[2];
    float *params;
    ono_ref_opt *opts; /* one per shard (optimizer_factory(params.len())) */
};

ono_ref_store *ono_ref_store_new(const float *init, size_t nparams, size_t shard_size,
                                 size_t nworkers, int kind, float lr, float momentum,
                                 float beta1, float beta2, float eps) {
    if (shard_size == 0) return NULL;
    ono_ref_store *s = (ono_ref_store *)calloc(1, sizeof(*s));
    s->nparams = nparams; s->shard_size = shard_size; s->nworkers = nworkers ? nworkers : 1;
    s->nshards = (nparams + shard_size - 1) / shard_size;
    s->grads[0] = (float *)calloc(nparams ? nparams : 1, sizeof(float));
    s->grads[1] = (float *)calloc(nparams ? nparams : 1, sizeof(float));
    s->params = (float *)malloc(sizeof(float) * (nparams ? nparams : 1));
    memcpy(s->params, init, nparams * sizeof(float));
    s->opts = (ono_ref_opt *)calloc(s->nshards ? s->nshards : 1, sizeof(ono_ref_opt));
    for (size_t k = 0; k < s->nshards; k++) {
        size_t lo = k * shard_size, hi = lo + shard_size > nparams ? nparams : lo + shard_size;
        ono_ref_opt_init(&s->opts[k], kind, hi - lo, lr, momentum, beta1, beta2, eps);
    }
    return s;
}
void ono_ref_store_free(ono_ref_store *s) {
    if (!s) return;
    for (size_t k = 0; k < s->nshards; k++) ono_ref_opt_free(&s->opts[k]);
    free(s->opts); free(s->grads[0]); free(s->grads[1]); free(s->params); free(s);
}
/* store.rs:84-91 + shard.rs:56-68: acc[active] += g (per shard, under its mutex) */
int ono_ref_store_accumulate(ono_ref_store *s, const float *g, size_t n) {
    if (n != s->nparams) return 1;
    float *acc = s->grads[s->active_idx];
    for (size_t i = 0; i < n; i++) acc[i] += g[i];
    return 0;
}
/* store.rs:93-108 + shard.rs:74-92: CAS `updating`, flip the active buffer,
 * then per shard g /= nworkers (if > 1), optimizer step, g.fill(0).          */
void ono_ref_store_update_params(ono_ref_store *s) {
    if (s->updating) return;
    s->updating = 1;
    int frozen = s->active_idx;
    s->active_idx ^= 1;
    for (size_t k = 0; k < s->nshards; k++) {
        size_t lo = k * s->shard_size;
        size_t hi = lo + s->shard_size > s->nparams ? s->nparams : lo + s->shard_size;
        float *g = s->grads[frozen] + lo;
        if (s->nworkers > 1) {
            float f = (float)s->nworkers;
            for (size_t i = 0; i < hi - lo; i++) g[i] /= f;
        }
        ono_ref_opt_update(&s->opts[k], g, s->params + lo, hi - lo);
        memset(g, 0, (hi - lo) * sizeof(float));
    }
    s->updating = 0;
}
int ono_ref_store_pull_params(ono_ref_store *s, float *out, size_t n) {
    if (n != s->nparams) return 1;
    memcpy(out, s->params, n * sizeof(float));
    return 0;
}
int ono_ref_store_active_idx(const ono_ref_store *s) { return s->active_idx; }
void ono_ref_store_set_updating(ono_ref_store *s, int u) { s->updating = u; }
size_t ono_ref_store_nshards(const ono_ref_store *s) { return s->nshards; }

/* WildStore (wild/store.rs:77-91, wild/shard.rs:43-58) */
struct ono_ref_wild {
    size_t nparams, shard_size, nshards;
    float *params;
    ono_ref_opt *opts;
};
ono_ref_wild *ono_ref_wild_new(const float *init, size_t nparams, size_t shard_size, int kind,
                               float lr, float momentum, float beta1, float beta2, float eps) {
    if (shard_size == 0) return NULL;
    ono_ref_wild *w = (ono_ref_wild *)calloc(1, sizeof(*w));
    w->nparams = nparams; w->shard_size = shard_size;
    w->nshards = (nparams + shard_size - 1) / shard_size;
    w->params = (float *)malloc(sizeof(float) * (nparams ? nparams : 1));
    memcpy(w->params, init, nparams * sizeof(float));
    w->opts = (ono_ref_opt *)calloc(w->nshards ? w->nshards : 1, sizeof(ono_ref_opt));
    for (size_t k = 0; k < w->nshards; k++) {
        size_t lo = k * shard_size, hi = lo + shard_size > nparams ? nparams : lo + shard_size;
        ono_ref_opt_init(&w->opts[k], kind, hi - lo, lr, momentum, beta1, beta2, eps);
    }
    return w;
}
void ono_ref_wild_free(ono_ref_wild *w) {
    if (!w) return;
    for (size_t k = 0; k < w->nshards; k++) ono_ref_opt_free(&w->opts[k]);
    free(w->opts); free(w->params); free(w);
}
int ono_ref_wild_accumulate(ono_ref_wild *w, const float *g, size_t n) {
    if (n != w->nparams) return 1;
    for (size_t k = 0; k < w->nshards; k++) {
        size_t lo = k * w->shard_size;
        size_t hi = lo + w->shard_size > w->nparams ? w->nparams : lo + w->shard_size;
        ono_ref_opt_update(&w->opts[k], g + lo, w->params + lo, hi - lo);
    }
    return 0;
}
int ono_ref_wild_pull_params(ono_ref_wild *w, float *out, size_t n) {
    if (n != w->nparams) return 1;
    memcpy(out, w->params, n * sizeof(float));
    return 0;
}

/* ------------------------------------------------------------------------- */
/* sparse codec, comms/src/sparse/protocol.rs:33-144 */
static int cmp_total(const void *a, const void *b) {
    /* f32::total_cmp on non-negative values (abs) == unsigned bit order */
    uint32_t x = f2u(*(const float *)a), y = f2u(*(const float *)b);
    int32_t sx = (int32_t)x, sy = (int32_t)y;
    sx ^= (int32_t)((uint32_t)(sx >> 31) >> 1);
    sy ^= (int32_t)((uint32_t)(sy >> 31) >> 1);
    return sx < sy ? -1 : sx > sy;
}
float ono_ref_sparse_threshold_full(const float *g, size_t n, float r) {
    if (n == 0) return 0.0f;
    if (n > 16384) return NAN; /* sample drawn by rand 0.9.4 StdRng: not restated */
    float *s = (float *)malloc(n * sizeof(float));
    for (size_t i = 0; i < n; i++) s[i] = fabsf(g[i]);
    qsort(s, n, sizeof(float), cmp_total);
    float kf = (float)n * (1.0f - r);
    size_t k = kf <= 0.0f ? 0 : (size_t)kf; /* `as usize` saturates */
    if (k > n - 1) k = n - 1;
    float t = s[k];
    free(s);
    const float min_pos_f16 = 6.103515625e-05f; /* f16::MIN_POSITIVE */
    return t > min_pos_f16 ? t : min_pos_f16;   /* f32::max; NaN-free input */
}
static void put_le(uint8_t *b, uint64_t v, int bytes) {
    for (int i = 0; i < bytes; i++) b[i] = (uint8_t)(v >> (8 * i));
}
/* protocol.rs:33-49 over a sample: values |g[idx[i]]|, total_cmp order of the
 * non-negative bit patterns (qsort; the rank statistic does not depend on how
 * select_nth_unstable_by gets there), then the NaN-ignoring f32::max.        */
float ono_ref_sparse_threshold_sample(const float *g, size_t n, const uint32_t *idx, size_t m, float r) {
    if (n == 0 || m == 0) return 0.0f;
    float *s = (float *)malloc(m * sizeof(float));
    for (size_t i = 0; i < m; i++) s[i] = fabsf(g[idx ? idx[i] : i]);
    qsort(s, m, sizeof(float), cmp_total);
    float kf = (float)m * (1.0f - r);
    size_t k = kf <= 0.0f ? 0 : (size_t)kf; /* `as usize` saturates */
    if (k > m - 1) k = m - 1;
    float t = s[k];
    free(s);
    const float min_pos_f16 = 6.103515625e-05f;
    return t > min_pos_f16 ? t : min_pos_f16; /* f32::max ignores a NaN t */
}

static uint64_t sm_next(uint64_t *x) {
    *x += 0x9E3779B97F4A7C15ULL;
    return mix64(*x);
}
/* Floyd: for j in len-m .. len: t = draw % (j+1); take t, or j if t was taken */
void ono_ref_sample_default(uint64_t *state, size_t len, uint32_t *idx, size_t m) {
    if (m >= len) {
        for (size_t i = 0; i < len; i++) idx[i] = (uint32_t)i;
        return;
    }
    /* membership: open addressing over a power-of-two table */
    size_t cap = 1;
    while (cap < 4 * m) cap <<= 1;
    uint32_t *tab = (uint32_t *)malloc(cap * sizeof(uint32_t));
    memset(tab, 0xFF, cap * sizeof(uint32_t));
    size_t c = 0;
    for (size_t j = len - m; j < len; j++) {
        uint32_t t = (uint32_t)(sm_next(state) % (uint64_t)(j + 1));
        for (int pass = 0; pass < 2; pass++) {
            size_t h = (size_t)(mix64(t) & (cap - 1));
            while (tab[h] != 0xFFFFFFFFu && tab[h] != t) h = (h + 1) & (cap - 1);
            if (tab[h] == 0xFFFFFFFFu) { tab[h] = t; idx[c++] = t; break; }
            t = (uint32_t)j; /* taken: take j (never taken before) */
        }
    }
    free(tab);
}

size_t ono_ref_grad_drop(uint8_t *buf, const float *g, size_t n, float threshold) {
    size_t o = 0, last_end = 0, i = 0;
    put_le(buf + o, (uint64_t)n, 8); o += 8;
    while (i < n) {
        if (fabsf(g[i]) >= threshold) {
            size_t start = i;
            while (i < n && fabsf(g[i]) >= threshold) i++;
            put_le(buf + o, (uint64_t)(start - last_end), 4); o += 4;
            put_le(buf + o, (uint64_t)(i - start), 4); o += 4;
            for (size_t j = start; j < i; j++) { put_le(buf + o, ono_ref_f32_to_f16(g[j]), 2); o += 2; }
            last_end = i;
        } else {
            i++;
        }
    }
    return o;
}
int ono_ref_grad_lift(float *g, size_t cap, size_t *out_len, const uint8_t *buf, size_t nb) {
    if (nb < 8) return -1;
    uint64_t total = 0;
    for (int i = 0; i < 8; i++) total |= (uint64_t)buf[i] << (8 * i);
    if (total > cap) return -2;
    memset(g, 0, total * sizeof(float));
    *out_len = total;
    size_t gi = 0, bi = 8;
    while (bi < nb) {
        if (nb - bi < 4) return -3;
        uint32_t off = buf[bi] | buf[bi + 1] << 8 | buf[bi + 2] << 16 | (uint32_t)buf[bi + 3] << 24;
        gi += off; bi += 4;
        if (nb - bi < 4) return -4;
        uint32_t cl = buf[bi] | buf[bi + 1] << 8 | buf[bi + 2] << 16 | (uint32_t)buf[bi + 3] << 24;
        bi += 4;
        if (gi > total || total - gi < cl) return -5;
        for (uint32_t j = 0; j < cl; j++) {
            if (nb - bi < 2) return -6;
            g[gi + j] = ono_ref_f16_to_f32((uint16_t)(buf[bi] | buf[bi + 1] << 8));
            bi += 2;
        }
        gi += cl;
    }
    return 0;
}

/* [u64 BE len][u32 BE kind][f16 LE...] — msg.rs:136-149 + sink.rs:41-50 */
size_t ono_ref_frame_dense(uint8_t *out, const uint16_t *h, size_t n, int is_last) {
    uint64_t len = 4 + 2 * (uint64_t)n;
    for (int i = 0; i < 8; i++) out[i] = (uint8_t)(len >> (56 - 8 * i));
    uint32_t kind = 1u + (is_last ? 1u : 0u);
    for (int i = 0; i < 4; i++) out[8 + i] = (uint8_t)(kind >> (24 - 8 * i));
    for (size_t i = 0; i < n; i++) { out[12 + 2 * i] = (uint8_t)h[i]; out[13 + 2 * i] = (uint8_t)(h[i] >> 8); }
    return 12 + 2 * n;
}

/* ------------------------------------------------------------------------- */
/* Synthetic gradients.  Classes by (h1>>32)%100:
 *   0 -> signed zero, 1 -> f16-subnormal magnitude, 2 -> exact f16 rounding
 *   tie, else ≈N(0, 0.0098^2) from a 4-term Irwin-Hall sum.                   */
void ono_ref_synth(float *out, size_t n, uint64_t seed, uint64_t rank, size_t offset) {
    const uint64_t G = 0x9E3779B97F4A7C15ULL;
    uint64_t key = mix64(seed + G * (rank + 1));
    const float scale = 0x1.3c1a2ep-22f;
    for (size_t j = 0; j < n; j++) {
        uint64_t i = (uint64_t)(offset + j);
        uint64_t h1 = mix64(key + G * (i + 1));
        uint64_t h2 = mix64(h1 ^ 0xD1B54A32D192ED03ULL);
        uint32_t cls = (uint32_t)((h1 >> 32) % 100u);
        uint32_t sign = (uint32_t)(h2 >> 63);
        float x;
        if (cls == 0) {
            x = u2f(sign << 31);
        } else if (cls == 1) {
            uint32_t m = (uint32_t)((h2 >> 8) & 0x3FFFFu);
            x = (float)m * 0x1p-32f;
            if (sign) x = -x;
        } else if (cls == 2) {
            uint32_t e = (uint32_t)((h2 >> 8) % 13u); /* unbiased exponent e-10 in [-10, 2] */
            uint32_t m10 = (uint32_t)((h2 >> 16) & 0x3FFu);
            x = u2f((sign << 31) | ((e - 10u + 127u) << 23) | (m10 << 13) | 0x1000u);
        } else {
            int32_t s4 = (int32_t)(h2 & 0xFFFF) + (int32_t)((h2 >> 16) & 0xFFFF) +
                         (int32_t)((h2 >> 32) & 0xFFFF) + (int32_t)((h2 >> 48) & 0xFFFF);
            x = (float)(s4 - 131070) * scale;
        }
        out[j] = x;
    }
}
