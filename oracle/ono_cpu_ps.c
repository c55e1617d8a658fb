/*
 * ono_cpu_ps.c — CPU BASELINE HARNESS (TEST INFRASTRUCTURE ONLY).
 *
 * SURVEY §8(d) CPU-baseline items (i) and (iii), restated from the reference:
 *   --mode hop : one scatter hop of the reference ring on one core —
 *                f16 encode of a chunk (compressor.rs:106-118), f16 decode into a
 *                handle-owned buffer (worker.rs:84-101), f32 add (worker_ring.rs:141-143)
 *   --mode ps  : BlockingStore accumulate (store.rs:84-91, shard.rs:56-68) of
 *                `workers` gradients + update_params (÷nworkers + GD, shard.rs:74-92),
 *                parallel over shards = 2 x threads (service/builder.rs:164-173) on
 *                `threads` pinned cores, the reference's rayon par_iter restated
 *                with pthreads.
 * prints one JSON line.
 */
#include "ono_oracle.h"

#include <pthread.h>
#include <sched.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

static double now(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

typedef struct {
    int id, nthreads;
    size_t n, shard;
    float *acc, *params;
    const float *grad;
    int phase; /* 0 accumulate, 1 update */
    float nworkers, lr;
} job_t;

static pthread_barrier_t g_start, g_done;
static volatile int g_quit;

static void *worker(void *arg) {
    job_t *j = (job_t *)arg;
    cpu_set_t cs;
    CPU_ZERO(&cs);
    CPU_SET(j->id % (int)sysconf(_SC_NPROCESSORS_ONLN), &cs);
    pthread_setaffinity_np(pthread_self(), sizeof cs, &cs);
    for (;;) {
        pthread_barrier_wait(&g_start);
        if (g_quit) break;
        size_t nsh = (j->n + j->shard - 1) / j->shard;
        for (size_t s = (size_t)j->id; s < nsh; s += (size_t)j->nthreads) { /* shard-parallel like par_iter */
            size_t lo = s * j->shard, hi = lo + j->shard > j->n ? j->n : lo + j->shard;
            float *a = j->acc + lo;
            if (j->phase == 0) {
                const float *g = j->grad + lo;
                for (size_t i = 0; i < hi - lo; i++) a[i] += g[i];
            } else {
                float *w = j->params + lo;
                for (size_t i = 0; i < hi - lo; i++) a[i] /= j->nworkers;
                for (size_t i = 0; i < hi - lo; i++) w[i] -= j->lr * a[i];
                memset(a, 0, (hi - lo) * sizeof(float));
            }
        }
        pthread_barrier_wait(&g_done);
    }
    return NULL;
}

int main(int argc, char **argv) {
    const char *mode = "hop";
    size_t n = (size_t)1 << 24;
    int threads = 16, workers = 2, rounds = 3;
    for (int a = 1; a < argc; a++) {
        if (!strcmp(argv[a], "--mode") && a + 1 < argc) mode = argv[++a];
        else if (!strcmp(argv[a], "--len") && a + 1 < argc) n = (size_t)strtoull(argv[++a], 0, 10);
        else if (!strcmp(argv[a], "--threads") && a + 1 < argc) threads = atoi(argv[++a]);
        else if (!strcmp(argv[a], "--workers") && a + 1 < argc) workers = atoi(argv[++a]);
        else if (!strcmp(argv[a], "--rounds") && a + 1 < argc) rounds = atoi(argv[++a]);
        else { fprintf(stderr, "bad arg %s\n", argv[a]); return 1; }
    }
    if (!strcmp(mode, "hop")) {
        float *chunk = malloc(n * 4), *acc = malloc(n * 4), *dec = malloc(n * 4);
        uint16_t *wire = malloc(n * 2);
        ono_ref_synth(chunk, n, 1, 0, 0);
        ono_ref_synth(acc, n, 2, 1, 0);
        double best = 1e30;
        for (int r = 0; r < rounds; r++) {
            double t0 = now();
            ono_ref_f16_encode(wire, chunk, n);         /* sender: compress_dense_grad */
            ono_ref_f16_decode(dec, wire, n);           /* receiver: recv_event decode */
            for (size_t i = 0; i < n; i++) acc[i] += dec[i]; /* chunks[i] += g */
            double t = now() - t0;
            if (t < best) best = t;
        }
        printf("{\"mode\": \"hop\", \"len\": %zu, \"threads\": 1, \"s_per_hop\": %.6f, \"gib_s\": %.4f}\n", n, best,
               n * 4.0 / best / (double)(1u << 30));
        return 0;
    }
    /* ps */
    size_t nsh = (size_t)threads * 2; /* shards = 2 x cores */
    if (nsh > n) nsh = n;
    size_t shard = (n + nsh - 1) / nsh;
    float *acc = calloc(n, 4), *params = malloc(n * 4);
    float **grads = malloc(sizeof(float *) * (size_t)workers);
    ono_ref_synth(params, n, 3, 9, 0);
    for (int w = 0; w < workers; w++) {
        grads[w] = malloc(n * 4);
        ono_ref_synth(grads[w], n, 4, (uint64_t)w, 0);
    }
    pthread_barrier_init(&g_start, NULL, (unsigned)threads + 1);
    pthread_barrier_init(&g_done, NULL, (unsigned)threads + 1);
    job_t *jobs = calloc((size_t)threads, sizeof(job_t));
    pthread_t *th = calloc((size_t)threads, sizeof(pthread_t));
    for (int t = 0; t < threads; t++) {
        jobs[t] = (job_t){t, threads, n, shard, acc, params, NULL, 0, (float)workers, 0.1f};
        pthread_create(&th[t], NULL, worker, &jobs[t]);
    }
    double best = 1e30;
    for (int r = 0; r < rounds; r++) {
        double t0 = now();
        for (int w = 0; w < workers; w++) {  /* one accumulate per worker, then the leader's update */
            for (int t = 0; t < threads; t++) { jobs[t].grad = grads[w]; jobs[t].phase = 0; }
            pthread_barrier_wait(&g_start);
            pthread_barrier_wait(&g_done);
        }
        for (int t = 0; t < threads; t++) jobs[t].phase = 1;
        pthread_barrier_wait(&g_start);
        pthread_barrier_wait(&g_done);
        double t = now() - t0;
        if (t < best) best = t;
    }
    g_quit = 1;
    pthread_barrier_wait(&g_start);
    for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
    printf("{\"mode\": \"ps\", \"len\": %zu, \"threads\": %d, \"workers\": %d, \"shards\": %zu, "
           "\"s_per_round\": %.6f, \"gib_s\": %.4f}\n",
           n, threads, workers, nsh, best, (double)workers * n * 4.0 / best / (double)(1u << 30));
    return 0;
}
