/*
 * ono_cpu_ring.c — CPU BASELINE / ORACLE HARNESS (TEST INFRASTRUCTURE ONLY).
 *
 * The reference CPU ring all-reduce, restated in C and run the way the
 * reference deploys it: n worker threads, each pinned to ONE core (reference
 * docker/gen_compose.py:9, CPUS=1 per node), connected prev->self->next over
 * loopback TCP, speaking the reference wire format
 *   [u64 BE len][u32 BE kind=1][len-4 bytes of f16 LE]   (msg.rs:120-151, sink.rs:37-58)
 * Per round each worker runs pull_grads() (worker_ring.rs:82-204):
 *   scatter: encode chunk i to f16 (compressor.rs:106-118) and send it while
 *            receiving prev's frame (try_join!, :122-123); zero chunk i (:133);
 *            decode into a handle-owned f32 buffer (worker.rs:84-101); add it
 *            into chunk i-1 (:141-143)
 *   gather:  grad[own] = residual[own]; forward / copy f16 chunks; then /= n.
 * Timed region = the pull_grads() rounds only (residual refill is outside).
 *
 * Serializer: Base (dense f16, default) or, with --sparse R, SparseCapable{R}
 * (compressor.rs:71-98): every push computes t = calculate_threshold(chunk, R)
 * (protocol.rs:33-49; sample from ono_ref_sample_default at --sparse-seed above
 * 16384 values) and the grad_drop stream of the values with |g| >= t
 * (:57-86); the stream goes out as a SparseGrad frame (kind 3) when it is no
 * longer than 2 bytes per value (compressor.rs:79), else the chunk goes out as
 * a DenseGrad (:84-89).  The ring follows the push (worker_ring.rs:125-134,
 * 177-193): sparse -> the scatter zeroes only the sent values, the gather keeps
 * only the sent values in grad and leaves the owned residual alone; dense ->
 * the scatter zeroes the chunk, the gather zeroes the owned residual at j == 0.
 * Either serializer receives both kinds: a SparseGrad lifts into the
 * zero-filled decode buffer (handles/worker.rs:102-108).
 *
 * usage: ono_cpu_ring --ranks N --len L --rounds R [--seed S] [--check] [--no-pin]
 * prints one JSON line: {"ranks":..,"len":..,"rounds":..,"s_per_round":..,"gib_s":..,"check":..}
 *
 * single-worker mode (one reference-style worker of a ring whose other members
 * run elsewhere — e.g. MI355X workers on ono_ring_create_tcp):
 *   ono_cpu_ring --rank R --ranks N --len L --next-port P [--listen-port Q] [--rounds R]
 *                [--seed S] [--out FILE]
 * prints {"port": Q} once listening, then runs like one thread above (its input is
 * ono_ref_synth(seed, rank R, round 0) every round) and writes grad ++ residual
 * (f32, 2*L values) of the last round to FILE.
 */
#include "ono_oracle.h"

#include <arpa/inet.h>
#include <errno.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <pthread.h>
#include <sched.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/socket.h>
#include <time.h>
#include <unistd.h>
#include <math.h>

typedef struct {
    int rank, n, rounds, pin;
    size_t len;
    uint64_t seed;
    int listen_fd, port_next, timer;
    float ratio;        /* 0: Base serializer, else SparseCapable{ratio} */
    uint64_t state;     /* the default sampler's stream */
    float *residual, *pristine, *grad;
    double elapsed;
} worker_t;

static pthread_barrier_t g_bar;
static double g_t0, g_total;

static double now(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

/* send `out` and receive one frame into `in` concurrently (try_join!) */
static int xchg(int fd_next, int fd_prev, const uint8_t *out, size_t out_n, uint8_t *in,
                size_t in_cap, size_t *in_n) {
    size_t sent = 0, got = 0, need = 8;
    int have_len = 0;
    while (sent < out_n || got < need) {
        struct pollfd p[2];
        int np = 0, is = -1, ir = -1;
        if (sent < out_n) { p[np].fd = fd_next; p[np].events = POLLOUT; is = np++; }
        if (got < need) { p[np].fd = fd_prev; p[np].events = POLLIN; ir = np++; }
        if (poll(p, (nfds_t)np, 60000) <= 0) return -1;
        if (is >= 0 && (p[is].revents & (POLLOUT | POLLERR | POLLHUP))) {
            ssize_t k = send(fd_next, out + sent, out_n - sent, MSG_NOSIGNAL);
            if (k < 0 && errno != EAGAIN) return -2;
            if (k > 0) sent += (size_t)k;
        }
        if (ir >= 0 && (p[ir].revents & (POLLIN | POLLERR | POLLHUP))) {
            ssize_t k = recv(fd_prev, in + got, need - got, 0);
            if (k == 0) return -3;
            if (k < 0 && errno != EAGAIN) return -4;
            if (k > 0) got += (size_t)k;
            if (!have_len && got >= 8) {
                uint64_t l = 0;
                for (int i = 0; i < 8; i++) l = (l << 8) | in[i];
                if (8 + l > in_cap) return -5;
                need = 8 + (size_t)l;
                have_len = 1;
            }
        }
    }
    *in_n = got;
    return 0;
}

static int connect_to(int port) {
    int fd = socket(AF_INET, SOCK_STREAM, 0);
    struct sockaddr_in a = {0};
    a.sin_family = AF_INET;
    a.sin_port = htons((uint16_t)port);
    a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
    for (int tries = 0; tries < 30000; tries++) {  /* 30 s: peers may start late */
        if (connect(fd, (struct sockaddr *)&a, sizeof a) == 0) return fd;
        close(fd);
        fd = socket(AF_INET, SOCK_STREAM, 0);
        usleep(1000);
    }
    close(fd);
    return -1;
}

static void set_nb(int fd) {
    int one = 1;
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
    fcntl(fd, F_SETFL, fcntl(fd, F_GETFL) | O_NONBLOCK);
}


/* push_grad (handles/worker.rs:157-174): the frame of this worker's serializer
 * for chunk ch; *sparse = 1 when it is a SparseGrad (push_grad's Some(*t)),
 * 0 for a DenseGrad (None). */
static size_t push_frame(worker_t *w, const float *ch, size_t cl, uint16_t *comp, uint8_t *frame, uint32_t *sidx,
                         float *t, int *sparse) {
    *sparse = 0;
    if (w->ratio > 0.0f) {
        const size_t m = cl < 16384 ? cl : 16384;
        if (cl > 16384) ono_ref_sample_default(&w->state, cl, sidx, m);
        *t = ono_ref_sparse_threshold_sample(ch, cl, cl > 16384 ? sidx : NULL, m, w->ratio);
        size_t nb = ono_ref_grad_drop(frame + 12, ch, cl, *t);
        if (nb <= cl * 2) { /* compressor.rs:79 */
            uint64_t len = 4 + (uint64_t)nb;
            for (int q = 0; q < 8; q++) frame[q] = (uint8_t)(len >> (56 - 8 * q));
            frame[8] = 0; frame[9] = 0; frame[10] = 0; frame[11] = 3; /* SparseGrad, is_last = false */
            *sparse = 1;
            return 12 + nb;
        }
    }
    ono_ref_f16_encode(comp, ch, cl); /* compress_dense_grad, compressor.rs:106-118 */
    return ono_ref_frame_dense(frame, comp, cl, 0);
}

/* recv_event (handles/worker.rs:82-108): a DenseGrad decodes, a SparseGrad
 * lifts into the zero-filled buffer; returns the values it holds. */
static size_t recv_grad(const uint8_t *b, size_t got, float *dec, size_t cap) {
    const uint8_t kind = b[11];
    if (kind == 1 || kind == 2) {
        size_t m = (got - 12) / 2;
        ono_ref_f16_decode(dec, (const uint16_t *)(b + 12), m);
        return m;
    }
    if (kind == 3 || kind == 4) {
        size_t m = 0;
        if (ono_ref_grad_lift(dec, cap, &m, b + 12, got - 12)) { fprintf(stderr, "sparse lift failed\n"); exit(3); }
        return m;
    }
    fprintf(stderr, "invalid worker event (kind %u)\n", kind);
    exit(3);
}

static void *worker_main(void *arg) {
    worker_t *w = (worker_t *)arg;
    if (w->pin) {  /* the rank-th CPU this process may run on (a box's cpuset need not start at CPU 0) */
        cpu_set_t allowed, cs;
        CPU_ZERO(&cs);
        if (sched_getaffinity(0, sizeof allowed, &allowed) == 0 && CPU_COUNT(&allowed) > 0) {
            int k = w->rank % CPU_COUNT(&allowed), c = 0;
            for (; c < CPU_SETSIZE; c++)
                if (CPU_ISSET(c, &allowed) && k-- == 0) break;
            CPU_SET(c, &cs);
        } else {
            long nc = sysconf(_SC_NPROCESSORS_ONLN);
            CPU_SET(w->rank % (nc > 0 ? nc : 1), &cs);
        }
        if (pthread_setaffinity_np(pthread_self(), sizeof cs, &cs) != 0) w->pin = 0;  /* reported: not pinned */
    }
    int n = w->n;
    int fd_next = -1, fd_prev = -1;
    if (n > 1) {
        fd_next = connect_to(w->port_next);
        fd_prev = accept(w->listen_fd, NULL, NULL);
        if (fd_next < 0 || fd_prev < 0) { fprintf(stderr, "connect failed\n"); exit(2); }
        set_nb(fd_next);
        set_nb(fd_prev);
    }
    size_t *off = (size_t *)malloc(sizeof(size_t) * (size_t)(n + 1));
    ono_ref_split_chunks(w->len, (size_t)n, off);
    size_t maxc = off[1] - off[0];
    const size_t cap = 12 + 8 + 10 * ((maxc + 1) / 2) + 2 * maxc + 16;  /* a frame of either kind */
    uint16_t *comp = (uint16_t *)malloc(2 * maxc + 16);           /* compression_buf */
    uint8_t *frame = (uint8_t *)malloc(cap);
    uint32_t *inbuf = (uint32_t *)malloc(cap);                      /* 4-B aligned, source.rs */
    float *dec = (float *)malloc(sizeof(float) * (maxc + 4));      /* handle-owned Vec<f32> */
    uint32_t *sidx = (uint32_t *)malloc(sizeof(uint32_t) * 16384);

    for (int round = 0; round < w->rounds; round++) {
        memcpy(w->residual, w->pristine, w->len * sizeof(float));
        pthread_barrier_wait(&g_bar);
        if (w->timer) g_t0 = now();
        /* ---- scatter ---- */
        int i = w->rank;
        for (int s = 0; s < n - 1; s++) {
            size_t cl = off[i + 1] - off[i];
            float t = 0.0f;
            int sparse = 0;
            size_t fl = push_frame(w, w->residual + off[i], cl, comp, frame, sidx, &t, &sparse);
            size_t got = 0;
            if (xchg(fd_next, fd_prev, frame, fl, (uint8_t *)inbuf, cap, &got)) {
                fprintf(stderr, "xchg failed\n"); exit(3);
            }
            if (sparse) { /* worker_ring.rs:126-132 */
                for (size_t j = 0; j < cl; j++) if (fabsf(w->residual[off[i] + j]) >= t) w->residual[off[i] + j] = 0.0f;
            } else {      /* :133 */
                memset(w->residual + off[i], 0, cl * sizeof(float));
            }
            i = (i + n - 1) % n;
            size_t m = recv_grad((const uint8_t *)inbuf, got, dec, off[i + 1] - off[i]);
            float *ch = w->residual + off[i];
            size_t k = off[i + 1] - off[i] < m ? off[i + 1] - off[i] : m;
            for (size_t j = 0; j < k; j++) ch[j] += dec[j];
        }
        /* ---- gather ---- */
        i = (w->rank + 1) % n;
        memcpy(w->grad + off[i], w->residual + off[i], (off[i + 1] - off[i]) * sizeof(float));
        if (n == 1) {
            memset(w->residual + off[i], 0, (off[i + 1] - off[i]) * sizeof(float));
        } else {
            for (int j = 0; j < n - 1; j++) {
                size_t cl = off[i + 1] - off[i];
                float t = 0.0f;
                int sparse = 0;
                size_t fl = push_frame(w, w->grad + off[i], cl, comp, frame, sidx, &t, &sparse);
                size_t got = 0;
                if (xchg(fd_next, fd_prev, frame, fl, (uint8_t *)inbuf, cap, &got)) {
                    fprintf(stderr, "xchg failed\n"); exit(3);
                }
                if (sparse) { /* :177-190; the owned residual is not reset (:178-184 commented out) */
                    for (size_t q = 0; q < cl; q++) if (fabsf(w->grad[off[i] + q]) < t) w->grad[off[i] + q] = 0.0f;
                } else if (j == 0) { /* :191-193 */
                    memset(w->residual + off[i], 0, cl * sizeof(float));
                }
                i = (i + n - 1) % n;
                size_t m = recv_grad((const uint8_t *)inbuf, got, dec, off[i + 1] - off[i]);
                if (m != off[i + 1] - off[i]) { fprintf(stderr, "gather: chunk length mismatch\n"); exit(3); }
                memcpy(w->grad + off[i], dec, m * sizeof(float));
            }
            ono_ref_normalize(w->grad, w->len, (size_t)n);
        }
        pthread_barrier_wait(&g_bar);
        if (w->timer) g_total += now() - g_t0;
    }
    if (fd_next >= 0) close(fd_next);
    if (fd_prev >= 0) close(fd_prev);
    free(off); free(comp); free(frame); free(inbuf); free(dec); free(sidx);
    return NULL;
}

static int listen_on(int port, int *bound) {
    int fd = socket(AF_INET, SOCK_STREAM, 0);
    int one = 1;
    setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
    struct sockaddr_in a = {0};
    a.sin_family = AF_INET;
    a.sin_port = htons((uint16_t)port);
    a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
    if (bind(fd, (struct sockaddr *)&a, sizeof a) || listen(fd, 4)) return -1;
    socklen_t sl = sizeof a;
    getsockname(fd, (struct sockaddr *)&a, &sl);
    *bound = ntohs(a.sin_port);
    return fd;
}

/* one worker of a ring whose other members are other processes */
static int single_worker(int rank, int n, size_t len, int rounds, uint64_t seed, int listen_port,
                         int next_port, const char *out, float ratio, uint64_t sstate) {
    worker_t w = {0};
    int port = 0;
    w.listen_fd = listen_on(listen_port, &port);
    if (w.listen_fd < 0) { perror("bind"); return 2; }
    printf("{\"port\": %d}\n", port);
    fflush(stdout);
    w.rank = rank; w.n = n; w.rounds = rounds; w.pin = 0; w.timer = 1;
    w.len = len; w.seed = seed; w.port_next = next_port; w.ratio = ratio; w.state = sstate;
    w.residual = (float *)malloc(len * sizeof(float));
    w.pristine = (float *)malloc(len * sizeof(float));
    w.grad = (float *)calloc(len, sizeof(float));
    ono_ref_synth(w.pristine, len, seed, (uint64_t)rank, 0);
    pthread_barrier_init(&g_bar, NULL, 1);
    worker_main(&w);
    if (out) {
        FILE *f = fopen(out, "wb");
        if (!f || fwrite(w.grad, sizeof(float), len, f) != len ||
            fwrite(w.residual, sizeof(float), len, f) != len) { perror("out"); return 5; }
        fclose(f);
    }
    double spr = g_total / rounds;
    printf("{\"rank\": %d, \"ranks\": %d, \"len\": %zu, \"rounds\": %d, \"s_per_round\": %.9f}\n",
           rank, n, len, rounds, spr);
    close(w.listen_fd);
    free(w.residual); free(w.pristine); free(w.grad);
    return 0;
}

int main(int argc, char **argv) {
    int n = 2, rounds = 3, check = 0, pin = 1, rank = -1, listen_port = 0, next_port = -1;
    float ratio = 0.0f;
    uint64_t sstate = 0;
    size_t len = 109386;
    uint64_t seed = 0x0402026;
    const char *out = NULL;
    for (int a = 1; a < argc; a++) {
        if (!strcmp(argv[a], "--ranks") && a + 1 < argc) n = atoi(argv[++a]);
        else if (!strcmp(argv[a], "--rank") && a + 1 < argc) rank = atoi(argv[++a]);
        else if (!strcmp(argv[a], "--listen-port") && a + 1 < argc) listen_port = atoi(argv[++a]);
        else if (!strcmp(argv[a], "--next-port") && a + 1 < argc) next_port = atoi(argv[++a]);
        else if (!strcmp(argv[a], "--out") && a + 1 < argc) out = argv[++a];
        else if (!strcmp(argv[a], "--len") && a + 1 < argc) len = (size_t)strtoull(argv[++a], 0, 10);
        else if (!strcmp(argv[a], "--rounds") && a + 1 < argc) rounds = atoi(argv[++a]);
        else if (!strcmp(argv[a], "--seed") && a + 1 < argc) seed = strtoull(argv[++a], 0, 0);
        else if (!strcmp(argv[a], "--check")) check = 1;
        else if (!strcmp(argv[a], "--sparse") && a + 1 < argc) ratio = (float)atof(argv[++a]);
        else if (!strcmp(argv[a], "--sparse-seed") && a + 1 < argc) sstate = strtoull(argv[++a], 0, 0);
        else if (!strcmp(argv[a], "--no-pin")) pin = 0;
        else { fprintf(stderr, "bad arg %s\n", argv[a]); return 1; }
    }
    if (ratio < 0.0f || ratio > 1.0f) { fprintf(stderr, "--sparse takes a ratio in (0, 1]\n"); return 1; }
    if (n < 1 || len < (size_t)n || rounds < 1) { fprintf(stderr, "need len >= ranks >= 1\n"); return 1; }
    if (rank >= 0) {
        if (rank >= n || (n > 1 && next_port <= 0)) { fprintf(stderr, "need rank < ranks, --next-port\n"); return 1; }
        return single_worker(rank, n, len, rounds, seed, listen_port, next_port, out, ratio, sstate);
    }
    worker_t *w = (worker_t *)calloc((size_t)n, sizeof(worker_t));
    int *ports = (int *)calloc((size_t)n, sizeof(int));
    for (int r = 0; r < n; r++) {
        w[r].listen_fd = listen_on(0, &ports[r]);
        if (w[r].listen_fd < 0) { perror("bind"); return 2; }
    }
    for (int r = 0; r < n; r++) {
        w[r].rank = r; w[r].n = n; w[r].rounds = rounds; w[r].pin = pin; w[r].timer = r == 0;
        w[r].len = len; w[r].seed = seed; w[r].port_next = ports[(r + 1) % n];
        w[r].residual = (float *)malloc(len * sizeof(float));
        w[r].pristine = (float *)malloc(len * sizeof(float));
        w[r].grad = (float *)calloc(len, sizeof(float));
        ono_ref_synth(w[r].pristine, len, seed, (uint64_t)r, 0);
    }
    pthread_barrier_init(&g_bar, NULL, (unsigned)n);
    pthread_t *th = (pthread_t *)calloc((size_t)n, sizeof(pthread_t));
    for (int r = 0; r < n; r++) pthread_create(&th[r], NULL, worker_main, &w[r]);
    for (int r = 0; r < n; r++) pthread_join(th[r], NULL);

    int ok = -1;
    if (check) { /* compare against the in-memory lockstep oracle, bit for bit */
        float **res = (float **)calloc((size_t)n, sizeof(float *));
        float **gr = (float **)calloc((size_t)n, sizeof(float *));
        for (int r = 0; r < n; r++) {
            res[r] = (float *)malloc(len * sizeof(float));
            gr[r] = (float *)calloc(len, sizeof(float));
            memcpy(res[r], w[r].pristine, len * sizeof(float));
        }
        ono_ref_ring_pull_grads(res, gr, n, len, 0);
        ok = 1;
        for (int r = 0; r < n; r++) {
            if (memcmp(gr[r], w[r].grad, len * sizeof(float))) ok = 0;
            if (memcmp(res[r], w[r].residual, len * sizeof(float))) ok = 0;
            free(res[r]); free(gr[r]);
        }
        free(res); free(gr);
    }
    double spr = g_total / rounds;
    int pinned = 0;  /* workers whose thread really got its one core */
    for (int r = 0; r < n; r++) pinned += w[r].pin;
    printf("{\"ranks\": %d, \"len\": %zu, \"rounds\": %d, \"pinned\": %d, \"workers_pinned\": %d, "
           "\"s_per_round\": %.9f, \"gib_s\": %.6f, \"check\": %d}\n",
           n, len, rounds, pin, pinned, spr, (double)len * 4.0 / spr / (double)(1ull << 30), ok);
    return ok == 0 ? 4 : 0;
}
