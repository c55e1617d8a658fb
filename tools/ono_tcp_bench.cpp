// ono_tcp_bench.cpp — the TCP edge timed from a plain C++ host (no Python in
// the process), the way the reference's Rust workers would drive it: n worker
// threads on one GPU, each an ono_ring_create_tcp manager over loopback TCP
// connections set up as the reference does (accept prev, connect next), each
// round = refill the residual in HBM (untimed) -> barrier -> pull_grads ->
// barrier.  Prints one JSON line with the median round time.
//
// --sparse R: every worker uses the SparseCapable{R} serializer (ono_ring_set_sparse);
// the line then also carries rank 0's per-round phase split (ono_ring_timing_phases:
// kernels, socket exchange, sparse codec) and the codec's share of the round.
//
// --phases 0: no phase timing (rank 0's per-launch event pairs cost host time inside every round, and the
// peers wait for rank 0: the round time without them is the one to quote; the phase split needs them).
//
// --dump PATH: rank 0's grad and residual after the last round (2 x len f32), for a checker to
// replay the rounds (residual k = synth(len, 0x0402026 + k, rank) for k = 0..rounds, sampler seed
// 0x5EED0000 + rank, carried across rounds).
//
//   make -C tools tcp_bench && tools/ono_tcp_bench --ranks 2 --len 109386 --rounds 200 [--sparse 0.1]
#include <hip/hip_runtime.h>

#include <arpa/inet.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <pthread.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "ono_reduce.h"

namespace {

int listen_any(int *port) {
    int fd = socket(AF_INET, SOCK_STREAM, 0);
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
    if (bind(fd, (sockaddr *)&a, sizeof a) || listen(fd, 4)) return -1;
    socklen_t sl = sizeof a;
    getsockname(fd, (sockaddr *)&a, &sl);
    *port = ntohs(a.sin_port);
    return fd;
}

int connect_to(int port) {
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_port = htons((uint16_t)port);
    a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
    for (int t = 0; t < 5000; t++) {
        int fd = socket(AF_INET, SOCK_STREAM, 0);
        if (connect(fd, (sockaddr *)&a, sizeof a) == 0) return fd;
        close(fd);
        usleep(1000);
    }
    return -1;
}

int g_sockbuf_kib = 0;  // --sockbuf: SO_SNDBUF / SO_RCVBUF of every ring socket (0: the system's autotuning)
void nodelay(int fd) {
    int one = 1;
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
    if (g_sockbuf_kib > 0) {
        int b = g_sockbuf_kib << 10;
        setsockopt(fd, SOL_SOCKET, SO_SNDBUF, &b, sizeof b);
        setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &b, sizeof b);
    }
}

}  // namespace

int main(int argc, char **argv) {
    int n = 2, rounds = 100;
    size_t len = 109386;
    float sparse = 0.0f;
    const char *dump = nullptr;
    int phases = 1;
    for (int a = 1; a < argc; a++) {
        if (!strcmp(argv[a], "--ranks") && a + 1 < argc) n = atoi(argv[++a]);
        else if (!strcmp(argv[a], "--len") && a + 1 < argc) len = strtoull(argv[++a], nullptr, 10);
        else if (!strcmp(argv[a], "--rounds") && a + 1 < argc) rounds = atoi(argv[++a]);
        else if (!strcmp(argv[a], "--sparse") && a + 1 < argc) sparse = (float)atof(argv[++a]);
        else if (!strcmp(argv[a], "--dump") && a + 1 < argc) dump = argv[++a];
        else if (!strcmp(argv[a], "--phases") && a + 1 < argc) phases = atoi(argv[++a]);
        else if (!strcmp(argv[a], "--sockbuf") && a + 1 < argc) g_sockbuf_kib = atoi(argv[++a]);
        else { fprintf(stderr, "bad arg %s\n", argv[a]); return 1; }
    }
    if (n < 2 || rounds < 1 || len < (size_t)n) { fprintf(stderr, "need ranks >= 2, len >= ranks\n"); return 1; }
    std::vector<int> lfd(n), port(n);
    for (int r = 0; r < n; r++)
        if ((lfd[r] = listen_any(&port[r])) < 0) { perror("listen"); return 2; }
    pthread_barrier_t bar;
    pthread_barrier_init(&bar, nullptr, (unsigned)n);
    std::vector<double> t(rounds, 0.0);
    std::vector<int> rc(n, ONO_OK);
    double ph_ms[ONO_PHASES] = {0};
    int64_t ph_n[ONO_PHASES] = {0};
    std::vector<std::thread> th;
    for (int r = 0; r < n; r++)
        th.emplace_back([&, r] {
            int nxt = connect_to(port[(r + 1) % n]);
            int prv = accept(lfd[r], nullptr, nullptr);
            if (nxt < 0 || prv < 0) { fprintf(stderr, "worker %d: connect failed\n", r); _exit(2); }
            nodelay(nxt);
            nodelay(prv);
            (void)hipSetDevice(0);
            hipStream_t s;
            if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) _exit(2);
            ono_ring *ring = nullptr;
            int e = ono_ring_create_tcp(&ring, r, n, len, 0, prv, nxt);
            if (e == ONO_OK && sparse > 0.0f) e = ono_ring_set_sparse(ring, sparse, 0x5EED0000ull + (uint64_t)r);
            for (int k = 0; k <= rounds && e == ONO_OK; k++) {  // round 0 is warmup
                if (k == 1 && r == 0 && phases) e = ono_ring_timing_enable(ring, 1);
                e = ono_synth_f32(ono_ring_residual(ring), len, 0x0402026 + k, (uint64_t)r, 0, s);
                if (e == ONO_OK) e = hipStreamSynchronize(s) == hipSuccess ? ONO_OK : ONO_E_HIP;
                pthread_barrier_wait(&bar);
                auto t0 = std::chrono::steady_clock::now();
                if (e == ONO_OK) e = ono_ring_pull_grads(ring, s);
                if (e == ONO_OK) e = hipStreamSynchronize(s) == hipSuccess ? ONO_OK : ONO_E_HIP;
                pthread_barrier_wait(&bar);
                if (r == 0 && k > 0)
                    t[k - 1] = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
            }
            if (e != ONO_OK) {  // the peers would wait for this worker's frames: end the tool
                fprintf(stderr, "worker %d: %s\n", r, ono_last_error());
                _exit(2);
            }
            if (r == 0 && e == ONO_OK && phases) e = ono_ring_timing_phases(ring, ph_ms, ph_n);
            if (r == 0 && e == ONO_OK && dump) {
                std::vector<float> h(2 * len);
                if (hipMemcpy(h.data(), ono_ring_grad(ring), len * 4, hipMemcpyDeviceToHost) != hipSuccess ||
                    hipMemcpy(h.data() + len, ono_ring_residual(ring), len * 4, hipMemcpyDeviceToHost) != hipSuccess)
                    e = ONO_E_HIP;
                FILE *f = e == ONO_OK ? fopen(dump, "wb") : nullptr;
                if (!f || fwrite(h.data(), 4, h.size(), f) != h.size()) e = ONO_E_IO;
                if (f) fclose(f);
            }
            rc[r] = e;
            if (ring) ono_ring_destroy(ring);
            (void)hipStreamDestroy(s);
            close(nxt);
            close(prv);
        });
    for (auto &x : th) x.join();
    for (int r = 0; r < n; r++) close(lfd[r]);
    for (int e : rc)
        if (e != ONO_OK) return 2;
    std::sort(t.begin(), t.end());
    const double med = t[t.size() / 2];
    double mean = 0;
    for (double x : t) mean += x;
    mean /= (double)t.size();
    // phase ms per round on rank 0 (events on its stream; the exchange and the codec block the host)
    const double kern = ph_ms[ONO_PHASE_KERNEL] / rounds, xchg = ph_ms[ONO_PHASE_RCCL] / rounds,
                 codec = ph_ms[ONO_PHASE_SPARSE_CODEC] / rounds;
    printf("{\"ranks\": %d, \"len\": %zu, \"rounds\": %d, \"sparse_r\": %g, \"s_per_round\": %.9f, "
           "\"s_per_round_mean\": %.9f, \"gib_s\": %.6f, \"phase_ms_per_round\": {\"kernel\": %.5f, "
           "\"exchange\": %.5f, \"sparse_codec\": %.5f}, \"codec_calls_per_round\": %.2f, "
           "\"codec_share_of_round\": %.4f, \"phases_timed\": %d}\n",
           n, len, rounds, (double)sparse, med, mean, (double)len * 4.0 / med / (double)(1ull << 30), kern, xchg, codec,
           (double)ph_n[ONO_PHASE_SPARSE_CODEC] / rounds, codec * 1e-3 / mean, phases);
    return 0;
}
