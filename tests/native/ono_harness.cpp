// ono_harness.cpp — a C++ host program driving libono_reduce.so through its
// C ABI only (include/ono_reduce.h), the way the reference's Rust crates would
// bind it.  It plays one WorkerRingManager round (n = 1 on this box: the
// device path of pull_grads) on host buckets, a three-worker ring over the
// TCP edge (socket pairs, one thread per worker, host buckets), and a
// BlockingStore + BarrierSync round with three worker threads, and checks all
// three against the C oracle.
//
//   make -C tests/native ono_harness && tests/native/ono_harness [n_elems]
// exit 0 = bit-exact, 1 = mismatch, 2 = library error.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>

#include <sys/socket.h>
#include <unistd.h>
#include <vector>

#include "ono_oracle.h"
#include "ono_reduce.h"

#define CHECK(call)                                                                   \
    do {                                                                              \
        int rc_ = (call);                                                             \
        if (rc_ != ONO_OK) {                                                          \
            fprintf(stderr, "%s -> %d: %s\n", #call, rc_, ono_last_error());         \
            return 2;                                                                 \
        }                                                                             \
    } while (0)

static bool same(const float *a, const float *b, size_t n) { return memcmp(a, b, n * sizeof(float)) == 0; }

int main(int argc, char **argv) {
    const size_t n = argc > 1 ? strtoull(argv[1], nullptr, 10) : 1000003;
    const uint64_t seed = 0x0402026;
    int devs = 0;
    CHECK(ono_device_count(&devs));
    if (devs < 1) { fprintf(stderr, "no GPU\n"); return 2; }

    // ---- ring: WorkerRingManager::new + pull_grads on host buckets (n = 1)
    std::vector<float> residual(n), grad(n), expect(n);
    ono_ref_synth(residual.data(), n, seed, 0, 0);
    expect = residual;  // n == 1: grad = residual, residual = 0 (worker_ring.rs:166-171)
    ono_ring *ring = nullptr;
    CHECK(ono_ring_create(&ring, 0, 1, n, 0, nullptr, ONO_WIRE_F16));
    CHECK(ono_ring_register_host(ring, residual.data(), n * sizeof(float)));
    CHECK(ono_ring_register_host(ring, grad.data(), n * sizeof(float)));
    CHECK(ono_ring_pull_grads_host(ring, residual.data(), grad.data(), n));
    bool ok = same(grad.data(), expect.data(), n);
    for (size_t i = 0; i < n; i++) ok &= residual[i] == 0.0f;
    CHECK(ono_ring_unregister_host(ring, residual.data()));
    CHECK(ono_ring_unregister_host(ring, grad.data()));
    CHECK(ono_ring_destroy(ring));
    printf("ring pull_grads_host (n=1, %zu elems): %s\n", n, ok ? "bit-exact" : "MISMATCH");

    // ---- TCP edge: three workers in one ring over socket pairs (builder.rs:272-311
    // hands each worker its prev/next connections), host buckets, f16 frames
    const int nr = 3;
    const size_t nt = 300007;
    int sp[nr][2];  // pair i carries worker i -> worker i+1
    for (auto &p : sp)
        if (socketpair(AF_UNIX, SOCK_STREAM, 0, p)) { perror("socketpair"); return 2; }
    std::vector<std::vector<float>> tres(nr, std::vector<float>(nt)), tgrad(nr, std::vector<float>(nt, 7.0f));
    for (int r = 0; r < nr; r++) ono_ref_synth(tres[r].data(), nt, seed + 9, (uint64_t)r, 0);
    std::vector<std::vector<float>> eres = tres, egrad(nr, std::vector<float>(nt));
    std::vector<int> trc(nr, ONO_OK);
    std::vector<std::thread> tw;
    for (int r = 0; r < nr; r++)
        tw.emplace_back([&, r] {
            ono_ring *tr = nullptr;
            int rc = ono_ring_create_tcp(&tr, r, nr, nt, 0, sp[(r + nr - 1) % nr][1], sp[r][0]);
            if (rc == ONO_OK) rc = ono_ring_pull_grads_host(tr, tres[r].data(), tgrad[r].data(), nt);
            if (rc != ONO_OK) fprintf(stderr, "worker %d: %s\n", r, ono_last_error());
            if (tr) ono_ring_destroy(tr);
            trc[r] = rc;
        });
    for (auto &t : tw) t.join();
    for (auto &p : sp) { close(p[0]); close(p[1]); }
    for (int rc : trc)
        if (rc != ONO_OK) return 2;
    {
        std::vector<float *> rp(nr), gp(nr);
        for (int r = 0; r < nr; r++) { rp[r] = eres[r].data(); gp[r] = egrad[r].data(); }
        ono_ref_ring_pull_grads(rp.data(), gp.data(), nr, nt, 0);
    }
    bool ok3 = true;
    for (int r = 0; r < nr; r++) ok3 &= same(tgrad[r].data(), egrad[r].data(), nt) && same(tres[r].data(), eres[r].data(), nt);
    printf("TCP edge ring (3 workers, socket pairs, %zu elems, host buckets): %s\n", nt, ok3 ? "bit-exact" : "MISMATCH");
    ok &= ok3;

    // ---- PS: BlockingStore + BarrierSync, three worker threads, Adam
    const int nw = 3, rounds = 4;
    const size_t np = 4099;
    std::vector<float> init(np);
    ono_ref_synth(init.data(), np, seed, 7, 0);
    ono_opt_spec opt{ONO_OPT_ADAM, 0.01f, 0.0f, 0.9f, 0.999f, 1e-8f};
    ono_store *store = nullptr;
    ono_sync *sync = nullptr;
    CHECK(ono_store_create(&store, ONO_STORE_BLOCKING, init.data(), np, 128, nw, &opt, 0));
    CHECK(ono_sync_create(&sync, ONO_SYNC_BARRIER, nw));
    for (int w = 1; w < nw; w++) CHECK(ono_sync_clone(sync));
    // integer-valued gradients: the accumulation order cannot change the sums
    std::vector<std::vector<float>> grads(nw * rounds, std::vector<float>(np));
    for (int k = 0; k < nw * rounds; k++) {
        ono_ref_synth(grads[k].data(), np, seed + k, 1, 0);
        for (auto &x : grads[k]) x = (float)(int)(x * 64.0f);
    }
    std::vector<std::vector<float>> pulled(nw * rounds, std::vector<float>(np));
    std::vector<int> rcs(nw, 0);
    std::vector<std::thread> ts;
    for (int w = 0; w < nw; w++)
        ts.emplace_back([&, w] {
            for (int r = 0; r < rounds && !rcs[w]; r++)
                rcs[w] = ono_sync_step(sync, store, grads[r * nw + w].data(), pulled[r * nw + w].data(), np);
            ono_sync_release(sync);
        });
    for (auto &t : ts) t.join();
    for (int w = 0; w < nw; w++)
        if (rcs[w]) { fprintf(stderr, "worker %d: %d %s\n", w, rcs[w], ono_last_error()); return 2; }
    ono_ref_store *ref = ono_ref_store_new(init.data(), np, 128, nw, ONO_REF_OPT_ADAM, 0.01f, 0.0f, 0.9f, 0.999f, 1e-8f);
    bool ok2 = true;
    std::vector<float> e(np);
    for (int r = 0; r < rounds; r++) {
        for (int w = 0; w < nw; w++) ono_ref_store_accumulate(ref, grads[r * nw + w].data(), np);
        ono_ref_store_update_params(ref);
        ono_ref_store_pull_params(ref, e.data(), np);
        for (int w = 0; w < nw; w++) ok2 &= same(pulled[r * nw + w].data(), e.data(), np);
    }
    ono_ref_store_free(ref);
    CHECK(ono_store_destroy(store));
    printf("BlockingStore + BarrierSync (3 threads, Adam, %d rounds): %s\n", rounds, ok2 ? "bit-exact" : "MISMATCH");
    return ok && ok2 ? 0 : 1;
}
