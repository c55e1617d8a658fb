// ono_xgmi_harness.cpp — the xGMI peer-access ring driven by a plain C++ host,
// one PROCESS per rank, through the C ABI only (no Python, no torch): the way
// a native Rust worker binary per GPU would use it.
//
// The parent forks n workers before anything touches the GPU; each worker
// creates its ring (ono_ring_create_xgmi), sends its 128-byte handle up a pipe,
// receives all n handles back (the parent plays the out-of-band control
// channel — the reference's ring links), connects, and runs host-fed rounds
// (ono_ring_pull_grads_host on registered host buckets, both wires), each
// checked bit for bit against the C oracle of the reference ring.
//
//   make -C tests/native ono_xgmi_harness && tests/native/ono_xgmi_harness [nranks] [n_elems] [device_stride]
// device_stride 0 puts every rank on device 0 (one-GPU box), 1 gives rank r device r.
// exit 0 = every rank bit-exact, 1 = mismatch, 2 = library / process error.
#include <sys/wait.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "ono_oracle.h"
#include "ono_reduce.h"

#define CHECK(call)                                                                   \
    do {                                                                              \
        int rc_ = (call);                                                             \
        if (rc_ != ONO_OK) {                                                          \
            fprintf(stderr, "rank %d: %s -> %d: %s\n", rank, #call, rc_, ono_last_error()); \
            return 2;                                                                 \
        }                                                                             \
    } while (0)

static bool io_all(int fd, void *buf, size_t len, bool wr) {
    char *p = static_cast<char *>(buf);
    while (len) {
        ssize_t k = wr ? write(fd, p, len) : read(fd, p, len);
        if (k <= 0) return false;
        p += k;
        len -= (size_t)k;
    }
    return true;
}

static int worker(int rank, int n, size_t len, int dev, int up, int down) {
    const uint64_t seed = 0x0402026;
    int rounds_ok = 0;
    for (int wire : {ONO_WIRE_F32, ONO_WIRE_F16}) {
        ono_ring *ring = nullptr;
        CHECK(ono_ring_create_xgmi(&ring, rank, n, len, dev, wire));
        uint8_t mine[ONO_XGMI_HANDLE_BYTES];
        CHECK(ono_ring_xgmi_handle(ring, mine));
        std::vector<uint8_t> all((size_t)n * ONO_XGMI_HANDLE_BYTES);
        if (!io_all(up, mine, sizeof mine, true) || !io_all(down, all.data(), all.size(), false)) return 2;
        CHECK(ono_ring_xgmi_connect(ring, all.data()));
        std::vector<float> res(len), grad(len);
        CHECK(ono_ring_register_host(ring, res.data(), len * sizeof(float)));
        CHECK(ono_ring_register_host(ring, grad.data(), len * sizeof(float)));
        for (int round = 0; round < 3; round++) {
            // every rank can regenerate every rank's bucket: the oracle ring runs here too
            std::vector<std::vector<float>> ins(n, std::vector<float>(len)), outs(n, std::vector<float>(len));
            std::vector<float *> ip(n), op(n);
            for (int r = 0; r < n; r++) {
                ono_ref_synth(ins[r].data(), len, seed + 100 * round + wire, (uint64_t)r, 0);
                ip[r] = ins[r].data();
                op[r] = outs[r].data();
            }
            res = ins[rank];
            if (ono_ref_ring_pull_grads(ip.data(), op.data(), n, len, wire == ONO_WIRE_F16 ? 0 : 1)) return 2;
            CHECK(ono_ring_pull_grads_host(ring, res.data(), grad.data(), len));
            bool ok = memcmp(grad.data(), outs[rank].data(), len * sizeof(float)) == 0;
            for (size_t i = 0; i < len && ok; i++) ok = res[i] == 0.0f;
            if (!ok) {
                fprintf(stderr, "rank %d wire %d round %d: MISMATCH\n", rank, wire, round);
                return 1;
            }
            rounds_ok++;
        }
        CHECK(ono_ring_unregister_host(ring, res.data()));
        CHECK(ono_ring_unregister_host(ring, grad.data()));
        CHECK(ono_ring_destroy(ring));  // collective: every rank destroys together
    }
    printf("rank %d: %d rounds bit-exact\n", rank, rounds_ok);
    fflush(stdout);  // the worker leaves through _exit()
    return 0;
}

int main(int argc, char **argv) {
    const int n = argc > 1 ? atoi(argv[1]) : 4;
    const size_t len = argc > 2 ? strtoull(argv[2], nullptr, 10) : 300007;
    const int stride = argc > 3 ? atoi(argv[3]) : 0;
    if (n < 2 || n > ONO_MAX_INPUTS) return 2;
    std::vector<int> up_r(n), down_w(n);
    std::vector<pid_t> pids(n);
    for (int r = 0; r < n; r++) {  // fork before any HIP call in this process
        int up[2], down[2];
        if (pipe(up) || pipe(down)) return 2;
        pid_t pid = fork();
        if (pid < 0) return 2;
        if (pid == 0) {
            close(up[0]);
            close(down[1]);
            fflush(stdout);
            _exit(worker(r, n, len, r * stride, up[1], down[0]));
        }
        close(up[1]);
        close(down[0]);
        up_r[r] = up[0];
        down_w[r] = down[1];
        pids[r] = pid;
    }
    // the control channel: two handle exchanges (one ring per wire)
    for (int ex = 0; ex < 2; ex++) {
        std::vector<uint8_t> all((size_t)n * ONO_XGMI_HANDLE_BYTES);
        bool ok = true;
        for (int r = 0; r < n && ok; r++) ok = io_all(up_r[r], all.data() + (size_t)r * ONO_XGMI_HANDLE_BYTES,
                                                      ONO_XGMI_HANDLE_BYTES, false);
        for (int r = 0; r < n && ok; r++) ok = io_all(down_w[r], all.data(), all.size(), true);
        if (!ok) break;
    }
    int worst = 0;
    for (int r = 0; r < n; r++) {
        int st = 0;
        waitpid(pids[r], &st, 0);
        int code = WIFEXITED(st) ? WEXITSTATUS(st) : 2;
        if (code > worst) worst = code;
    }
    printf("xgmi harness: %d ranks x %zu elems: %s\n", n, len, worst == 0 ? "bit-exact" : "FAILED");
    return worst;
}
