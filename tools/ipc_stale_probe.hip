// ipc_stale_probe.hip — what a peer reads through a fresh IPC import of an
// exchange region (the round-4 pool-release wrong result).
//
// Two processes on one GPU (forked before either touches HIP, no exec):
//   A (exporter)  per trial: hipMalloc an ordinary buffer M, fill it with
//                 pattern P1 (plain stores) and read every line of it from
//                 workgroups on every XCD (so the XCDs' L2s hold its lines),
//                 hipFree M; then allocate the exchange region R exactly as
//                 ono_xgmi.cpp does (hipExtMallocWithFlags, uncached), write
//                 P2 with system-scope stores + vmcnt(0), read it back through
//                 its own mapping, export it.
//   B (importer)  imports R, reads every line from every XCD with the
//                 system-scope loads the pull kernel uses, and classifies each
//                 word: P2 (right), P1 (a line of M's earlier use: a stale L2
//                 line of the same physical page), or other.
//   Then A rewrites R with P3 (system-scope stores) and B reads it again: P2
//   there means B's own earlier reads left lines its next kernel hits (the
//   within-ring case: the result slot rewritten every round).
//   Optional purge step in B before its first read (argv[2]):
//     0 none, 1 = one workgroup per CU runs a system-scope acquire fence
//     (buffer_inv sc0 sc1) before the read kernel.
// Mode "fbc" / "cbf" (argv[4]): the release order of ono_xgmi_pool_release.
//   fbc (free before close): A frees its exported region while B still has it
//   imported, then B closes the import (the BO's last reference drops in B);
//   cbf (close before free): B closes first, then A frees.  Right after, A
//   allocates fresh regions of the same size, writes them with system-scope
//   stores and reads them back 64 times over a few ms through its own
//   (uncached) mapping: a word that changes after it was written means the
//   released region's memory was still being written (e.g. cleared) after it
//   had been handed out again.
// Mode "ring" (argv[4]): the exchange protocol itself, no host in the loop.
//   A writes round k's pattern into R with system-scope stores (+ vmcnt(0)),
//   stores k into R's flag a (release, system) and spins until flag b >= k;
//   B (importer) spins until flag a >= k, reads every line of R from every XCD
//   and classifies it (round k right, round k-1 stale), stores k into flag b.
//   Every step is a kernel queued back to back on one stream per process, as
//   the ring's rounds are.  argv[2] picks B's load: 0 volatile (sc0 sc1, the
//   pull kernel's), 1 sc0 sc1 nt, 2 a system-scope acquire fence per wave first.
// Prints one line per trial and a summary.  usage: ipc_stale_probe [trials] [purge] [mib] [cache|fbc|cbf|ring]
#include <hip/hip_runtime.h>

#include <sys/wait.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) {                                                                 \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));   \
            _exit(3);                                                                           \
        }                                                                                       \
    } while (0)

constexpr int kBlock = 64;
constexpr int kXcd = 8;

__device__ __forceinline__ uint32_t pat(uint32_t kind, uint32_t trial, uint32_t i) {
    return (kind << 28) | ((trial & 0xFFu) << 20) | (i & 0xFFFFFu);
}

// one 16-B vector per lane; plain stores (cacheable) or system-scope stores
template <bool SYS>
__global__ __launch_bounds__(kBlock) void fill(uint32_t *p, size_t nwords, uint32_t kind, uint32_t trial) {
    const size_t v = (size_t)blockIdx.x * kBlock + threadIdx.x;
    if (4 * v + 3 < nwords) {
        typedef uint32_t u4 __attribute__((ext_vector_type(4)));
        u4 x = {pat(kind, trial, 4 * v), pat(kind, trial, 4 * v + 1), pat(kind, trial, 4 * v + 2),
                pat(kind, trial, 4 * v + 3)};
        if (SYS) *(volatile __attribute__((address_space(1))) u4 *)(p + 4 * v) = x;
        else *(u4 *)(p + 4 * v) = x;
    }
    if (SYS) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// Every segment of kBlock vectors is read by kXcd consecutive workgroups
// (blockIdx % 8 lands on a different XCD under round-robin dispatch), so each
// XCD's L2 sees every line.  Words classified by their kind nibble and trial.
template <bool SYS>
__global__ __launch_bounds__(kBlock) void readall(const uint32_t *p, size_t nwords, uint32_t want_kind,
                                                  uint32_t stale_kind, uint32_t trial, unsigned long long *cnt) {
    const size_t seg = blockIdx.x / kXcd;
    const size_t v = seg * kBlock + threadIdx.x;
    unsigned long long good = 0, stale = 0, other = 0;
    if (4 * v + 3 < nwords) {
        typedef uint32_t u4 __attribute__((ext_vector_type(4)));
        u4 x = SYS ? *(const volatile __attribute__((address_space(1))) u4 *)(p + 4 * v) : *(const u4 *)(p + 4 * v);
        uint32_t w[4] = {x.x, x.y, x.z, x.w};
        for (int k = 0; k < 4; k++) {
            const uint32_t i = (uint32_t)(4 * v + k);
            if (w[k] == pat(want_kind, trial, i)) good++;
            else if (w[k] == pat(stale_kind, trial, i)) stale++;
            else other++;
        }
    }
    if (good) atomicAdd(cnt + 0, good);
    if (stale) atomicAdd(cnt + 1, stale);
    if (other) atomicAdd(cnt + 2, other);
}

__global__ __launch_bounds__(kBlock) void purge_kernel() {
    if (threadIdx.x == 0) __atomic_thread_fence(__ATOMIC_SEQ_CST);  // system scope: buffer_wbl2 + buffer_inv sc0 sc1
}

struct Counts {
    unsigned long long good, stale, other;
};

Counts read_counts(const uint32_t *p, size_t nwords, uint32_t want, uint32_t stale, uint32_t trial, bool sys) {
    unsigned long long *d = nullptr;
    CK(hipMalloc(&d, 3 * sizeof(unsigned long long)));
    CK(hipMemset(d, 0, 3 * sizeof(unsigned long long)));
    const unsigned blocks = (unsigned)((nwords / 4 + kBlock - 1) / kBlock) * kXcd;
    if (sys) hipLaunchKernelGGL(readall<true>, dim3(blocks), dim3(kBlock), 0, 0, p, nwords, want, stale, trial, d);
    else hipLaunchKernelGGL(readall<false>, dim3(blocks), dim3(kBlock), 0, 0, p, nwords, want, stale, trial, d);
    CK(hipGetLastError());
    Counts c{};
    CK(hipMemcpy(&c, d, sizeof c, hipMemcpyDeviceToHost));
    CK(hipFree(d));
    return c;
}

void fill_buf(uint32_t *p, size_t nwords, uint32_t kind, uint32_t trial, bool sys) {
    const unsigned blocks = (unsigned)((nwords / 4 + kBlock - 1) / kBlock);
    if (sys) hipLaunchKernelGGL(fill<true>, dim3(blocks), dim3(kBlock), 0, 0, p, nwords, kind, trial);
    else hipLaunchKernelGGL(fill<false>, dim3(blocks), dim3(kBlock), 0, 0, p, nwords, kind, trial);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
}

bool rd(int fd, void *b, size_t n) {
    size_t got = 0;
    while (got < n) {
        ssize_t k = read(fd, (char *)b + got, n - got);
        if (k <= 0) return false;
        got += (size_t)k;
    }
    return true;
}
bool wr(int fd, const void *b, size_t n) { return write(fd, b, n) == (ssize_t)n; }

int exporter(int to_b, int from_b, int trials, size_t bytes) {
    CK(hipSetDevice(0));
    const size_t nw = bytes / 4;
    unsigned long long tot_self_bad = 0;
    for (int t = 0; t < trials; t++) {
        uint32_t *m = nullptr;
        CK(hipMalloc(&m, bytes));
        fill_buf(m, nw, 1, t, false);
        Counts cm = read_counts(m, nw, 1, 0, t, false);  // every XCD's L2 now holds M's lines
        CK(hipFree(m));
        uint32_t *r = nullptr;
        CK(hipExtMallocWithFlags((void **)&r, bytes, hipDeviceMallocUncached));
        fill_buf(r, nw, 2, t, true);
        Counts self = read_counts(r, nw, 2, 1, t, true);
        tot_self_bad += self.stale + self.other;
        hipIpcMemHandle_t h;
        CK(hipIpcGetMemHandle(&h, r));
        if (!wr(to_b, &h, sizeof h)) return 4;
        char ack;
        if (!rd(from_b, &ack, 1)) return 5;  // B has read P2
        fill_buf(r, nw, 3, t, true);
        if (!wr(to_b, "3", 1)) return 6;
        if (!rd(from_b, &ack, 1)) return 7;  // B has read P3 and closed its import
        CK(hipFree(r));
        printf("A trial %d: M read ok %llu/%zu; own mapping of R: right %llu stale(P1) %llu other %llu\n", t, cm.good,
               nw, self.good, self.stale, self.other);
        fflush(stdout);
    }
    printf("A summary: own-mapping wrong words %llu\n", tot_self_bad);
    fflush(stdout);
    return 0;
}

int importer(int from_a, int to_a, int trials, size_t bytes, int purge) {
    CK(hipSetDevice(0));
    const size_t nw = bytes / 4;
    unsigned long long stale1 = 0, other1 = 0, stale2 = 0, other2 = 0;
    int trials_stale1 = 0, trials_stale2 = 0;
    for (int t = 0; t < trials; t++) {
        hipIpcMemHandle_t h;
        if (!rd(from_a, &h, sizeof h)) return 4;
        void *p = nullptr;
        CK(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess));
        if (purge == 1) {
            hipLaunchKernelGGL(purge_kernel, dim3(256 * kXcd), dim3(kBlock), 0, 0);
            CK(hipDeviceSynchronize());
        }
        Counts c1 = read_counts((const uint32_t *)p, nw, 2, 1, t, true);
        if (!wr(to_a, "2", 1)) return 5;
        char ack;
        if (!rd(from_a, &ack, 1)) return 6;
        Counts c2 = read_counts((const uint32_t *)p, nw, 3, 2, t, true);
        CK(hipIpcCloseMemHandle(p));
        if (!wr(to_a, "c", 1)) return 7;
        stale1 += c1.stale;
        other1 += c1.other;
        stale2 += c2.stale;
        other2 += c2.other;
        trials_stale1 += c1.stale > 0;
        trials_stale2 += c2.stale > 0;
        printf("B trial %d: first read right %llu P1(stale) %llu other %llu | after rewrite right %llu P2(stale) %llu "
               "other %llu\n", t, c1.good, c1.stale, c1.other, c2.good, c2.stale, c2.other);
        fflush(stdout);
    }
    printf("B summary (purge %d): fresh import stale words %llu in %d/%d trials, other %llu; rewritten slot stale %llu "
           "in %d/%d trials, other %llu\n", purge, stale1, trials_stale1, trials, other1, stale2, trials_stale2, trials,
           other2);
    fflush(stdout);
    return 0;
}

// release-order probe, exporter side
int rel_exporter(int to_b, int from_b, int trials, size_t bytes, bool free_first) {
    CK(hipSetDevice(0));
    const size_t nw = bytes / 4;
    unsigned long long bad_tot = 0;
    int bad_trials = 0;
    for (int t = 0; t < trials; t++) {
        uint32_t *r = nullptr;
        CK(hipExtMallocWithFlags((void **)&r, bytes, hipDeviceMallocUncached));
        fill_buf(r, nw, 4, t, true);
        hipIpcMemHandle_t h;
        CK(hipIpcGetMemHandle(&h, r));
        if (!wr(to_b, &h, sizeof h)) return 4;
        char ack;
        if (!rd(from_b, &ack, 1)) return 5;  // imported and read once
        if (free_first) {
            CK(hipFree(r));
            if (!wr(to_b, "f", 1)) return 6;
            if (!rd(from_b, &ack, 1)) return 7;  // closed: the BO's last reference dropped in B
        } else {
            if (!wr(to_b, "c", 1)) return 6;
            if (!rd(from_b, &ack, 1)) return 7;  // closed
            CK(hipFree(r));
        }
        // fresh regions right away (several, so that one gets the released pages)
        constexpr int kFresh = 4;
        uint32_t *f[kFresh];
        for (int k = 0; k < kFresh; k++) {
            CK(hipExtMallocWithFlags((void **)&f[k], bytes, hipDeviceMallocUncached));
            fill_buf(f[k], nw, 5, t * kFresh + k, true);
        }
        unsigned long long bad = 0;
        for (int rep = 0; rep < 64; rep++)
            for (int k = 0; k < kFresh; k++) {
                Counts c = read_counts(f[k], nw, 5, 4, t * kFresh + k, true);
                bad += c.stale + c.other;
            }
        for (int k = 0; k < kFresh; k++) CK(hipFree(f[k]));
        bad_tot += bad;
        bad_trials += bad > 0;
        printf("A trial %d (%s): words of fresh regions changed after being written: %llu\n", t,
               free_first ? "free before close" : "close before free", bad);
        fflush(stdout);
    }
    printf("A summary (%s): %llu changed words in %d/%d trials\n", free_first ? "free before close" : "close before free",
           bad_tot, bad_trials, trials);
    fflush(stdout);
    return 0;
}

int rel_importer(int from_a, int to_a, int trials, size_t bytes) {
    CK(hipSetDevice(0));
    const size_t nw = bytes / 4;
    for (int t = 0; t < trials; t++) {
        hipIpcMemHandle_t h;
        if (!rd(from_a, &h, sizeof h)) return 4;
        void *p = nullptr;
        CK(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess));
        Counts c = read_counts((const uint32_t *)p, nw, 4, 0, t, true);
        if (c.other) printf("B trial %d: import read %llu wrong words\n", t, c.other);
        if (!wr(to_a, "i", 1)) return 5;
        char ack;
        if (!rd(from_a, &ack, 1)) return 6;
        CK(hipIpcCloseMemHandle(p));
        if (!wr(to_a, "c", 1)) return 7;
    }
    return 0;
}

// ---- mode ring ----
constexpr size_t kFlagPage = 4096;
__global__ __launch_bounds__(64) void ring_write(uint32_t *data, size_t nwords, uint32_t k) {
    const size_t v = (size_t)blockIdx.x * kBlock + threadIdx.x;
    if (4 * v + 3 < nwords) {
        typedef uint32_t u4 __attribute__((ext_vector_type(4)));
        u4 x = {pat(6, k, 4 * v), pat(6, k, 4 * v + 1), pat(6, k, 4 * v + 2), pat(6, k, 4 * v + 3)};
        *(volatile __attribute__((address_space(1))) u4 *)(data + 4 * v) = x;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}
// lane 0: optionally store `mine` (release, system), then spin until *theirs >= want (acquire, system)
__global__ __launch_bounds__(64) void ring_flag(uint64_t *mine, uint64_t val, const uint64_t *theirs, uint64_t want,
                                                uint32_t *err) {
    if (threadIdx.x) return;
    __atomic_thread_fence(__ATOMIC_SEQ_CST);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (mine) __hip_atomic_store(mine, val, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    if (theirs) {
        const uint64_t t0 = wall_clock64();
        while (__hip_atomic_load(theirs, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < want) {
            if (wall_clock64() - t0 > 100000000ull * 5) {  // 5 s at 100 MHz
                __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                break;
            }
            __builtin_amdgcn_s_sleep(2);
        }
    }
    __atomic_thread_fence(__ATOMIC_SEQ_CST);
}
template <int LOAD>
__global__ __launch_bounds__(kBlock) void ring_read(const uint32_t *p, size_t nwords, uint32_t k,
                                                    unsigned long long *cnt) {
    typedef uint32_t u4 __attribute__((ext_vector_type(4)));
    if constexpr (LOAD == 2) __atomic_thread_fence(__ATOMIC_SEQ_CST);
    const size_t seg = blockIdx.x / kXcd;
    const size_t v = seg * kBlock + threadIdx.x;
    unsigned long long stale = 0, other = 0;
    if (4 * v + 3 < nwords) {
        u4 x;
        if constexpr (LOAD == 1) {
            asm volatile("global_load_dwordx4 %0, %1, off sc0 sc1 nt\n\ts_waitcnt vmcnt(0)" : "=v"(x) : "v"(p + 4 * v) : "memory");
        } else {
            x = *(const volatile __attribute__((address_space(1))) u4 *)(p + 4 * v);
        }
        uint32_t w[4] = {x.x, x.y, x.z, x.w};
        for (int j = 0; j < 4; j++) {
            const uint32_t i = (uint32_t)(4 * v + j);
            if (w[j] == pat(6, k, i)) continue;
            if (w[j] == pat(6, k - 1, i)) stale++;
            else other++;
        }
    }
    if (stale) atomicAdd(cnt + 0, stale);
    if (other) atomicAdd(cnt + 1, other);
}

int ring_a(int to_b, int from_b, int rounds, size_t bytes) {
    CK(hipSetDevice(0));
    const size_t nw = bytes / 4;
    uint8_t *r = nullptr;
    CK(hipExtMallocWithFlags((void **)&r, kFlagPage + bytes, hipDeviceMallocUncached));
    CK(hipMemset(r, 0, kFlagPage + bytes));
    uint32_t *err = nullptr;
    CK(hipHostMalloc((void **)&err, 4, hipHostMallocMapped | hipHostMallocCoherent));
    *err = 0;
    CK(hipDeviceSynchronize());
    hipIpcMemHandle_t h;
    CK(hipIpcGetMemHandle(&h, r));
    if (!wr(to_b, &h, sizeof h)) return 4;
    char ack;
    if (!rd(from_b, &ack, 1)) return 5;
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    uint64_t *fa = (uint64_t *)r, *fb = (uint64_t *)(r + 8);
    uint32_t *data = (uint32_t *)(r + kFlagPage);
    const unsigned blocks = (unsigned)((nw / 4 + kBlock - 1) / kBlock);
    for (int k = 1; k <= rounds; k++) {
        hipLaunchKernelGGL(ring_write, dim3(blocks), dim3(kBlock), 0, s, data, nw, (uint32_t)k);
        hipLaunchKernelGGL(ring_flag, dim3(1), dim3(64), 0, s, fa, (uint64_t)k, fb, (uint64_t)k, err);
    }
    CK(hipStreamSynchronize(s));
    printf("A: %d rounds, err %u\n", rounds, *err);
    fflush(stdout);
    if (!rd(from_b, &ack, 1)) return 6;  // B closed its import
    CK(hipFree(r));
    return *err ? 8 : 0;
}

int ring_b(int from_a, int to_a, int rounds, size_t bytes, int load) {
    CK(hipSetDevice(0));
    const size_t nw = bytes / 4;
    hipIpcMemHandle_t h;
    if (!rd(from_a, &h, sizeof h)) return 4;
    uint8_t *r = nullptr;
    CK(hipIpcOpenMemHandle((void **)&r, h, hipIpcMemLazyEnablePeerAccess));
    uint32_t *err = nullptr;
    CK(hipHostMalloc((void **)&err, 4, hipHostMallocMapped | hipHostMallocCoherent));
    *err = 0;
    unsigned long long *cnt = nullptr;  // per round: stale, other
    CK(hipMalloc(&cnt, 2 * sizeof(unsigned long long) * (rounds + 1)));
    CK(hipMemset(cnt, 0, 2 * sizeof(unsigned long long) * (rounds + 1)));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    CK(hipDeviceSynchronize());
    if (!wr(to_a, "r", 1)) return 5;
    uint64_t *fa = (uint64_t *)r, *fb = (uint64_t *)(r + 8);
    const uint32_t *data = (const uint32_t *)(r + kFlagPage);
    const unsigned blocks = (unsigned)((nw / 4 + kBlock - 1) / kBlock) * kXcd;
    for (int k = 1; k <= rounds; k++) {
        hipLaunchKernelGGL(ring_flag, dim3(1), dim3(64), 0, s, nullptr, 0ull, fa, (uint64_t)k, err);
        if (load == 1) hipLaunchKernelGGL(ring_read<1>, dim3(blocks), dim3(kBlock), 0, s, data, nw, (uint32_t)k, cnt + 2 * k);
        else if (load == 2) hipLaunchKernelGGL(ring_read<2>, dim3(blocks), dim3(kBlock), 0, s, data, nw, (uint32_t)k, cnt + 2 * k);
        else hipLaunchKernelGGL(ring_read<0>, dim3(blocks), dim3(kBlock), 0, s, data, nw, (uint32_t)k, cnt + 2 * k);
        hipLaunchKernelGGL(ring_flag, dim3(1), dim3(64), 0, s, fb, (uint64_t)k, nullptr, 0ull, err);
    }
    CK(hipStreamSynchronize(s));
    std::vector<unsigned long long> c(2 * (rounds + 1));
    CK(hipMemcpy(c.data(), cnt, c.size() * sizeof(c[0]), hipMemcpyDeviceToHost));
    unsigned long long st = 0, ot = 0;
    int rs = 0, ro = 0, first = -1;
    for (int k = 1; k <= rounds; k++) {
        st += c[2 * k];
        ot += c[2 * k + 1];
        rs += c[2 * k] > 0;
        ro += c[2 * k + 1] > 0;
        if ((c[2 * k] || c[2 * k + 1]) && first < 0) first = k;
    }
    printf("B (load %d, %zu KiB, %d rounds): stale words %llu in %d rounds, other %llu in %d rounds, first bad round %d, "
           "err %u\n", load, bytes >> 10, rounds, st, rs, ot, ro, first, *err);
    fflush(stdout);
    CK(hipIpcCloseMemHandle(r));
    if (!wr(to_a, "c", 1)) return 6;
    return *err ? 8 : 0;
}

int main(int argc, char **argv) {
    const int trials = argc > 1 ? atoi(argv[1]) : 16;
    const int purge = argc > 2 ? atoi(argv[2]) : 0;
    const size_t bytes = (size_t)(argc > 3 ? atoi(argv[3]) : 2) << 20;
    const char *mode = argc > 4 ? argv[4] : "cache";
    const bool rel = strcmp(mode, "fbc") == 0 || strcmp(mode, "cbf") == 0;
    if (strcmp(mode, "ring") == 0) {
        int ab[2], ba[2];
        if (pipe(ab) || pipe(ba)) return 2;
        pid_t a = fork();
        if (a == 0) _exit(ring_a(ab[1], ba[0], trials, bytes));
        pid_t b = fork();
        if (b == 0) _exit(ring_b(ab[0], ba[1], trials, bytes, purge));
        int sa = 0, sb = 0;
        waitpid(a, &sa, 0);
        waitpid(b, &sb, 0);
        printf("exit A %d B %d\n", WEXITSTATUS(sa), WEXITSTATUS(sb));
        return (WIFEXITED(sa) && WEXITSTATUS(sa) == 0 && WIFEXITED(sb) && WEXITSTATUS(sb) == 0) ? 0 : 1;
    }
    int ab[2], ba[2];
    if (pipe(ab) || pipe(ba)) return 2;
    pid_t a = fork();
    if (a == 0)
        _exit(rel ? rel_exporter(ab[1], ba[0], trials, bytes, strcmp(mode, "fbc") == 0)
                  : exporter(ab[1], ba[0], trials, bytes));
    pid_t b = fork();
    if (b == 0) _exit(rel ? rel_importer(ab[0], ba[1], trials, bytes) : importer(ab[0], ba[1], trials, bytes, purge));
    int sa = 0, sb = 0;
    waitpid(a, &sa, 0);
    waitpid(b, &sb, 0);
    printf("exit A %d B %d\n", WEXITSTATUS(sa), WEXITSTATUS(sb));
    return (WIFEXITED(sa) && WEXITSTATUS(sa) == 0 && WIFEXITED(sb) && WEXITSTATUS(sb) == 0) ? 0 : 1;
}
