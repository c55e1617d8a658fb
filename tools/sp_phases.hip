// sp_phases — where a stream-ordered sparse drop's time goes (measurement build, not the product).
//
// Compiles the library's sparse codec source with ONO_SP_STAMP defined: every sp_image workgroup
// and every sp_move wave stores {start, mid, end} real-time stamps (100 MHz) and its XCC id.
// Runs K stream-ordered drops of 64 MiB gradients (6 in turn, ~10 % kept in isolated runs like the
// bench's) back to back between two events, then reports for the last drop, per kernel: the span
// (first start -> last end), when units start (dispatch), how long they live, the mid stamp
// (sp_move: its loads landed and its prefix known; sp_image: its last tile imaged) and the
// per-XCD last end.
//
// Then the same for K stream-ordered lifts (pattern path) of the last drop's wire into 6 outputs
// in turn: pl_fused stamped per workgroup (ONO_LIFT_FUSED=0: pl_index and pl_place).
//
// usage: sp_phases [MiB=64] [K=24]
#define ONO_SP_STAMP 1
#include "../oxidized-neural-orchestra_amd/csrc/ono_sparse.hip"

#include <cmath>
#include <cstdarg>
#include <cstdio>

namespace ono {
int set_error(int code, const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    fprintf(stderr, "error %d: ", code);
    vfprintf(stderr, fmt, ap);
    fprintf(stderr, "\n");
    va_end(ap);
    return code;
}
int hip_error(hipError_t e, const char *what, const char *file, int line) {
    fprintf(stderr, "%s: %s (%s:%d)\n", what, hipGetErrorString(e), file, line);
    return ONO_E_HIP;
}
}  // namespace ono

#define CK(x)                                                                            \
    do {                                                                                 \
        hipError_t e_ = (x);                                                             \
        if (e_ != hipSuccess) {                                                          \
            fprintf(stderr, "%s: %s (line %d)\n", #x, hipGetErrorString(e_), __LINE__); \
            exit(1);                                                                     \
        }                                                                                \
    } while (0)

// |x| uniform in [0, 1): with threshold 0.9 about 10 % kept, in runs of mean length 1.1
__global__ void gen(float *g, size_t n, uint32_t seed) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        uint32_t h = (uint32_t)i * 0x9E3779B1u ^ seed;
        h ^= h >> 15; h *= 0x85EBCA77u; h ^= h >> 13; h *= 0xC2B2AE3Du; h ^= h >> 16;
        const float u = (h >> 8) * (1.0f / 16777216.0f);
        g[i] = (h & 1) ? -u : u;
    }
}

static double pct(std::vector<double> v, double p) {
    if (v.empty()) return 0;
    std::sort(v.begin(), v.end());
    return v[std::min(v.size() - 1, (size_t)(p * (v.size() - 1) + 0.5))];
}

static void report(const char *name, const std::vector<uint4> &st, uint64_t base) {
    // stamps: x = low 32 bits of start, y = mid - start, z = end - start, w = XCC
    std::vector<double> start, life, mid, end;
    double xend[16] = {0};
    const double us = 0.01;  // 100 MHz ticks -> us
    uint32_t b32 = (uint32_t)base;
    for (const uint4 &s : st) {
        const double t0 = (double)(uint32_t)(s.x - b32) * us;
        start.push_back(t0);
        life.push_back(s.z * us);
        mid.push_back(s.y * us);
        end.push_back(t0 + s.z * us);
        xend[s.w & 15] = std::max(xend[s.w & 15], t0 + s.z * us);
    }
    const double first_end = pct(end, 0.0);
    size_t late = 0;
    for (double t : start) late += t > first_end;
    printf("%-9s units %6zu | start p0 %6.2f p50 %6.2f p90 %6.2f max %6.2f | life p10 %5.2f p50 %5.2f p90 %5.2f "
           "max %5.2f | mid p50 %5.2f | end p50 %6.2f p90 %6.2f max %6.2f | started after the first end %zu\n",
           name, st.size(), pct(start, 0), pct(start, 0.5), pct(start, 0.9), pct(start, 1), pct(life, 0.1),
           pct(life, 0.5), pct(life, 0.9), pct(life, 1), pct(mid, 0.5), pct(end, 0.5), pct(end, 0.9), pct(end, 1),
           late);
    printf("%-9s per-XCD last end:", name);
    for (int x = 0; x < 8; x++) printf(" %6.2f", xend[x]);
    printf("\n");
}

int main(int argc, char **argv) {
    // argv[1]: MiB, or eN for N elements (e54693: a config-1 chunk); argv[3] = "pinned": the TCP ring's form —
    // the blocking drop (its in-kernel completion) into a pinned coherent buffer, timed on the host per call
    const bool by_elems = argc > 1 && argv[1][0] == 'e';
    const size_t mib = argc > 1 && !by_elems ? (size_t)atoi(argv[1]) : 64;
    const int K = argc > 2 ? atoi(argv[2]) : 24, NG = 6;
    const size_t n = by_elems ? (size_t)strtoull(argv[1] + 1, nullptr, 10) : mib << 18;
    const bool pinned = argc > 3 && !strcmp(argv[3], "pinned");
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    std::vector<float *> gs(NG);
    for (int i = 0; i < NG; i++) {
        CK(hipMalloc((void **)&gs[i], n * sizeof(float)));
        hipLaunchKernelGGL(gen, dim3(4096), dim3(256), 0, s, gs[i], n, 0x5EED0u + 77u * i);
    }
    const size_t cap = ono_sparse_max_bytes(n);
    uint8_t *buf;
    uint64_t *nbd;
    if (pinned) CK(hipHostMalloc((void **)&buf, cap + 64, hipHostMallocCoherent));
    else CK(hipMalloc((void **)&buf, cap));
    CK(hipMalloc((void **)&nbd, 8));
    const float thr = 0.9f;
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    float ms = 0;
    uint64_t wire = 0;
    if (pinned) {  // blocking calls, as the TCP ring's push makes them
        size_t nb = 0;
        for (int i = 0; i < 2 * K; i++)
            if (drop_launch(buf, cap, &nb, nullptr, gs[i % NG], n, thr, s)) return 1;
        std::vector<double> us;
        for (int i = 0; i < K; i++) {
            const auto t0 = std::chrono::steady_clock::now();
            if (drop_launch(buf, cap, &nb, nullptr, gs[i % NG], n, thr, s)) return 1;
            us.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
        }
        printf("# sp_phases: %zu values, %d blocking drops into pinned coherent memory: %.2f us per call (host, median), "
               "wire %zu B\n", n, K, pct(us, .5), nb);
        wire = nb;
    } else {
    for (int i = 0; i < 2 * K; i++)
        if (drop_launch(buf, cap, nullptr, nbd, gs[i % NG], n, thr, s)) return 1;
    CK(hipStreamSynchronize(s));
    for (int i = 0; i < 8; i++) drop_launch(buf, cap, nullptr, nbd, gs[i % NG], n, thr, s);
    CK(hipEventRecord(a, s));
    for (int i = 0; i < K; i++) drop_launch(buf, cap, nullptr, nbd, gs[i % NG], n, thr, s);
    CK(hipEventRecord(b, s));
    CK(hipEventSynchronize(b));
    CK(hipEventElapsedTime(&ms, a, b));
    CK(hipMemcpy(&wire, nbd, 8, hipMemcpyDeviceToHost));
    const double per = ms * 1e3 / K, bytes = 4.0 * n + (double)wire;
    printf("# sp_phases: %zu values, %d stream-ordered drops over %d gradients, tiles/workgroup %zu: %.2f us per drop "
           "(events), wire %llu B, %.1f GB/s = %.3f of 8 TB/s\n",
           n, K, NG, kImageTpw, per, (unsigned long long)wire, bytes / per * 1e-3,
           bytes / per * 1e-3 / 8000.0);
    }
    const size_t ntiles = (n + kTile - 1) / kTile, nwg = (ntiles + kImageTpw - 1) / kImageTpw;
    if (drop_fused() && ntiles <= drop_one_launch_tiles()) {  // the one-launch encoder: per tile {start, look-back done, end} + ticket and image times
        std::vector<uint4> d1(ntiles), d1b(ntiles);
        CK(hipMemcpyFromSymbol(d1.data(), HIP_SYMBOL(g_sp_stamp_d1), ntiles * sizeof(uint4)));
        CK(hipMemcpyFromSymbol(d1b.data(), HIP_SYMBOL(g_sp_stamp_d1b), ntiles * sizeof(uint4)));
        uint32_t b = d1[0].x;
        for (const uint4 &v : d1) b = (int32_t)(v.x - b) < 0 ? v.x : b;
        printf("# times in us from sp_drop1's first workgroup start (the last drop; mid: look-back done)\n");
        report("sp_drop1", d1, b);
        std::vector<double> tk, img, lb, wr, dist;
        for (size_t i = 0; i < ntiles; i++) {
            tk.push_back(d1b[i].x * 0.01);
            img.push_back((d1b[i].y - d1b[i].x) * 0.01);
            lb.push_back(((double)d1[i].y - d1b[i].y) * 0.01);
            wr.push_back(((double)d1[i].z - d1[i].y) * 0.01);
            dist.push_back(std::fabs((double)d1b[i].z - (double)i));
        }
        printf("sp_drop1 ticket p50 %.2f p90 %.2f max %.2f | image p50 %.2f p90 %.2f max %.2f | look-back p50 %.2f p90 "
               "%.2f max %.2f | write p50 %.2f p90 %.2f max %.2f | |block - ticket| p50 %.0f max %.0f\n",
               pct(tk, .5), pct(tk, .9), pct(tk, 1), pct(img, .5), pct(img, .9), pct(img, 1), pct(lb, .5), pct(lb, .9),
               pct(lb, 1), pct(wr, .5), pct(wr, .9), pct(wr, 1), pct(dist, .5), pct(dist, 1));
        std::vector<double> l0, l1;
        for (size_t i = 1; i < ntiles; i++) {
            l0.push_back(((double)d1b[i].w - d1b[i].y) * 0.01);
            l1.push_back(((double)d1[i].y - d1b[i].w) * 0.01);
        }
        printf("sp_drop1 own-group look-back p50 %.2f p90 %.2f max %.2f | earlier groups p50 %.2f p90 %.2f max %.2f\n",
               pct(l0, .5), pct(l0, .9), pct(l0, 1), pct(l1, .5), pct(l1, .9), pct(l1, 1));
        {
            std::vector<uint4> d1c(ntiles);
            CK(hipMemcpyFromSymbol(d1c.data(), HIP_SYMBOL(g_sp_stamp_d1c), ntiles * sizeof(uint4)));
            std::vector<double> p0, p1, lat;
            for (size_t i = 1; i < ntiles; i++) {
                p0.push_back(d1c[i].x);
                p1.push_back(d1c[i].z);
                if (d1c[i].x + d1c[i].z) lat.push_back((d1c[i].y + d1c[i].w) * 0.01 / (d1c[i].x + d1c[i].z));
            }
            printf("sp_drop1 lane-0 polls own group p50 %.0f p90 %.0f max %.0f | earlier groups p50 %.0f p90 %.0f max %.0f | "
                   "per-poll load time p10 %.2f p50 %.2f p90 %.2f max %.2f us\n",
                   pct(p0, .5), pct(p0, .9), pct(p0, 1), pct(p1, .5), pct(p1, .9), pct(p1, 1), pct(lat, .1), pct(lat, .5),
                   pct(lat, .9), pct(lat, 1));
        }
        printf("sp_drop1 tile: start/imaged/own-group/done/end (us)");
        for (size_t i : {(size_t)0, (size_t)1, (size_t)63, (size_t)64, (size_t)127, (size_t)448, (size_t)511, (size_t)512,
                         (size_t)575, (size_t)1023, (size_t)1024, (size_t)2047, (size_t)2048, (size_t)4095, (size_t)4096}) {
            if (i >= ntiles) continue;
            const double st = (double)(uint32_t)(d1[i].x - b) * 0.01;
            printf(" %zu:%.1f/%.1f/%.1f/%.1f/%.1f", i, st, st + d1b[i].y * 0.01, st + d1b[i].w * 0.01, st + d1[i].y * 0.01,
                   st + d1[i].z * 0.01);
        }
        printf("\n");
        // the time line by tile index: start and end of every 512th tile
        printf("sp_drop1 tile:start/lookback/end");
        for (size_t i = 0; i < ntiles; i += std::max<size_t>(1, ntiles / 16))
            printf(" %zu:%.1f/%.1f/%.1f", i, (double)(uint32_t)(d1[i].x - b) * 0.01,
                   (double)(uint32_t)(d1[i].x - b) * 0.01 + d1[i].y * 0.01,
                   (double)(uint32_t)(d1[i].x - b) * 0.01 + d1[i].z * 0.01);
        printf("\n");
        return 0;
    }
    if (drop_emit()) {  // sp_count per workgroup (mid: its waves' values loaded), sp_emit per wave
        const size_t ncw = count_grid(ntiles);
        std::vector<uint4> sc(ncw), se(ntiles);
        CK(hipMemcpyFromSymbol(sc.data(), HIP_SYMBOL(g_sp_stamp_img), ncw * sizeof(uint4)));
        CK(hipMemcpyFromSymbol(se.data(), HIP_SYMBOL(g_sp_stamp_mov), ntiles * sizeof(uint4)));
        uint32_t base = sc[0].x;
        for (const uint4 &v : sc) base = (int32_t)(v.x - base) < 0 ? v.x : base;
        printf("# times in us from sp_count's first workgroup start (the last drop; sp_emit mid: its loads in)\n");
        report("sp_count", sc, base);
        report("sp_emit", se, base);
        return 0;
    }
    std::vector<uint4> si(nwg), sm(ntiles);
    CK(hipMemcpyFromSymbol(si.data(), HIP_SYMBOL(g_sp_stamp_img), nwg * sizeof(uint4)));
    CK(hipMemcpyFromSymbol(sm.data(), HIP_SYMBOL(g_sp_stamp_mov), ntiles * sizeof(uint4)));
    uint32_t base = si[0].x;
    for (const uint4 &v : si) base = (int32_t)(v.x - base) < 0 ? v.x : base;
    printf("# times in us from sp_image's first workgroup start (the last drop of the timed loop)\n");
    report("sp_image", si, base);
    report("sp_move", sm, base);

    // the stream-ordered lift (pattern path) of the last drop's wire, into 6 outputs in turn
    const size_t nb = (size_t)wire;
    std::vector<float *> outs(NG);
    for (int i = 0; i < NG; i++) CK(hipMalloc((void **)&outs[i], n * sizeof(float)));
    uint64_t *status, ticket = 0;
    CK(hipMalloc((void **)&status, 8));
    CK(hipMemset(status, 0, 8));
    for (int i = 0; i < 2 * K; i++)
        if (ono_sparse_lift_dev_async(outs[i % NG], n, buf, nb, status, &ticket, s)) return 1;
    CK(hipStreamSynchronize(s));
    for (int i = 0; i < 8; i++) ono_sparse_lift_dev_async(outs[i % NG], n, buf, nb, status, &ticket, s);
    CK(hipEventRecord(a, s));
    for (int i = 0; i < K; i++) ono_sparse_lift_dev_async(outs[i % NG], n, buf, nb, status, &ticket, s);
    CK(hipEventRecord(b, s));
    CK(hipEventSynchronize(b));
    CK(hipEventElapsedTime(&ms, a, b));
    uint64_t st = 0;
    CK(hipMemcpy(&st, status, 8, hipMemcpyDeviceToHost));
    const double lper = ms * 1e3 / K, lbytes = 4.0 * n + (double)nb;
    printf("# lift: %d stream-ordered lifts: %.2f us per lift (events), %.1f GB/s = %.3f of 8 TB/s, refused %d\n", K,
           lper, lbytes / lper * 1e-3, lbytes / lper * 1e-3 / 8000.0, (int)(st == ticket));
    const size_t T = ((nb - 8) / 2 + kPatU - 1) / kPatU;
    std::vector<uint4> spi(T), spp(T);
    CK(hipMemcpyFromSymbol(spi.data(), HIP_SYMBOL(g_sp_stamp_pli), T * sizeof(uint4)));
    CK(hipMemcpyFromSymbol(spp.data(), HIP_SYMBOL(g_sp_stamp_plp), T * sizeof(uint4)));
    // one launch (pl_fused, the default up to kPatDirect tiles) stamps only pl_place's array: start, after
    // its last stores issued, end
    const bool fused = spi[0].x == 0 && spi[0].z == 0;
    if (fused && T > 2048) spp.resize((T + 2) / 3);  // (three tiles per workgroup above 2048 tiles)
    const std::vector<uint4> &first = fused ? spp : spi;
    base = first[0].x;
    for (const uint4 &v : first) base = (int32_t)(v.x - base) < 0 ? v.x : base;
    if (fused) {
        printf("# times in us from pl_fused's first workgroup start (the last lift; mid: its last stores issued)\n");
        report("pl_fused", spp, base);
        const size_t nwg = spp.size();
        std::vector<uint4> plf(nwg);
        CK(hipMemcpyFromSymbol(plf.data(), HIP_SYMBOL(g_sp_stamp_plf), nwg * sizeof(uint4)));
        std::vector<double> r1;
        for (const uint4 &v : plf) r1.push_back(v.z * 0.01);
        printf("pl_fused first tile's look-back done: p10 %.2f p50 %.2f p90 %.2f max %.2f us from start\n", pct(r1, 0.1),
               pct(r1, 0.5), pct(r1, 0.9), pct(r1, 1));
    } else {
        printf("# times in us from pl_index's first workgroup start (the last lift; mid: pl_index after its scan, "
               "pl_place after its prologue)\n");
        report("pl_index", spi, base);
        report("pl_place", spp, base);
    }
    return 0;
}
