// read_ceiling — how fast one kernel can read a 64 MiB gradient, from HBM (6 buffers in turn: 384 MiB
// > the 256 MiB Infinity Cache) and from the cache (one buffer again): the floor sp_count's read sits on.
// Shapes: coalesced grid-stride float4 (k workgroups per CU), and the count's lane-per-128-B shape.
// usage: read_ceiling [MiB=64]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)
typedef float f4 __attribute__((ext_vector_type(4)));

// coalesced: consecutive lanes read consecutive 16 B, grid-stride, U vectors per thread per step
template <int U>
__global__ __launch_bounds__(256) void rd_coal(const f4 *__restrict__ g, size_t n4, float t, unsigned *out) {
    unsigned c = 0;
    const size_t stride = (size_t)gridDim.x * 256 * U;
    for (size_t i = (size_t)blockIdx.x * 256 * U + threadIdx.x; i < n4; i += stride) {
        f4 v[U];
#pragma unroll
        for (int u = 0; u < U; u++) v[u] = i + 256 * u < n4 ? g[i + 256 * u] : f4{0, 0, 0, 0};
#pragma unroll
        for (int u = 0; u < U; u++) c += (fabsf(v[u].x) >= t) + (fabsf(v[u].y) >= t) + (fabsf(v[u].z) >= t) + (fabsf(v[u].w) >= t);
    }
    if (c == 0xFFFFFFFFu) out[0] = c;
}
// the count's shape: a wave per 2048-value tile, lane l reads values 32 l .. 32 l + 31 (8 x 16 B)
__global__ __launch_bounds__(256) void rd_lane(const f4 *__restrict__ g, size_t ntiles, float t, unsigned *out) {
    unsigned c = 0;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (size_t tile = (size_t)blockIdx.x * 4 + wave; tile < ntiles; tile += (size_t)gridDim.x * 4) {
        const f4 *p = g + tile * 512 + lane * 8;
        f4 v[8];
#pragma unroll
        for (int q = 0; q < 8; q++) v[q] = p[q];
#pragma unroll
        for (int q = 0; q < 8; q++) c += (fabsf(v[q].x) >= t) + (fabsf(v[q].y) >= t) + (fabsf(v[q].z) >= t) + (fabsf(v[q].w) >= t);
    }
    if (c == 0xFFFFFFFFu) out[0] = c;
}

int main(int argc, char **argv) {
    const size_t mib = argc > 1 ? atoi(argv[1]) : 64, n = mib << 18, n4 = n / 4, ntiles = n / 2048;
    const int NB = 6, K = 24;
    std::vector<f4 *> b(NB);
    for (auto &p : b) { CK(hipMalloc((void **)&p, n * 4)); CK(hipMemset(p, 0x3f, n * 4)); }
    unsigned *out;
    CK(hipMalloc((void **)&out, 4));
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    auto run = [&](const char *name, int rot, auto launch) {
        for (int i = 0; i < 12; i++) launch(b[i % rot]);
        CK(hipEventRecord(e0));
        for (int i = 0; i < K; i++) launch(b[i % rot]);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        const double us = ms * 1e3 / K;
        printf("%-28s %s  %7.2f us per read  %5.2f TB/s\n", name, rot > 1 ? "HBM  " : "cache", us, n * 4.0 / us * 1e-6);
    };
    for (int rot : {NB, 1}) {
        for (int k : {2, 4, 8}) {
            char nm[64];
            snprintf(nm, 64, "coalesced U=4 %d wg/CU", k);
            run(nm, rot, [&](f4 *p) { hipLaunchKernelGGL(rd_coal<4>, dim3(cus * k), dim3(256), 0, 0, p, n4, 0.9f, out); });
            snprintf(nm, 64, "coalesced U=1 %d wg/CU", k);
            run(nm, rot, [&](f4 *p) { hipLaunchKernelGGL(rd_coal<1>, dim3(cus * k), dim3(256), 0, 0, p, n4, 0.9f, out); });
            snprintf(nm, 64, "lane-128B %d wg/CU", k);
            run(nm, rot, [&](f4 *p) { hipLaunchKernelGGL(rd_lane, dim3(cus * k), dim3(256), 0, 0, p, ntiles, 0.9f, out); });
        }
        run("coalesced U=1 one-shot", rot, [&](f4 *p) { hipLaunchKernelGGL(rd_coal<1>, dim3((n4 + 255) / 256), dim3(256), 0, 0, p, n4, 0.9f, out); });
        run("lane-128B one-shot", rot, [&](f4 *p) { hipLaunchKernelGGL(rd_lane, dim3(ntiles / 4), dim3(256), 0, 0, p, ntiles, 0.9f, out); });
    }
    return 0;
}
