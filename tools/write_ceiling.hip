// write_ceiling — how long the drop's wire write (15 MB, one ~1.9 KB range per 2048-value tile, the
// ranges back to back at 2-B granularity) takes on its own: (a) a coalesced 16-B fill of the same
// bytes by a grid-stride kernel, (b) one wave per range as sp_emit stores it (16-B chunks of the
// destination; the two chunks shared with the neighbours unit by unit), (c) (b) with every range
// 16-B aligned (no shared chunks).  One event pair around K launches each.
// usage: write_ceiling [tiles=8192] [units_per_tile=941]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)
typedef unsigned u4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void fill16(u4 *p, size_t n16) {
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256)
        __builtin_nontemporal_store(u4{1u, 2u, 3u, 4u}, p + i);
}
// wave t writes units [t * U, t * U + U) of a u16 array (ALIGN: [t * U16, ...) with U16 = U rounded up to 8)
template <bool ALIGN>
__global__ __launch_bounds__(256) void ranges(uint16_t *w, size_t ntiles, unsigned U) {
    const size_t t = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const unsigned lane = threadIdx.x & 63;
    if (t >= ntiles) return;
    const size_t U16 = ALIGN ? (U + 7) / 8 * 8 : U;
    const size_t u0 = t * U16, u1 = u0 + U;
    const size_t c0 = u0 / 8, c1 = (u1 + 7) / 8;  // destination chunks touched
    for (size_t c = c0 + lane; c < c1; c += 64) {
        const bool whole = c * 8 >= u0 && c * 8 + 8 <= u1;
        if (whole) __builtin_nontemporal_store(u4{5u, 6u, 7u, 8u}, (u4 *)(w + 8 * c));
        else
            for (int i = 0; i < 8; i++) {
                const size_t u = c * 8 + i;
                if (u >= u0 && u < u1) w[u] = (uint16_t)u;
            }
    }
}

__global__ __launch_bounds__(512) void empty512(uint16_t *w) { if (threadIdx.x == 1023) w[0] = 0; }
__global__ __launch_bounds__(1024) void empty1024(uint16_t *w) { if (threadIdx.x == 2047) w[0] = 0; }

int main(int argc, char **argv) {
    const size_t ntiles = argc > 1 ? atoi(argv[1]) : 8192;
    const unsigned U = argc > 2 ? atoi(argv[2]) : 941;
    const size_t bytes = ntiles * ((U + 7) / 8 * 8) * 2 + 64;
    const int K = 24, NB = 6;
    uint16_t *b[NB];
    for (auto &p : b) { CK(hipMalloc((void **)&p, bytes)); CK(hipMemset(p, 0, bytes)); }
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    auto run = [&](const char *name, auto launch) {
        for (int i = 0; i < 12; i++) launch(b[i % NB]);
        CK(hipEventRecord(e0));
        for (int i = 0; i < K; i++) launch(b[i % NB]);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        const double us = ms * 1e3 / K, mb = ntiles * (double)U * 2;
        printf("%-40s %7.2f us per launch  %5.2f TB/s (%.1f MB)\n", name, us, mb / us * 1e-6, mb * 1e-6);
    };
    const size_t n16 = ntiles * (size_t)U * 2 / 16;
    for (int k : {4, 8}) {
        char nm[64];
        snprintf(nm, 64, "coalesced fill, %d wg/CU", k);
        run(nm, [&](uint16_t *p) { hipLaunchKernelGGL(fill16, dim3(cus * k), dim3(256), 0, 0, (u4 *)p, n16); });
    }
    run("wave per range, back to back (emit)", [&](uint16_t *p) {
        hipLaunchKernelGGL(ranges<false>, dim3((ntiles + 3) / 4), dim3(256), 0, 0, p, ntiles, U); });
    run("wave per range, 16-B aligned ranges", [&](uint16_t *p) {
        hipLaunchKernelGGL(ranges<true>, dim3((ntiles + 3) / 4), dim3(256), 0, 0, p, ntiles, U); });
    run("empty kernel, same grid", [&](uint16_t *p) {
        hipLaunchKernelGGL(ranges<false>, dim3((ntiles + 3) / 4), dim3(256), 0, 0, p, 0, U); });
    run("empty kernel, half the workgroups x 512", [&](uint16_t *p) {
        hipLaunchKernelGGL(empty512, dim3((ntiles + 7) / 8), dim3(512), 0, 0, p); });
    run("empty kernel, a quarter x 1024", [&](uint16_t *p) {
        hipLaunchKernelGGL(empty1024, dim3((ntiles + 15) / 16), dim3(1024), 0, 0, p); });
    run("empty kernel, 1 workgroup", [&](uint16_t *p) {
        hipLaunchKernelGGL(ranges<false>, dim3(1), dim3(256), 0, 0, p, 0, U); });
    return 0;
}
