// cu_hog.hip (TEST INFRASTRUCTURE) — holds CU slots from another process for a
// bounded time: `cu_hog WGS MS` launches WGS one-wave workgroups, each taking
// the whole 160 KiB of a CU's LDS (so nothing else that uses LDS fits beside
// it), spinning on the wall clock for MS milliseconds; prints "running" once
// the kernel has started and "done" when it ends.  Used by
// tests/test_gpu_sparse_pattern.py to show that the one-launch lift's
// residency bound turns a grid that cannot become resident into a quick
// refusal instead of a ~10 ms poll.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>

__global__ void hog(uint64_t ticks, unsigned *started) {
    extern __shared__ unsigned lds[];
    if (threadIdx.x == 0) {
        lds[0] = blockIdx.x;
        __hip_atomic_fetch_add(started, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    const uint64_t t0 = wall_clock64();
    while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(127);
    if (lds[0] == 0xFFFFFFFFu) started[1] = 1;  // (keeps the LDS allocation live)
}

int main(int argc, char **argv) {
    const int wgs = argc > 1 ? atoi(argv[1]) : 192;
    const int ms = argc > 2 ? atoi(argv[2]) : 300;
    const size_t lds = 160 * 1024;
    if (hipFuncSetAttribute((const void *)hog, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess) {
        fprintf(stderr, "cannot request %zu B of LDS\n", lds);
        return 2;
    }
    unsigned *started = nullptr;
    if (hipHostMalloc((void **)&started, 2 * sizeof(unsigned), hipHostMallocMapped | hipHostMallocCoherent) !=
        hipSuccess)
        return 2;
    started[0] = started[1] = 0;
    unsigned *dev = nullptr;
    (void)hipHostGetDevicePointer((void **)&dev, started, 0);
    hipLaunchKernelGGL(hog, dim3(wgs), dim3(64), lds, 0, (uint64_t)ms * 100000ull, dev);
    if (hipGetLastError() != hipSuccess) return 3;
    const auto t0 = std::chrono::steady_clock::now();
    while (*(volatile unsigned *)&started[0] < (unsigned)wgs &&
           std::chrono::steady_clock::now() - t0 < std::chrono::milliseconds(ms))
        std::this_thread::sleep_for(std::chrono::microseconds(50));
    printf("running %u\n", *(volatile unsigned *)&started[0]);
    fflush(stdout);
    if (hipDeviceSynchronize() != hipSuccess) return 4;
    printf("done\n");
    return 0;
}
