// Microbenchmark: device-scope atomic claim throughput / latency on MI355X.
// Each wave does K dependent fetch_adds (lane 0) on counter (wave % NC) *
// stride; reports total kernel time and per-atomic latency per wave.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

__global__ void claims(unsigned *ctr, int nc, int k, unsigned long long *lat)
{
    const unsigned gid = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
    unsigned *c = ctr + (gid % nc) * 64;
    unsigned v = 0;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < k; ++i)
    {
        unsigned r = 0;
        if ((threadIdx.x & 63) == 0)
            r = __hip_atomic_fetch_add(c + (v & 0), 1u, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
        v += __builtin_amdgcn_readfirstlane(r);
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if ((threadIdx.x & 63) == 0)
        lat[gid] = (t1 - t0) / k + (v == 0xffffffffu);
}

__global__ void polls(unsigned long long *flags, int k, unsigned long long *lat)
{
    const unsigned gid = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
    unsigned long long v = 0;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < k; ++i)
    {
        unsigned idx = (gid * 7 + i * 64 + (threadIdx.x & 63) + (unsigned) (v & 1)) & 16383;
        v += __hip_atomic_load(&flags[idx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if ((threadIdx.x & 63) == 0)
        lat[gid] = (t1 - t0) / k + (v == 12345);
}

int main()
{
    unsigned *ctr;
    unsigned long long *lat, *flags;
    const int blocks = 256, threads = 768, waves = blocks * threads / 64;
    hipMalloc(&ctr, 64 * 64 * 4 * 8);
    hipMalloc(&lat, waves * 8);
    hipMalloc(&flags, 16384 * 8);
    hipMemset(flags, 0, 16384 * 8);
    unsigned long long *h = (unsigned long long *) malloc(waves * 8);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    int ncs[] = {1, 8, 64, 512};
    for (int ki = 0; ki < 2; ++ki)
    for (int nci = 0; nci < 4; ++nci)
    {
        int nc = ncs[nci], k = ki ? 16 : 4;
        for (int rep = 0; rep < 3; ++rep)
        {
            hipMemset(ctr, 0, 64 * 64 * 4 * 8);
            hipEventRecord(e0);
            hipLaunchKernelGGL(claims, dim3(blocks), dim3(threads), 0, 0, ctr, nc, k, lat);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
        }
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        hipMemcpy(h, lat, waves * 8, hipMemcpyDeviceToHost);
        double s = 0; unsigned long long mx = 0;
        for (int i = 0; i < waves; ++i) { s += h[i]; if (h[i] > mx) mx = h[i]; }
        printf("claims: counters %3d, %2d per wave (%d total): kernel %7.1f us, per-atomic latency mean %6.0f max %6llu cyc\n",
               nc, k, k * waves, ms * 1e3, s / waves, mx);
    }
    for (int k = 1; k <= 16; k *= 4)
    {
        for (int rep = 0; rep < 3; ++rep)
        {
            hipEventRecord(e0);
            hipLaunchKernelGGL(polls, dim3(blocks), dim3(threads), 0, 0, flags, k, lat);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
        }
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        hipMemcpy(h, lat, waves * 8, hipMemcpyDeviceToHost);
        double s = 0; unsigned long long mx = 0;
        for (int i = 0; i < waves; ++i) { s += h[i]; if (h[i] > mx) mx = h[i]; }
        printf("polls: %2d dependent 64-lane agent loads per wave: kernel %7.1f us, latency mean %6.0f max %6llu cyc\n",
               k, ms * 1e3, s / waves, mx);
    }
    // empty-ish kernel launch time
    for (int rep = 0; rep < 3; ++rep)
    {
        hipEventRecord(e0);
        hipLaunchKernelGGL(claims, dim3(blocks), dim3(threads), 0, 0, ctr, 64, 0, lat);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
    }
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    printf("empty kernel (256 x 768): %.1f us\n", ms * 1e3);
    return 0;
}
