// empty_launch.hip -- what a follow-on launch that exits at once costs a
// stream: K iterations of a ~50 us busy kernel (one workgroup of 768
// threads per CU, 153 KB of LDS, like the codec kernels), alone and each
// followed by an early-exit kernel of the same grid (every wave reads one
// flag word and leaves), or of a one-workgroup grid.  Wall time per
// iteration from events around the K iterations.
// Build: hipcc -O3 --offload-arch=gfx950 -o empty_launch empty_launch.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ __launch_bounds__(768) void busy(unsigned *out, unsigned iters)
{
    __shared__ unsigned lds[38000];
    unsigned v = threadIdx.x;
    for (unsigned i = 0; i < iters; ++i)
    {
        lds[(v * 7 + i) % 38000] = v;
        v = v * 1664525u + lds[(v + i * 13) % 38000];
    }
    if (v == 0x12345678u)
        out[0] = v;
}

__global__ __launch_bounds__(768) void early(const unsigned *flag, unsigned *out)
{
    __shared__ unsigned lds[38000];
    if (__builtin_expect(flag[0] == 0, 1))
        return;
    lds[threadIdx.x] = 1;
    __syncthreads();
    out[blockIdx.x] = lds[threadIdx.x ^ 1];
}

int main()
{
    int ncu = 0;
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    unsigned *buf;
    hipMalloc(&buf, 1 << 20);
    hipMemset(buf, 0, 1 << 20);
    hipStream_t st;
    hipStreamCreate(&st);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const int K = 200;
    for (unsigned iters : {4000u, 8000u})
        for (int mode = 0; mode < 3; ++mode)
        {
            for (int w = 0; w < 2; ++w)
            {
                hipEventRecord(a, st);
                for (int k = 0; k < K; ++k)
                {
                    hipLaunchKernelGGL(busy, dim3(ncu), dim3(768), 0, st, buf + 64, iters);
                    if (mode == 1)
                        hipLaunchKernelGGL(early, dim3(ncu), dim3(768), 0, st, buf, buf + 1024);
                    if (mode == 2)
                        hipLaunchKernelGGL(early, dim3(1), dim3(768), 0, st, buf, buf + 1024);
                }
                hipEventRecord(b, st);
                hipEventSynchronize(b);
                float ms = 0;
                hipEventElapsedTime(&ms, a, b);
                if (w)
                    printf("busy iters %u, follow-on %s: %.2f us per iteration\n", iters,
                           mode == 0 ? "none" : mode == 1 ? "early-exit, full grid"
                                                         : "early-exit, 1 workgroup",
                           1e3 * ms / K);
            }
        }
    return 0;
}
