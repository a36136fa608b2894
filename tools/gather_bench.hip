// Microbenchmark: random 8-byte gathers from a table of T bytes (L2- or MALL-resident),
// one per lane per position, versus LDS random ds_read_b64 of a 128 KB table.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ __launch_bounds__(1024) void g_gather(const uint2 *tab, uint32_t mask, uint32_t iters, uint32_t *out)
{
    uint32_t x = blockIdx.x * 1024u + threadIdx.x, acc = 0;
    for (uint32_t i = 0; i < iters; i++) {
        x = x * 1664525u + 1013904223u;
        uint2 w = tab[(x >> 8) & mask];
        acc += w.x ^ w.y;
    }
    out[blockIdx.x * 1024u + threadIdx.x] = acc;
}
__global__ __launch_bounds__(1024) void g_lds(const uint2 *tab, uint32_t iters, uint32_t *out)
{
    __shared__ uint2 f[16384];
    for (uint32_t i = threadIdx.x; i < 16384; i += 1024) f[i] = tab[i];
    __syncthreads();
    uint32_t x = blockIdx.x * 1024u + threadIdx.x, acc = 0;
    for (uint32_t i = 0; i < iters; i++) {
        x = x * 1664525u + 1013904223u;
        uint2 w = f[(x >> 8) & 16383u];
        acc += w.x ^ w.y;
    }
    out[blockIdx.x * 1024u + threadIdx.x] = acc;
}
int main()
{
    uint2 *tab; uint32_t *out;
    hipMalloc(&tab, 256u << 20); hipMemset(tab, 1, 256u << 20);
    hipMalloc(&out, 256 * 1024 * 4);
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    const uint32_t iters = 4096;
    for (uint32_t kb : {256u, 1024u, 2048u, 4096u, 16384u, 65536u, 262144u}) {
        uint32_t words = kb * 1024u / 8u;
        hipLaunchKernelGGL(g_gather, dim3(256), dim3(1024), 0, 0, tab, words - 1, 64u, out);
        hipEventRecord(a);
        hipLaunchKernelGGL(g_gather, dim3(256), dim3(1024), 0, 0, tab, words - 1, iters, out);
        hipEventRecord(b); hipEventSynchronize(b);
        float ms; hipEventElapsedTime(&ms, a, b);
        double n = 256.0 * 1024 * iters;
        printf("global table %7u KB: %.3f ms  %.1f G gathers/s\n", kb, ms, n / ms / 1e6);
    }
    hipLaunchKernelGGL(g_lds, dim3(256), dim3(1024), 0, 0, tab, 64u, out);
    hipEventRecord(a);
    hipLaunchKernelGGL(g_lds, dim3(256), dim3(1024), 0, 0, tab, iters, out);
    hipEventRecord(b); hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    printf("LDS 128 KB table: %.3f ms  %.1f G reads/s\n", ms, 256.0 * 1024 * iters / ms / 1e6);
    return 0;
}
