// Host cost of hipLaunchKernelGGL against the kernel-argument size (the pipeline's argument blocks
// are 700-930 bytes): N back-to-back launches of a trivial kernel on one stream, host time per
// launch and the drain time per kernel.  usage: ./launch_bench   (built: hipcc -O2 --offload-arch=gfx950)
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

template <int N>
struct Args {
    unsigned long long w[N / 8];
};
template <int N>
__global__ void k_touch(Args<N> a, unsigned *out)
{
    if (a.w[0] == 12345ull && threadIdx.x == 0) out[blockIdx.x] = 1u;
}

template <int N>
static void run(hipStream_t s, unsigned *out, int iters, int grid)
{
    Args<N> a{};
    for (int i = 0; i < 50; i++) hipLaunchKernelGGL(k_touch<N>, dim3(grid), dim3(256), 0, s, a, out);
    hipStreamSynchronize(s);
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < iters; i++) {
        a.w[1] = (unsigned long long)i;
        hipLaunchKernelGGL(k_touch<N>, dim3(grid), dim3(256), 0, s, a, out);
    }
    const auto t1 = std::chrono::steady_clock::now();
    hipStreamSynchronize(s);
    const auto t2 = std::chrono::steady_clock::now();
    const double h = std::chrono::duration<double, std::micro>(t1 - t0).count() / iters;
    const double d = std::chrono::duration<double, std::micro>(t2 - t0).count() / iters;
    std::printf("args %5d B grid %5d: host %.2f us/launch, launch..drain %.2f us/kernel\n", N, grid, h, d);
}

int main()
{
    hipStream_t s;
    hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    unsigned *out;
    hipMalloc(&out, 4096 * 4);
    for (int grid : {1, 256, 1024}) {
        run<16>(s, out, 4000, grid);
        run<256>(s, out, 4000, grid);
        run<768>(s, out, 4000, grid);
        run<1024>(s, out, 4000, grid);
        run<2048>(s, out, 4000, grid);
    }
    hipFree(out);
    return 0;
}
