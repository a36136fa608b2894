// Dependent-launch gaps on one stream (DESIGN §4 "next factors" (6)): the idle time between two
// kernels of the context stream as a function of the kernel-argument size, whether the arguments
// change between launches, the first kernel's grid and how much it wrote.  Run under
//   rocprofv3 --kernel-trace -d DIR -o gap -- ./gap_bench
// and read the gaps with tools/gap_summary.py.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

struct Big { uint64_t w[100]; };  // 800 bytes, like the pipeline's argument structs

template <int P> __global__ void k_small(uint32_t *p, uint32_t v) { if (threadIdx.x == 0 && blockIdx.x == 0 && v == 0xFFFFFFFFu) p[P] = v; }
template <int P> __global__ void k_big(Big b, uint32_t *p) { if (threadIdx.x == 0 && blockIdx.x == 0 && b.w[99] == 0xFFFFFFFFu) p[0] = P; }
__global__ void k_big2(Big b, uint32_t *p) { if (threadIdx.x == 0 && blockIdx.x == 0 && b.w[98] == 0xFFFFFFFFu) p[0] = 2; }
__global__ void k_write(uint4 *p, size_t n)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        p[i] = make_uint4((uint32_t)i, 1, 2, 3);
}
// holds the stream for ~2 ms so that the host has enqueued a whole phase before it runs (the gaps
// measured behind it are the device's, not the host's launch rate)
__global__ void k_spin(long long cycles)
{
    const long long t0 = wall_clock64();
    while (wall_clock64() - t0 < cycles) __builtin_amdgcn_s_sleep(8);
}
__global__ void k_grid(uint32_t *p, uint32_t v) { if (v == 0xFFFFFFFFu) p[blockIdx.x] = v; }

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

int main()
{
    uint32_t *d;
    uint4 *w;
    const size_t nw = (64u << 20) / sizeof(uint4);
    CK(hipMalloc(&d, 4096));
    CK(hipMalloc(&w, nw * sizeof(uint4)));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipStream_t hs;
    CK(hipStreamCreateWithFlags(&hs, hipStreamNonBlocking));
    hipEvent_t ev;
    CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    uint4 *w2;
    CK(hipMalloc(&w2, nw * sizeof(uint4)));
    Big b{};
    // warm up every kernel
    k_small<0><<<1, 64, 0, s>>>(d, 0);
    k_small<5><<<1, 64, 0, s>>>(d, 0);
    k_small<6><<<1, 64, 0, s>>>(d, 0);
    k_small<7><<<1, 64, 0, s>>>(d, 0);
    k_big<1><<<1, 64, 0, s>>>(b, d);
    k_big<2><<<1, 64, 0, s>>>(b, d);
    k_big<3><<<1, 64, 0, s>>>(b, d);
    k_big2<<<1, 64, 0, s>>>(b, d);
    k_write<<<1024, 256, 0, s>>>(w, nw);
    k_grid<<<4096, 256, 0, s>>>(d, 0);
    CK(hipStreamSynchronize(s));
    // each phase enqueued whole before it runs: a long head kernel keeps the host ahead
    for (int phase = 0; phase < 8; phase++) {
        k_spin<<<1, 64, 0, s>>>(200000);  // 2 ms at the 100 MHz wall clock
        k_write<<<1024, 256, 0, s>>>(w, nw);
        if (phase == 7)  // another stream's long kernel beside the chain
            for (int r = 0; r < 8; r++) k_write<<<256, 256, 0, hs>>>(w2, nw);  // head: 64 MiB written (the host enqueues behind it)
        for (int i = 0; i < 20; i++) {
            switch (phase) {
            case 0: k_small<0><<<1, 64, 0, s>>>(d, (uint32_t)i); break;          // 12-byte args
            case 1: b.w[0] = (uint64_t)i; k_big<1><<<1, 64, 0, s>>>(b, d); break; // 800 bytes, changing
            case 2: k_big<2><<<1, 64, 0, s>>>(b, d); break;                       // 800 bytes, the same
            case 3:  // alternating kernels, the same 800 bytes
                if (i & 1) k_big2<<<1, 64, 0, s>>>(b, d); else k_big<3><<<1, 64, 0, s>>>(b, d);
                break;
            case 4: k_grid<<<4096, 256, 0, s>>>(d, (uint32_t)i); break;       // wide grid
            case 5:  // a kernel that wrote 64 MiB before each small one
                k_write<<<1024, 256, 0, s>>>(w, nw);
                k_small<5><<<1, 64, 0, s>>>(d, (uint32_t)i);
                break;
            case 6:  // an event recorded after each kernel (a marker packet between them)
                k_small<6><<<1, 64, 0, s>>>(d, (uint32_t)i);
                CK(hipEventRecord(ev, s));
                break;
            case 7: k_small<7><<<1, 64, 0, s>>>(d, (uint32_t)i); break;
            }
        }
        CK(hipStreamSynchronize(s));
        CK(hipStreamSynchronize(hs));
    }
    CK(hipGetLastError());
    printf("done\n");
    return 0;
}
