// Calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE on gfx950 for the access patterns of the encode
// pipeline's kernels (MI355X_MICROARCH.md: FETCH_SIZE reports half the bytes of a 16 B/lane streaming
// read; other widths are uncalibrated).  Each kernel moves a known number of bytes of a 2 GiB buffer
// (8x the Infinity Cache, so the reads reach HBM), and prints it; tools/pmc_calib.py divides the
// counters of each dispatch by it.
//   build: hipcc -O3 --offload-arch=gfx950 tools/fetch_calib.hip -o tools/fetch_calib
//   run:   rocprofv3 --pmc FETCH_SIZE -- tools/fetch_calib   (and WRITE_SIZE, TCC_EA0_RDREQ... passes)
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

static constexpr size_t BUF = 2ull << 30;  // 2 GiB
static constexpr uint32_t GRID = 2048, BLK = 256;

// streaming reads: every byte of [0, n) once, W bytes per lane per access, coalesced
template <int W>
__global__ __launch_bounds__(BLK) void c_read(const uint8_t *p, size_t n, uint32_t *sink)
{
    uint32_t acc = 0;
    const size_t stride = (size_t)GRID * BLK * W;
    for (size_t o = ((size_t)blockIdx.x * BLK + threadIdx.x) * W; o < n; o += stride) {
        if (W == 32) {
            const uint4 a = *(const uint4 *)(p + o), b = *(const uint4 *)(p + o + 16);
            acc += a.x ^ a.y ^ a.z ^ a.w ^ b.x ^ b.y ^ b.z ^ b.w;
        } else if (W == 16) {
            const uint4 a = *(const uint4 *)(p + o);
            acc += a.x ^ a.y ^ a.z ^ a.w;
        } else if (W == 8) {
            const uint2 a = *(const uint2 *)(p + o);
            acc += a.x ^ a.y;
        } else if (W == 4) {
            acc += *(const uint32_t *)(p + o);
        } else {
            acc += p[o];
        }
    }
    if (acc == 0x12345678u) sink[0] = acc;  // (never: keeps the loads)
}

// random gathers: `count` accesses of W bytes at W-aligned addresses spread over the buffer (a
// multiplicative walk; distinct 128-byte lines with high probability)
template <int W>
__global__ __launch_bounds__(BLK) void c_gather(const uint8_t *p, uint32_t per_thread, uint32_t *sink)
{
    uint64_t x = ((uint64_t)blockIdx.x * BLK + threadIdx.x) * 0x9E3779B97F4A7C15ull + 1;
    uint32_t acc = 0;
    for (uint32_t i = 0; i < per_thread; i++) {
        x = x * 6364136223846793005ull + 1442695040888963407ull;
        const size_t o = ((x >> 20) % (BUF / 128)) * 128;  // a line's first W bytes
        if (W == 16) {
            const uint4 a = *(const uint4 *)(p + o);
            acc += a.x ^ a.y ^ a.z ^ a.w;
        } else if (W == 8) {
            const uint2 a = *(const uint2 *)(p + o);
            acc += a.x ^ a.y;
        } else {
            acc += *(const uint32_t *)(p + o);
        }
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

// streaming writes: every byte of [0, n) once, W bytes per lane
template <int W>
__global__ __launch_bounds__(BLK) void c_write(uint8_t *p, size_t n)
{
    const size_t stride = (size_t)GRID * BLK * W;
    for (size_t o = ((size_t)blockIdx.x * BLK + threadIdx.x) * W; o < n; o += stride) {
        if (W == 16) *(uint4 *)(p + o) = make_uint4((uint32_t)o, 1, 2, 3);
        else if (W == 8) *(uint2 *)(p + o) = make_uint2((uint32_t)o, 1);
        else if (W == 4) *(uint32_t *)(p + o) = (uint32_t)o;
        else p[o] = (uint8_t)o;
    }
}

int main()
{
    uint8_t *p;
    uint32_t *sink;
    if (hipMalloc(&p, BUF) != hipSuccess || hipMalloc(&sink, 4) != hipSuccess) return 1;
    hipMemset(p, 7, BUF);
    hipDeviceSynchronize();
    const size_t n = 1ull << 30;  // 1 GiB read or written per streaming dispatch
    const uint32_t per = 64;      // gathers per thread: GRID * BLK * 64 = 33.5 M accesses
    const double g = (double)GRID * BLK * per;
    printf("kernel,known_bytes,what\n");
    hipLaunchKernelGGL(c_read<32>, dim3(GRID), dim3(BLK), 0, 0, p, n, sink);
    printf("c_read<32>,%zu,32 B per lane (two 16-B loads)\n", n);
    hipLaunchKernelGGL(c_read<16>, dim3(GRID), dim3(BLK), 0, 0, p + n, n, sink);
    printf("c_read<16>,%zu,16 B per lane\n", n);
    hipLaunchKernelGGL(c_read<8>, dim3(GRID), dim3(BLK), 0, 0, p, n, sink);
    printf("c_read<8>,%zu,8 B per lane\n", n);
    hipLaunchKernelGGL(c_read<4>, dim3(GRID), dim3(BLK), 0, 0, p + n, n, sink);
    printf("c_read<4>,%zu,4 B per lane\n", n);
    hipLaunchKernelGGL(c_read<1>, dim3(GRID), dim3(BLK), 0, 0, p, n / 4, sink);
    printf("c_read<1>,%zu,1 B per lane\n", n / 4);
    hipLaunchKernelGGL(c_gather<16>, dim3(GRID), dim3(BLK), 0, 0, p, per, sink);
    printf("c_gather<16>,%.0f,random 16-B reads (bytes used; one 128-B line each)\n", g * 16);
    hipLaunchKernelGGL(c_gather<8>, dim3(GRID), dim3(BLK), 0, 0, p, per, sink);
    printf("c_gather<8>,%.0f,random 8-B reads (bytes used; one 128-B line each)\n", g * 8);
    hipLaunchKernelGGL(c_gather<4>, dim3(GRID), dim3(BLK), 0, 0, p, per, sink);
    printf("c_gather<4>,%.0f,random 4-B reads (bytes used; one 128-B line each)\n", g * 4);
    hipLaunchKernelGGL(c_write<16>, dim3(GRID), dim3(BLK), 0, 0, p, n);
    printf("c_write<16>,%zu,16 B per lane\n", n);
    hipLaunchKernelGGL(c_write<8>, dim3(GRID), dim3(BLK), 0, 0, p + n, n);
    printf("c_write<8>,%zu,8 B per lane\n", n);
    hipLaunchKernelGGL(c_write<4>, dim3(GRID), dim3(BLK), 0, 0, p, n);
    printf("c_write<4>,%zu,4 B per lane\n", n);
    hipLaunchKernelGGL(c_write<1>, dim3(GRID), dim3(BLK), 0, 0, p + n, n / 4);
    printf("c_write<1>,%zu,1 B per lane\n", n / 4);
    printf("gathers,%.0f,accesses per gather kernel\n", g);
    return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
