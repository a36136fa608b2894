// Microbenchmark: k_blockhash-style hashing of every aligned 2048-byte block of a 512 MiB arena
// (cfg5 sub-batch size) alone on the GPU, in variants of the load/compute structure.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -o tools/bh_bench tools/bh_bench.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#include "../wanproxy_amd/csrc/xc_device.h"

using namespace xc;

constexpr int BLK = 8;

// MODE 0: as k_blockhash (one-shot wave, 8 blocks, all 16 loads then the hash)
// MODE 1: loads only (xor of the words)
// MODE 2: nontemporal loads + hash
// MODE 3: compute only (no loads: registers from the lane id)
// MODE 4: two groups per wave, the second group's loads issued before the first is hashed
// MODE 5: persistent waves (grid = PER_CU workgroups per CU) striding over the groups, the next
//         group's loads in flight while the current one is hashed
template <int MODE, int WAVES>
__global__ __launch_bounds__(64 * WAVES) void k_bh(const uint8_t *in, uint32_t ngroups, uint64_t *out)
{
    const uint32_t per = MODE == 4 ? 2u : 1u;
    const uint32_t g0 = (blockIdx.x * WAVES + (threadIdx.x >> 6)) * per;
    if (g0 >= ngroups) return;
    const uint32_t l = lane_id();
    if (MODE == 5) {
        const uint32_t stride = gridDim.x * WAVES;
        uint32_t g = g0;
        uint32_t x[BLK][8], xn[BLK][8];
        auto load = [&](uint32_t gg, uint32_t y[BLK][8]) {
            const uint8_t *p = in + (size_t)gg * BLK * XC_SEG;
#pragma unroll
            for (int i = 0; i < BLK; i++) {
                const uint4 *q = (const uint4 *)(p + (size_t)i * XC_SEG + 32u * l);
                const uint4 a = q[0], b = q[1];
                y[i][0] = a.x; y[i][1] = a.y; y[i][2] = a.z; y[i][3] = a.w;
                y[i][4] = b.x; y[i][5] = b.y; y[i][6] = b.z; y[i][7] = b.w;
            }
        };
        load(g, x);
        for (;;) {
            const uint32_t gn = g + stride < ngroups ? g + stride : g;
            load(gn, xn);
            const uint64_t h = block_group_hash<BLK>(x);
            if (l < BLK) out[(size_t)g * BLK + l] = h;
            if (gn == g) break;
            g = gn;
#pragma unroll
            for (int i = 0; i < BLK; i++)
#pragma unroll
                for (int k = 0; k < 8; k++) x[i][k] = xn[i][k];
        }
        return;
    }
    uint32_t w[BLK][8];
    (void)w;
    if (MODE == 3) {
        uint32_t v[BLK][8];
        for (int i = 0; i < BLK; i++)
            for (int k = 0; k < 8; k++) v[i][k] = (g0 * 0x9E3779B1u) ^ (l * 0x85EBCA6Bu) ^ (uint32_t)(i * 8 + k);
        const uint64_t h = block_group_hash<BLK>(v);
        if (l < BLK) out[(size_t)g0 * BLK + l] = h;
        return;
    }
    for (uint32_t r = 0; r < per; r++) {
        const uint32_t g = g0 + r;
        const uint8_t *p = in + (size_t)g * BLK * XC_SEG;
        uint32_t x[BLK][8];
#pragma unroll
        for (int i = 0; i < BLK; i++) {
            typedef uint32_t v4u __attribute__((ext_vector_type(4)));
            const v4u *q = (const v4u *)(p + (size_t)i * XC_SEG + 32u * l);
            v4u a, b;
            if (MODE == 2) { a = __builtin_nontemporal_load(q); b = __builtin_nontemporal_load(q + 1); }
            else { a = q[0]; b = q[1]; }
            x[i][0] = a.x; x[i][1] = a.y; x[i][2] = a.z; x[i][3] = a.w;
            x[i][4] = b.x; x[i][5] = b.y; x[i][6] = b.z; x[i][7] = b.w;
        }
        if (MODE == 1) {
            uint32_t s = 0;
            for (int i = 0; i < BLK; i++)
                for (int k = 0; k < 8; k++) s ^= x[i][k];
            if (l < BLK) out[(size_t)g * BLK + l] = s;
            continue;
        }
        const uint64_t h = block_group_hash<BLK>(x);
        if (l < BLK) out[(size_t)g * BLK + l] = h;
    }
}

static const int BLKC = BLK;

static uint8_t *g_flush;
__global__ void k_flush(uint4 *p, size_t n)
{
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) p[i] = make_uint4(i, 0, 0, 0);
}

template <int MODE, int WAVES, int PER_CU = 0>
static double run(const uint8_t *d_in, uint32_t ngroups, uint64_t *d_out, const char *name)
{
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const uint32_t per = MODE == 4 ? 2u : 1u;
    const uint32_t waves = (ngroups + per - 1) / per;
    uint32_t grid = (waves + WAVES - 1) / WAVES;
    if (PER_CU) grid = PER_CU * 256;
    float best = 1e30f, sum = 0;
    for (int rep = 0; rep < 8; rep++) {
        // cold caches, as in the pipeline: 1 GiB of stores evict the input from L2 and MALL
        hipLaunchKernelGGL(k_flush, dim3(4096), dim3(256), 0, 0, (uint4 *)g_flush, ((size_t)1 << 30) / 16);
        hipEventRecord(e0);
        hipLaunchKernelGGL((k_bh<MODE, WAVES>), dim3(grid), dim3(64 * WAVES), 0, 0, d_in, ngroups, d_out);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        if (rep >= 2 && ms < best) best = ms;
        if (rep >= 2) sum += ms;
    }
    const double bytes = (double)ngroups * BLKC * XC_SEG;
    printf("%-40s best %7.1f us  mean %7.1f us  %6.2f TB/s\n", name, best * 1e3, sum / 6 * 1e3,
           bytes / (best * 1e-3) / 1e12);
    return best;
}

int main()
{
    const size_t n = (size_t)512 << 20;
    const uint32_t ngroups = (uint32_t)(n / (BLKC * XC_SEG));
    uint8_t *d_in;
    uint64_t *d_out, *d_ref;
    hipMalloc(&d_in, n);
    hipMalloc(&d_out, (size_t)ngroups * BLKC * 8);
    hipMalloc(&d_ref, (size_t)ngroups * BLKC * 8);
    hipMalloc(&g_flush, (size_t)1 << 30);
    {
        std::vector<uint32_t> h(n / 4);
        uint64_t s = 0x5555;
        for (auto &x : h) {
            s += 0x9E3779B97F4A7C15ull;
            uint64_t z = s;
            z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
            z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
            x = (uint32_t)(z ^ (z >> 31));
        }
        hipMemcpy(d_in, h.data(), n, hipMemcpyHostToDevice);
    }
        run<0, 4>(d_in, ngroups, d_ref, "hash, 4 waves/WG (k_blockhash)");
    run<0, 8>(d_in, ngroups, d_out, "hash, 8 waves/WG");
    run<0, 16>(d_in, ngroups, d_out, "hash, 16 waves/WG");
    run<1, 4>(d_in, ngroups, d_out, "loads only, 4 waves/WG");
    run<2, 4>(d_in, ngroups, d_out, "hash, nt loads");
    run<5, 4, 2>(d_in, ngroups, d_out, "persistent prefetch, 2 WG/CU");
    run<5, 4, 3>(d_in, ngroups, d_out, "persistent prefetch, 3 WG/CU");
    run<5, 4, 4>(d_in, ngroups, d_out, "persistent prefetch, 4 WG/CU");
    run<4, 4>(d_in, ngroups, d_out, "hash, 2 groups per wave");
    std::vector<uint64_t> a((size_t)ngroups * BLKC), b(a.size());
    hipMemcpy(a.data(), d_ref, a.size() * 8, hipMemcpyDeviceToHost);
    hipMemcpy(b.data(), d_out, b.size() * 8, hipMemcpyDeviceToHost);
    printf("2-groups variant matches: %s\n", a == b ? "yes" : "NO");
    run<3, 4>(d_in, ngroups, d_out, "compute only");
    return 0;
}
