// Microbenchmark: VALU issue rate per instruction form used by the scan's rolling hash (no
// memory traffic; 8 independent chains per lane, forms forced with inline asm).
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/valu_bench tools/valu_bench.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

template <int FORM>
__global__ __launch_bounds__(1024) void k(uint32_t *out, uint32_t iters, uint32_t seed)
{
    uint32_t a[8], b[8];
    for (int i = 0; i < 8; i++) { a[i] = seed * (threadIdx.x + i); b[i] = seed ^ (threadIdx.x * 7 + i); }
    for (uint32_t it = 0; it < iters; it++) {
#pragma unroll
        for (int j = 0; j < 8; j++) {
#pragma unroll
            for (int i = 0; i < 8; i++) {
                if (FORM == 0) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b[i]));
                if (FORM == 1) asm volatile("v_sub_u32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1" : "+v"(a[i]) : "v"(b[i]));
                if (FORM == 2) asm volatile("v_lshl_add_u32 %0, %0, 20, %1" : "+v"(a[i]) : "v"(b[i]));
                if (FORM == 3) asm volatile("v_lshlrev_b32_sdwa %0, 11, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_2" : "=v"(a[i]) : "v"(b[i] + a[i]));
                if (FORM == 4) asm volatile("v_dot4_u32_u8 %0, %1, %1, %0" : "+v"(a[i]) : "v"(b[i]));
                if (FORM == 5) asm volatile("v_bfe_u32 %0, %1, 8, 8" : "=v"(a[i]) : "v"(a[i] ^ b[i]));
                if (FORM == 6) asm volatile("v_add3_u32 %0, %0, %1, %1" : "+v"(a[i]) : "v"(b[i]));
                if (FORM == 7) asm volatile("v_mad_u32_u24 %0, %1, %1, %0" : "+v"(a[i]) : "v"(b[i]));
                if (FORM == 8) asm volatile("v_lshrrev_b32 %0, %1, %0" : "+v"(a[i]) : "v"(b[i]));
                if (FORM == 9) asm volatile("v_bitop3_b32 %0, %0, 1, %1 bitop3:0x80" : "+v"(a[i]) : "v"(b[i]));
            }
        }
    }
    uint32_t x = 0;
    for (int i = 0; i < 8; i++) x ^= a[i];
    if (x == 0x12345678u) out[threadIdx.x] = x;
}

template <int FORM>
static void run(uint32_t *out, const char *name)
{
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const uint32_t iters = 4000;
    float ms = 0;
    for (int rep = 0; rep < 2; rep++) {
        hipEventRecord(e0);
        hipLaunchKernelGGL(k<FORM>, dim3(256), dim3(1024), 0, 0, out, iters, 12345u);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        hipEventElapsedTime(&ms, e0, e1);
    }
    const double ins = 256.0 * 16 * iters * 64;  // wave-instructions
    printf("%-22s %7.3f ms  %6.3f wave-instr/ns  (%.2f cyc/instr/SIMD @2.4GHz)\n", name, ms, ins / ms / 1e6,
           1024.0 * 2.4 / (ins / ms / 1e6));
}

int main()
{
    uint32_t *out;
    if (hipMalloc(&out, 4096 * 4) != hipSuccess) return 1;
    run<0>(out, "v_add_u32");
    run<1>(out, "v_sub_u32_sdwa");
    run<2>(out, "v_lshl_add_u32");
    run<3>(out, "v_lshlrev_b32_sdwa");
    run<4>(out, "v_dot4_u32_u8");
    run<5>(out, "v_bfe_u32");
    run<6>(out, "v_add3_u32");
    run<7>(out, "v_mad_u32_u24");
    run<8>(out, "v_lshrrev_b32");
    run<9>(out, "v_bitop3_b32");
    return 0;
}
