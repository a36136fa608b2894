// xc_device.h — wave64 primitives and the XCodec window-hash arithmetic for gfx950.
//
// The hash (xcodec/xcodec_hash.h:32-164) of the 2048-byte window ending at p depends
// only on the window's bytes.  With w = byte+1 and
// f = ffs(byte):
//   S1 = sum w_i,   S2 = sum (p+1-i) w_i        (same for f)   all mod 2^32
//   bytes_hash = (S1w << 20) + S2w,  bits_hash = (S1f << 16) + S2f
//   H = (uint64(bits_hash) << 36) + bytes_hash
// so H.lo32 == bytes_hash and H.hi32 == bits_hash << 4.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define XC_SEG 2048u
#define XC_MAGIC 0xF1u

namespace xc {

__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }

// ---- DPP wave scans (gfx9 DPP: row_shr 1/2/4/8, row_bcast 15/31) ----------------
template <int CTRL, int ROWMASK>
__device__ __forceinline__ uint32_t dpp0(uint32_t x)
{
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, ROWMASK, 0xf, false);
}

// Inclusive prefix sum over the 64 lanes (mod 2^32).
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x)
{
    x += dpp0<0x111, 0xf>(x);  // row_shr:1
    x += dpp0<0x112, 0xf>(x);  // row_shr:2
    x += dpp0<0x114, 0xf>(x);  // row_shr:4
    x += dpp0<0x118, 0xf>(x);  // row_shr:8
    x += dpp0<0x142, 0xa>(x);  // row_bcast:15 -> rows 1,3
    x += dpp0<0x143, 0xc>(x);  // row_bcast:31 -> rows 2,3
    return x;
}

// OR over the 64 lanes, result in lane 63 (same DPP pattern as the scan).
__device__ __forceinline__ uint32_t wave_incl_or(uint32_t x)
{
    x |= dpp0<0x111, 0xf>(x);
    x |= dpp0<0x112, 0xf>(x);
    x |= dpp0<0x114, 0xf>(x);
    x |= dpp0<0x118, 0xf>(x);
    x |= dpp0<0x142, 0xa>(x);
    x |= dpp0<0x143, 0xc>(x);
    return x;
}

__device__ __forceinline__ uint32_t readlane(uint32_t x, int l)
{
    return (uint32_t)__builtin_amdgcn_readlane((int)x, l);
}

__device__ __forceinline__ uint32_t wave_sum(uint32_t x) { return readlane(wave_incl_scan(x), 63); }

__device__ __forceinline__ uint64_t ballot(bool p) { return __ballot(p); }

// Number of set bits of m below this lane.
__device__ __forceinline__ uint32_t mbcnt(uint64_t m)
{
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

__device__ __forceinline__ uint32_t uniform(uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); }

// ---- byte helpers -------------------------------------------------------------
__device__ __forceinline__ uint32_t ffs8(uint32_t b) { return b ? (uint32_t)__builtin_ctz(b) + 1u : 0u; }

// 32 bytes at an arbitrary address as 8 little-endian dwords (aligned loads + alignbyte).
__device__ __forceinline__ void load32_unaligned(const uint8_t *p, uint32_t out[8])
{
    uintptr_t a = (uintptr_t)p;
    const uint32_t *w = (const uint32_t *)(a & ~(uintptr_t)3);
    uint32_t sh = (uint32_t)(a & 3);
    uint32_t d[9];
#pragma unroll
    for (int k = 0; k < 9; k++) d[k] = w[k];
#pragma unroll
    for (int k = 0; k < 8; k++) out[k] = __builtin_amdgcn_alignbyte(d[k + 1], d[k], sh);
}

// The same for a lane's part of a 2048-byte window that may end where its allocation ends: the
// ninth word only when p is unaligned (it then holds the part's last bytes; an aligned part ends
// on a word boundary).
__device__ __forceinline__ void load32_window(const uint8_t *p, uint32_t out[8])
{
    const uintptr_t a = (uintptr_t)p;
    const uint32_t *w = (const uint32_t *)(a & ~(uintptr_t)3);
    const uint32_t sh = (uint32_t)(a & 3);
    uint32_t d[9];
#pragma unroll
    for (int k = 0; k < 8; k++) d[k] = w[k];
    d[8] = sh ? w[8] : 0u;
#pragma unroll
    for (int k = 0; k < 8; k++) out[k] = __builtin_amdgcn_alignbyte(d[k + 1], d[k], sh);
}

// Per-lane partial sums of 32 bytes at local offsets 0..31:
//   A = sum w, B = sum j*w for w = byte+1   (and the same with f = ffs(byte))
struct Sums4 {
    uint32_t aw, bw, af, bf;
};

// ffs per byte uses v_ffbl_b32 on the zero-extended byte (SDWA src0_sel), which the hardware
// defines as 0xFFFFFFFF for a zero byte: ffbl + 1 == ffs(byte) with ffs(0) == 0
// (xcodec/xcodec_hash.h:95-96) and no compare/select.  Inline asm: the compiler's cttz would add
// the zero test back.
// ffs of the four bytes of x, packed as bytes: each byte's ffbl is written into its own byte of
// the result (SDWA dst_sel, the other bytes preserved), giving ffs - 1 with 0xFF for a zero
// byte; a carry-free per-byte +1 (0xFF + 1 wraps to 0 = ffs(0)) finishes ffs.
__device__ __forceinline__ uint32_t ffs_bytes(uint32_t x)
{
    uint32_t p;
    asm("v_ffbl_b32_sdwa %0, %1 dst_sel:BYTE_0 dst_unused:UNUSED_PAD src0_sel:BYTE_0" : "=v"(p) : "v"(x));
    asm("v_ffbl_b32_sdwa %0, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_1" : "+v"(p) : "v"(x));
    asm("v_ffbl_b32_sdwa %0, %1 dst_sel:BYTE_2 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_2" : "+v"(p) : "v"(x));
    asm("v_ffbl_b32_sdwa %0, %1 dst_sel:BYTE_3 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_3" : "+v"(p) : "v"(x));
    return ((p & 0x7F7F7F7Fu) + 0x01010101u) ^ (p & 0x80808080u);
}

__device__ __forceinline__ Sums4 chunk_sums32(const uint32_t w[8])
{
    Sums4 s = {0, 0, 0, 0};
    uint32_t sb = 0, jb = 0, sf = 0, jf = 0;
#pragma unroll
    for (int d = 0; d < 8; d++) {
        // weights (4d, 4d+1, 4d+2, 4d+3) packed as bytes
        const uint32_t wt = (uint32_t)(4 * d) * 0x01010101u + 0x03020100u;
        sb = __builtin_amdgcn_udot4(w[d], 0x01010101u, sb, false);
        jb = __builtin_amdgcn_udot4(w[d], wt, jb, false);
        // f = ffs per byte (0..8), packed: plain and j-weighted byte dot products
        const uint32_t f = ffs_bytes(w[d]);
        sf = __builtin_amdgcn_udot4(f, 0x01010101u, sf, false);
        jf = __builtin_amdgcn_udot4(f, wt, jf, false);
    }
    s.aw = sb + 32u;         // sum (b+1)
    s.bw = jb + 496u;        // sum j*(b+1), sum j = 496
    s.af = sf;               // sum ffs(b)
    s.bf = jf;               // sum j*ffs(b)
    return s;
}

// Lane permutation by a DPP control (quad_perm, row_mirror, row_half_mirror, ...).
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_perm(uint32_t x)
{
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, 0xf, 0xf, false);
}

// Full hash of a 2048-byte window held as 32 bytes per lane (lane l: bytes 32l..32l+31);
// every lane returns the result.
__device__ __forceinline__ uint64_t wave_hash_regs(const uint32_t w[8])
{
    const uint32_t l = lane_id();
    Sums4 s = chunk_sums32(w);
    const uint32_t k = XC_SEG - 32u * l;  // weight of this lane's byte 0 is (2048 - 32l)
    // transposed reduction of the 4 sums: permlane swaps over lane bits 5 and 4 leave value
    // 2 bit5 + bit4 in each 16-lane row, then a row sum
    uint32_t v0 = s.aw, v1 = k * s.aw - s.bw, v2 = s.af, v3 = k * s.af - s.bf;
    {
        const auto r = __builtin_amdgcn_permlane32_swap(v0, v2, false, false);
        const auto q = __builtin_amdgcn_permlane32_swap(v1, v3, false, false);
        v0 = r[0] + r[1];  // lanes < 32: value 0, lanes >= 32: value 2
        v1 = q[0] + q[1];  // lanes < 32: value 1, lanes >= 32: value 3
        const auto t = __builtin_amdgcn_permlane16_swap(v0, v1, false, false);
        v0 = t[0] + t[1];  // row r holds value r
    }
    v0 += dpp_perm<0x140>(v0);  // row_mirror
    v0 += dpp_perm<0x141>(v0);  // row_half_mirror
    v0 += dpp_perm<0x4E>(v0);   // quad_perm [2,3,0,1]
    v0 += dpp_perm<0xB1>(v0);   // quad_perm [1,0,3,2]: every lane of row r: the sum of value r
    const uint32_t s1w = readlane(v0, 0), s2w = readlane(v0, 16);
    const uint32_t s1f = readlane(v0, 32), s2f = readlane(v0, 48);
    uint32_t bytes_hash = (s1w << 20) + s2w;
    uint32_t bits_hash = (s1f << 16) + s2f;
    return ((uint64_t)bits_hash << 36) + (uint64_t)bytes_hash;
}

// Full hash of the 2048 bytes at p (any alignment); every lane returns the result.
__device__ __forceinline__ uint64_t wave_window_hash(const uint8_t *p)
{
    uint32_t w[8];
    load32_window(p + 32u * lane_id(), w);
    return wave_hash_regs(w);
}

// Butterfly step: each lane keeps half of its values, the partner (an involution differing in
// `bit` of the lane id) sends the other half.  After it, lane l holds half as many sums.
template <int H, int CTRL>
__device__ __forceinline__ void bfly_dpp(uint32_t v[], uint32_t bit)
{
#pragma unroll
    for (int i = 0; i < H; i++) {
        const uint32_t send = bit ? v[i] : v[i + H], keep = bit ? v[i + H] : v[i];
        v[i] = keep + dpp_perm<CTRL>(send);
    }
}

// Transposed wave reduction of 32 values per lane: lane l returns the 64-lane sum of value
// (l >> 1) & 31.  Butterflies over the lane bits 5, 4 (v_permlane32/16_swap: no selects), 3, 2
// (row_mirror, row_half_mirror: partners differ in that bit, and in lower ones, which the later
// steps cover), 1, 0 (quad_perm): 70 VALU instead of 32 separate 6-step scans.
__device__ __forceinline__ uint32_t wave_sums32(uint32_t v[32])
{
    const uint32_t l = lane_id();
#pragma unroll
    for (int i = 0; i < 16; i++) {  // lanes < 32 keep value i, lanes >= 32 value i + 16
        const auto r = __builtin_amdgcn_permlane32_swap(v[i], v[i + 16], false, false);
        v[i] = r[0] + r[1];
    }
#pragma unroll
    for (int i = 0; i < 8; i++) {   // even rows keep value i, odd rows value i + 8
        const auto r = __builtin_amdgcn_permlane16_swap(v[i], v[i + 8], false, false);
        v[i] = r[0] + r[1];
    }
    bfly_dpp<4, 0x140>(v, (l >> 3) & 1u);  // row_mirror: lane j <-> 15 - j
    bfly_dpp<2, 0x141>(v, (l >> 2) & 1u);  // row_half_mirror: lane j <-> 7 - j
    bfly_dpp<1, 0x4E>(v, (l >> 1) & 1u);   // quad_perm [2,3,0,1]
    return v[0] + dpp_perm<0xB1>(v[0]);    // quad_perm [1,0,3,2]
}

// Hashes of G = 8 blocks held as 32 bytes per lane (w[i]: block i): lane i (< 8) receives block
// i's hash.  The 4 window sums of the 8 blocks are reduced together (wave_sums32): value 4 i + c
// lands in lanes 8 i + 2 c (and + 1).
template <int G>
__device__ __forceinline__ uint64_t block_group_hash(const uint32_t w[G][8])
{
    static_assert(G == 8, "8 blocks x 4 sums fill the 32-value transposed reduction");
    const uint32_t l = lane_id();
    uint32_t v[32];
    const uint32_t k = XC_SEG - 32u * l;  // weight of this lane's byte 0 is (2048 - 32l)
#pragma unroll
    for (int i = 0; i < G; i++) {
        const Sums4 s = chunk_sums32(w[i]);
        v[4 * i + 0] = s.aw;
        v[4 * i + 1] = k * s.aw - s.bw;
        v[4 * i + 2] = s.af;
        v[4 * i + 3] = k * s.af - s.bf;
    }
    const uint32_t sum = wave_sums32(v);
    const int src = (int)(8u * (l & 7u));
    const uint32_t s1w = (uint32_t)__shfl((int)sum, src), s2w = (uint32_t)__shfl((int)sum, src + 2);
    const uint32_t s1f = (uint32_t)__shfl((int)sum, src + 4), s2f = (uint32_t)__shfl((int)sum, src + 6);
    const uint32_t bytes_hash = (s1w << 20) + s2w, bits_hash = (s1f << 16) + s2f;
    return ((uint64_t)bits_hash << 36) + (uint64_t)bytes_hash;
}

// The words of n <= G consecutive 16-byte-aligned blocks at p (lane l: bytes 32 l .. 32 l + 31 of
// each; zeros past n), all loads issued together.
template <int G, bool NT = false>
__device__ __forceinline__ void wave_load_blocks(const uint8_t *p, uint32_t n, uint32_t (&w)[G][8])
{
    const uint32_t l = lane_id();
    typedef uint32_t v4u __attribute__((ext_vector_type(4)));
#pragma unroll
    for (int i = 0; i < G; i++) {
#pragma unroll
        for (int k = 0; k < 8; k++) w[i][k] = 0u;
        if ((uint32_t)i < n) {
            const v4u *q = (const v4u *)(p + (size_t)i * XC_SEG + 32u * l);
            v4u x, y;
            if (NT) {  // (streamed once: the L2 keeps the filters the other stream's kernels read)
                x = __builtin_nontemporal_load(q);
                y = __builtin_nontemporal_load(q + 1);
            } else {
                x = q[0];
                y = q[1];
            }
            w[i][0] = x.x; w[i][1] = x.y; w[i][2] = x.z; w[i][3] = x.w;
            w[i][4] = y.x; w[i][5] = y.y; w[i][6] = y.z; w[i][7] = y.w;
        }
    }
}

// Hashes of n <= 8 consecutive 16-byte-aligned blocks at p: lane i (< n) receives block i's hash.
template <int G>
__device__ __forceinline__ uint64_t wave_block_hashes(const uint8_t *p, uint32_t n)
{
    uint32_t w[G][8];
    wave_load_blocks<G>(p, n, w);
    return block_group_hash<G>(w);
}

// 2048-byte equality of two windows (any alignment); wave-uniform result.
__device__ __forceinline__ bool wave_equal2048(const uint8_t *a, const uint8_t *b)
{
    const uint32_t l = lane_id();
    uint32_t x[8], y[8];
    load32_window(a + 32u * l, x);
    load32_window(b + 32u * l, y);
    uint32_t diff = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) diff |= x[k] ^ y[k];
    return ballot(diff != 0) == 0;
}

// Wave-cooperative copy of n bytes, any alignments.  Body uses 16-byte aligned stores;
// head/tail bytes are single-byte stores (never a read-modify-write of a neighbour's word).
__device__ __forceinline__ void wave_copy(uint8_t *dst, const uint8_t *src, uint32_t n)
{
    const uint32_t l = lane_id();
    uintptr_t d = (uintptr_t)dst;
    uint32_t head = (uint32_t)((16u - (d & 15u)) & 15u);
    if (head > n) head = n;
    if (l < head) dst[l] = src[l];
    uint32_t body = (n - head) & ~15u;
    for (uint32_t o = head + 16u * l; o < head + body; o += 1024u) {
        const uint8_t *s = src + o;
        uintptr_t a = (uintptr_t)s;
        const uint32_t *w = (const uint32_t *)(a & ~(uintptr_t)3);
        uint32_t sh = (uint32_t)(a & 3);
        uint32_t v0 = w[0], v1 = w[1], v2 = w[2], v3 = w[3], v4 = sh ? w[4] : 0u;
        uint4 o4;
        o4.x = __builtin_amdgcn_alignbyte(v1, v0, sh);
        o4.y = __builtin_amdgcn_alignbyte(v2, v1, sh);
        o4.z = __builtin_amdgcn_alignbyte(v3, v2, sh);
        o4.w = __builtin_amdgcn_alignbyte(v4, v3, sh);
        *(uint4 *)(dst + o) = o4;
    }
    uint32_t t0 = head + body;
    if (t0 + l < n) dst[t0 + l] = src[t0 + l];
}

// 16 bytes at an arbitrary address (aligned dword loads + alignbyte).
__device__ __forceinline__ uint4 load16_unaligned(const uint8_t *p)
{
    const uintptr_t a = (uintptr_t)p;
    const uint32_t *w = (const uint32_t *)(a & ~(uintptr_t)3);
    const uint32_t sh = (uint32_t)(a & 3);
    const uint32_t v0 = w[0], v1 = w[1], v2 = w[2], v3 = w[3], v4 = sh ? w[4] : 0u;
    return make_uint4(__builtin_amdgcn_alignbyte(v1, v0, sh), __builtin_amdgcn_alignbyte(v2, v1, sh),
                      __builtin_amdgcn_alignbyte(v3, v2, sh), __builtin_amdgcn_alignbyte(v4, v3, sh));
}

// A 2048-byte payload from src (any alignment) to the wire at out (any alignment) and to a
// cache slot (16-byte aligned), split into a load half and a store half so that a wave can
// have several payloads in flight.  Every store is a whole 16-byte aligned store except the
// wire copy's head and tail bytes; the wire-aligned reads of src hit the cache.
#ifndef XC_NT_STORE
#define XC_NT_STORE 1
#endif
struct PayloadRegs {
    uint4 a0, a1;  // slot-aligned chunks: src + 16 l, src + 1024 + 16 l
};

// The loads only (the wire-aligned chunks are made from a0 / a1 at the store, so that the registers
// of a payload in flight are its 32 bytes per lane, not twice that: the emit's occupancy).
__device__ __forceinline__ void payload_load(const uint8_t *src, const uint8_t *out, PayloadRegs &r)
{
    (void)out;
    const uint32_t l = lane_id();
    if (((uintptr_t)src & 15u) == 0u) {  // (aligned blocks, segment-store slots): one load each
        r.a0 = *(const uint4 *)(src + 16u * l);
        r.a1 = *(const uint4 *)(src + 1024u + 16u * l);
    } else {
        r.a0 = load16_unaligned(src + 16u * l);
        r.a1 = load16_unaligned(src + 1024u + 16u * l);
    }
}

// Byte x (< 16) of a uint4 whose four words are wave-uniform.
__device__ __forceinline__ uint32_t byte_of4(uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3, uint32_t x)
{
    const uint32_t w = x < 4u ? w0 : x < 8u ? w1 : x < 12u ? w2 : w3;
    return (w >> (8u * (x & 3u))) & 0xffu;
}

// The wire-aligned chunks of a payload for a wire address with `head` bytes to its next 16-byte
// boundary: lane l's chunk is bytes head .. head + 15 of (chunk l, chunk l + 1), the next lane's words
// by a DPP wave shift (lane 63's successor: lane 0 of the second half), then a funnel by head bytes;
// no second read of src.
__device__ __forceinline__ void payload_wire(const PayloadRegs &r, uint32_t head, uint4 &b0, uint4 &b1)
{
    b0 = r.a0;
    b1 = r.a1;
    if (!head) return;
    const uint32_t c0[4] = {r.a0.x, r.a0.y, r.a0.z, r.a0.w}, c1[4] = {r.a1.x, r.a1.y, r.a1.z, r.a1.w};
    uint32_t n0[4], n1[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const uint32_t first1 = readlane(c1[k], 0);
        n0[k] = (uint32_t)__builtin_amdgcn_update_dpp((int)first1, (int)c0[k], 0x130, 0xf, 0xf, false);  // wave_shl:1
        n1[k] = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)c1[k], 0x130, 0xf, 0xf, false);
    }
    const uint32_t dh = head >> 2, bh = 8u * (head & 3u);
    auto fun = [&](const uint32_t (&c)[4], const uint32_t (&nx)[4]) {
        uint32_t d[8] = {c[0], c[1], c[2], c[3], nx[0], nx[1], nx[2], nx[3]};
        uint32_t o[5];
#pragma unroll
        for (int k = 0; k < 5; k++)  // dwords dh .. dh + 4 of the 32 bytes (dh uniform)
            o[k] = dh == 0 ? d[k] : dh == 1 ? d[k + 1] : dh == 2 ? d[k + 2] : d[min(k + 3, 7)];
        uint4 v;
        v.x = bh ? (o[0] >> bh) | (o[1] << (32u - bh)) : o[0];
        v.y = bh ? (o[1] >> bh) | (o[2] << (32u - bh)) : o[1];
        v.z = bh ? (o[2] >> bh) | (o[3] << (32u - bh)) : o[2];
        v.w = bh ? (o[3] >> bh) | (o[4] << (32u - bh)) : o[3];
        return v;
    };
    b0 = fun(c0, n0);
    b1 = fun(c1, n1);
}

// 16-byte store, non-temporal (the wire bytes and the segment store are not read back by this
// pass; cfg5 A/B +1.6 %, profiles/r04/ab_nt_store.txt); -DXC_NT_STORE=0: plain stores
__device__ __forceinline__ void store16(void *p, const uint4 &v)
{
#if XC_NT_STORE
    typedef uint32_t v4u __attribute__((ext_vector_type(4)));
    v4u x = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(x, (v4u *)p);
#else
    *(uint4 *)p = v;
#endif
}

__device__ __forceinline__ void payload_store(uint8_t *out, uint8_t *seg, const PayloadRegs &r)
{
    const uint32_t l = lane_id();
    const uint32_t head = (uint32_t)((16u - ((uintptr_t)out & 15u)) & 15u);
    const uint32_t nbody = (XC_SEG - head) >> 4;
    const uint32_t t0 = head + 16u * nbody;
    if (seg) {
        store16((uint4 *)seg + l, r.a0);
        store16((uint4 *)seg + l + 64u, r.a1);
    }
    uint4 b0, b1;
    payload_wire(r, head, b0, b1);
    if (l < nbody) store16(out + head + 16u * l, b0);
    if (l + 64u < nbody) store16(out + head + 1024u + 16u * l, b1);
    // the head bytes (payload 0 .. head - 1: lane 0's first chunk) and the tail bytes (t0 .. 2047: lane
    // 63's last chunk), from the registers (no byte loads)
    if (head) {
        const uint32_t h0 = readlane(r.a0.x, 0), h1 = readlane(r.a0.y, 0), h2 = readlane(r.a0.z, 0), h3 = readlane(r.a0.w, 0);
        if (l < head) out[l] = (uint8_t)byte_of4(h0, h1, h2, h3, l);
        const uint32_t e0 = readlane(r.a1.x, 63), e1 = readlane(r.a1.y, 63), e2 = readlane(r.a1.z, 63), e3 = readlane(r.a1.w, 63);
        if (t0 + l < XC_SEG) out[t0 + l] = (uint8_t)byte_of4(e0, e1, e2, e3, t0 + l - (XC_SEG - 16u));
    }
}

__device__ __forceinline__ void payload_store_seg(uint8_t *seg, const PayloadRegs &r)
{
    const uint32_t l = lane_id();
    ((uint4 *)seg)[l] = r.a0;
    ((uint4 *)seg)[l + 64u] = r.a1;
}

__device__ __forceinline__ void wave_copy_payload(uint8_t *out, uint8_t *seg, const uint8_t *src)
{
    PayloadRegs r;
    payload_load(src, out, r);
    payload_store(out, seg, r);
}

// ---- membership sets -------------------------------------------------------------
// A set of 64-bit hashes: level-1 bitmap (LDS-loaded by the scan), exact lo32 set,
// full-key table with a 64-bit value.  Used for the cache (value = segment index)
// and for a batch's declarations (value = buffer<<32 | declaration position, min-wins).
// Level-1 filter: a blocked k=2 Bloom filter of 36864 32-bit words (144 KB: with the scan's
// 16 KB of positive queues it fills a CU's 160 KB of LDS).  lo32 (the hash's bytes_hash half)
// picks word floor(lo[31:8] * 36864 / 2^24) (one full-rate v_mul_hi_u32_u24); the key sets
// bits lo[4:0] and lo[9:5] of that word.  One ds_read_b32 per tested position.
#define XC_FILT_WORDS 36864u  // in 32-bit words (a multiple of 4096)
#define XC_EMPTY64 0xFFFFFFFFFFFFFFFFull           // H never has bits 32..35 set

// Level-2 filter: a blocked k=2 Bloom filter of 2^19 32-bit words (2 MB, sized to stay in an
// XCD's L2) keyed by a remix g of lo32, independent of the level-1 bits: word g >> 13, bits g[4:0]
// and g[9:5] (one 4-byte read per test).  XC_L2_WORDS counts 8-byte units of its storage.
#define XC_L2_WORDS (1u << 18)

__device__ __forceinline__ uint32_t l2_mix(uint32_t lo)
{
    uint32_t g = (lo ^ (lo >> 15)) * 0x2C1B3C6Du;
    return g ^ (g >> 12);
}

// lo from l2_mix(lo) (both steps invert: an xorshift, and a multiply by an odd constant)
__device__ __forceinline__ uint32_t l2_unmix(uint32_t g)
{
    g ^= (g >> 12) ^ (g >> 24);
    g *= 0x64EA2D65u;  // 0x2C1B3C6D^-1 mod 2^32
    return g ^ (g >> 15) ^ (g >> 30);
}

__device__ __forceinline__ uint32_t l2_word(uint32_t g) { return g >> 13; }
__device__ __forceinline__ bool l2_test(uint32_t w, uint32_t g)
{
    return ((w >> (g & 31u)) & (w >> ((g >> 5) & 31u)) & 1u) != 0u;
}

struct DevSet {
    uint32_t *filt;     // XC_FILT_WORDS
    uint32_t *l2;       // 2 * XC_L2_WORDS (level-2 filter)
    uint32_t *lo_keys;  // lo32 set (0 = empty; a zero key is flagged in *lo_zero)
    uint32_t *lo_zero;
    uint32_t lo_mask;
    uint32_t mask;      // full table
    uint64_t *keys;
    uint64_t *vals;
};

// Word of a filter of `words` words (XC_FILT_WORDS >> fold: the folded image, whose word w is the
// OR of the full image's words w << fold ..): floor(lo[23:0] * words / 2^24), one full-rate
// v_mul_hi_u32_u24 on lo itself (the unit ignores lo[31:24]; both operands must be provably
// 24-bit, or the compiler emits the quarter-rate 32-bit v_mul_hi_u32).
__device__ __forceinline__ uint32_t filt_word_n(uint32_t lo, uint32_t words)
{
    return (uint32_t)(((uint64_t)(lo & 0xFFFFFFu) * (uint64_t)((words << 8) & 0xFFFFFFu)) >> 32);
}
__device__ __forceinline__ uint32_t filt_word(uint32_t lo) { return filt_word_n(lo, XC_FILT_WORDS); }
// The key's two bits in its word: lo[4:0] and lo[31:27] (outside the bits that pick the word).
__device__ __forceinline__ uint32_t filt_mask(uint32_t lo) { return (1u << (lo & 31u)) | (1u << (lo >> 27)); }
__device__ __forceinline__ uint32_t filt_test_n(const uint32_t *f, uint32_t lo, uint32_t words)
{
    const uint32_t w = f[filt_word_n(lo, words)];
    return (w >> (lo & 31u)) & (w >> (lo >> 27)) & 1u;
}
__device__ __forceinline__ uint32_t filt_test(const uint32_t *f, uint32_t lo) { return filt_test_n(f, lo, XC_FILT_WORDS); }
__device__ __forceinline__ uint32_t lo_slot(uint32_t lo, uint32_t mask) { return (lo * 0x9E3779B1u) >> 5 & mask; }
__device__ __forceinline__ uint32_t key_slot(uint64_t h, uint32_t mask)
{
    uint32_t lo = (uint32_t)h, hi = (uint32_t)(h >> 32);
    return ((lo * 0x9E3779B1u) ^ (hi * 0x85EBCA6Bu)) >> 5 & mask;
}

__device__ __forceinline__ bool set_has_lo(const DevSet &s, uint32_t lo)
{
    if (lo == 0u) return *s.lo_zero != 0u;
    uint32_t i = lo_slot(lo, s.lo_mask);
    for (;;) {
        uint32_t k = s.lo_keys[i];
        if (k == lo) return true;
        if (k == 0u) return false;
        i = (i + 1u) & s.lo_mask;
    }
}

// A cache entry evicted by the COSS tier (xc_coss.cpp) keeps its key with this bit in its value:
// absent to every lookup, revived by the next insert of the key.
#define XC_DEAD (1ull << 63)
// The undo record's lo slot of an insert that revived an evicted key: undoing it evicts the key
// again (clearing the key would cut the probe chains of keys inserted after it).
#define XC_REVIVED 0xFFFFFFFEu

// Returns true and *val if present (and not evicted).
__device__ __forceinline__ bool set_find(const DevSet &s, uint64_t h, uint64_t *val)
{
    uint32_t i = key_slot(h, s.mask);
    for (;;) {
        uint64_t k = s.keys[i];
        if (k == h) {
            const uint64_t v = s.vals[i];
            if (v & XC_DEAD) return false;
            *val = v;
            return true;
        }
        if (k == XC_EMPTY64) return false;
        i = (i + 1u) & s.mask;
    }
}

// Insert (h, val).  Returns 1 if newly inserted, 0 if h was present.  With min_merge the
// value is atomicMin-merged (vals must start at ~0); otherwise a fresh value is stored.
// *slot_out / *lo_slot_out receive the full-table slot and the newly used lo32 slot
// (NONE when the lo32 key was already present) for undo logs.
__device__ __forceinline__ int set_insert(const DevSet &s, uint64_t h, uint64_t val, bool min_merge,
                                          uint32_t *slot_out, uint32_t *lo_slot_out)
{
    // filter bits first: their atomics return nothing, so none waits, and setting them again
    // for a key already present changes nothing
    {
        const uint32_t lo = (uint32_t)h;
        atomicOr(&s.filt[filt_word(lo)], filt_mask(lo));
        const uint32_t g = l2_mix(lo);
        atomicOr(&s.l2[l2_word(g)], (1u << (g & 31u)) | (1u << ((g >> 5) & 31u)));
    }
    uint32_t i = key_slot(h, s.mask);
    int fresh = 0;
    for (;;) {
        uint64_t prev = atomicCAS((unsigned long long *)&s.keys[i], (unsigned long long)XC_EMPTY64,
                                  (unsigned long long)h);
        if (prev == XC_EMPTY64) { fresh = 1; break; }
        if (prev == h) break;
        i = (i + 1u) & s.mask;
    }
    bool revived = false;
    if (min_merge) {
        atomicMin((unsigned long long *)&s.vals[i], (unsigned long long)val);
    } else if (fresh || (s.vals[i] & XC_DEAD)) {
        revived = !fresh;  // an evicted key comes back: its undo record restores the eviction
        s.vals[i] = val;
    }
    if (slot_out) *slot_out = i;
    uint32_t los = revived ? XC_REVIVED : 0xFFFFFFFFu;
    if (fresh) {
        uint32_t lo = (uint32_t)h;
        if (lo == 0u) atomicOr(s.lo_zero, 1u);
        else {
            uint32_t j = lo_slot(lo, s.lo_mask);
            for (;;) {
                uint32_t prev = atomicCAS(&s.lo_keys[j], 0u, lo);
                if (prev == 0u) { los = j; break; }
                if (prev == lo) break;
                j = (j + 1u) & s.lo_mask;
            }
        }
    }
    if (lo_slot_out) *lo_slot_out = los;
    return fresh;
}

// set_insert into the keys and values alone (no filter bits, no lo32 key): a declaration set read
// only through set_find (an anchor-scanned sub-batch's, block_predict); values atomicMin-merged.
__device__ __forceinline__ void set_insert_kv(const DevSet &s, uint64_t h, uint64_t val, uint32_t *slot_out)
{
    uint32_t i = key_slot(h, s.mask);
    for (;;) {
        const uint64_t prev = atomicCAS((unsigned long long *)&s.keys[i], (unsigned long long)XC_EMPTY64,
                                        (unsigned long long)h);
        if (prev == XC_EMPTY64 || prev == h) break;
        i = (i + 1u) & s.mask;
    }
    atomicMin((unsigned long long *)&s.vals[i], (unsigned long long)val);
    *slot_out = i;
}

// ---- anchor index -----------------------------------------------------------------
// A content-defined index that finds every window equal to an indexed segment without testing
// every window end against the key set.  G(p) = sum_{k<32} b[p-k] 2^k mod 2^32
// is a shift-add hash of the 32 bytes ending at p.  Position p is an anchor when p >= 63 (its
// 64-byte context lies inside the buffer, or the segment) and G(p) < 2^26 (1/64 of random
// positions); its fingerprint hashes G(p) and G(p - 32), i.e. the 64 bytes ending at p.  A
// segment's anchor is its last anchor j (63 <= j <= 2047), indexed as key fp << 11 | j.  If the
// window ending at q equals the segment, the input position a = q - 2047 + j has the same 64-byte
// context, so it is an anchor with the same fingerprint: the index proposes q = a + 2047 - j.
// Segments without an anchor (a 1.6e-14 chance for random bytes; constant runs of some values)
// keep the cache out of anchor mode (the exact scan, xc_runtime.hip).
#define ANC_G_LIMIT (1u << 26)
#define NONE_U32 0xFFFFFFFFu
#define ANC_NONE 0xFFFFFFFFFFFFFFFFull
#define ANC_FILT_WORDS (1u << 18)  // 1 MB anchor filter (k = 2 bits in a 32-bit word): stays in an XCD's L2

__device__ __forceinline__ uint64_t anc_fp(uint32_t g, uint32_t g2)
{
    const uint64_t k = ((uint64_t)g2 << 26) | (g & (ANC_G_LIMIT - 1u));
    return (k * 0x9E3779B97F4A7C15ull) >> 19;  // 45 bits
}
__device__ __forceinline__ uint64_t anc_key(uint64_t fp, uint32_t j) { return (fp << 11) | j; }
__device__ __forceinline__ uint32_t anc_mix(uint64_t fp) { return (uint32_t)(fp ^ (fp >> 21)) * 0x2C1B3C6Du; }
__device__ __forceinline__ uint32_t anc_home(uint64_t fp, uint32_t mask) { return (uint32_t)((fp * 0xD6E8FEB86659FD93ull) >> 37) & mask; }
__device__ __forceinline__ uint32_t anc_fword(uint32_t g) { return g >> 14; }
__device__ __forceinline__ uint32_t anc_fbits(uint32_t g) { return (1u << (g & 31u)) | (1u << ((g >> 5) & 31u)); }
__device__ __forceinline__ bool anc_ftest(uint32_t w, uint32_t g) { return ((w >> (g & 31u)) & (w >> ((g >> 5) & 31u)) & 1u) != 0u; }

// An anchor table: open addressing over keys fp << 11 | j, home slot by fp only (a probe walks
// the chain from home(fp) to the first empty slot and takes every key with that fingerprint).
struct AncSet {
    uint64_t *keys;  // mask + 1 slots, XC_EMPTY64 = empty
    uint32_t *filt;  // ANC_FILT_WORDS
    uint32_t mask;
};

// Insert key (fingerprint fp): the slot it took, or NONE when the key was there already.
__device__ __forceinline__ uint32_t anc_insert(const AncSet &s, uint64_t key)
{
    const uint64_t fp = key >> 11;
    const uint32_t g = anc_mix(fp);
    atomicOr(&s.filt[anc_fword(g)], anc_fbits(g));
    uint32_t i = anc_home(fp, s.mask);
    for (;;) {
        const uint64_t prev = atomicCAS((unsigned long long *)&s.keys[i], (unsigned long long)XC_EMPTY64,
                                        (unsigned long long)key);
        if (prev == XC_EMPTY64) return i;
        if (prev == key) return 0xFFFFFFFFu;
        i = (i + 1u) & s.mask;
    }
}

// G at a lane's last position from its 32 bytes alone: sum_i b_i 2^(31 - i) (byte dot products
// with weights 8, 4, 2, 1 per dword, Horner over the dwords).
__device__ __forceinline__ uint32_t gear32(const uint32_t w[8])
{
    uint32_t s = 0;
#pragma unroll
    for (int d = 0; d < 8; d++) s = (s << 4) + __builtin_amdgcn_udot4(w[d], 0x01020408u, 0u, false);
    return s;
}

// G at the lane's position -1 (the last of the lane before; lane 0: `first`).
__device__ __forceinline__ uint32_t gear_prev(uint32_t sf, uint32_t first)
{
    const uint32_t l = lane_id();
    const uint32_t up = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(4u * ((l + 63u) & 63u)), (int)sf);
    return l == 0 ? first : up;
}

// Anchor mask of the lane's 32 positions (bit 31 - t: position t of the lane is an anchor, before
// any position bound); TILE: G of every position into tile[t * XC_TILE_ROW + lane] too.
// Per position, all full-rate VOP2/VOPC but one: g + g, then the byte added straight from its
// dword (SDWA byte select: no extraction), and m = 2 m + (g < 2^26) as a compare into VCC and an
// add with carry-in (the compiler's select + or forms are VOP3).  The compare of position t is
// issued before the next position's two adds, so its VCC is read by the carry-in add two
// instructions later (gfx950 wants a wait state between a VALU write of VCC and its read as carry).
template <int K>
__device__ __forceinline__ uint32_t gear_cmp_step(uint32_t &m, uint32_t g, uint32_t w)
{
    static_assert(K >= 0 && K < 4, "byte");
    uint32_t gn;
#define XC_GEAR_STEP(SEL)                                                                                       \
    asm("v_cmp_gt_u32_e32 vcc, 0x4000000, %2\n\t"                                                              \
        "v_add_u32_e32 %0, %2, %2\n\t"                                                                         \
        "v_add_u32_sdwa %0, %0, %3 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:" SEL "\n\t"    \
        "v_addc_co_u32_e32 %1, vcc, %1, %1, vcc"                                                               \
        : "=&v"(gn), "+v"(m) : "v"(g), "v"(w) : "vcc")
    if (K == 0) XC_GEAR_STEP("BYTE_0");
    else if (K == 1) XC_GEAR_STEP("BYTE_1");
    else if (K == 2) XC_GEAR_STEP("BYTE_2");
    else XC_GEAR_STEP("BYTE_3");
#undef XC_GEAR_STEP
    return gn;
}
static_assert(ANC_G_LIMIT == 0x4000000u, "gear_cmp_step's literal");

// m after the last position: its compare, a wait state, the carry-in add.
__device__ __forceinline__ uint32_t mask_last(uint32_t m, uint32_t g)
{
    asm("v_cmp_gt_u32_e32 vcc, 0x4000000, %1\n\ts_nop 0\n\tv_addc_co_u32_e32 %0, vcc, %0, %0, vcc"
        : "+v"(m) : "v"(g) : "vcc");
    return m;
}

// (a row of 64 values and one pad word: the anchor pass gathers G(p) and G(p - 32) of a lane's
// several anchors, at different t, from different banks)
#define XC_TILE_ROW 65u
template <bool TILE>
__device__ __forceinline__ uint32_t gear_mask(const uint32_t w[8], uint32_t g, uint32_t *tile)
{
    const uint32_t l = lane_id();
    // position 0: its G from g (no mask bit before it: the first step's compare shifts in a bit
    // for "position -1" that the final shift-out below drops)
    uint32_t m = 0;
#pragma unroll
    for (int d = 0; d < 8; d++) {
        g = gear_cmp_step<0>(m, g, w[d]);
        if (TILE) tile[(4 * d + 0) * XC_TILE_ROW + l] = g;
        g = gear_cmp_step<1>(m, g, w[d]);
        if (TILE) tile[(4 * d + 1) * XC_TILE_ROW + l] = g;
        g = gear_cmp_step<2>(m, g, w[d]);
        if (TILE) tile[(4 * d + 2) * XC_TILE_ROW + l] = g;
        g = gear_cmp_step<3>(m, g, w[d]);
        if (TILE) tile[(4 * d + 3) * XC_TILE_ROW + l] = g;
    }
    // 32 compares so far: position -1 (shifted out of the word by the 32nd) and positions 0..30
    return mask_last(m, g);
}

// G at position t (wave-uniform, < 32) of every lane, from G at position -1.
__device__ __forceinline__ uint32_t gear_at(const uint32_t w[8], uint32_t g, uint32_t t)
{
#pragma unroll
    for (int d = 0; d < 8; d++) {
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const uint32_t gn = (g << 1) + ((w[d] >> (8 * k)) & 0xffu);
            g = (uint32_t)(4 * d + k) <= t ? gn : g;
        }
    }
    return g;
}

// Anchor mask of the lane's 32 positions below `lim` (bit 31 - t: position t), from G at position -1
// (the plain form of gear_mask for the other levels of a segment's key).
__device__ __forceinline__ uint32_t gear_mask_below(const uint32_t w[8], uint32_t g, uint32_t lim)
{
    uint32_t m = 0;
#pragma unroll
    for (int d = 0; d < 8; d++) {
#pragma unroll
        for (int k = 0; k < 4; k++) {
            g = (g << 1) + ((w[d] >> (8 * k)) & 0xffu);
            m = (m << 1) | (g < lim ? 1u : 0u);
        }
    }
    return m;
}

// The segment's key from its anchor mask m (one level): its last anchor j >= 63, or ANC_NONE.
__device__ __forceinline__ uint64_t seg_key_of_mask(const uint32_t w[8], uint32_t gi, uint32_t m)
{
    const uint32_t l = lane_id();
    // positions 32 l + t >= 63: lanes >= 2 all, lane 1 only t = 31 (bit 0)
    m = l >= 2u ? m : (l == 1u ? (m & 1u) : 0u);
    // the last anchor: the highest lane with one, its lowest bit (largest t)
    const uint32_t j = m ? 32u * l + 31u - (uint32_t)__builtin_ctz(m) : 0u;
    const uint64_t has = ballot(m != 0u);
    if (!has) return ANC_NONE;
    const int lj = 63 - __builtin_clzll(has);
    const uint32_t jj = readlane(j, lj), t = jj & 31u;
    const uint32_t g = gear_at(w, gi, t);
    return anc_key(anc_fp(readlane(g, lj), readlane(g, lj - 1)), jj);
}

// wave_seg_anchor's key by one lane (a rare case inside a lane-per-block kernel): G(p) and G(p - 32)
// by two rolling sums, the last position of each level.
__device__ __forceinline__ uint64_t seg_key_serial(const uint8_t *seg)
{
    uint32_t g1 = 0, g2 = 0, j[3] = {NONE_U32, NONE_U32, NONE_U32}, a[3] = {0, 0, 0}, c[3] = {0, 0, 0};
    for (uint32_t p = 0; p < XC_SEG; p++) {
        g1 = (g1 << 1) + seg[p];
        g2 = (g2 << 1) + (p >= 32u ? seg[p - 32u] : 0u);
        if (p < 63u) continue;
#pragma unroll
        for (int v = 0; v < 3; v++)
            if (g1 < (ANC_G_LIMIT << v)) {
                j[v] = p;
                a[v] = g1;
                c[v] = g2;
            }
    }
#pragma unroll
    for (int v = 0; v < 3; v++)
        if (j[v] != NONE_U32) return anc_key(anc_fp(a[v], c[v]), j[v]);
    return ANC_NONE;
}

// The anchor key of a 2048-byte segment held as 32 bytes per lane (lane l: bytes 32 l .. 32 l + 31),
// or ANC_NONE; every lane returns it.  Level 0: its last anchor (G < 2^26).  A segment with none
// (anchors cluster: about one random segment in 10^7) takes its last position with G < 2^27, or
// with G < 2^28 (levels 1, 2): the anchor scan finds those through the gap windows (k_aprop);
// ANC_NONE past level 2 (a constant run of most byte values, say).
__device__ __forceinline__ uint64_t wave_seg_anchor(const uint32_t w[8])
{
    const uint32_t gi = gear_prev(gear32(w), 0u);
    const uint64_t k0 = seg_key_of_mask(w, gi, gear_mask<false>(w, gi, nullptr));
    if (k0 != ANC_NONE) return k0;
    const uint64_t k1 = seg_key_of_mask(w, gi, gear_mask_below(w, gi, ANC_G_LIMIT << 1));
    if (k1 != ANC_NONE) return k1;
    return seg_key_of_mask(w, gi, gear_mask_below(w, gi, ANC_G_LIMIT << 2));
}

}  // namespace xc
