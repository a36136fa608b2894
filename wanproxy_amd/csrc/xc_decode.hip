// xc_decode.hip — XCodec batch decoder for gfx950 (CDNA4).
//
// Reference: XCodecDecoder::decode (xcodec/xcodec_decoder.cc:76-176), one call per stream,
// streams in index order, one shared XCodecMemoryCache.  Pipeline:
//
//   k_dtok     one wave per stream: F1 search in 4 KiB windows loaded two ahead -> tokens
//              (literal run [lb, le) with F1 00 escapes, then the op at le); every EXTRACT
//              payload hashed as it is passed (H, xcodec_hash.h:166-174) and entered in the
//              batch provider table, min-merged by (stream, token).  With the input ready it
//              runs on a side stream beside the previous run's emit; else also the run's
//              prologue and round 0's cache probes (k_dtok<true, true>)
//   k_dres1    later rounds only: EXTRACT vs the cache (equal -> ok, different -> collision,
//              decode returns false, xcodec_decoder.cc:120-132; absent -> candidate provider)
//   k_dres2    every token against cache + earlier providers: REF data source or unknown
//              (xcodec_decoder.cc:142-166); later duplicate EXTRACTs compared with the first;
//              per stream the first token that stops the decode, ENTER ordinals.  Round 0
//              after an early parse: the prologue and the EXTRACT cache probes too
//   k_dfin     workgroup 0: the cache slots of the ENTER tokens; the others: round
//              consistency (a provider past its own stream's stop: the host re-resolves, rare)
//   k_demit    unescape literals, copy EXTRACT payloads (first-seen ones into their cache
//              slots too), gather REF segments; enter the first-seen hashes in the cache
#include <hip/hip_runtime.h>
#include <sched.h>

#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/xcodec_hip.h"
#include "xc_kernels.h"
#include "xc_env.h"

namespace xc {

constexpr uint32_t T_EXTRACT = 1, T_REF = 2, T_END = 3, T_WAIT = 4, T_BADOP = 5;
constexpr uint32_t R_OKCACHE = 1, R_ENTER = 2, R_OKPROV = 3, R_UNKNOWN = 4, R_COLL = 5, R_PENDING = 6;
constexpr uint64_t SRC_PROV = 1ull << 63;

struct DecDev {
    const uint8_t *in;
    const uint64_t *in_off;
    const uint32_t *in_len;
    uint32_t ns;
    const uint32_t *tok_base;  // [ns]
    uint32_t *tok_cnt;         // [ns]
    uint32_t *t_lb, *t_le, *t_op, *t_stat;
    uint64_t *t_h, *t_src;
    uint32_t *s_stop;          // executed tokens per stream (the stop token included: its literal runs)
    uint32_t *s_lim;           // tokens eligible as EXTRACT providers this round
    uint32_t *s_slot;          // first cache slot of the stream's entered segments
    uint2 *s_cnt;              // executed (REF, EXTRACT) tokens of the stream (k_dfin sums them)
    uint32_t *s_xp;            // an executed token of the stream has a provider in another stream
    uint8_t *out;
    const uint64_t *out_off;
    const uint64_t *out_cap;
    uint64_t *out_len, *consumed, *unknown;
    int32_t *status, *has_unknown;
    DevSet cache;
    SegStore segs;
    uint32_t *seg_count;
    uint32_t seg_cap;
    uint2 *undo;
    DevSet dset;
    DevSet dset_other;          // k_dres2<true> clears it (when clr_full): the other token set's table,
    uint32_t clr_lo, clr_full;  // whose last reader, the run before's k_dres2, is done
    uint32_t *ctl;
    int count;                 // k_dfin: count executed REF / EXTRACT tokens into ctl
    uint32_t *ctl_host;        // k_dfin: publish the control words here (mapped host memory)
};

enum : uint32_t {
    DCTL_FIX = 0, DCTL_ERR = 1, DCTL_NENTER = 2, DCTL_NREF = 3, DCTL_NEXTRACT = 4,
    DCTL_MAYBE = 5,   // k_dfin: an output may not fit (workgroup 0's sum of k_dres2's flags)
    DCTL_TICKET = 6,  // k_dfin's finished workgroups (its last one resets it)
    DCTL_WORDS = 8
};
// DCTL_ERR bits: 1 an output capacity is too small (k_demit), 2 the cache is full (k_dfin),
// 4 an output may not fit (k_dres2's bound: the words are then final only after k_demit)
constexpr uint32_t DERR_MAYBE_OUT = 4u;

// The control words to the run's mapped host buffer, the last word (unused: the host's sentinel)
// cleared only after the others are visible (one thread).
__device__ __forceinline__ void dctl_publish(const DecDev &D)
{
    if (!D.ctl_host) return;
    __threadfence();
    for (uint32_t i = 0; i + 1u < DCTL_WORDS; i++) D.ctl_host[i] = __atomic_load_n(&D.ctl[i], __ATOMIC_RELAXED);
    __threadfence_system();
    D.ctl_host[DCTL_WORDS - 1] = 0u;
    __threadfence_system();
}

// Emit kernels stand down while a resolution round asks for another one.
__device__ __forceinline__ bool fix_pending(const DecDev &D)
{
    return __builtin_amdgcn_readfirstlane((int)*(volatile const uint32_t *)&D.ctl[DCTL_FIX]) != 0;
}

__device__ __forceinline__ void dclear_range(const DecDev &D, uint32_t n_lo, uint32_t n_full, uint32_t i0,
                                             uint32_t stride);
__device__ __forceinline__ void dset_clear_range(const DevSet &s, uint32_t n_lo, uint32_t n_full, uint32_t i0,
                                                 uint32_t stride);

// Streaming tokenizer (round 3): the stream is read in 4 KiB windows, two windows ahead of the
// one being tokenized (lane l: bytes 64 l .. 64 l + 63 of a window, 4 dwordx4 loads), so the
// per-EXTRACT load latency of the 1 KiB windows (one dependent round trip per payload skipped)
// becomes a stream of independent loads.  Each window's F1 positions are a 64-bit mask per lane
// (lane l: positions 64 l ..); its bytes go to the wave's LDS copy, from which the op byte and a
// REF's hash bytes are read (a token whose 10 bytes cross the window's end reads them from memory).
// Token semantics: xcodec_decoder.cc:85-173.
constexpr uint32_t DTOK_WIN = 4096;

__device__ __forceinline__ uint32_t magic_mask4(uint32_t d)
{
    // bytes equal to F1: x = d ^ F1F1F1F1 has zero bytes there; exact per-byte zero test
    const uint32_t x = d ^ 0xF1F1F1F1u;
    const uint32_t t = ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x) & 0x80808080u;  // bit 7 of each zero byte
    return ((t >> 7) & 1u) | ((t >> 14) & 2u) | ((t >> 21) & 4u) | ((t >> 28) & 8u);
}

__device__ __forceinline__ void dtok_load(uint4 (&v)[4], const uint8_t *s, uint32_t w0)
{
    const uint4 *q = (const uint4 *)(s + w0 + 64u * lane_id());
#pragma unroll
    for (int i = 0; i < 4; i++) v[i] = q[i];
}

// The window's F1 mask of lane l (bit i: position w0 + 64 l + i), positions < n only.
__device__ __forceinline__ uint64_t dtok_mask(const uint4 (&v)[4], uint32_t w0, uint32_t n)
{
    uint64_t m = 0;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const uint32_t d[4] = {v[i].x, v[i].y, v[i].z, v[i].w};
#pragma unroll
        for (int k = 0; k < 4; k++) m |= (uint64_t)magic_mask4(d[k]) << (16 * i + 4 * k);
    }
    const uint32_t base = w0 + 64u * lane_id();
    if (n < base + 64u) m = n <= base ? 0ull : m & ((1ull << (n - base)) - 1ull);
    return m;
}

// The batch provider table's insert: the least (stream, token) per hash (xcodec_decoder.cc:101-132,
// the first EXTRACT of a hash provides it). set_find reads only the keys and values, so the
// decoder's tables keep no filters: one CAS claim and one atomicMin.
__device__ __forceinline__ void prov_insert(const DevSet &s, uint64_t h, uint64_t val)
{
    uint32_t i = key_slot(h, s.mask);
    for (;;) {
        const uint64_t prev = atomicCAS((unsigned long long *)&s.keys[i], (unsigned long long)XC_EMPTY64,
                                        (unsigned long long)h);
        if (prev == XC_EMPTY64 || prev == h) break;
        i = (i + 1u) & s.mask;
    }
    atomicMin((unsigned long long *)&s.vals[i], (unsigned long long)val);
}

__device__ __forceinline__ uint64_t dreadlane64(uint64_t x, int l)
{
    return ((uint64_t)readlane((uint32_t)(x >> 32), l) << 32) | readlane((uint32_t)x, l);
}

// Bytes x .. x + 31 of the stream from the wave's 8 KiB LDS ring (position p at ring byte p & 8191):
// three aligned 16-byte reads and a funnel by x & 15 (uniform across the wave when x = start + 32 l).
__device__ __forceinline__ void ring_read32(const uint32_t *ring, uint32_t x, uint32_t (&o)[8])
{
    const uint32_t b = x & (2u * DTOK_WIN - 1u), a16 = b & ~15u, dsh = (b >> 2) & 3u, sh = b & 3u;
    uint32_t d[12];
#pragma unroll
    for (int i = 0; i < 3; i++) {
        const uint4 v = *(const uint4 *)((const uint8_t *)ring + ((a16 + 16u * i) & (2u * DTOK_WIN - 1u)));
        d[4 * i] = v.x; d[4 * i + 1] = v.y; d[4 * i + 2] = v.z; d[4 * i + 3] = v.w;
    }
#pragma unroll
    for (int k = 0; k < 8; k++) {
        const uint32_t lo = dsh == 0 ? d[k] : dsh == 1 ? d[k + 1] : dsh == 2 ? d[k + 2] : d[k + 3];
        const uint32_t hi = dsh == 0 ? d[k + 1] : dsh == 1 ? d[k + 2] : dsh == 2 ? d[k + 3] : d[k + 4];
        o[k] = __builtin_amdgcn_alignbyte(hi, lo, sh);
    }
}

// first: also the run's prologue, spread over the tokenizer's threads (the control words, every
// stream's provider limit and, unless HASH, the round-0 batch provider table): launches less.
// HASH: round 0 of the provider resolution too (k_dres1<true>'s work, xcodec_hash.h:166-174 and
// xcodec_decoder.cc:101-132): every EXTRACT payload is hashed from the wave's LDS ring of the two
// latest windows as the tokenizer passes it (no second read of the payloads), and 64 at a time the
// cache probes, collisions and batch-table inserts run lane-parallel (the batch table was cleared by
// k_dclear before this kernel: its inserts must not race with a clear).
// PROBE = false (with HASH): the parse alone, input-only work (tokens and every EXTRACT's hash): it
// runs on a side stream as soon as a run is submitted with its input ready, beside the previous
// run's emit; k_dres2<true> then does round 0's cache probes on the context stream.
template <bool HASH, bool PROBE>
__global__ __launch_bounds__(64) void k_dtok(DecDev D, int fill, int first, uint32_t n_lo, uint32_t n_full)
{
    __shared__ uint32_t win[(HASH ? 2u : 1u) * DTOK_WIN / 4 + 8];
    const uint32_t j = blockIdx.x;
    if (first) {
        if (j == 0 && threadIdx.x < DCTL_WORDS) D.ctl[threadIdx.x] = 0u;
        if (j < D.ns && threadIdx.x == 0) D.s_lim[j] = 0xFFFFFFFFu;
        if (!HASH) dclear_range(D, n_lo, n_full, j * 64u + threadIdx.x, gridDim.x * 64u);
    }
    if (j >= D.ns) return;
    const uint8_t *s = D.in + D.in_off[j];
    const uint32_t n = D.in_len[j];
    const uint32_t tb = fill ? D.tok_base[j] : 0u;
    const uint32_t l = lane_id();
    constexpr uint32_t RING = (HASH ? 2u : 1u) * DTOK_WIN - 1u;  // ring byte mask
    uint32_t nt = 0, lb = 0, p = 0;
    auto put = [&](uint32_t op, uint32_t le, uint64_t h) {
        if (fill && l == 0) {
            D.t_lb[tb + nt] = lb;
            D.t_le[tb + nt] = le;
            D.t_op[tb + nt] = op;
            if (!HASH || op != T_EXTRACT) D.t_h[tb + nt] = h;  // (HASH: the probes write it)
        }
        nt++;
    };
    // HASH: lane i holds the i-th EXTRACT of the current batch of 64 (hash, token, payload start)
    uint64_t xh = 0;
    uint32_t xt = 0, xx = 0, xn = 0;
    uint32_t pend_x = NONE, pend_t = 0;  // an EXTRACT whose payload ends in the next window
    auto flush = [&]() {
        const bool ex = l < xn;
        if (!PROBE) {
            // every EXTRACT into the batch table (cleared before the parse): the table is consulted
            // only for hashes the cache lacks, and a hash the cache holds is held for every token
            // that carries it, so entering those too changes no answer (k_dres2<true> probes the cache)
            if (ex) prov_insert(D.dset, xh, ((uint64_t)j << 32) | xt);  // (round 0: no limit)
            if (ex && fill) D.t_h[tb + xt] = xh;
            xn = 0;
            return;
        }
        uint64_t v = 0;
        uint32_t st = 0;
        const bool hit = ex && set_find(D.cache, xh, &v);
        if (ex && !hit) {
            st = R_PENDING;
            prov_insert(D.dset, xh, ((uint64_t)j << 32) | xt);  // (round 0: no limit)
        }
        for (uint64_t mh = ballot(hit); mh; mh &= mh - 1) {  // a cached hash: the bytes (rare)
            const int fh = __ffsll((unsigned long long)mh) - 1;
            const bool eq = wave_equal2048(s + readlane(xx, fh), seg_at(D.segs, dreadlane64(v, fh)));
            if ((int)l == fh) st = eq ? R_OKCACHE : R_COLL;
        }
        if (ex && fill) {
            D.t_h[tb + xt] = xh;
            D.t_stat[tb + xt] = st;
            D.t_src[tb + xt] = st == R_OKCACHE ? v : 0;
        }
        xn = 0;
    };
    auto hash_at = [&](uint32_t x, uint32_t t) {  // payload x .. x + 2047, inside the ring
        uint32_t w8[8];
        ring_read32(win, x + 32u * l, w8);
        const uint64_t h = wave_hash_regs(w8);
        if (l == xn) { xh = h; xt = t; xx = x; }
        if (++xn == 64u) flush();
    };
    const uint32_t nw = (n + DTOK_WIN - 1u) / DTOK_WIN;
    // (only windows that start inside the stream are read: past the last, it is read again)
    const uint32_t last = nw ? (nw - 1u) * DTOK_WIN : 0u;
    uint4 v0[4], v1[4], v2[4];
    dtok_load(v0, s, 0u);
    dtok_load(v1, s, min(DTOK_WIN, last));
    // window k from cur (its loads issued two windows earlier); window k + 2's loads into fut (the
    // set of window k - 1): three statically named sets, so no register copy waits on a load in flight
    auto step = [&](uint4 (&cur)[4], uint4 (&fut)[4], uint32_t k) -> bool {
        const uint32_t w0 = k * DTOK_WIN;
        dtok_load(fut, s, min(w0 + 2u * DTOK_WIN, last));  // (unconditional: a static vmcnt)
        const uint64_t mask = dtok_mask(cur, w0, n);
        // the window into LDS (the previous window's readers are done: every read was waited for;
        // HASH: the ring's other half keeps the window before)
        uint4 *wl = (uint4 *)((uint8_t *)win + (w0 & RING)) + 4u * l;
#pragma unroll
        for (int i = 0; i < 4; i++) wl[i] = cur[i];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (HASH && pend_x != NONE) {  // its payload ends in this window
            hash_at(pend_x, pend_t);
            pend_x = NONE;
        }
        const uint32_t base = w0 + 64u * l;
        for (;;) {
            uint64_t mm = mask;
            if (p > base) mm = p - base >= 64u ? 0ull : mm & (~0ull << (p - base));
            const uint64_t b = ballot(mm != 0ull);
            if (!b) return false;  // no F1 in [p, window end): the literal run goes on
            const int f = __ffsll((unsigned long long)b) - 1;
            const uint64_t mf = ((uint64_t)readlane((uint32_t)(mm >> 32), f) << 32) | readlane((uint32_t)mm, f);
            const uint32_t q = w0 + 64u * (uint32_t)f + (uint32_t)__builtin_ctzll(mf);
            if (q + 1u >= n) { put(T_WAIT, q, 0); return true; }
            const uint32_t r = q + 1u - w0;  // the op byte's window offset (<= 4096)
            uint32_t op;
            uint64_t h = 0;
            if (r + 9u <= DTOK_WIN) {  // op and 8 hash bytes inside the window
                const uint32_t i = ((q + 1u) & RING) >> 2, o = r & 3u;
                const uint32_t d0 = win[i], d1 = win[i + 1u], d2 = win[i + 2u];
                op = (d0 >> (8u * o)) & 0xffu;
                // hash bytes r + 1 .. r + 8: bytes o + 1 .. o + 8 of d0 d1 d2
                const uint32_t a = o + 1u;  // 1..4
                const uint32_t lo = a == 4u ? d1 : __builtin_amdgcn_alignbyte(d1, d0, a);
                const uint32_t hi = a == 4u ? d2 : __builtin_amdgcn_alignbyte(d2, d1, a);
                h = ((uint64_t)__builtin_bswap32(lo) << 32) | __builtin_bswap32(hi);
            } else {
                op = s[q + 1u];
                if (op == 0x02u && n - q >= 10u)
                    for (uint32_t k2 = 0; k2 < 8; k2++) h = (h << 8) | s[q + 2u + k2];
            }
            if (op == 0x00u) { p = q + 2u; continue; }  // escape: stays inside the literal run
            if (op == 0x01u) {
                if (n - q < 2u + XC_SEG) { put(T_WAIT, q, 0); return true; }
                const uint32_t t = nt;
                put(T_EXTRACT, q, 0);
                if (HASH) {
                    if (q + 2u + XC_SEG <= w0 + DTOK_WIN) hash_at(q + 2u, t);
                    else { pend_x = q + 2u; pend_t = t; }  // (the window's last token)
                }
                lb = p = q + 2u + XC_SEG;
                continue;
            }
            if (op == 0x02u) {
                if (n - q < 10u) { put(T_WAIT, q, 0); return true; }
                put(T_REF, q, h);
                lb = p = q + 10u;
                continue;
            }
            put(T_BADOP, q, 0);
            return true;
        }
    };
    bool done = false;
    for (uint32_t k = 0; k < nw && !done; k += 3u) {
        done = step(v0, v2, k);
        if (!done && k + 1u < nw) done = step(v1, v0, k + 1u);
        if (!done && k + 2u < nw) done = step(v2, v1, k + 2u);
    }
    if (!done) put(T_END, n, 0);
    if (HASH && xn) flush();
    if (l == 0) D.tok_cnt[j] = nt;
}
template __global__ void k_dtok<true, true>(DecDev, int, int, uint32_t, uint32_t);
template __global__ void k_dtok<true, false>(DecDev, int, int, uint32_t, uint32_t);

// k_dres1 / k_dres2 grids: (streams, DRES_WAVES), wave y taking tokens y, y + DRES_WAVES, ...
#ifndef XC_DRES_WAVES
#define XC_DRES_WAVES 4
#endif
constexpr uint32_t DRES_WAVES = XC_DRES_WAVES;

// EXTRACTs against the cache; absent ones become provider candidates in the batch table.
// HASH (round 0): the payloads' hashes H first (xcodec_hash.h:166-174), kept in t_h.
// A payload's 2048 bytes as raw dword loads (lane l: bytes 32 l ..), aligned only when used, so
// that the next payload's loads stay in flight while the current one is hashed and looked up.
struct RawWin {
    uint32_t d[9];
    uint32_t sh;
};

__device__ __forceinline__ void raw_load(RawWin &r, const uint8_t *p)
{
    const uintptr_t a = (uintptr_t)(p + 32u * lane_id());
    const uint32_t *w = (const uint32_t *)(a & ~(uintptr_t)3);
    r.sh = (uint32_t)(a & 3);
#pragma unroll
    for (int k = 0; k < 9; k++) r.d[k] = w[k];  // (the ninth dword: the input arena has slack)
}

__device__ __forceinline__ void raw_align(const RawWin &r, uint32_t out[8])
{
#pragma unroll
    for (int k = 0; k < 8; k++) out[k] = __builtin_amdgcn_alignbyte(r.d[k + 1], r.d[k], r.sh);
}


template <bool HASH>
__global__ __launch_bounds__(64) void k_dres1(DecDev D)
{
    const uint32_t j = blockIdx.x;
    if (j >= D.ns) return;
    const uint8_t *s = D.in + D.in_off[j];
    const uint32_t tb = D.tok_base[j], n = D.tok_cnt[j];
    const uint32_t lim = D.s_lim[j];
    if (HASH) {
        // round 0: the wave's tokens 64 at a time (lane i: token t0 + i * gridDim.y): their
        // EXTRACT payloads hashed in token order with the next payload's loads issued before this
        // one is used, then every probe and insert at once, one lane per token
        const uint32_t l = lane_id();
        for (uint32_t t0 = blockIdx.y; t0 < n; t0 += 64u * gridDim.y) {
            const uint32_t tl = t0 + l * gridDim.y;
            const bool ex = tl < n && D.t_op[tb + tl] == T_EXTRACT;
            const uint32_t le = ex ? D.t_le[tb + tl] : 0u;
            uint64_t m = ballot(ex);
            if (!m) continue;
            int f = __ffsll((unsigned long long)m) - 1;
            RawWin cur, nxt;
            raw_load(cur, s + readlane(le, f) + 2u);
            // the hashes, wave-wide, each kept by its token's lane
            uint64_t hl = 0;
            for (uint64_t mm = m;;) {
                mm &= mm - 1;
                const int fn = mm ? __ffsll((unsigned long long)mm) - 1 : -1;
                if (fn >= 0) raw_load(nxt, s + readlane(le, fn) + 2u);
                uint32_t w[8];
                raw_align(cur, w);
                const uint64_t h = wave_hash_regs(w);
                if ((int)l == f) hl = h;
                if (fn < 0) break;
                cur = nxt;
                f = fn;
            }
            // the cache probes and the batch table's inserts, lane-parallel
            uint64_t v = 0;
            uint32_t st = 0;
            const bool hit = ex && set_find(D.cache, hl, &v);
            if (ex && !hit) {
                st = R_PENDING;
                if (tl < lim) prov_insert(D.dset, hl, ((uint64_t)j << 32) | tl);
            }
            // a cached hash: its payload against the cached segment, wave-wide (rare)
            for (uint64_t mh = ballot(hit); mh; mh &= mh - 1) {
                const int fh = __ffsll((unsigned long long)mh) - 1;
                const bool eq = wave_equal2048(s + readlane(le, fh) + 2u, seg_at(D.segs, dreadlane64(v, fh)));
                if ((int)l == fh) st = eq ? R_OKCACHE : R_COLL;
            }
            if (ex) {
                D.t_h[tb + tl] = hl;
                D.t_stat[tb + tl] = st;
                D.t_src[tb + tl] = st == R_OKCACHE ? v : 0;
            }
        }
        return;
    }
    for (uint32_t t = blockIdx.y; t < n; t += gridDim.y) {
        if (uniform(D.t_op[tb + t]) != T_EXTRACT) continue;
        const uint8_t *pay = s + D.t_le[tb + t] + 2u;
        uint64_t h;
        if (HASH) {
            h = wave_window_hash(pay);
            if (lane_id() == 0) D.t_h[tb + t] = h;
        } else {
            h = D.t_h[tb + t];
        }
        uint64_t v;
        uint32_t st;
        if (set_find(D.cache, h, &v)) {
            st = wave_equal2048(pay, seg_at(D.segs, v)) ? R_OKCACHE : R_COLL;
        } else {
            st = R_PENDING;
            if (lane_id() == 0 && t < lim) prov_insert(D.dset, h, ((uint64_t)j << 32) | t);
        }
        if (lane_id() == 0) {
            D.t_stat[tb + t] = st;
            D.t_src[tb + t] = st == R_OKCACHE ? v : 0;
        }
    }
}


// Provider resolution in (stream, token) order, and the stream's stop: one wave per stream, one lane
// per token (every probe of 64 tokens in flight together); an EXTRACT with an earlier provider then
// takes a wave-wide 2048-byte comparison (rare: the same new segment twice in a batch). The first
// token that stops the decode (terminal, unknown REF or colliding EXTRACT) ends the walk; the
// stream's executed token count, status / consumed bytes, and the ordinal of every first-seen
// EXTRACT (ENTER) among its executed tokens, kept in t_src (unused for ENTER tokens); s_slot[j] =
// the stream's ENTER count (k_dfin prefixes it). Tokens past the stop are left as they were: no
// later kernel reads them.
// PROBE (round 0 after an early parse, k_dtok<true, false>): round 0's cache probes in the same
// pass, so the context stream runs no kernel between the parse and this one: the run's prologue
// (control words, provider limits, the other token set's table cleared) and every EXTRACT's cache
// probe (a hit's payload compared wave-wide: rare; xcodec_decoder.cc:101-132) before its provider
// lookup (a separate probe kernel: cfg4 1398-1399 against 1428-1435 GiB/s, ab/dres2_probe_r6dp.txt).
// The output-bound flag goes to k_dfin in bit 31 of s_cnt[j].x (no atomic on a control word
// that workgroup 0 zeroes here).
template <bool PROBE>
__global__ __launch_bounds__(64) void k_dres2(DecDev D)
{
    const uint32_t l = lane_id(), j = blockIdx.x;
    if (PROBE) {
        if (j == 0 && threadIdx.x < DCTL_WORDS) D.ctl[threadIdx.x] = 0u;
        if (D.clr_full) dset_clear_range(D.dset_other, D.clr_lo, D.clr_full, j * 64u + l, gridDim.x * 64u);
        if (j < D.ns && threadIdx.x == 0) D.s_lim[j] = 0xFFFFFFFFu;
    }
    if (j >= D.ns) return;
    const uint8_t *s = D.in + D.in_off[j];
    const uint32_t tb = D.tok_base[j], n = D.tok_cnt[j];
    const uint64_t cap = D.out_cap[j];
    uint32_t stop = n, nr = 0, ne = 0, nent = 0;
    uint32_t sop = T_END, sle = 0;  // the stopping token's op and end (its lane's registers)
    uint64_t sh = 0;
    bool xprov = false;  // an executed token with a provider in another stream (k_dfin checks it)
    uint64_t lit = 0;  // literal bytes of the executed tokens and the stop token (escapes counted twice)
    for (uint32_t t0 = 0; t0 < n; t0 += 64u) {
        const uint32_t t = t0 + l;
        uint32_t op = T_END, ll = 0, le = 0;
        if (t < n) {
            op = D.t_op[tb + t];
            le = D.t_le[tb + t];
            ll = le - D.t_lb[tb + t];
        }
        const uint64_t self = ((uint64_t)j << 32) | t;
        uint32_t st = 0;
        uint64_t src = 0, pv = 0, h = 0;
        bool wst = false, wsrc = false, cmp = false, chit = false;
        if (op == T_EXTRACT) {
            h = D.t_h[tb + t];
            if (PROBE) {  // the cache first; a hit's bytes are compared below
                chit = set_find(D.cache, h, &pv);
                st = chit ? R_COLL : R_PENDING;
                wst = wsrc = true;
            } else {
                st = D.t_stat[tb + t];  // (round 0's cache probe, or k_dres1's)
            }
            if (st == R_PENDING) {
                uint64_t v;
                st = R_ENTER;
                wst = wsrc = true;
                if (set_find(D.dset, h, &v) && v < self) {
                    cmp = true;
                    pv = v;
                    src = SRC_PROV | v;
                }
            }
        } else if (op == T_REF) {
            h = D.t_h[tb + t];
            uint64_t v;
            st = R_UNKNOWN;
            wst = wsrc = true;
            if (set_find(D.cache, h, &v)) {
                st = R_OKCACHE;
                src = v;
            } else if (set_find(D.dset, h, &v) && v < self) {
                st = R_OKPROV;
                src = SRC_PROV | v;
            }
        } else if (t < n) {
            wst = true;
        }
        if (PROBE)  // a cached hash: the payload against the cached segment, wave-wide (rare)
            for (uint64_t m = ballot(chit); m; m &= m - 1) {
                const int f = __ffsll((unsigned long long)m) - 1;
                const bool eq = wave_equal2048(s + readlane(le, f) + 2u, seg_at(D.segs, dreadlane64(pv, f)));
                if ((int)l == f) {
                    st = eq ? R_OKCACHE : R_COLL;
                    src = eq ? pv : 0;
                }
            }
        for (uint64_t m = ballot(cmp); m; m &= m - 1) {
            const int f = __ffsll((unsigned long long)m) - 1;
            const uint64_t v = dreadlane64(pv, f);
            const uint32_t pj = (uint32_t)(v >> 32), pt = (uint32_t)v;
            const uint8_t *pp = D.in + D.in_off[pj] + D.t_le[D.tok_base[pj] + pt] + 2u;
            const bool eq = wave_equal2048(s + readlane(le, f) + 2u, pp);
            if ((int)l == f) st = eq ? R_OKPROV : R_COLL;
        }
        // the first token of these 64 that stops the decode
        const uint64_t brk = ballot(t < n && ((op != T_EXTRACT && op != T_REF) || st == R_UNKNOWN || st == R_COLL));
        const uint32_t k = brk ? (uint32_t)__ffsll((unsigned long long)brk) - 1u : 64u;
        lit += wave_sum(l <= k ? ll : 0u);
        const bool ex = l < k && t < n;
        xprov |= ballot(ex && (st == R_OKPROV || st == R_COLL) && (src & SRC_PROV) &&
                        (uint32_t)((src >> 32) & 0x7FFFFFFFu) != j) != 0ull;
        nr += (uint32_t)__popcll(ballot(ex && op == T_REF));
        ne += (uint32_t)__popcll(ballot(ex && op == T_EXTRACT));
        const uint64_t em = ballot(ex && st == R_ENTER);
        if (ex && st == R_ENTER) src = nent + mbcnt(em);
        nent += (uint32_t)__popcll(em);
        if (wst) D.t_stat[tb + t] = st;
        if (wsrc) D.t_src[tb + t] = src;
        if (brk) {
            stop = t0 + k;
            sop = readlane(op, k);
            sle = readlane(le, k);
            sh = dreadlane64(h, k);
            break;
        }
    }
    // the output is at most the literal bytes plus a segment per executed EXTRACT / REF: when
    // that may exceed the capacity, only k_demit's exact sizes decide (no early publication)
    const uint32_t maybe_out = lit + (uint64_t)XC_SEG * (nr + ne) > cap ? 0x80000000u : 0u;
    if (l == 0) {
        // stop = the stopping token; its literal is output
        D.s_stop[j] = stop + 1u;
        D.s_slot[j] = nent;  // (k_dfin prefixes the counts and ORs the flags into DCTL_ERR)
        D.s_cnt[j] = make_uint2(nr | maybe_out, ne);
        D.s_xp[j] = xprov ? 1u : 0u;
        int32_t status = 1, hu = 0;
        uint64_t cons = sle, unk = 0;
        if (sop == T_BADOP) status = 0;
        else if (sop == T_REF) { hu = 1; unk = sh; }                        // unknown REF
        else if (sop == T_EXTRACT) { status = 0; cons = sle + 2u; }         // collision
        D.status[j] = status;
        D.consumed[j] = cons;
        D.has_unknown[j] = hu;
        D.unknown[j] = unk;
    }
}

__device__ __forceinline__ void dset_clear_range(const DevSet &s, uint32_t n_lo, uint32_t n_full, uint32_t i0,
                                                 uint32_t stride)
{
    // (keys and values only: prov_insert and set_find use nothing else)
    (void)n_lo;
    const uint4 ones = make_uint4(~0u, ~0u, ~0u, ~0u);
    for (uint32_t i = i0; i < n_full / 2; i += stride) {
        ((uint4 *)s.keys)[i] = ones;
        ((uint4 *)s.vals)[i] = ones;
    }
}

__device__ __forceinline__ void dclear_range(const DecDev &D, uint32_t n_lo, uint32_t n_full, uint32_t i0,
                                             uint32_t stride)
{
    dset_clear_range(D.dset, n_lo, n_full, i0, stride);
}

// A resolution round's fresh batch provider table, its FIX flag and the token counters.
__global__ void k_dclear(DecDev D, uint32_t n_lo, uint32_t n_full)
{
    const uint32_t i0 = blockIdx.x * blockDim.x + threadIdx.x;
    dclear_range(D, n_lo, n_full, i0, gridDim.x * blockDim.x);
    if (i0 == 0) {
        D.ctl[DCTL_FIX] = 0u;
        D.ctl[DCTL_NREF] = 0u;
        D.ctl[DCTL_NEXTRACT] = 0u;
        D.ctl[DCTL_TICKET] = 0u;
    }
}


__global__ void k_dlim(DecDev D, int init)
{
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j < D.ns) D.s_lim[j] = init ? 0xFFFFFFFFu : D.s_stop[j] - 1u;
}

__device__ __forceinline__ uint32_t count_magic_d(const uint8_t *p, uint32_t n)
{
    uint32_t c = 0;
    for (uint32_t o = 4u * lane_id(); o < n; o += 256u) {
#pragma unroll
        for (uint32_t k = 0; k < 4; k++)
            if (o + k < n) c += p[o + k] == XC_MAGIC ? 1u : 0u;
    }
    return wave_sum(c);
}

// Unescape a literal run: every F1 is followed by the escape's 00, which is dropped.
__device__ __forceinline__ void write_unescaped(uint8_t *dst, const uint8_t *p, uint32_t n)
{
    uint32_t o = 0;
    for (uint32_t x = 0; x < n; x += 256u) {
        const uint32_t s = x + 4u * lane_id();
        uint32_t v[4], keep = 0, cnt = 0;
#pragma unroll
        for (uint32_t k = 0; k < 4; k++) {
            const uint32_t i = s + k;
            v[k] = i < n ? p[i] : 0u;
            const bool drop = i >= n || (i > 0 && p[i - 1] == XC_MAGIC);
            if (!drop) { keep |= 1u << k; cnt++; }
        }
        const uint32_t inc = wave_incl_scan(cnt);
        uint32_t q = o + inc - cnt;
#pragma unroll
        for (uint32_t k = 0; k < 4; k++)
            if (keep & (1u << k)) dst[q++] = (uint8_t)v[k];
        o += readlane(inc, 63);
    }
}

constexpr uint32_t DMAX_TOK = 2048;
constexpr uint32_t DEMIT_WAVES = 4;
// payloads a wave has in flight: 3 (one box, bench.py --only cfg4: 1491-1497 against 1469-1484 GiB/s at
// 2, profiles/r06/ab/demit_pay3_r6dg.txt; 4 and 6 were slower, demit_pay_r6l.txt)
#ifndef XC_DEMIT_PAY
#define XC_DEMIT_PAY 3
#endif
constexpr uint32_t DEMIT_PAY = XC_DEMIT_PAY;


// Output offsets (executed tokens only), then the bytes.  One workgroup (DEMIT_WAVES waves) per
// stream, tokens in blocks of DMAX_TOK: sizes lane-parallel (one token per lane; escapes counted
// only in non-empty literal runs), a prefix, then each wave writes a contiguous token group with
// DEMIT_PAY 2048-byte copies in flight.
__global__ __launch_bounds__(64 * DEMIT_WAVES) void k_demit(DecDev D)
{
    if (fix_pending(D)) return;
    __shared__ uint64_t off[DMAX_TOK + 1];
    __shared__ uint64_t base_off;
    const uint32_t j = blockIdx.x;
    if (j >= D.ns) return;
    const uint32_t wave = threadIdx.x >> 6, l = lane_id();
    const uint8_t *s = D.in + D.in_off[j];
    uint8_t *out = D.out + D.out_off[j];
    const uint32_t tb = D.tok_base[j];
    const uint32_t lim = min(D.tok_cnt[j], D.s_stop[j]);
    if (threadIdx.x == 0) base_off = 0;
    bool ovf = false;  // (uniform: an output past its capacity ends the writes)
    for (uint32_t t0 = 0; t0 < lim; t0 += DMAX_TOK) {
        const uint32_t nb = min(DMAX_TOK, lim - t0);
        __syncthreads();
        for (uint32_t i0 = wave * 64u; i0 < nb; i0 += 64u * DEMIT_WAVES) {
            const uint32_t i = i0 + l, t = t0 + i;
            uint32_t lb = 0, le = 0, op = T_END;
            if (i < nb) { lb = D.t_lb[tb + t]; le = D.t_le[tb + t]; op = D.t_op[tb + t]; }
            uint32_t sz = le - lb;
            for (uint64_t m = ballot(le > lb); m; m &= m - 1) {
                const int f = __ffsll((unsigned long long)m) - 1;
                const uint32_t flb = readlane(lb, f), fle = readlane(le, f);
                const uint32_t c = count_magic_d(s + flb, fle - flb);
                if ((int)l == f) sz -= c;
            }
            if (t + 1u != lim && (op == T_EXTRACT || op == T_REF)) sz += XC_SEG;
            if (i < nb) off[i] = sz;
        }
        __syncthreads();
        if (wave == 0) {
            uint64_t carry = base_off;
            for (uint32_t i0 = 0; i0 < nb; i0 += 64u) {
                const uint32_t i = i0 + l;
                const uint32_t v = i < nb ? (uint32_t)off[i] : 0u;
                const uint32_t inc = wave_incl_scan(v);
                if (i < nb) off[i] = carry + inc - v;
                carry += readlane(inc, 63);
            }
            if (l == 0) { off[nb] = carry; base_off = carry; }
        }
        __syncthreads();
        if (off[nb] > D.out_cap[j]) {
            if (threadIdx.x == 0) atomicOr(&D.ctl[DCTL_ERR], 1u);
            ovf = true;
            break;
        }
        // wave w: tokens [w G, (w+1) G) of the block, one per lane
        const uint32_t G = (nb + DEMIT_WAVES - 1u) / DEMIT_WAVES;
        const uint32_t g_end = min(nb, (wave + 1u) * G);
        for (uint32_t g0 = wave * G; g0 < g_end; g0 += 64u) {
            const uint32_t i = g0 + l, t = t0 + i;
            const bool live = i < g_end;
            uint32_t lb = 0, le = 0, op = T_END;
            uint64_t from = 0;  // source of the token's 2048 bytes
            uint64_t seg = 0;   // first-seen EXTRACT: its cache slot (k_dfin), written here too
            if (live) {
                lb = D.t_lb[tb + t];
                le = D.t_le[tb + t];
                op = t + 1u == lim ? T_END : D.t_op[tb + t];  // the stop token: its literal only
                if (op == T_EXTRACT) {
                    from = (uint64_t)(uintptr_t)(s + le + 2u);
                    if (D.t_stat[tb + t] == R_ENTER) {
                        const uint32_t idx = D.s_slot[j] + (uint32_t)D.t_src[tb + t];
                        if (idx < D.seg_cap) seg = (uint64_t)(uintptr_t)seg_at(D.segs, idx);
                    }
                } else if (op == T_REF) {
                    const uint64_t src = D.t_src[tb + t];
                    if (src & SRC_PROV) {
                        const uint32_t pj = (uint32_t)((src >> 32) & 0x7FFFFFFFu), pt = (uint32_t)src;
                        from = (uint64_t)(uintptr_t)(D.in + D.in_off[pj] + D.t_le[D.tok_base[pj] + pt] + 2u);
                    } else {
                        from = (uint64_t)(uintptr_t)seg_at(D.segs, src);
                    }
                }
            }
            for (uint64_t m = ballot(live && le > lb); m; m &= m - 1) {
                const int f = __ffsll((unsigned long long)m) - 1;
                const uint32_t flb = readlane(lb, f);
                write_unescaped(out + off[readlane(i, f)], s + flb, readlane(le, f) - flb);
            }
            // DEMIT_PAY payloads in flight (their loads first, then the stores)
            for (uint64_t m = ballot(from != 0); m;) {
                int f[DEMIT_PAY];
                PayloadRegs r[DEMIT_PAY];
#pragma unroll
                for (int k = 0; k < (int)DEMIT_PAY; k++) {
                    f[k] = m ? __ffsll((unsigned long long)m) - 1 : -1;
                    if (m) m &= m - 1;
                    if (f[k] >= 0)
                        payload_load((const uint8_t *)(uintptr_t)dreadlane64(from, f[k]), nullptr, r[k]);
                }
#pragma unroll
                for (int k = 0; k < (int)DEMIT_PAY; k++)
                    if (f[k] >= 0)
                        payload_store(out + off[readlane(i, f[k]) + 1u] - XC_SEG,
                                      (uint8_t *)(uintptr_t)dreadlane64(seg, f[k]), r[k]);
            }
        }
    }
    __syncthreads();
    if (threadIdx.x == 0 && !ovf) D.out_len[j] = base_off;
    // XCodecMemoryCache::enter for the first-seen EXTRACT payloads (xcodec_decoder.cc:133-135),
    // whose slots this workgroup filled above; one thread per token
    const uint32_t clim = min(D.tok_cnt[j], D.s_stop[j] - 1u);
    for (uint32_t t = threadIdx.x; t < clim; t += 64u * DEMIT_WAVES) {
        if (D.t_stat[tb + t] != R_ENTER) continue;
        const uint32_t idx = D.s_slot[j] + (uint32_t)D.t_src[tb + t];
        if (idx >= D.seg_cap) continue;
        uint32_t s1, s2;
        set_insert(D.cache, D.t_h[tb + t], idx, false, &s1, &s2);
        D.undo[idx] = make_uint2(s1, s2);
    }
}

// The end of a resolution round. Workgroup 0 takes the cache slots of the streams' ENTER tokens:
// the exclusive prefix of the per-stream counts k_dres2 left in s_slot, on top of the current
// segment count.  Beside it the other workgroups check the round's consistency, one wave per
// stream: every provider used by an executed token must itself be executed, and (after round 0)
// the executed tokens must be exactly the eligible providers.  The last workgroup to finish (a
// ticket in the control words) commits the segment count unless another round is due, and
// publishes the control words.  (The slots after the checks, in the last workgroup: k_dfin
// 13.6 us a cfg4 step, ab/dfin_split_r6dfs.txt: 1430-1437 against 1467-1473 GiB/s.)
constexpr uint32_t DFIN_WAVES = 16, DFIN_REG = 8, DFIN_GRID = 128;
__global__ __launch_bounds__(64 * DFIN_WAVES) void k_dfin(DecDev D, int round)
{
    __shared__ uint32_t wsum[DFIN_WAVES];
    __shared__ uint2 csum[DFIN_WAVES];
    __shared__ uint32_t last;
    const uint32_t wave = threadIdx.x >> 6, l = lane_id();
    const uint32_t start = *D.seg_count;
    if (blockIdx.x == 0) {
        // workgroup 0: the slots, at once (a FIX decided by the others leaves them unused): a
        // contiguous range of streams per thread, its sums, a block prefix, its slots (up to
        // DFIN_REG streams per thread with every load in flight at once)
        const uint32_t per = (D.ns + 64u * DFIN_WAVES - 1u) / (64u * DFIN_WAVES);
        const uint32_t j0 = min(D.ns, threadIdx.x * per), j1 = min(D.ns, j0 + per);
        uint32_t sum = 0, nr = 0, ne = 0;  // ENTER tokens; executed REF / EXTRACT tokens (decode statistics)
        uint32_t mo = 0;                   // k_dres2's output-bound flags (bit 31 of s_cnt.x)
        uint32_t v[DFIN_REG];
        if (per <= DFIN_REG) {
            uint2 c[DFIN_REG];
#pragma unroll
            for (uint32_t k = 0; k < DFIN_REG; k++) {
                const bool in = j0 + k < j1;
                v[k] = in ? D.s_slot[j0 + k] : 0u;
                c[k] = in ? D.s_cnt[j0 + k] : make_uint2(0, 0);
            }
#pragma unroll
            for (uint32_t k = 0; k < DFIN_REG; k++) {
                sum += v[k];
                nr += c[k].x & 0x7FFFFFFFu;
                mo |= c[k].x;
                ne += c[k].y;
            }
        } else {
            for (uint32_t j = j0; j < j1; j++) {
                sum += D.s_slot[j];
                const uint2 c = D.s_cnt[j];
                nr += c.x & 0x7FFFFFFFu;
                mo |= c.x;
                ne += c.y;
            }
        }
        const uint32_t inc = wave_incl_scan(sum);
        nr = wave_sum(nr) | (ballot(mo >> 31) ? 0x80000000u : 0u);
        ne = wave_sum(ne);
        if (l == 63) wsum[wave] = inc;
        if (l == 0) csum[wave] = make_uint2(nr, ne);
        __syncthreads();
        uint32_t o = start + inc - sum;
        for (uint32_t k = 0; k < wave; k++) o += wsum[k];
        if (per <= DFIN_REG) {
#pragma unroll
            for (uint32_t k = 0; k < DFIN_REG; k++)
                if (j0 + k < j1) {
                    D.s_slot[j0 + k] = o;
                    o += v[k];
                }
        } else {
            for (uint32_t j = j0; j < j1; j++) {
                const uint32_t x = D.s_slot[j];
                D.s_slot[j] = o;
                o += x;
            }
        }
        if (threadIdx.x == 0) {  // (the totals for the last workgroup)
            uint32_t tot = 0, mw = 0;
            uint2 t = make_uint2(0, 0);
            for (uint32_t k = 0; k < DFIN_WAVES; k++) {
                tot += wsum[k];
                t.x += csum[k].x & 0x7FFFFFFFu;
                mw |= csum[k].x;
                t.y += csum[k].y;
            }
            D.ctl[DCTL_MAYBE] = mw >> 31;
            if (D.count) {
                D.ctl[DCTL_NREF] = t.x;
                D.ctl[DCTL_NEXTRACT] = t.y;
            }
            D.ctl[DCTL_NENTER] = tot;
        }
    } else {
        // the others: the round's consistency, each wave a stride of streams (a grid of at most
        // DFIN_GRID + 1 workgroups: every workgroup takes a ticket below, and device-scope atomics
        // on one word serialize across the XCDs)
        for (uint32_t j = (blockIdx.x - 1u) * DFIN_WAVES + wave; j < D.ns; j += (gridDim.x - 1u) * DFIN_WAVES) {
            const uint32_t tb = D.tok_base[j], ex = D.s_stop[j] - 1u, xp = D.s_xp[j];
            if (round > 0 && l == 0 && ex != D.s_lim[j]) atomicOr(&D.ctl[DCTL_FIX], 1u);
            if (!xp) continue;  // (no provider in another stream: nothing to check)
            for (uint32_t t = l; t < ex; t += 64u) {
                const uint64_t src = D.t_src[tb + t];
                const uint32_t st = D.t_stat[tb + t];
                if ((st == R_OKPROV || st == R_COLL) && (src & SRC_PROV)) {
                    const uint32_t pj = (uint32_t)((src >> 32) & 0x7FFFFFFFu), pt = (uint32_t)src;
                    if (pt + 1u >= D.s_stop[pj]) atomicOr(&D.ctl[DCTL_FIX], 1u);
                }
            }
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence();  // (release: this workgroup's FIX, or workgroup 0's slots and totals)
        last = atomicAdd(&D.ctl[DCTL_TICKET], 1u) == gridDim.x - 1u;
    }
    __syncthreads();
    if (!last || threadIdx.x != 0) return;
    __threadfence();  // (acquire: every workgroup's words)
    D.ctl[DCTL_TICKET] = 0u;
    if (fix_pending(D)) {  // another resolution round: the host decides it now
        dctl_publish(D);
        return;
    }
    const uint32_t carry = start + D.ctl[DCTL_NENTER];
    *D.seg_count = carry;
    if (D.ctl[DCTL_MAYBE]) D.ctl[DCTL_ERR] |= DERR_MAYBE_OUT;
    if (carry > D.seg_cap) D.ctl[DCTL_ERR] |= 2u;
    // final unless an output may overflow (k_demit then sets bit 1): the rest of the run
    // changes no control word
    if (!(D.ctl[DCTL_ERR] & DERR_MAYBE_OUT)) dctl_publish(D);
}

}  // namespace xc

using namespace xc;

// ------------------------------------------------------------------ host side ----------
// A decode plan (xc_dplan) fixes the stream lengths and output capacities of a batch and owns
// every device array, so xc_decode_run is device resident: one host round trip to decide the
// provider rounds (normally a single round), none for allocation.
//
// Token capacity: every EXTRACT / REF token consumes >= 10 input bytes and a stream ends in one
// terminal token (END / WAIT / bad op), so a stream of n bytes has <= n/10 + 1 tokens; the
// tokenizer writes them straight into per-stream slices (no counting pass).  Only EXTRACTs
// (>= 2050 bytes each) enter the batch provider table, which is sized by that bound.

// The cache object is defined in xc_runtime.hip; these accessors expose what we need.
extern "C" void xc__cache_count_unknown(xc_cache *c);
extern "C" int64_t xc__cache_host_count(xc_cache *c);
extern "C" int xc__cache_truncate(xc_cache *c, uint64_t keep);
extern "C" void xc__cache_set_host_count(xc_cache *c, int64_t n);
extern "C" int xc__cache_reserve(xc_cache *c, uint64_t extra);
extern "C" uint32_t xc__cache_gen(xc_cache *c);
extern "C" int xc__cache_devset(xc_cache *c, void *devset, SegStore *segs, uint32_t **count, uint32_t *cap,
                                uint2 **undo, void **stream, int *dev);
extern "C" int xc__set_error(int code, const char *msg);
extern "C" hipError_t xc__spin_wait(hipEvent_t ev);
extern "C" bool xc__query_due(int64_t *t0);
extern "C" int xc__dalloc(void **p, uint64_t bytes);
extern "C" int xc__halloc(void **p, uint64_t bytes);
extern "C" void xc__pfree(void *p);

#define DHIP(x)                                                                          \
    do {                                                                                 \
        hipError_t e_ = (x);                                                             \
        if (e_ != hipSuccess) return xc__set_error(XC_EDEVICE, hipGetErrorString(e_));   \
    } while (0)

template <class T>
static hipError_t dalloc(T **p, size_t n)
{
    // the runtime's caching pool (xc_runtime.hip): no hipMalloc per call
    return xc__dalloc((void **)p, std::max<size_t>(n, 1) * sizeof(T)) == XC_OK ? hipSuccess : hipErrorOutOfMemory;
}

struct xc_dplan {
    xc_cache *cache = nullptr;
    hipStream_t s = nullptr;
    int dev = 0;
    uint32_t ns = 0;
    std::vector<uint64_t> ioff, ooff;
    uint64_t in_bytes = 0, out_bytes = 0, in_total = 0, ntok = 0;
    uint32_t n_full = 0, n_lo = 0;
    DecDev D{};
    xc_decode_stats stats{};
    std::vector<void *> owned;
    uint32_t *h_ctl = nullptr;    // pinned copy of the control words (the run's host wait)
    uint32_t *d_hctl = nullptr;   // its device address (k_dfin publishes there)
    hipEvent_t ev_ctl = nullptr;
    int completion = XC_COMPLETE_RUN;  // xc_dplan_set_completion
    uint32_t cache_gen = 0;       // the cache arrays D holds (they move when the cache grows)
    std::vector<uint32_t> tok_base;  // host copy [ns + 1]
    bool internal = false;        // run by xc_decode_batch_host (its replay takes a XC__SLOW run)
    // xc_dplan_set_input_ready: runs parse their input on the side stream ps as soon as they are
    // submitted, beside the previous run's emit; the tokenizer's arrays alternate between two sets
    // (tset[k]: tok_cnt, t_lb, t_le, t_op, t_h) so that the parse never writes what a run before it
    // still reads. Set k's last readers are the kernels of the run two back, which precede the
    // run before's k_dfin on the context stream: once that run returned from its emit (settled),
    // the parse needs no event; else it waits for an event recorded on the context stream then
    bool input_ready = false;
    struct TokSet {
        uint32_t *tok_cnt = nullptr, *t_lb = nullptr, *t_le = nullptr, *t_op = nullptr;
        uint64_t *t_h = nullptr;
    } tset[2];
    int tcur = 0;
    hipStream_t ps = nullptr;
    hipEvent_t ev_parsed = nullptr, ev_free = nullptr;
    bool settled = false;
    // the batch provider tables of the two token sets: an early run's parse enters its EXTRACTs in
    // dsets[tcur], which the early run before it cleared in its k_dres2 (clean[tcur]; done before
    // the parse starts, as above), or else the side stream clears first
    DevSet dsets[2] = {};
    bool clean[2] = {false, false};
    uint64_t early_runs = 0;
    template <class T>
    int alloc(T **p, size_t n)
    {
        if (dalloc(p, n) != hipSuccess) return xc__set_error(XC_ENOMEM, "device allocation failed");
        owned.push_back((void *)*p);
        return XC_OK;
    }
};

extern "C" int xc_dplan_set_completion(xc_dplan *p, int mode)
{
    if (!p || (mode != XC_COMPLETE_RUN && mode != XC_COMPLETE_STREAM)) return xc__set_error(XC_EINVAL, "completion mode");
    p->completion = mode;
    return XC_OK;
}

extern "C" int xc_dplan_set_input_ready(xc_dplan *p, int ready)
{
    if (!p) return xc__set_error(XC_EINVAL, "null");
    p->input_ready = ready != 0;
    return XC_OK;
}

extern "C" void xc__cache_plan_gone_dec(xc_cache *c, void *dplan);
extern "C" int xc__cache_run_start(xc_cache *c, int *slow);
extern "C" void xc__cache_run_done_dec(xc_cache *c, void *dplan);
struct xc_memmodel;
extern "C" xc_memmodel *xc__cache_mem(xc_cache *c);
extern "C" int xc__mem_decode_batch(xc_memmodel *m, const uint8_t *in, const uint64_t *in_off,
                                    const uint64_t *in_len, uint64_t nbuf, uint8_t *out, const uint64_t *out_off,
                                    const uint64_t *out_cap, uint64_t *out_len, uint64_t *consumed, int32_t *status,
                                    uint64_t *unknown, int32_t *has_unknown);
constexpr int XC__SLOW = -1000;  // (xc_runtime.hip)

extern "C" int xc_dplan_destroy(xc_dplan *p)
{
    if (!p) return XC_OK;
    hipSetDevice(p->dev);
    if (p->cache) xc__cache_plan_gone_dec(p->cache, p);  // (its tokens are the window's record)
    hipStreamSynchronize(p->s);
    if (p->ps) hipStreamSynchronize(p->ps);
    for (void *x : p->owned) xc__pfree(x);
    if (p->h_ctl) xc__pfree(p->h_ctl);
    if (p->ev_ctl) hipEventDestroy(p->ev_ctl);
    if (p->ev_parsed) hipEventDestroy(p->ev_parsed);
    if (p->ev_free) hipEventDestroy(p->ev_free);
    if (p->ps) hipStreamDestroy(p->ps);
    delete p;
    return XC_OK;
}

extern "C" int xc_decode_plan_create(xc_cache *c, const uint64_t *in_len, const uint64_t *out_cap, uint64_t nbuf,
                                     xc_dplan **out)
{
    if (!c || !out || (nbuf && (!in_len || !out_cap))) return xc__set_error(XC_EINVAL, "null");
    if (nbuf > (1u << 24)) return xc__set_error(XC_EINVAL, "too many streams");
    xc_dplan *p = new xc_dplan();
    DecDev &D = p->D;
    void *streamv = nullptr;
    uint32_t cap = 0;
    int rc = xc__cache_devset(c, &D.cache, &D.segs, &D.seg_count, &cap, &D.undo, &streamv, &p->dev);
    if (rc) { delete p; return rc; }
    p->cache = c;
    p->cache_gen = xc__cache_gen(c);
    p->s = (hipStream_t)streamv;
    D.seg_cap = cap;
    const uint32_t ns = (uint32_t)nbuf;
    p->ns = D.ns = ns;
    p->ioff.resize(ns);
    p->ooff.resize(ns);
    std::vector<uint32_t> ilen(ns), tbase(ns);
    uint64_t itot = 0, otot = 0, ntok = 0, nprov = 0;
    for (uint32_t j = 0; j < ns; j++) {
        if (in_len[j] > 0xFFFFFF00ull) { xc_dplan_destroy(p); return xc__set_error(XC_EINVAL, "stream too long"); }
        p->ioff[j] = itot;
        itot += (in_len[j] + 255) / 256 * 256;
        p->in_total += in_len[j];
        ilen[j] = (uint32_t)in_len[j];
        p->ooff[j] = otot;
        otot += (out_cap[j] + 255) / 256 * 256;
        tbase[j] = (uint32_t)ntok;
        ntok += in_len[j] / 10 + 2;
        nprov += in_len[j] / (XC_SEG + 2) + 1;
    }
    if (ntok > 0xFFFFFFF0ull) { xc_dplan_destroy(p); return xc__set_error(XC_EINVAL, "batch too large"); }
    p->tok_base.assign(tbase.begin(), tbase.begin() + ns);
    p->tok_base.push_back((uint32_t)ntok);
    p->in_bytes = itot + 4096;  // the tokenizer's 256-byte windows read past a stream's end
    p->out_bytes = otot + 256;
    p->ntok = ntok;
    p->n_full = 1024;
    while (p->n_full < 2 * nprov + 2) p->n_full <<= 1;
    p->n_lo = 1024;
    while (p->n_lo < 4 * nprov + 4) p->n_lo <<= 1;
    uint64_t *d_ioff, *d_ooff, *d_ocap;
    uint32_t *d_ilen, *d_tbase;
#define DA(ptr, n) if ((rc = p->alloc(ptr, n))) { xc_dplan_destroy(p); return rc; }
    if (hipSetDevice(p->dev) != hipSuccess) { xc_dplan_destroy(p); return xc__set_error(XC_EDEVICE, "hipSetDevice"); }
    // the five per-stream layout arrays in one device block, uploaded by one copy from pinned staging
    // (five pageable copies cost ~10 us each of a small call's host time)
    uint8_t *d_lay = nullptr;
    const size_t lay = (size_t)std::max<uint32_t>(ns, 1) * 32u;
    DA(&d_lay, lay);
    d_ioff = (uint64_t *)d_lay;
    d_ooff = d_ioff + std::max<uint32_t>(ns, 1);
    d_ocap = d_ooff + std::max<uint32_t>(ns, 1);
    d_ilen = (uint32_t *)(d_ocap + std::max<uint32_t>(ns, 1));
    d_tbase = d_ilen + std::max<uint32_t>(ns, 1);
    DA(&D.tok_cnt, ns); DA(&D.s_stop, ns); DA(&D.s_slot, ns); DA(&D.s_cnt, ns); DA(&D.s_lim, ns); DA(&D.ctl, DCTL_WORDS);
    DA(&D.s_xp, ns);
    DA(&D.t_lb, ntok); DA(&D.t_le, ntok); DA(&D.t_op, ntok); DA(&D.t_stat, ntok); DA(&D.t_h, ntok);
    DA(&D.t_src, ntok);
    // The batch provider tables (two when the parse runs ahead, dsets[1] below) are keys and values
    // only: prov_insert / set_find / dset_clear_range read nothing else.  Their filter and lo32 arrays
    // stay null, so set_insert / set_has_lo on them would fault at once rather than probe stale words.
    DevSet &ds = D.dset;
    ds.filt = nullptr; ds.l2 = nullptr; ds.lo_keys = nullptr; ds.lo_zero = nullptr;
    DA(&ds.keys, p->n_full); DA(&ds.vals, p->n_full);
#undef DA
    ds.mask = p->n_full - 1;
    ds.lo_mask = p->n_lo - 1;
    p->dsets[0] = ds;
    const hipStream_t s = p->s;
    if (ns) {
        uint8_t *h_lay = nullptr;
        if (xc__halloc((void **)&h_lay, lay)) { xc_dplan_destroy(p); return xc__set_error(XC_ENOMEM, "pinned allocation failed"); }
        const size_t n1 = std::max<uint32_t>(ns, 1);
        memcpy(h_lay, p->ioff.data(), ns * 8);
        memcpy(h_lay + 8 * n1, p->ooff.data(), ns * 8);
        memcpy(h_lay + 16 * n1, out_cap, ns * 8);
        memcpy(h_lay + 24 * n1, ilen.data(), ns * 4);
        memcpy(h_lay + 28 * n1, tbase.data(), ns * 4);
        const hipError_t e = hipMemcpyAsync(d_lay, h_lay, lay, hipMemcpyHostToDevice, s);
        const hipError_t e2 = hipStreamSynchronize(s);
        xc__pfree(h_lay);
        DHIP(e);
        DHIP(e2);
    } else {
        DHIP(hipStreamSynchronize(s));
    }
    p->tset[0] = {D.tok_cnt, D.t_lb, D.t_le, D.t_op, D.t_h};
    D.in_off = d_ioff;
    D.in_len = d_ilen;
    D.tok_base = d_tbase;
    D.out_off = d_ooff;
    D.out_cap = d_ocap;
    D.count = 1;
    *out = p;
    return XC_OK;
}

extern "C" int xc_dplan_layout(xc_dplan *p, uint64_t *in_off, uint64_t *out_off, uint64_t *in_bytes,
                               uint64_t *out_bytes)
{
    if (!p) return xc__set_error(XC_EINVAL, "null");
    if (in_off) std::copy(p->ioff.begin(), p->ioff.end(), in_off);
    if (out_off) std::copy(p->ooff.begin(), p->ooff.end(), out_off);
    if (in_bytes) *in_bytes = p->in_bytes;
    if (out_bytes) *out_bytes = p->out_bytes;
    return XC_OK;
}

extern "C" int xc_dplan_stats(xc_dplan *p, xc_decode_stats *st)
{
    if (!p || !st) return xc__set_error(XC_EINVAL, "null");
    *st = p->stats;
    return XC_OK;
}

extern "C" int xc_decode_run(xc_dplan *p, const uint8_t *d_in, uint8_t *d_out, uint64_t *d_out_len,
                             uint64_t *d_consumed, int32_t *d_status, uint64_t *d_unknown, int32_t *d_has_unknown)
{
    if (!p) return xc__set_error(XC_EINVAL, "null");
    const uint32_t ns = p->ns;
    if (ns == 0) return XC_OK;
    if (!d_in || !d_out || !d_out_len || !d_consumed || !d_status || !d_unknown || !d_has_unknown)
        return xc__set_error(XC_EINVAL, "null");
    DHIP(hipSetDevice(p->dev));
    {   // the recent window (xc_memcache.cpp): the cache's pending run first; with a hash entered
        // twice that may answer other bytes than the device holds, the host path replays the run
        int slow = 0;
        int r = xc__cache_run_start(p->cache, &slow);
        if (r) return r;
        if (slow && p->internal) return xc__set_error(XC__SLOW, "a hash entered twice is in the recent window");
        if (slow)
            return xc__set_error(XC_EINVAL, "device-resident decode on a cache with a hash entered twice by a "
                                            "stateful stream: run it through xc_decode_batch_host");
    }
    // the parse of this run's input on the side stream at once (input ready), into the token set the
    // run before this one did not use (its last reader, two runs back, is long done)
    // (round 0's hashes are taken by the tokenizer as it passes each payload: a separate k_dres1<true>
    // measured cfg4 914 against 940 GiB/s; the round-2 1 KiB-window tokenizer 905 against 928, §5.1)
    const bool early = p->input_ready && !p->internal;
    if (early) {
        if (!p->ps) {  // (the second token set, the side stream and its events, once)
            xc_dplan::TokSet &t1 = p->tset[1];
            const size_t nt = std::max<uint64_t>(p->ntok, 1);
            int ra = XC_OK;
            if ((ra = p->alloc(&t1.tok_cnt, std::max<uint32_t>(ns, 1))) || (ra = p->alloc(&t1.t_lb, nt)) ||
                (ra = p->alloc(&t1.t_le, nt)) || (ra = p->alloc(&t1.t_op, nt)) || (ra = p->alloc(&t1.t_h, nt)))
                return ra;  // (what was allocated goes with the plan)
            DevSet &d1 = p->dsets[1];
            d1 = p->dsets[0];
            if ((ra = p->alloc(&d1.keys, p->n_full)) || (ra = p->alloc(&d1.vals, p->n_full)))  // (keys, values)
                return ra;
            DHIP(hipEventCreateWithFlags(&p->ev_parsed, hipEventDisableTiming));
            DHIP(hipEventCreateWithFlags(&p->ev_free, hipEventDisableTiming));
            DHIP(hipStreamCreateWithFlags(&p->ps, hipStreamNonBlocking));
        }
        p->tcur ^= 1;
        const xc_dplan::TokSet &t = p->tset[p->tcur];
        p->D.tok_cnt = t.tok_cnt;
        p->D.t_lb = t.t_lb;
        p->D.t_le = t.t_le;
        p->D.t_op = t.t_op;
        p->D.t_h = t.t_h;
        p->D.dset = p->dsets[p->tcur];
        DecDev Dp = p->D;
        Dp.in = d_in;
        if (!p->settled) {
            DHIP(hipEventRecord(p->ev_free, p->s));
            DHIP(hipStreamWaitEvent(p->ps, p->ev_free, 0));
        }
        if (!p->clean[p->tcur])  // (not left clean by an early run: cleared here)
            hipLaunchKernelGGL(k_dclear, dim3(512), dim3(256), 0, p->ps, Dp, p->n_lo, p->n_full);
        p->clean[p->tcur] = false;
        auto parse = k_dtok<true, false>;
        hipLaunchKernelGGL(parse, dim3(ns), dim3(64), 0, p->ps, Dp, 1, 0, p->n_lo, p->n_full);
        DHIP(hipGetLastError());
        DHIP(hipEventRecord(p->ev_parsed, p->ps));
        p->early_runs++;
    } else {
        p->clean[p->tcur] = false;  // (this run's tokenizer enters into p->D.dset = dsets[tcur])
    }

    DecDev D = p->D;
    D.in = d_in;
    D.out = d_out;
    D.out_len = d_out_len;
    D.consumed = d_consumed;
    D.status = d_status;
    D.unknown = d_unknown;
    D.has_unknown = d_has_unknown;
    const hipStream_t s = p->s;
    uint32_t ctl[DCTL_WORDS] = {};
    int rounds = 0;
    // room for every EXTRACT of the batch (>= 2050 input bytes each): the cache grows, never fills
    int rcr = xc__cache_reserve(p->cache, p->in_total / (XC_SEG + 2) + 1);
    if (rcr) return rcr;
    if (p->cache_gen != xc__cache_gen(p->cache)) {  // it grew: its arrays moved
        void *streamv = nullptr;
        int dev = 0;
        DecDev &PD = p->D;
        if ((rcr = xc__cache_devset(p->cache, &PD.cache, &PD.segs, &PD.seg_count, &PD.seg_cap, &PD.undo, &streamv,
                                    &dev)))
            return rcr;
        D.cache = PD.cache;
        D.segs = PD.segs;
        D.seg_count = PD.seg_count;
        D.seg_cap = PD.seg_cap;
        D.undo = PD.undo;
        p->cache_gen = xc__cache_gen(p->cache);
    }
    // the run enters segments: the host's copy of the count is stale until the run's totals
    const int64_t count0 = xc__cache_host_count(p->cache);
    xc__cache_count_unknown(p->cache);
    // tokens, with the prologue (control words, provider limits, round 0's provider table)
    if (!early) {  // (the batch table cleared before the tokenizer inserts into it)
        hipLaunchKernelGGL(k_dclear, dim3(512), dim3(256), 0, s, D, p->n_lo, p->n_full);
        DHIP(hipGetLastError());
    }
    // round 0 behind the side stream's parse: k_dres2<true> takes the prologue and the cache probes
    // (and clears the other set's table for the next early run on it)
    DecDev Dq = D;
    if (early) {
        DHIP(hipStreamWaitEvent(s, p->ev_parsed, 0));
        Dq.dset_other = p->dsets[p->tcur ^ 1];
        Dq.clr_lo = p->n_lo;
        Dq.clr_full = p->n_full;
    } else {
        hipLaunchKernelGGL((k_dtok<true, true>), dim3(std::max<uint32_t>(ns, 256u)), dim3(64), 0, s, D, 1, 1, p->n_lo, p->n_full);
    }
    DHIP(hipGetLastError());
    // one provider-resolution round (a fresh batch table each time; round 0's came with k_dtok)
    auto resolve_round = [&](int r) -> int {
        if (r > 0) {
            hipLaunchKernelGGL(k_dclear, dim3(512), dim3(256), 0, s, D, p->n_lo, p->n_full);
            DHIP(hipGetLastError());
            hipLaunchKernelGGL(k_dres1<false>, dim3(ns, DRES_WAVES), dim3(64), 0, s, D);
        }
        DHIP(hipGetLastError());
        // (a wave per stream; round 0 after an early parse: with the prologue and the cache probes)
        if (early && r == 0) hipLaunchKernelGGL(k_dres2<true>, dim3(ns), dim3(64), 0, s, Dq);
        else hipLaunchKernelGGL(k_dres2<false>, dim3(ns), dim3(64), 0, s, D);
        DHIP(hipGetLastError());
        return XC_OK;
    };
    // output and cache commit: these kernels return at once while DCTL_FIX is set, so round 0
    // and the emit are enqueued together and the host waits once in the common case
    int rc0 = XC_OK;
    auto emit = [&](int r) -> int {
        if (!p->h_ctl) {
            if ((rc0 = xc__halloc((void **)&p->h_ctl, DCTL_WORDS * 4))) return rc0;
            void *dp = nullptr;
            DHIP(hipHostGetDevicePointer(&dp, p->h_ctl, 0));
            p->d_hctl = (uint32_t *)dp;
            DHIP(hipEventCreateWithFlags(&p->ev_ctl, hipEventDisableTiming));
        }
        // stream-ordered completion: k_dfin publishes the words when they are final (a sentinel
        // in the last word, cleared last) and the host returns while k_demit runs
        const bool pub = p->completion == XC_COMPLETE_STREAM;
        DecDev Da = D;
        if (pub) {
            p->h_ctl[DCTL_WORDS - 1] = 0xFFFFFFFFu;
            Da.ctl_host = p->d_hctl;
        }
        // (XC_DFIN_GRID, -DXC_ABLATIONS builds: another grid)
        static const uint32_t dfin_grid = abl_env("XC_DFIN_GRID") ? (uint32_t)atoi(abl_env("XC_DFIN_GRID")) : DFIN_GRID;
        hipLaunchKernelGGL(k_dfin, dim3(1u + std::max(1u, std::min(dfin_grid, (ns + DFIN_WAVES - 1) / DFIN_WAVES))),
                           dim3(64 * DFIN_WAVES), 0, s, Da, r);  // (workgroup 0: the slots)
        DHIP(hipGetLastError());  // (slots first: k_demit fills them)
        hipLaunchKernelGGL(k_demit, dim3(ns), dim3(64 * DEMIT_WAVES), 0, s, D);
        DHIP(hipGetLastError());
        if (pub) {
            int64_t t0 = 0;
            for (int i = 0;; i++) {
                if (*(volatile const uint32_t *)(p->h_ctl + DCTL_WORDS - 1) == 0u) {
                    __atomic_thread_fence(__ATOMIC_ACQUIRE);
                    memcpy(ctl, p->h_ctl, DCTL_WORDS * 4);
                    return XC_OK;
                }
                if ((i & 255) == 255) {
                    if (xc__query_due(&t0)) {  // (a query enqueues a marker: only after ~2 ms)
                        const hipError_t e = hipStreamQuery(s);
                        if (e == hipSuccess) break;  // drained without a publication: read the words
                        if (e != hipErrorNotReady) DHIP(e);
                    }
                    if (i >= 4096) sched_yield();
                }
            }
        }
        // through a pinned buffer, then a spin on an event: back within a few us of the copy
        DHIP(hipMemcpyAsync(p->h_ctl, D.ctl, DCTL_WORDS * 4, hipMemcpyDeviceToHost, s));
        DHIP(hipEventRecord(p->ev_ctl, s));
        DHIP(xc__spin_wait(p->ev_ctl));  // (polls, yielding the core after ~20 us)
        memcpy(ctl, p->h_ctl, DCTL_WORDS * 4);
        return XC_OK;
    };
    int rc;
    p->settled = false;
    if ((rc = resolve_round(0)) || (rc = emit(0))) return rc;
    p->settled = true;  // (this run's k_dfin ran: every kernel of the run before is done)
    while (ctl[DCTL_FIX]) {
        // a provider lies past its own stream's stop: re-resolve with the executed prefixes
        // as the only eligible providers, until the executed sets agree
        if (++rounds > 64) return xc__set_error(XC_EDEVICE, "decode provider resolution did not converge");
        hipLaunchKernelGGL(k_dlim, dim3((ns + 255) / 256), dim3(256), 0, s, D, 0);
        DHIP(hipGetLastError());
        if ((rc = resolve_round(rounds)) || (rc = emit(rounds))) return rc;
    }
    p->stats.in_bytes = p->in_total;
    p->stats.n_ref = ctl[DCTL_NREF];
    p->stats.n_extract = ctl[DCTL_NEXTRACT];
    p->stats.n_entered = ctl[DCTL_NENTER];
    p->stats.rounds = (uint32_t)rounds + 1u;
    if (ctl[DCTL_ERR] & 2u) {
        const uint32_t c = D.seg_cap;  // the committed prefix stays; the count is clamped
        hipMemcpyAsync(D.seg_count, &c, 4, hipMemcpyHostToDevice, s);
        hipStreamSynchronize(s);
        return xc__set_error(XC_ENOSPC, "device cache capacity exhausted");
    }
    if (ctl[DCTL_ERR] & 1u) {
        // An output overflowed: k_demit stopped that stream's copies, so some of the slots k_dfin gave
        // its ENTER tokens were never filled.  The run is rolled back whole: the cache is left as it
        // was before the call (the tables rebuilt from the first count0 entries, as a COSS roll back
        // does), and no hit of the run reaches the recent window.
        DHIP(hipStreamSynchronize(s));
        int64_t before = count0;
        if (before < 0) {
            uint64_t n = 0;
            if ((rc = xc_cache_count(p->cache, &n))) return rc;
            before = (int64_t)n - (int64_t)ctl[DCTL_NENTER];
        }
        if (ctl[DCTL_NENTER] && (rc = xc__cache_truncate(p->cache, (uint64_t)before))) return rc;
        return xc__set_error(XC_EINVAL, "output capacity too small");
    }
    // (k_dfin advanced the count by exactly the entered segments: a later restore or reserve
    // needs no device read)
    if (count0 >= 0) xc__cache_set_host_count(p->cache, count0 + ctl[DCTL_NENTER]);
    if (early) p->clean[p->tcur ^ 1] = true;
    xc__cache_run_done_dec(p->cache, p);
    return XC_OK;
}

// A finished run's lookup hits in the reference's order (xcodec_decoder.cc:120-166): per stream,
// its executed EXTRACT and REF tokens that found the hash (in the cache or entered by an earlier
// EXTRACT of the batch), and an EXTRACT it stopped on as a collision.
extern "C" int xc__dplan_hits(void *dp, uint64_t **hits, uint64_t *n, int *complete)
{
    xc_dplan *p = (xc_dplan *)dp;
    *complete = 1;
    *n = 0;
    *hits = nullptr;
    const uint32_t ns = p->ns;
    if (!ns) return XC_OK;
    DHIP(hipSetDevice(p->dev));
    std::vector<uint32_t> op(p->ntok), st(p->ntok), stop(ns);
    std::vector<uint64_t> th(p->ntok);
    DHIP(hipMemcpyAsync(op.data(), p->D.t_op, p->ntok * 4, hipMemcpyDeviceToHost, p->s));
    DHIP(hipMemcpyAsync(st.data(), p->D.t_stat, p->ntok * 4, hipMemcpyDeviceToHost, p->s));
    DHIP(hipMemcpyAsync(th.data(), p->D.t_h, p->ntok * 8, hipMemcpyDeviceToHost, p->s));
    DHIP(hipMemcpyAsync(stop.data(), p->D.s_stop, ns * 4, hipMemcpyDeviceToHost, p->s));
    DHIP(hipStreamSynchronize(p->s));
    std::vector<uint64_t> v;
    for (uint32_t j = 0; j < ns; j++) {
        const uint32_t tb = p->tok_base[j], ex = std::min(stop[j], p->tok_base[j + 1] - tb);
        for (uint32_t t = 0; t < ex; t++) {
            const uint32_t o = op[tb + t], r = st[tb + t];
            const bool executed = t + 1u < ex;
            if ((o == T_EXTRACT || o == T_REF) && executed && (r == R_OKCACHE || r == R_OKPROV)) v.push_back(th[tb + t]);
            else if (o == T_EXTRACT && !executed && r == R_COLL) v.push_back(th[tb + t]);
        }
    }
    *hits = (uint64_t *)malloc(std::max<size_t>(v.size(), 1) * 8);
    if (!*hits) return xc__set_error(XC_ENOMEM, "host allocation failed");
    std::copy(v.begin(), v.end(), *hits);
    *n = v.size();
    return XC_OK;
}

extern "C" int xc_decode_batch_host(xc_cache *c, const uint8_t *in, const uint64_t *in_off, const uint64_t *in_len,
                                    uint64_t nbuf, uint8_t *out, const uint64_t *out_off, const uint64_t *out_cap,
                                    uint64_t *out_len, uint64_t *consumed, int32_t *status, uint64_t *unknown,
                                    int32_t *has_unknown)
{
    if (!c || (nbuf && (!in || !in_off || !in_len || !out || !out_off || !out_cap || !out_len || !consumed ||
                        !status || !unknown || !has_unknown)))
        return xc__set_error(XC_EINVAL, "null");
    if (nbuf == 0) return XC_OK;
    xc_dplan *p = nullptr;
    int rc = xc_decode_plan_create(c, in_len, out_cap, nbuf, &p);
    if (rc) return rc;
    const uint32_t ns = p->ns;
    const hipStream_t s = p->s;
    p->internal = true;
    uint8_t *h_in = nullptr, *h_out = nullptr, *d_in = nullptr, *d_out = nullptr, *h_res = nullptr, *d_res = nullptr;
    uint64_t *d_u64 = nullptr;  // out_len | consumed | unknown
    int32_t *d_i32 = nullptr;   // status | has_unknown   (one block: one copy back into pinned h_res)
    const size_t res_bytes = (size_t)ns * (3 * 8 + 2 * 4);
    auto run = [&]() -> int {
        if (xc__halloc((void **)&h_in, p->in_bytes) || xc__halloc((void **)&h_out, p->out_bytes) ||
            xc__halloc((void **)&h_res, res_bytes))
            return XC_ENOMEM;
        DHIP(dalloc(&d_in, p->in_bytes));
        DHIP(dalloc(&d_out, p->out_bytes));
        DHIP(dalloc(&d_res, res_bytes));
        d_u64 = (uint64_t *)d_res;
        d_i32 = (int32_t *)(d_u64 + 3 * (size_t)ns);
        // (the padding between streams needs no clearing: the tokenizer clips every window to its
        // stream's length)
        for (uint32_t j = 0; j < ns; j++) memcpy(h_in + p->ioff[j], in + in_off[j], in_len[j]);
        DHIP(hipMemcpyAsync(d_in, h_in, p->in_bytes, hipMemcpyHostToDevice, s));
        int r = xc_decode_run(p, d_in, d_out, d_u64, d_u64 + ns, d_i32, d_u64 + 2 * ns, d_i32 + ns);
        if (r) return r;
        DHIP(hipMemcpyAsync(h_out, d_out, p->out_bytes, hipMemcpyDeviceToHost, s));
        DHIP(hipMemcpyAsync(h_res, d_res, res_bytes, hipMemcpyDeviceToHost, s));
        DHIP(hipStreamSynchronize(s));
        const uint64_t *u64 = (const uint64_t *)h_res;
        const int32_t *i32 = (const int32_t *)(u64 + 3 * (size_t)ns);
        for (uint32_t j = 0; j < ns; j++) {
            out_len[j] = u64[j];
            consumed[j] = u64[ns + j];
            unknown[j] = u64[2 * ns + j];
            status[j] = i32[j];
            has_unknown[j] = i32[ns + j];
            memcpy(out + out_off[j], h_out + p->ooff[j], out_len[j]);
        }
        return XC_OK;
    };
    rc = run();
    hipStreamSynchronize(s);
    xc__pfree(h_in);
    xc__pfree(h_out);
    xc__pfree(h_res);
    xc__pfree(d_in);
    xc__pfree(d_out);
    xc__pfree(d_res);
    xc_dplan_destroy(p);
    if (rc == XC__SLOW)  // a hash entered twice: the recent window's replay (xc_memcache.cpp)
        rc = xc__mem_decode_batch(xc__cache_mem(c), in, in_off, in_len, nbuf, out, out_off, out_cap, out_len, consumed,
                                  status, unknown, has_unknown);
    return rc;
}

// The replay engines' device batch (the cache's hooks stand aside while they run).
extern "C" int xc__decode_batch_host_raw(xc_cache *c, const uint8_t *in, const uint64_t *in_off,
                                         const uint64_t *in_len, uint64_t nbuf, uint8_t *out,
                                         const uint64_t *out_off, const uint64_t *out_cap, uint64_t *out_len,
                                         uint64_t *consumed, int32_t *status, uint64_t *unknown,
                                         int32_t *has_unknown)
{
    return xc_decode_batch_host(c, in, in_off, in_len, nbuf, out, out_off, out_cap, out_len, consumed, status,
                                unknown, has_unknown);
}
