// xc_encode.hip — XCodec batch encoder kernels for gfx950 (CDNA4).
//
// Reference path: XCodecEncoder::encode/flush (xcodec/xcodec_encoder.cc:60-260) over a
// shared XCodecMemoryCache (xcodec/xcodec_cache.h:162-211).  DESIGN.md explains the
// pipeline; in short, per sub-batch of buffers:
//
//   k_scan(S)     every window end p: lo32 of H(p) by the rolling recurrence, level-1 LDS
//                 bitmap, exact lo32 probe -> sparse/dense event layer S (cache hits)
//   k_resolve(S)  per event: full 64-bit H, cache probe, 2048-byte compare -> EQUAL / COLL
//   k_walk        per buffer: the sequential candidate/declare/reference state machine
//                 (xcodec_encoder.cc:77-170) over the sparse events -> tokens
//                 (block-parallel when no event between aligned windows decides anything),
//                 then H(segment) of declarations no event supplied (xcodec_hash.h:166-174)
//                 into the declaration set D
//   k_scan(D), k_resolve(D), k_walk  until D stops growing (self references)
//   k_emit        tokens -> F1-escaped wire bytes; EXTRACT payloads entered in the cache
//
// Buffers are processed as if in index order against one cache: a buffer whose lookups
// would have hit an earlier buffer's new declaration is detected (first_cross) and the
// host re-runs the batch from that buffer after committing everything before it.
#include "xc_kernels.h"

// Timing ablations (XC_ABL_BH, XC_ABL_EMIT: the results are wrong) only in builds with
// -DXC_ABLATIONS=1 (tools/build_variant.sh, xc_env.h): production kernels carry no such branch.
#include "xc_env.h"

namespace xc {

// ---------------------------------------------------------------- k_scan ----------------

__device__ __forceinline__ void scan_record(const ScanArgs &a, uint32_t c, uint32_t c0, bool match, uint32_t pos,
                                            uint32_t &ev_n, bool &dense)
{
    uint64_t m = ballot(match);
    if (!m) return;
    const uint32_t k = (uint32_t)__popcll(m);
    const uint32_t W = a.P.chunk_len / 32u;
    if (!dense && ev_n + k <= EV_CAP) {
        if (match) a.L.pos[c * EV_CAP + ev_n + mbcnt(m)] = pos;
        ev_n += k;
        return;
    }
    if (!dense) {
        dense = true;
        uint32_t *bits = a.L.bits + (size_t)c * W;
        for (uint32_t i = lane_id(); i < W; i += 64u) bits[i] = 0u;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        for (uint32_t i = lane_id(); i < ev_n; i += 64u) {
            uint32_t q = a.L.pos[c * EV_CAP + i] - c0;
            atomicOr(&bits[q >> 5], 1u << (q & 31u));
        }
    }
    if (match) {
        uint32_t q = pos - c0;
        atomicOr(&a.L.bits[(size_t)c * W + (q >> 5)], 1u << (q & 31u));
    }
}

// Exact lo32 membership for queued filter positives, split in two halves so the global
// probe latency overlaps the next 2048-position iteration: issue() moves up to 128 queued
// (position, lo32) pairs into registers and starts their lo32-set loads (two consecutive
// slots each); complete() consumes them one iteration later.
// Exact lo32 membership for queued level-1 positives, split in two halves so the latency
// overlaps the next 2048-position iteration: issue() moves up to 128 queued (position, lo32)
// pairs into registers and starts their level-2 filter loads (one 8-byte L2 read each);
// complete() tests them one iteration later and probes the exact lo32 sets for survivors.
// Exact lo32 membership in set | set2: the first slots of both tables are loaded together.
__device__ __forceinline__ bool scan_has_lo(const ScanArgs &a, uint32_t lo)
{
    if (lo == 0u) return *a.set.lo_zero != 0u || (a.has2 && *a.set2.lo_zero != 0u);
    uint32_t i1 = lo_slot(lo, a.set.lo_mask), i2 = a.has2 ? lo_slot(lo, a.set2.lo_mask) : 0u;
    uint32_t k1 = a.set.lo_keys[i1];
    uint32_t k2 = a.has2 ? a.set2.lo_keys[i2] : 0u;
    while (k1 != 0u && k1 != lo) {
        i1 = (i1 + 1u) & a.set.lo_mask;
        k1 = a.set.lo_keys[i1];
    }
    if (k1 == lo) return true;
    while (k2 != 0u && k2 != lo) {
        i2 = (i2 + 1u) & a.set2.lo_mask;
        k2 = a.set2.lo_keys[i2];
    }
    return k2 == lo;
}

struct Pending {
    uint32_t n;          // entries (uniform); 0 = nothing pending
    uint32_t c, c0;      // chunk the entries belong to
    uint32_t pos[2], lo[2];  // lo: l2_mix of the window's lo32
    uint32_t w[2];
};

__device__ __forceinline__ void pend_issue(const ScanArgs &a, Pending &pd, const uint2 *queue, uint32_t qn,
                                           uint32_t c, uint32_t c0)
{
    pd.n = qn;
    pd.c = c;
    pd.c0 = c0;
    // every lane loads (empty slots: word 0), so the count of outstanding loads is static and
    // the compiler can keep these in flight across the next iteration
#pragma unroll
    for (int s = 0; s < 2; s++) {
        const uint32_t i = lane_id() + 64u * s;
        const uint2 e = queue[i];
        const bool v = i < qn;
        pd.pos[s] = v ? e.x : 0u;
        pd.lo[s] = l2_mix(e.y);  // (kept mixed: the exact probe unmixes its few survivors)
        pd.w[s] = a.l2[v ? l2_word(pd.lo[s]) : 0u];
    }
}

template <int MODE>
__device__ __forceinline__ void pend_complete(const ScanArgs &a, Pending &pd, uint32_t &ev_n, bool &dense)
{
#pragma unroll
    for (int s = 0; s < 2; s++) {
        if (64u * s >= pd.n) break;
        const uint32_t i = lane_id() + 64u * s;
        bool match = false;
        if (i < pd.n && l2_test(pd.w[s], pd.lo[s])) {
            const uint32_t x = l2_unmix(pd.lo[s]);
            match = MODE == 5 ? x == 0x12345u : scan_has_lo(a, x);
        }
        scan_record(a, pd.c, pd.c0, match, pd.pos[s], ev_n, dense);
    }
    pd.n = 0;
}

template <int MODE>
__device__ __forceinline__ void scan_flush(const ScanArgs &a, uint2 *queue, uint32_t &qn, uint32_t c, uint32_t c0,
                                           uint32_t &ev_n, bool &dense)
{
    if (MODE == 4) {  // ablation: queue appends only
        qn = 0;
        return;
    }
    static_assert(Q_CAP == 128u, "Pending holds 2 x 64 entries");
    // Q_CAP = 2 x 64: every entry's level-2 word is in flight before the first test
    Pending f;
    pend_issue(a, f, queue, qn, c, c0);
    pend_complete<MODE>(a, f, ev_n, dense);
    qn = 0;
}

// Exclusive-scan helpers for the per-lane chunk sums of one 2048-byte block.
struct BlockSums {
    uint32_t preA, preC, totA, totC;
};

__device__ __forceinline__ BlockSums block_sums(const uint32_t w[8], uint32_t l)
{
    uint32_t sb = 0, jb = 0;
#pragma unroll
    for (int d = 0; d < 8; d++) {
        const uint32_t wt = (uint32_t)(4 * d) * 0x01010101u + 0x03020100u;
        sb = __builtin_amdgcn_udot4(w[d], 0x01010101u, sb, false);
        jb = __builtin_amdgcn_udot4(w[d], wt, jb, false);
    }
    const uint32_t A = sb + 32u;               // sum (b+1) over the lane's 32 bytes
    const uint32_t C = 32u * l * A + jb + 496u; // 32*l*A + sum j*(b+1)
    const uint32_t ia = wave_incl_scan(A), ic = wave_incl_scan(C);
    BlockSums s;
    s.totA = readlane(ia, 63);
    s.totC = readlane(ic, 63);
    s.preA = ia - A;
    s.preC = ic - C;
    return s;
}

__device__ __forceinline__ void load32_aligned(const uint8_t *p, uint32_t w[8])
{
    // streamed once: non-temporal, so the level-2 filter keeps its place in L2
    typedef uint32_t v4u __attribute__((ext_vector_type(4)));
    const v4u *q = (const v4u *)p;
    const v4u x = __builtin_nontemporal_load(q), y = __builtin_nontemporal_load(q + 1);
    w[0] = x.x; w[1] = x.y; w[2] = x.z; w[3] = x.w;
    w[4] = y.x; w[5] = y.y; w[6] = y.z; w[7] = y.w;
}

// The blocks a chunk starts from: pw = the 2048 bytes before its first iteration's block
// (block 0 when c0 == 0), w = that block, wn = the one after (prefetch ring, 2 deep).
__device__ __forceinline__ void first_blocks(const uint8_t *base, uint32_t c0, uint32_t l, uint32_t pw[8],
                                             uint32_t w[8], uint32_t wn[8])
{
    const uint32_t s = c0 == 0 ? XC_SEG : c0;
    load32_aligned(base + s - XC_SEG + 32u * l, pw);
    load32_aligned(base + s + 32u * l, w);
    load32_aligned(base + s + XC_SEG + 32u * l, wn);  // may lie past the buffer: arena slack
}

__device__ __forceinline__ const uint8_t *desc_base(const ScanArgs &a, const uint4 &d)
{
    return a.P.in + (((uint64_t)uniform(d.w) << 32) | uniform(d.z));
}

// A half-iteration with more level-1 positives than this probes the level-2 filter directly from
// every lane (one round trip) instead of queueing them for the next iteration's batch.
#ifndef XC_DIRECT_MIN
#define XC_DIRECT_MIN Q_CAP
#endif
// Level-2 loads of the direct path in flight at once (16 spills registers).
#ifndef XC_DIRECT_GROUP
#define XC_DIRECT_GROUP 8
#endif

template <int MODE>
__global__ __launch_bounds__(64 * SCAN_WAVES) void k_scan(ScanArgs a)
{
    if (aborted(a.P)) return;
    __shared__ uint32_t filt[XC_FILT_WORDS];
    __shared__ uint2 queues[SCAN_WAVES][Q_CAP];
    const uint32_t wave = threadIdx.x >> 6;
    uint2 *queue = queues[wave];
    const uint32_t l = lane_id();

    const uint32_t fw = a.filt_words;

    // Work distribution: waves take runs of a.unit consecutive chunks from a counter (chunks
    // of one buffer continue the block stream and its prefetch without a restart), the next run
    // always claimed one run ahead.  Dynamic, because the cost of a chunk varies (REF shadows,
    // filter positives) and other kernels may hold some CUs when the scan starts.
    // The first run of every wave is static (wave g: run g), so only the look-ahead claims
    // contend on the counter.
    // When the static first runs cover every chunk (small batches) no wave claims: claims from
    // thousands of waves at once serialize on the counter's one address.
    const uint32_t nwaves = gridDim.x * SCAN_WAVES;
    const bool dynamic = nwaves * a.unit < a.ck_hi - a.ck_lo;
    auto claim = [&]() -> uint32_t {
        if (!dynamic) return a.ck_hi;
        uint32_t t = 0;
        if (l == 0) t = atomicAdd(&a.P.ctl[CTL_SCAN_NEXT], a.unit);
        return a.ck_lo + nwaves * a.unit + uniform(t);
    };
    uint32_t c = a.ck_lo + (blockIdx.x * SCAN_WAVES + wave) * a.unit;
    const bool idle = c >= a.ck_hi;  // (a wave without chunks still loads its share of the image)
    uint32_t c_end = 0, c_nxt = 0, gblk = 0;
    uint4 dsc = make_uint4(0, 0, 0, 0), dn = dsc;
    uint32_t pw[8], w[8], wn[8];
    if (!idle) {
        // the first chunk's descriptor and blocks before the level-1 image: their memory latency
        // overlaps the image's copy (a small batch's waves scan 2 blocks each: the prologue counts)
        c_end = min(c + a.unit, a.ck_hi);
        c_nxt = claim();
        // chunk descriptors: {c0, c1, arena offset lo, hi}; the next one is always in flight
        dsc = a.P.chunk_desc[c];
        gblk = a.shadow ? uniform(a.P.chunk_blk[c]) : 0u;
        first_blocks(desc_base(a, dsc), uniform(dsc.x), l, pw, w, wn);
        dn = a.P.chunk_desc[c + 1u < c_end ? c + 1u : min(c_nxt, a.ck_hi - 1u)];
    }
    // the level-1 image (the first round's is cache | predicted declarations, folded for small
    // key counts: a multiple of 4 words)
    for (uint32_t i = threadIdx.x * 4u; i < fw; i += 256u * SCAN_WAVES)
        *(uint4 *)(filt + i) = *(const uint4 *)(a.filt + i);
    __syncthreads();
    if (idle) return;

    Pending pd;
    pd.n = 0;
    uint32_t sink = 0;  // MODE 3 ablation: filter tests kept alive without queueing
    uint32_t prev_c = NONE, prev_ev = 0;
    bool prev_dense = false;

    for (;;) {
        const uint32_t c0 = uniform(dsc.x), c1 = uniform(dsc.y) & 0x3FFFFFFFu;
        const uint8_t *base = desc_base(a, dsc);
        const bool in_run = c + 1u < c_end;
        const bool has_next = in_run || c_nxt < a.ck_hi;
        // the next chunk continues this one (same run and buffer, starts at c1): keep streaming
        const bool contig = in_run && (uniform(dsc.y) >> 31) != 0u;
        uint32_t ev_n = 0, qn = 0;
        bool dense = false;
        // REF-shadow flags of the chunk's iterations, one load per chunk (lane j: the block before
        // s = c0 + 2048 j), instead of a dependent load at every iteration
        uint32_t sflag = 0;
        if (a.shadow) {
            const uint32_t sj = c0 + XC_SEG * l;
            if (l < CHUNK_BLOCKS && sj >= XC_SEG && sj < c1) sflag = a.P.blk_pref[gblk + (sj >> 11) - 1u];
        }

        BlockSums ps = block_sums(pw, l);
        uint32_t s = c0;
        if (c0 == 0) {
            // window ending at 2047 = the whole first block (every chunk has len >= 2048); an
            // aligned window is always an event: its block is cached or a predicted declaration
            scan_record(a, c, c0, l == 0u, XC_SEG - 1u, ev_n, dense);
            s = XC_SEG;
        }

        const bool next_long = (uniform(dsc.y) >> 30 & 1u) != 0u;  // next chunk passes c1 + 2048
        for (; s < c1; s += XC_SEG) {
            // prefetch ring: w = block s (ready), wn = block s+2048 (in flight), wn2 = block
            // s+4096 issued now when the stream reaches it.  Unconditional (re-reads block s
            // otherwise): a conditional load makes the compiler drain every outstanding load.
            uint32_t wn2[8];
            const bool need2 = s + 2u * XC_SEG < c1 || (contig && (s + 2u * XC_SEG == c1 || next_long));
            load32_aligned(base + (need2 ? s + 2u * XC_SEG : s) + 32u * l, wn2);
            const BlockSums cs = block_sums(w, l);
            // REF shadow: the block before s is a predicted REF, after which the reference looks
            // nothing up until s + 2047 (recorded below); k_walk verifies the REF happened
            const bool shadowed = a.shadow && ((ballot(blk_cached(sflag)) >> ((s - c0) >> 11)) & 1u) != 0u;
            // window ending just before this lane's first position q = s + 32 l:
            // out-chunks of lanes >= l (previous block) + in-chunks of lanes < l.
            const uint32_t sufA = ps.totA - ps.preA, sufC = ps.totC - ps.preC;
            const uint32_t S1 = sufA + cs.preA;
            const uint32_t S2 = (XC_SEG + 32u * l) * sufA - sufC + 32u * l * cs.preA - cs.preC;
            if (MODE == 2) sink = sink * 31u + (S1 ^ S2);
            uint32_t U = S1 - XC_SEG;          // S1 - 2048
            uint32_t V = S2 + 0x80000000u;     // S2 + (2048 << 20)
            const uint32_t q = s + 32u * l;
            const uint32_t vmask = (q + 32u <= c1) ? 0xFFFFFFFFu : (q >= c1 ? 0u : ((1u << (c1 - q)) - 1u));
#pragma unroll
            for (int half = 0; half < (MODE == 2 ? 0 : 2); half++) {
                if (shadowed) break;
                uint32_t lo[16];
                uint32_t hit = 0;
#pragma unroll
                for (int d = 0; d < 4; d++) {
#pragma unroll
                    for (int k = 0; k < 4; k++) {
                        const uint32_t ib = (w[half * 4 + d] >> (8 * k)) & 0xffu;
                        const uint32_t ob = (pw[half * 4 + d] >> (8 * k)) & 0xffu;
                        U += ib - ob;
                        V += U + (uint32_t)__mul24((int)ob, -2048);
                        const uint32_t x = (U << 20) + V;
                        lo[d * 4 + k] = x;
                        if (MODE == 0 || MODE >= 3) hit |= filt_test_n(filt, x, fw) << (d * 4 + k);
                        else hit |= (x == 0x12345678u) ? 1u << (d * 4 + k) : 0u;
                    }
                }
                hit &= vmask >> (16 * half);
                if (half == 1 && l == 63u) hit &= 0x7FFFu;  // aligned window: recorded below
                if (MODE == 3) { sink = sink * 31u + hit; hit = 0; }
                const uint32_t cnt = (uint32_t)__popc(hit);
                const uint32_t incl = wave_incl_scan(cnt);
                const uint32_t tot = readlane(incl, 63);
                if (tot && qn + tot <= Q_CAP && tot <= XC_DIRECT_MIN) {
                    // lane-parallel append: this lane's hits go to [qn + excl, qn + excl + cnt);
                    // (offsets j unrolled: lo[j] stays a static register)
                    uint32_t slot = qn + incl - cnt;
#pragma unroll
                    for (int j = 0; j < 16; j++) {
                        if ((hit >> j) & 1u) {
                            queue[slot] = make_uint2(q + 16u * half + (uint32_t)j, lo[j]);
                            slot++;
                        }
                    }
                    qn += tot;
                } else if (tot) {
                    // more positives than the queue holds (a dense filter late in a run): every
                    // lane probes its own level-2 words directly, all loads in flight before the
                    // first test (one round trip for the half instead of a flush per 128)
                    if (MODE == 4) {
                        sink = sink * 31u + hit;
                    } else {
                        // lo[j] becomes its level-2 mix in place (inverted for the rare survivors);
                        // every lane loads (word 0 for non-positives: one coalesced request), so all
                        // 16 loads are in flight and the tests wait for them in order, branch-free
                        uint32_t pm = 0;
#pragma unroll
                        for (int g0 = 0; g0 < 16; g0 += XC_DIRECT_GROUP) {  // (groups: registers)
                            uint32_t w2[XC_DIRECT_GROUP];
#pragma unroll
                            for (int j = 0; j < XC_DIRECT_GROUP; j++) {
                                lo[g0 + j] = l2_mix(lo[g0 + j]);
                                w2[j] = a.l2[((hit >> (g0 + j)) & 1u) ? l2_word(lo[g0 + j]) : 0u];
                            }
#pragma unroll
                            for (int j = 0; j < XC_DIRECT_GROUP; j++)
                                pm |= (uint32_t)l2_test(w2[j], lo[g0 + j]) << (g0 + j);
                        }
                        pm &= hit;
                        // level-2 survivors (few): each lane its lowest one per round, exact lo32 sets
                        for (;;) {
                            const bool any = pm != 0u;
                            if (!ballot(any)) break;
                            const uint32_t j = any ? (uint32_t)__builtin_ctz(pm) : 0u;
                            pm &= pm - 1u;
                            uint32_t g = lo[0];
#pragma unroll
                            for (int jj = 1; jj < 16; jj++) g = j == (uint32_t)jj ? lo[jj] : g;
                            const uint32_t x = l2_unmix(g);
                            const bool match = any && (MODE == 5 ? x == 0x12345u : scan_has_lo(a, x));
                            scan_record(a, c, c0, match, q + 16u * half + j, ev_n, dense);
                        }
                    }
                }
            }
            // the aligned window ending at s + 2047 is an event without a probe: k_blockpredict
            // put its block in the declaration set unless the cache holds it (k_resolve decides)
            scan_record(a, c, c0, l == 63u && s + XC_SEG - 1u < c1, s + XC_SEG - 1u, ev_n, dense);
            // iteration boundary: finish the previous probe batch, start this one
            if (pd.n) {
                if (pd.c == c) {
                    pend_complete<MODE>(a, pd, ev_n, dense);
                } else {
                    pend_complete<MODE>(a, pd, prev_ev, prev_dense);
                    if (l == 0) a.L.cnt[prev_c] = prev_dense ? (EV_DENSE | prev_ev) : prev_ev;
                    if (l == 0 && prev_dense) atomicAdd(&a.P.ctl[CTL_DENSE], 1u);
                    prev_c = NONE;
                }
            }
            if (MODE == 4) { sink = sink * 31u + qn + queue[l & 63u].y; qn = 0; }
            pend_issue(a, pd, queue, qn, c, c0);  // (also when empty: a static load count)
            qn = 0;
#pragma unroll
            for (int d = 0; d < 8; d++) { pw[d] = w[d]; w[d] = wn[d]; wn[d] = wn2[d]; }
            ps = cs;
        }
        if (qn) {  // chunk whose only position is 2047: no iteration ran
            if (pd.n) {
                if (pd.c == c) pend_complete<MODE>(a, pd, ev_n, dense);
                else {
                    pend_complete<MODE>(a, pd, prev_ev, prev_dense);
                    if (l == 0) a.L.cnt[prev_c] = prev_dense ? (EV_DENSE | prev_ev) : prev_ev;
                    if (l == 0 && prev_dense) atomicAdd(&a.P.ctl[CTL_DENSE], 1u);
                    prev_c = NONE;
                }
            }
            pend_issue(a, pd, queue, qn, c, c0);
            qn = 0;
        }
        // chunk end: its count is final now, or once its pending probes complete
        if (pd.n && pd.c == c) {
            prev_c = c;
            prev_ev = ev_n;
            prev_dense = dense;
        } else {
            if (l == 0) a.L.cnt[c] = dense ? (EV_DENSE | ev_n) : ev_n;
            if (l == 0 && dense) atomicAdd(&a.P.ctl[CTL_DENSE], 1u);
        }
        if (!has_next) break;
        if (in_run) {
            c += 1u;
        } else {
            c = c_nxt;
            c_end = min(c + a.unit, a.ck_hi);
            c_nxt = claim();
        }
        dsc = dn;
        if (a.shadow) gblk = uniform(a.P.chunk_blk[c]);
        if (!contig) first_blocks(desc_base(a, dsc), uniform(dsc.x), l, pw, w, wn);
        dn = a.P.chunk_desc[c + 1u < c_end ? c + 1u : min(c_nxt, a.ck_hi - 1u)];
    }
    if (MODE >= 2 && sink == 0x7FFFFFF0u - a.ck_hi) a.P.ctl[CTL_ERROR] = sink;  // never true; keeps ablations honest
    if (pd.n) {
        if (pd.c == prev_c) {
            pend_complete<MODE>(a, pd, prev_ev, prev_dense);
            if (l == 0) a.L.cnt[prev_c] = prev_dense ? (EV_DENSE | prev_ev) : prev_ev;
            if (l == 0 && prev_dense) atomicAdd(&a.P.ctl[CTL_DENSE], 1u);
        }
    }
}

template __global__ void k_scan<0>(ScanArgs);
template __global__ void k_scan<1>(ScanArgs);
template __global__ void k_scan<2>(ScanArgs);
template __global__ void k_scan<3>(ScanArgs);
template __global__ void k_scan<4>(ScanArgs);
template __global__ void k_scan<5>(ScanArgs);

// ---------------------------------------------------------------- k_ascan ---------------
// The first-round scan of an anchor-scanned sub-batch.  Its events are the
// aligned windows (always events, as in k_scan) and the window ends the anchor index proposes: an
// input anchor record (fingerprint fp, position a, a run of n) whose fingerprint the cache or the
// predicted declarations index as (fp, j) proposes q = a + k + 2047 - j for k < n.  Every window
// equal to an indexed segment is among them (superset: k_resolve decides each exactly).
//
// k_aprop: one thread per record (a workgroup per k_blockhash group of the sub-batch): the
// combined anchor filter (amix, 2 MB, L2-resident), for its few positives the two tables, and
// every proposal (not aligned, not in a predicted REF's shadow) appended to its chunk's list
// (pcnt / pq).  k_aevents: one lane per chunk writes the aligned windows (no proposal: the common
// case); a chunk with proposals is sorted and merged by its whole wave in an LDS bitmask.

// A proposal: window end q of buffer b (chunk list of its chunk), unless aligned (an event anyway)
// or in a predicted REF's shadow.
__device__ __forceinline__ void propose(const PlanDev &P, const AScanArgs &a, uint32_t b, uint32_t q)
{
    if (((q + 1u) & (XC_SEG - 1u)) == 0u) return;
    const uint32_t cblk = P.blk_base[b];
    if (a.shadow && q >= XC_SEG && blk_cached(P.blk_pref[cblk + (q >> 11) - 1u])) return;
    const uint32_t c = P.buf_chunk0[b] + q / P.chunk_len;
    const uint32_t slot = atomicAdd(&a.pcnt[c], 1u);
    if (slot < PROP_CAP) a.pq[(size_t)c * PROP_CAP + slot] = q;
}

// Gap windows.  A segment without a level-0 anchor is indexed by a later level's
// (its last position j with G < 2^27, or < 2^28: wave_seg_anchor), and a window equal to it has no
// input anchor at offsets 63 .. 2047: its end q has none in [q - 1984, q].  So the input positions
// of every run of at least 1985 positions without an input anchor (between two records, before a
// buffer's first) are probed with their own fingerprints where G < 2^28.  k_aprop's threads note
// the gaps (gap_note), its workgroup probes them together (gap_probe).  A cache segment with no key
// at all (anc_bad: past level 2) sends a sub-batch with a gap to the exact scan.
constexpr uint32_t GAP_MAX = 16;  // gaps per k_aprop workgroup (more: the exact scan)
struct GapList {
    uint32_t n;
    uint32_t b[GAP_MAX], lo[GAP_MAX], hi[GAP_MAX];
};

// The first input anchor of buffer b at or after group g (its groups up to the sub-batch's end), or
// the buffer's length.
__device__ __forceinline__ uint32_t next_anchor(const PlanDev &P, const AScanArgs &a, uint32_t g, uint32_t b,
                                                uint32_t len)
{
    for (; g < a.g_hi; g++) {
        const uint2 gr = P.blk_grp[g];
        if (gr.x != b) break;
        const uint32_t f = P.ainfo[g].x;
        if (f != NONE) return gr.y * XC_SEG + f;
    }
    return len;
}

// Anchor-free positions lo .. hi (inclusive) of buffer b: a gap when they hold a window's 1985.
__device__ __forceinline__ void gap_note(const PlanDev &P, GapList &G, uint32_t b, uint32_t lo, uint32_t hi, bool hard)
{
    if (hi < lo || hi - lo + 1u < XC_SEG - 63u) return;
    if (hard) {
        atomicOr(&P.ctl[CTL_AFAIL], 8u);
        return;
    }
    const uint32_t k = atomicAdd(&G.n, 1u);
    if (k < GAP_MAX) {
        G.b[k] = b;
        G.lo[k] = lo;
        G.hi[k] = hi;
    } else {
        atomicOr(&P.ctl[CTL_AFAIL], 8u);
    }
}

// The gaps a flagged group (REC_GAP) answers for, from k_blockhash's records: those inside it; the
// one after its last anchor (to the buffer's next); the one before its first anchor when the group
// before it (which would answer for it) is not flagged, or the buffer's leading one (positions
// below 63 are no anchors); a group without an anchor answers for the gap across it when the group
// before it has anchors and is not flagged.  Each gap is noted once.
__device__ __forceinline__ void gaps_of_group(const PlanDev &P, const AScanArgs &a, GapList &G, uint32_t g, uint2 gr,
                                              bool hard)
{
    // (every load at once: the group's record, its neighbours', the buffer's length)
    const uint32_t b = gr.x, gpos = gr.y * XC_SEG;
    const bool has_prev = gr.y != 0u, has_next = g + 1u < a.g_hi;
    const uint4 inf = P.ainfo[g];
    const uint4 pr = has_prev ? P.ainfo[g - 1u] : make_uint4(NONE, NONE, 0u, 1u);
    const uint4 nx = has_next ? P.ainfo[g + 1u] : make_uint4(NONE, NONE, 0u, 1u);
    const uint2 nxgr = has_next ? P.blk_grp[g + 1u] : make_uint2(NONE, 0u);
    const uint32_t len = P.buf_len[b];
    if (inf.z > AGAP_CAP) {
        atomicOr(&P.ctl[CTL_AFAIL], 8u);
        return;
    }
    for (uint32_t j = 0; j < inf.z; j++) {
        const uint2 v = P.agap[g * AGAP_CAP + j];
        gap_note(P, G, b, gpos + v.x + 1u, gpos + v.y - 1u, hard);
    }
    // the buffer's first input anchor after this group (or its length)
    uint32_t next = len;
    if (nxgr.x == b) next = nx.x != NONE ? nxgr.y * XC_SEG + nx.x : next_anchor(P, a, g + 2u, b, len);
    if (inf.y != NONE) gap_note(P, G, b, gpos + inf.y + 1u, next - 1u, hard);
    const uint32_t first = inf.x != NONE ? gpos + inf.x : next;
    if (!has_prev) gap_note(P, G, b, 63u, first - 1u, hard);
    else if (!pr.w && pr.y != NONE) gap_note(P, G, b, gpos - BLK_GROUP * XC_SEG + pr.y + 1u, first - 1u, hard);
}

// Wave 0 of k_aprop's workgroup over one gap: lane t takes a stretch of its positions, G(p) and G(p - 32) by two
// rolling sums over the bytes (31 bytes of history each), and probes the fingerprints of the
// positions with G < 2^28 (the combined filter first, then both tables).
__device__ __forceinline__ void gap_probe(const PlanDev &P, const AScanArgs &a, uint32_t b, uint32_t lo, uint32_t hi)
{
    const uint8_t *base = P.in + P.buf_off[b];
    const uint32_t len = P.buf_len[b], n = hi - lo + 1u, S = (n + 63u) / 64u;
    const uint32_t p0 = lo + lane_id() * S, p1 = min(p0 + S, hi + 1u);
    if (p0 >= p1) return;
    uint32_t g1 = 0, g2 = 0;
    for (uint32_t p = p0 - 31u; p < p1; p++) {
        g1 = (g1 << 1) + base[p];
        g2 = (g2 << 1) + base[p - 32u];
        if (p < p0 || g1 >= (ANC_G_LIMIT << 2)) continue;
        const uint64_t fp = anc_fp(g1, g2);
        const uint32_t mx = anc_mix(fp);
        if (!anc_ftest(P.amix[anc_fword(mx)], mx)) continue;
        for (int tb = 0; tb < 2; tb++) {
            const AncSet &T = tb ? P.danc : P.canc;
            for (uint32_t kk = anc_home(fp, T.mask);; kk = (kk + 1u) & T.mask) {
                const uint64_t key = T.keys[kk];
                if (key == XC_EMPTY64) break;
                if ((key >> 11) != fp) continue;
                const uint32_t j = (uint32_t)key & 2047u, q = p + (XC_SEG - 1u) - j;
                if (p >= j && q < len) propose(P, a, b, q);
            }
        }
    }
}

// The proposals of record r (fingerprint fp, its positions) for the indexed key (fp, j).
__device__ __forceinline__ void propose_key(const PlanDev &P, const AScanArgs &a, uint64_t key, uint32_t ap,
                                            uint32_t nr, uint32_t len, uint32_t ck0, uint32_t cblk)
{
    const uint32_t j = (uint32_t)key & 2047u;
    for (uint32_t e = 0; e < nr; e++) {
        const uint32_t aa = ap + e, q = aa + (XC_SEG - 1u) - j;
        if (aa < j || q >= len || ((q + 1u) & (XC_SEG - 1u)) == 0u) continue;
        // REF shadow: the 2047 window ends after a predicted REF are not looked up
        if (a.shadow && q >= XC_SEG && blk_cached(P.blk_pref[cblk + (q >> 11) - 1u])) continue;
        const uint32_t c = ck0 + q / P.chunk_len;
        const uint32_t slot = atomicAdd(&a.pcnt[c], 1u);
        if (slot < PROP_CAP) a.pq[(size_t)c * PROP_CAP + slot] = q;
    }
}

// A record that passed the combined filter: the cache's and the declarations' anchor tables, both
// chains walked together (their loads in flight at once), every key with its fingerprint proposing.
__device__ __forceinline__ void aprop_probe(const PlanDev &P, const AScanArgs &a, uint64_t r, uint2 gr)
{
    const uint64_t fp = r >> 19;
    const uint32_t b = gr.x, gpos = gr.y * XC_SEG;
    const uint32_t len = P.buf_len[b], ck0 = P.buf_chunk0[b], cblk = P.blk_base[b];
    const uint32_t ap = gpos + (((uint32_t)r >> 5) & 0x3FFFu), nr = ((uint32_t)r & 31u) + 1u;
    uint32_t kc = anc_home(fp, P.canc.mask), kd = anc_home(fp, P.danc.mask);
    uint64_t yc = P.canc.keys[kc], yd = P.danc.keys[kd];
    while (yc != XC_EMPTY64 || yd != XC_EMPTY64) {
        if (yc != XC_EMPTY64) {
            if ((yc >> 11) == fp) propose_key(P, a, yc, ap, nr, len, ck0, cblk);
            kc = (kc + 1u) & P.canc.mask;
            yc = P.canc.keys[kc];
        }
        if (yd != XC_EMPTY64) {
            if ((yd >> 11) == fp) propose_key(P, a, yd, ap, nr, len, ck0, cblk);
            kd = (kd + 1u) & P.danc.mask;
            yd = P.danc.keys[kd];
        }
    }
}

// (APROP_GROUPS groups per workgroup, xc_kernels.h: every thread's record and filter loads of all
// of them in flight together; one group per workgroup left the kernel latency-bound, and 2 beat 4
// and 8 once the side stream's block hashing ran beside it: cfg5 A/B +0.8 %, aprop 0.61 -> 0.53 ms)
// A thread's records i and i + 256 of each group are loaded with the counts, before they are known
// (REC_CAP >= 512: in bounds; the slots past a count are masked after): a group has ~200 records.
constexpr uint32_t APROP_SPEC = 2;
static_assert(REC_CAP >= 256u * APROP_SPEC, "k_aprop's speculative record loads stay in bounds");
__global__ __launch_bounds__(256) void k_aprop(AScanArgs a)
{
    const PlanDev &P = a.P;
    if (aborted(P)) return;
    __shared__ GapList G;
    // a cached segment without any key (anc_bad): a sub-batch with a gap takes the exact scan
    const bool hard = uniform(*(volatile const uint32_t *)P.anc_bad) != 0u;
    const uint32_t g0 = a.g_lo + blockIdx.x * APROP_GROUPS;
    uint32_t cnt[APROP_GROUPS];
    uint2 gr[APROP_GROUPS];
    uint64_t r[APROP_SPEC][APROP_GROUPS];
#pragma unroll
    for (uint32_t k = 0; k < APROP_GROUPS; k++) {
        const bool ok = g0 + k < a.g_hi;
        cnt[k] = ok ? P.rec_cnt[g0 + k] : 0u;
        gr[k] = ok ? P.blk_grp[g0 + k] : make_uint2(0u, 0u);
#pragma unroll
        for (uint32_t u = 0; u < APROP_SPEC; u++)
            r[u][k] = ok ? P.rec[(size_t)(g0 + k) * REC_CAP + 256u * u + threadIdx.x] : ~0ull;
    }
    uint32_t gflag = 0;  // groups whose anchor record k_aprop reads (REC_GAP)
#pragma unroll
    for (uint32_t k = 0; k < APROP_GROUPS; k++) {
        gflag |= (cnt[k] & REC_GAP) ? 1u << k : 0u;
        cnt[k] &= ~REC_GAP;
    }
    bool ovf = false;
#pragma unroll
    for (uint32_t k = 0; k < APROP_GROUPS; k++) ovf |= (cnt[k] & REC_OVF) != 0u;
    if (ovf) {  // records overflowed (a long run of one byte value, say): the exact scan
        if (threadIdx.x == 0) atomicOr(&P.ctl[CTL_AFAIL], 4u);
        return;
    }
    // the gaps of the workgroup's groups: wave 0 (lane k: group g0 + k) notes them from
    // k_blockhash's record of them, then probes them, before its share of the records (nothing of
    // it stays live across the record loop: the kernel keeps its register count and occupancy)
    if (gflag && threadIdx.x < 64u) {  // (rare: ~50 flagged groups per 512 MiB sub-batch of random data)
        if (threadIdx.x == 0) G.n = 0;
        if (threadIdx.x < APROP_GROUPS && ((gflag >> threadIdx.x) & 1u))
            gaps_of_group(P, a, G, g0 + threadIdx.x, P.blk_grp[g0 + threadIdx.x], hard);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const uint32_t ng = min(uniform(G.n), GAP_MAX);
        for (uint32_t k = 0; k < ng; k++) gap_probe(P, a, G.b[k], G.lo[k], G.hi[k]);
    }
    uint32_t fw[APROP_SPEC][APROP_GROUPS];
#pragma unroll
    for (uint32_t u = 0; u < APROP_SPEC; u++)
#pragma unroll
        for (uint32_t k = 0; k < APROP_GROUPS; k++) {
            if (256u * u + threadIdx.x >= cnt[k]) r[u][k] = ~0ull;
            fw[u][k] = P.amix[r[u][k] != ~0ull ? anc_fword(anc_mix(r[u][k] >> 19)) : 0u];
        }
#pragma unroll
    for (uint32_t u = 0; u < APROP_SPEC; u++)
#pragma unroll
        for (uint32_t k = 0; k < APROP_GROUPS; k++)
            if (r[u][k] != ~0ull && anc_ftest(fw[u][k], anc_mix(r[u][k] >> 19))) aprop_probe(P, a, r[u][k], gr[k]);
    // (more than 512 records in a group: rare for random data)
    uint32_t cmax = 0;
#pragma unroll
    for (uint32_t k = 0; k < APROP_GROUPS; k++) cmax = max(cmax, cnt[k]);
    for (uint32_t i = 256u * APROP_SPEC + threadIdx.x; i < cmax; i += 256u) {
        uint64_t rr[APROP_GROUPS];
        uint32_t fv[APROP_GROUPS];
#pragma unroll
        for (uint32_t k = 0; k < APROP_GROUPS; k++) rr[k] = i < cnt[k] ? P.rec[(size_t)(g0 + k) * REC_CAP + i] : ~0ull;
#pragma unroll
        for (uint32_t k = 0; k < APROP_GROUPS; k++) fv[k] = P.amix[rr[k] != ~0ull ? anc_fword(anc_mix(rr[k] >> 19)) : 0u];
#pragma unroll
        for (uint32_t k = 0; k < APROP_GROUPS; k++)
            if (rr[k] != ~0ull && anc_ftest(fv[k], anc_mix(rr[k] >> 19))) aprop_probe(P, a, rr[k], gr[k]);
    }
}

__global__ __launch_bounds__(256) void k_aevents(AScanArgs a)
{
    const PlanDev &P = a.P;
    __shared__ uint32_t bitsl[4][CHUNK_BLOCKS * XC_SEG / 32];
    const uint32_t wave = threadIdx.x >> 6, l = lane_id();
    const uint32_t c = a.ck_lo + blockIdx.x * 256u + threadIdx.x;
    const bool live = c < a.ck_hi;
    if (aborted(P)) {
        if (live) a.pcnt[c] = 0u;
        return;
    }
    uint32_t c0 = 0, c1 = 0, n = 0;
    if (live) {
        const uint4 d = P.chunk_desc[c];
        c0 = d.x;
        c1 = d.y & 0x3FFFFFFFu;
        n = a.pcnt[c];
    }
    if (n > PROP_CAP) {
        atomicOr(&P.ctl[CTL_AFAIL], 16u);
        n = 0;
    }
    if (live && n == 0) {  // the aligned windows only (k_resolve sorts nothing: they are in order)
        uint32_t k = 0;
        for (uint32_t q = c0 + (XC_SEG - 1u); q < c1; q += XC_SEG) a.L.pos[c * EV_CAP + k++] = q;
        a.L.cnt[c] = k;
    }
    // chunks with proposals: each by the whole wave (LDS bitmask: sorted, deduplicated)
    uint32_t *bm = bitsl[wave];
    const uint32_t W = P.chunk_len / 32u;
    for (uint64_t m = ballot(live && n > 0); m; m &= m - 1) {
        const int f = __ffsll((unsigned long long)m) - 1;
        const uint32_t cc = readlane(c, f), cs = readlane(c0, f), ce = readlane(c1, f), nn = readlane(n, f);
        for (uint32_t i = l; i < W; i += 64u) bm[i] = 0u;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        for (uint32_t q = cs + (XC_SEG - 1u) + XC_SEG * l; q < ce; q += 64u * XC_SEG)
            atomicOr(&bm[(q - cs) >> 5], 1u << ((q - cs) & 31u));
        if (l < nn) {
            const uint32_t q = a.pq[(size_t)cc * PROP_CAP + l];
            atomicOr(&bm[(q - cs) >> 5], 1u << ((q - cs) & 31u));
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        uint32_t tot = 0;
        for (uint32_t i = l; i < W; i += 64u) tot += (uint32_t)__popc(bm[i]);
        tot = wave_sum(tot);
        if (tot <= EV_CAP) {
            uint32_t base = 0;
            for (uint32_t i0 = 0; i0 < W; i0 += 64u) {
                const uint32_t i = i0 + l;
                uint32_t v = i < W ? bm[i] : 0u;
                const uint32_t k = (uint32_t)__popc(v), incl = wave_incl_scan(k);
                uint32_t o = base + incl - k;
                while (v) {
                    const uint32_t bit = (uint32_t)__builtin_ctz(v);
                    v &= v - 1u;
                    a.L.pos[cc * EV_CAP + o++] = cs + 32u * i + bit;
                }
                base += readlane(incl, 63);
            }
            if (l == 0) a.L.cnt[cc] = tot;
        } else {
            for (uint32_t i = l; i < W; i += 64u) a.L.bits[(size_t)cc * W + i] = bm[i];
            if (l == 0) {
                a.L.cnt[cc] = EV_DENSE | EV_CAP;
                atomicAdd(&P.ctl[CTL_DENSE], 1u);
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    if (live) a.pcnt[c] = 0u;  // (clean for the next sub-batch)
}

// ------------------------------------------------------------- k_resolve ----------------
// One wave per chunk: sort the sparse list, then resolve every event exactly.

// Resolve the window ending at q of buffer b: full hash (from the aligned-block table when the
// window is a block), then the cache (EQUAL / COLL) and / or the declaration set (MATCH).
__device__ __forceinline__ uint32_t resolve_one(const PlanDev &P, int dmode, uint32_t b, const uint8_t *base,
                                                uint32_t q, uint64_t *h_out, uint64_t *val_out)
{
    const uint8_t *win = base + q - (XC_SEG - 1u);
    uint64_t h;
    if (((q + 1u) & (XC_SEG - 1u)) == 0u && P.blk_h) {
        const uint32_t bi = uniform(P.blk_base[b]) + (q + 1u) / XC_SEG - 1u;
        h = ((uint64_t)uniform((uint32_t)(P.blk_h[bi] >> 32)) << 32) | uniform((uint32_t)P.blk_h[bi]);
    } else {
        h = wave_window_hash(win);
    }
    *h_out = h;
    uint64_t v = 0;
    if (dmode != 1 && set_find(P.cache, h, &v)) {
        *val_out = v;
        return wave_equal2048(win, seg_at(P.segs, v)) ? ST_EQUAL : ST_COLL;
    }
    if (dmode != 0 && set_find(P.dset, h, &v)) {
        *val_out = v;
        return ST_MATCH;
    }
    *val_out = 0;
    return ST_MISS;
}

__device__ __forceinline__ uint64_t readlane64(uint64_t x, int l)
{
    return ((uint64_t)readlane((uint32_t)(x >> 32), l) << 32) | readlane((uint32_t)x, l);
}

__global__ __launch_bounds__(64 * RES_WAVES) void k_resolve(ResolveArgs a)
{
    // the scan that ran before has handed out all its work: reset its counter for the next
    // scan (before the abort check, so a redone sub-batch starts from a clean counter)
    if (blockIdx.x == 0 && threadIdx.x == 0) a.P.ctl[CTL_SCAN_NEXT] = 0u;
    if (aborted(a.P)) return;
    if (blockIdx.x == 0 && threadIdx.x == 0) {  // the walk that follows reports afresh
        a.P.ctl[CTL_GREW] = 0u;
        a.P.ctl[CTL_FIRST_CROSS] = NONE;
        a.P.ctl[CTL_SHADOW] = 0u;
    }
    const uint32_t c = a.ck_lo + blockIdx.x * RES_WAVES + (threadIdx.x >> 6);
    if (c >= a.ck_hi) return;
    const uint32_t cnt = a.L.cnt[c];
    if (cnt == 0 || (cnt & EV_DENSE)) return;
    const PlanDev &P = a.P;
    const uint32_t l = lane_id();
    const bool live = l < cnt;
    const uint2 ck = P.chunks[c];
    const uint8_t *base = P.in + P.buf_off[ck.x];
    // sort: lane l ends up holding the event of rank l
    const uint32_t p0 = live ? a.L.pos[c * EV_CAP + l] : NONE;
    uint32_t rank = 0;
    for (uint32_t k = 0; k < cnt; k++) rank += readlane(p0, (int)k) < p0 ? 1u : 0u;
    const uint32_t q = (uint32_t)__builtin_amdgcn_ds_permute((int)(4u * (live ? rank : l)), (int)p0);
    // full hashes: aligned windows from the block table (lane-parallel), the rest per wave.  On
    // the first round (dmode 2) k_blockpredict already probed the cache for every aligned block
    // of a buffer without carried state and entered the others in D: their slots come from
    // blk_pref (the cache does not change between k_blockpredict and this kernel).
    const bool aligned = live && ((q + 1u) & (XC_SEG - 1u)) == 0u && P.blk_h;
    const bool pref_ok = a.dmode == 2 && !stream_carried(P, ck.x);
    uint64_t h = 0;
    uint32_t pref = 0, bcmp = 0;
    if (aligned) {
        const uint32_t gi = P.chunk_blk[c] + (q + 1u) / XC_SEG - 1u;
        h = P.blk_h[gi];
        if (pref_ok) {
            pref = P.blk_pref[gi];
            bcmp = P.blk_cmp[gi];
        }
    }
    for (uint64_t m = ballot(live && !aligned); m; m &= m - 1) {
        const int f = __ffsll((unsigned long long)m) - 1;
        const uint32_t qf = readlane(q, f);
        const uint64_t hf = wave_window_hash(base + qf - (XC_SEG - 1u));
        if ((int)l == f) h = hf;
    }
    // cache then declaration-set probes, lane-parallel
    uint64_t v = 0;
    uint32_t st = ST_MISS;
    const bool known = pref != 0u;  // (aligned and pref_ok)
    bool compared = false;  // k_blockhash compared the block with the same cached segment
    if (known) {
        if (blk_cached(pref)) {
            compared = bcmp != 0u && (bcmp & ~BC_DIFF) == pref;
            st = compared && (bcmp & BC_DIFF) ? ST_COLL : ST_EQUAL;  // (else until the comparison below)
            v = pref - 1u;
        } else {
            st = ST_MATCH;
            v = P.dset.vals[pref & ~BP_DECL];
        }
    }
    if (live && !known && a.dmode != 1 && set_find(P.cache, h, &v)) st = ST_EQUAL;
    if (live && !known && st == ST_MISS && a.dmode != 0) {
        if (set_find(P.dset, h, &v)) st = ST_MATCH;
        else v = 0;
    }
    // 2048-byte comparisons against the cached segments: up to 4 per pass, all loads in flight
    for (uint64_t m = ballot(st == ST_EQUAL && !compared); m;) {
        int f[4];
        uint32_t x[4][8], y[4][8];
#pragma unroll
        for (int g = 0; g < 4; g++) {
            f[g] = m ? __ffsll((unsigned long long)m) - 1 : -1;
            if (m) m &= m - 1;
            if (f[g] >= 0) {
                const uint32_t qf = readlane(q, f[g]);
                const uint64_t vf = readlane64(v, f[g]);
                const uint8_t *wp = base + qf - (XC_SEG - 1u) + 32u * l;
                if (((qf + 1u) & (XC_SEG - 1u)) == 0u) load32_aligned(wp, x[g]);  // a block: 2 x 16 B
                else load32_unaligned(wp, x[g]);
                const uint4 *sp = (const uint4 *)(seg_at(P.segs, vf) + 32u * l);
                const uint4 s0 = sp[0], s1 = sp[1];
                y[g][0] = s0.x; y[g][1] = s0.y; y[g][2] = s0.z; y[g][3] = s0.w;
                y[g][4] = s1.x; y[g][5] = s1.y; y[g][6] = s1.z; y[g][7] = s1.w;
            }
        }
#pragma unroll
        for (int g = 0; g < 4; g++) {
            if (f[g] < 0) continue;
            uint32_t diff = 0;
#pragma unroll
            for (int k = 0; k < 8; k++) diff |= x[g][k] ^ y[g][k];
            if (ballot(diff != 0u) && (int)l == f[g]) st = ST_COLL;
        }
    }
    if (live) {
        const uint32_t i = c * EV_CAP + l;
        a.L.pos[i] = q;
        a.L.stat[i] = st;
        a.L.h[i] = h;
        a.L.val[i] = v;
    }
}

// ---------------------------------------------------------------- k_walk ----------------
// Walk cursor over one layer of one buffer: the current chunk's sorted sparse events live
// in registers, lane i holding event i, so finding the next event is one ballot.
struct Cursor {
    uint32_t k, cnt, cs;  // chunk index, count|EV_DENSE, first position (uniform)
    uint32_t pos, stat;   // lane-held event (pos = NONE past cnt)
    uint64_t h, v;
};

__device__ __forceinline__ void cur_load(const PlanDev &P, const Layer &L, Cursor &c, uint32_t ck1)
{
    c.pos = NONE;
    if (c.k >= ck1) return;
    c.cnt = uniform(L.cnt[c.k]);
    c.cs = uniform(P.chunks[c.k].y);
    const uint32_t l = lane_id();
    if (!(c.cnt & EV_DENSE) && l < c.cnt) {
        const uint32_t i = c.k * EV_CAP + l;
        c.pos = L.pos[i];
        c.stat = L.stat[i];
        c.h = L.h[i];
        c.v = L.val[i];
    }
}

__device__ __forceinline__ Cursor cur_begin(const PlanDev &P, const Layer &L, uint32_t ck0, uint32_t ck1)
{
    Cursor c;
    c.k = ck0;
    c.cnt = 0;
    c.cs = 0;
    c.stat = 0;
    c.h = c.v = 0;
    cur_load(P, L, c, ck1);
    return c;
}

// First set bit at chunk offset >= from, or NONE.
__device__ __forceinline__ uint32_t dense_find(const uint32_t *bits, uint32_t from, uint32_t W)
{
    const uint32_t l = lane_id();
    for (uint32_t w0 = from >> 5; w0 < W; w0 += 64u) {
        const uint32_t wi = w0 + l;
        uint32_t v = wi < W ? bits[wi] : 0u;
        if (wi == (from >> 5)) v &= ~0u << (from & 31u);
        const uint64_t m = ballot(v != 0u);
        if (m) {
            const int f = __ffsll((unsigned long long)m) - 1;
            const uint32_t vv = readlane(v, f);
            return (w0 + (uint32_t)f) * 32u + (uint32_t)(__builtin_ctz(vv));
        }
    }
    return NONE;
}

// Next event position >= p in the layer (chunks [cur.k, ck1) of one buffer), or NONE.
__device__ __forceinline__ uint32_t next_event(const PlanDev &P, const Layer &L, Cursor &cur, uint32_t ck1,
                                               uint32_t p)
{
    const uint32_t W = P.chunk_len / 32u;
    while (cur.k < ck1) {
        if (cur.cnt & EV_DENSE) {
            const uint32_t from = p > cur.cs ? p - cur.cs : 0u;
            if (from < P.chunk_len) {
                const uint32_t r = dense_find(L.bits + (size_t)cur.k * W, from, W);
                if (r != NONE) return cur.cs + r;
            }
        } else {
            const uint64_t m = ballot(cur.pos != NONE && cur.pos >= p);
            if (m) return readlane(cur.pos, __ffsll((unsigned long long)m) - 1);
        }
        cur.k++;
        cur_load(P, L, cur, ck1);
    }
    return NONE;
}

struct EvInfo {
    uint32_t st;
    uint64_t h, v;
};


// Event of the layer exactly at q, or st = NONE.
__device__ __forceinline__ EvInfo event_at(const PlanDev &P, const Layer &L, Cursor &cur, uint32_t ck1, uint32_t q,
                                           int dmode, uint32_t b, const uint8_t *base)
{
    EvInfo e;
    e.st = NONE;
    e.h = 0;
    e.v = 0;
    if (next_event(P, L, cur, ck1, q) != q) return e;
    if (cur.cnt & EV_DENSE) {
        e.st = resolve_one(P, dmode, b, base, q, &e.h, &e.v);
    } else {
        const int f = __ffsll((unsigned long long)ballot(cur.pos == q)) - 1;
        e.st = readlane(cur.stat, f);
        e.h = readlane64(cur.h, f);
        e.v = readlane64(cur.v, f);
    }
    return e;
}

constexpr uint32_t R_MISS = 0, R_HIT = 1, R_COLL = 2;

// The sequential walk of buffer b (one wave).
__device__ __forceinline__ void walk_seq(const WalkArgs &a, uint32_t b, uint64_t *walk_lds)
{
    // declarations of this buffer (sized by the plan's longest buffer, so short buffers leave
    // room for many walk waves per CU) and the aligned REFs emitted, one bit per block
    uint64_t *d_hash = walk_lds;
    uint32_t *d_cand = (uint32_t *)(walk_lds + a.max_decl);
    uint32_t *d_known = d_cand + a.max_decl;
    uint32_t *ref_done = d_known + a.max_decl;
    const PlanDev &P = a.P;
    const uint32_t l = lane_id();
    const uint32_t len = P.buf_len[b];
    const uint8_t *base = P.in + P.buf_off[b];
    const uint32_t ck0 = P.buf_chunk0[b], ck1 = P.buf_chunk0[b + 1];
    const uint32_t tb = P.tok_base[b];
    const uint32_t tcap = 2u * (len / XC_SEG) + 3u;
    Cursor cs = cur_begin(P, P.S, ck0, ck1);  // cache + predicted declarations
    Cursor cd = cur_begin(P, P.D, ck0, a.use_d ? ck1 : ck0);
    uint32_t ntok = 0, nd = 0;
    uint32_t basep = 0;
    int cand = -1;
    uint64_t cand_h = 0;
    uint32_t cand_known = 0;
    uint32_t p = XC_SEG - 1u;
    bool cross = false;
    bool noflush = false;
    if (P.stream_st) {
        // a stream's pending source_: window ends below start were looked up by earlier calls
        // (xcodec_encoder.cc:72-118), a pending candidate carries over (its hash: decl_hash)
        const uint4 st = P.stream_st[b];
        p = max(p, uniform(st.x));
        if (uniform(st.y) != NONE) cand = (int)uniform(st.y);
        noflush = (uniform(st.z) & SF_NOFLUSH) != 0u;
    }

    if (a.shadow)
        for (uint32_t i = l; i < a.max_decl / 32u + 1u; i += 64u) ref_done[i] = 0u;
    uint32_t n_ext = 0, n_ref = 0;
    auto emit = [&](uint32_t op, uint32_t lb, uint32_t le, uint32_t seg, uint32_t dpos, uint64_t h,
                    uint32_t known) {
        n_ext += op == OP_EXTRACT ? 1u : 0u;
        n_ref += op == OP_REF ? 1u : 0u;
        if (a.shadow && op == OP_REF && (seg & (XC_SEG - 1u)) == 0u && l == 0) {
            const uint32_t k = seg / XC_SEG;  // the REF covers aligned block k
            ref_done[k >> 5] |= 1u << (k & 31u);
        }
        if (ntok < tcap && l == 0) {
            P.tok_op[tb + ntok] = op;
            P.tok_known[tb + ntok] = known;
            P.tok_lb[tb + ntok] = lb;
            P.tok_le[tb + ntok] = le;
            P.tok_seg[tb + ntok] = seg;
            P.tok_dpos[tb + ntok] = dpos;
            P.tok_h[tb + ntok] = h;
        }
        ntok++;
    };

    // Own declarations with a known hash equal to h (lanes search 64 at a time).
    auto own_decl = [&](uint64_t h) -> uint32_t {
        for (uint32_t i0 = 0; i0 < nd; i0 += 64u) {
            const uint32_t i = i0 + l;
            const uint64_t m = ballot(i < nd && d_known[i] && d_hash[i] == h);
            if (m) return i0 + (uint32_t)(__ffsll((unsigned long long)m) - 1);
        }
        return NONE;
    };

    // Lookup at q (xcodec_encoder.cc:89-118 + xcodec_cache.h:190-210): the cache as of the
    // batch start, or a segment this buffer declared earlier.  Layer S holds cache hits
    // (EQUAL / COLL) and predicted-declaration matches (MATCH); layer D, used only when the
    // walk declared hashes nobody predicted, holds matches against every declaration.
    // (layer D, when present, is the fresher view: table values can only have decreased)
    auto decl_info = [&](uint32_t q, EvInfo s) -> EvInfo {
        if (!a.use_d) return s;
        return event_at(P, P.D, cd, ck1, q, 1, b, base);
    };
    // A candidate whose hash a declaration-set match supplies: 1, or 2 when the entry is a later
    // buffer's (its predicted declaration of the same bytes): this buffer declares them first, so
    // the set must hold this buffer's declaration (decl_hash enters it and asks for another round,
    // in which that later buffer sees it as an earlier buffer's declaration: a cross-buffer case).
    auto known_of = [&](const EvInfo &d) -> uint32_t { return (uint32_t)(d.v >> 32) > b ? 2u : 1u; };
    uint32_t n_coll = 0;
    // a lookup hit with other bytes: record it, with the candidate pending then (NONE: none)
    auto coll = [&](uint32_t q, uint64_t h) {
        if (P.coll && n_coll < COLL_CAP && l == 0)
            P.coll[b * COLL_CAP + n_coll] =
                make_uint4(q, (uint32_t)h, (uint32_t)(h >> 32), cand >= 0 ? (uint32_t)cand : NONE);
        n_coll++;
    };
    auto lookup = [&](uint32_t q, uint64_t *hout) -> uint32_t {
        EvInfo s = event_at(P, P.S, cs, ck1, q, 2, b, base);
        if (s.st == ST_EQUAL) { *hout = s.h; return R_HIT; }
        if (s.st == ST_COLL) { coll(q, s.h); return R_COLL; }
        EvInfo d = decl_info(q, s);
        if (d.st != ST_MATCH) return R_MISS;
        const uint32_t i = own_decl(d.h);
        if (i != NONE) {
            *hout = d.h;
            if (wave_equal2048(base + q - (XC_SEG - 1u), base + d_cand[i])) return R_HIT;
            coll(q, d.h);
            return R_COLL;
        }
        if ((uint32_t)(d.v >> 32) < b) cross = true;  // an earlier buffer declared it
        return R_MISS;
    };

    if (cand >= 0) {  // the carried candidate's hash, when a resolved event supplies it
        const uint32_t q = (uint32_t)cand + XC_SEG - 1u;
        const EvInfo d = decl_info(q, event_at(P, P.S, cs, ck1, q, 2, b, base));
        if (d.st == ST_MATCH) { cand_known = known_of(d); cand_h = d.h; }
    }
    while (p < len) {
        if (cand < 0) {
            uint64_t h = 0;
            const uint32_t r = lookup(p, &h);
            if (r == R_HIT) {
                emit(OP_REF, basep, p - (XC_SEG - 1u), p - (XC_SEG - 1u), 0, h, 1);
                basep = p + 1u;
                p = basep + (XC_SEG - 1u);
                continue;
            }
            if (r == R_COLL) { p++; continue; }
            cand = (int)(p - (XC_SEG - 1u));
            cand_known = 0;
            cand_h = 0;
            {
                const EvInfo d = decl_info(p, event_at(P, P.S, cs, ck1, p, 2, b, base));
                if (d.st == ST_MATCH) { cand_known = known_of(d); cand_h = d.h; }
            }
            p++;
            continue;
        }
        const uint32_t dp = (uint32_t)cand + 2u * XC_SEG - 1u;
        uint32_t e = next_event(P, P.S, cs, ck1, p);
        if (a.use_d) e = min(e, next_event(P, P.D, cd, ck1, p));
        if (e < dp && e < len) {
            uint64_t h = 0;
            const uint32_t r = lookup(e, &h);
            if (r == R_HIT) {
                emit(OP_REF, basep, e - (XC_SEG - 1u), e - (XC_SEG - 1u), 0, h, 1);
                basep = e + 1u;
                cand = -1;
                p = basep + (XC_SEG - 1u);
            } else {
                p = e + 1u;
            }
            continue;
        }
        if (dp >= len) break;
        // declaration (xcodec_encoder.cc:77-82, 203-215)
        emit(OP_EXTRACT, basep, (uint32_t)cand, (uint32_t)cand, dp, cand_h, cand_known);
        if (nd < a.max_decl) {
            if (l == 0) {
                d_cand[nd] = (uint32_t)cand;
                d_hash[nd] = cand_h;
                d_known[nd] = cand_known;
            }
            nd++;
        }
        basep = (uint32_t)cand + XC_SEG;
        cand = -1;
        p = dp;
    }
    if (noflush) {
        // encode() returns here: the candidate and the bytes from basep stay in source_
        if (l == 0) P.stream_res[b] = make_uint2(basep, cand >= 0 ? (uint32_t)cand : NONE);
        emit(OP_END, basep, basep, 0, 0, 0, 0);
    } else {
        // flush (xcodec_encoder.cc:175-201)
        if (cand >= 0) {
            emit(OP_EXTRACT, basep, (uint32_t)cand, (uint32_t)cand, DPOS_FLUSH, cand_h, cand_known);
            basep = (uint32_t)cand + XC_SEG;
        }
        emit(OP_END, basep, len, 0, 0, 0, 0);
        if (P.stream_res && l == 0) P.stream_res[b] = make_uint2(len, NONE);
    }
    if (a.shadow) {
        // every predicted REF whose following block the scan skipped must have been emitted
        // (ref_done was written by this wave's lane 0: a wave-level barrier orders it)
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const uint32_t nblk = len / XC_SEG, bb = P.blk_base[b];
        bool miss = false;
        for (uint32_t k = l; k < nblk; k += 64u)
            if ((k + 1u) * XC_SEG < len && blk_cached(P.blk_pref[bb + k]) && !((ref_done[k >> 5] >> (k & 31u)) & 1u))
                miss = true;
        if (ballot(miss) && l == 0) atomicOr(&P.ctl[CTL_SHADOW], 1u);
    }
    if (l == 0) {
        P.tok_cnt[b] = ntok;
        P.buf_next[b] = n_ext;
        P.buf_nref[b] = n_ref;
        if (P.coll_cnt) P.coll_cnt[b] = n_coll;
        if (n_coll) atomicOr(&P.ctl[CTL_COLLS], 1u);
        if (ntok > tcap) atomicOr(&P.ctl[CTL_ERROR], ERR_TOKENS);
        if (cross) atomicMin(&P.ctl[CTL_FIRST_CROSS], b);
    }
}

// ------------------------------------------------------------ walk_blocks ----------------
// The first-round walk of a buffer whose events decide nothing between its aligned windows
// (hit-free data and block-aligned repeats: every cfg workload), lane-parallel.  In k_walk's
// state machine (xcodec_encoder.cc:77-170) a lookup with no candidate pending happens only at
// aligned positions p_k = 2048k + 2047 as long as every aligned lookup either
//   hits the cache with equal bytes -> REF of block k (the hash resets; next lookup p_{k+1}), or
//   misses                          -> candidate = block k, declared at p_{k+1} = cand + 4095
//                                      (or by flush() for the last block) just before p_{k+1}
//                                      is looked up,
// and every unaligned event in between is a plain miss (a lo32 match whose full hash is
// absent: it changes nothing).  Then block k's token depends on the event at p_k alone.  The
// reduction fails on a collision (the next candidate becomes unaligned), an unaligned event
// that is a hit / collision / declaration match, a dense chunk, or a block repeating an earlier
// new block of the same buffer (a self-REF that needs a byte compare; the declaration set's
// min-merged value tells).  Such buffers take the sequential walk.
// Returns false (nothing written that the sequential walk would not rewrite) when the
// reduction does not apply to buffer b.  The buffer's chunks are shared by the workgroup's
// a.waves waves (groups of WB_GROUP chunks round-robin), combined through LDS.
struct WalkShared {
    uint32_t fail, cross, n_ext, n_ref;
    uint32_t n_unk;  // EXTRACTs whose hash no event supplied (decl_hash's work)
};

__device__ __forceinline__ bool walk_blocks(const WalkArgs &a, uint32_t b, WalkShared &sh)
{
    const PlanDev &P = a.P;
    const uint32_t l = lane_id(), wave = threadIdx.x >> 6;
    const uint32_t len = P.buf_len[b];
    const uint32_t nblk = len / XC_SEG;
    const uint32_t ck0 = P.buf_chunk0[b], ck1 = P.buf_chunk0[b + 1];
    const uint32_t tb = P.tok_base[b];
    if (!stream_plain(P, b)) return false;  // carried state: the sequential walk
    if (threadIdx.x == 0) sh = WalkShared{0u, 0u, 0u, 0u, 0u};
    __syncthreads();
    bool ok = true, cross = false;
    uint32_t n_ext = 0, n_ref = 0, n_unk = 0;
    // chunks in groups of WB_GROUP: every load of a group is issued before any is used (a buffer
    // of short chunks would otherwise pay one memory round trip per chunk)
    constexpr uint32_t WB_GROUP = 4;
    for (uint32_t cg = ck0 + wave * WB_GROUP; cg < ck1 && ballot(!ok) == 0; cg += a.waves * WB_GROUP) {
        if (a.waves > 1 && *(volatile uint32_t *)&sh.fail) break;  // another wave gave up
        uint32_t cnt[WB_GROUP], q[WB_GROUP], st[WB_GROUP];
        uint64_t hh[WB_GROUP], vv[WB_GROUP];
#pragma unroll
        for (uint32_t i = 0; i < WB_GROUP; i++) {
            cnt[i] = 0u;
            q[i] = st[i] = 0u;
            hh[i] = vv[i] = 0u;
            if (cg + i < ck1) {  // (uniform) entries past the count are loaded but never used
                const uint32_t e = (cg + i) * EV_CAP + l;
                cnt[i] = uniform(P.S.cnt[cg + i]);
                q[i] = P.S.pos[e];
                st[i] = P.S.stat[e];
                hh[i] = P.S.h[e];
                vv[i] = P.S.val[e];
            }
        }
#pragma unroll
        for (uint32_t i = 0; i < WB_GROUP; i++) {
            const uint32_t c = cg + i;
            if (c >= ck1) break;
            const uint32_t c0 = (c - ck0) * P.chunk_len;
            const uint32_t want = min(c0 + P.chunk_len, len) / XC_SEG - c0 / XC_SEG;  // aligned ends
            if (cnt[i] & EV_DENSE) { ok = false; break; }
            bool aligned = false;
            if (l < cnt[i]) {
                aligned = ((q[i] + 1u) & (XC_SEG - 1u)) == 0u;
                if (!aligned) {
                    if (st[i] != ST_MISS) ok = false;
                } else {
                    const uint32_t k = q[i] / XC_SEG;
                    const uint64_t h = hh[i], v = vv[i];
                    const uint32_t dpos = q[i] + XC_SEG;  // declaration point cand + 4095
                    if (st[i] == ST_COLL) ok = false;
                    if (st[i] == ST_MATCH && (uint32_t)(v >> 32) == b && (uint32_t)v < dpos) ok = false;  // self-REF
                    if (st[i] == ST_MATCH && (uint32_t)(v >> 32) < b) cross = true;
                    const uint32_t t = tb + k;
                    if (st[i] == ST_EQUAL) {
                        P.tok_op[t] = OP_REF;
                        P.tok_known[t] = 1u;
                        P.tok_dpos[t] = 0u;
                        P.tok_h[t] = h;
                        n_ref++;
                    } else {
                        P.tok_op[t] = OP_EXTRACT;
                        P.tok_known[t] = st[i] == ST_MATCH ? 1u : 0u;
                        n_unk += st[i] == ST_MATCH ? 0u : 1u;
                        P.tok_dpos[t] = dpos < len ? dpos : DPOS_FLUSH;
                        P.tok_h[t] = st[i] == ST_MATCH ? h : 0u;
                        n_ext++;
                    }
                    P.tok_lb[t] = k * XC_SEG;
                    P.tok_le[t] = k * XC_SEG;
                    P.tok_seg[t] = k * XC_SEG;
                }
            }
            if ((uint32_t)__popcll(ballot(aligned)) != want) ok = false;  // each aligned end, once
        }
    }
    const bool wave_fail = ballot(!ok) != 0;  // (every lane's verdict: ballots run on all lanes)
    n_ext = wave_sum(n_ext);
    n_ref = wave_sum(n_ref);
    n_unk = wave_sum(n_unk);
    const bool any_cross = ballot(cross) != 0;
    if (l == 0) {
        if (wave_fail) atomicOr(&sh.fail, 1u);
        if (any_cross) atomicOr(&sh.cross, 1u);
        atomicAdd(&sh.n_ext, n_ext);
        atomicAdd(&sh.n_ref, n_ref);
        atomicAdd(&sh.n_unk, n_unk);
    }
    __syncthreads();
    if (sh.fail) return false;
    if (threadIdx.x == 0) {
        uint32_t t = tb + nblk;  // END: the tail after the last block, escaped by flush()
        uint32_t end = len, n_ext = sh.n_ext, n_unk = sh.n_unk;
        uint2 res = make_uint2(len, NONE);  // flushed: source_ empty
        if (stream_noflush(P, b)) {
            // encode() without flush() (xcodec_encoder.cc:60-170): the last block's candidate is
            // due at cand + 4095 >= len, so it stays pending with the bytes from it in source_;
            // after a REF of the last block the tail stays in source_ (no candidate)
            end = nblk * XC_SEG;
            res = make_uint2(end, NONE);
            if (nblk && P.tok_op[t - 1u] == OP_EXTRACT) {
                t--;
                end -= XC_SEG;
                res = make_uint2(end, end);
                n_ext--;
                n_unk -= P.tok_known[t] == 1u ? 0u : 1u;
            }
            P.tok_cnt[b] = t - tb + 1u;
        } else {
            P.tok_cnt[b] = nblk + 1u;
        }
        P.tok_op[t] = OP_END;
        P.tok_known[t] = 0u;
        P.tok_lb[t] = t == tb + nblk ? nblk * XC_SEG : end;
        P.tok_le[t] = end;
        P.tok_seg[t] = 0u;
        P.tok_dpos[t] = 0u;
        P.tok_h[t] = 0u;
        P.buf_next[b] = n_ext;
        P.buf_nref[b] = sh.n_ref;
        sh.n_unk = n_unk;
        if (P.coll_cnt) P.coll_cnt[b] = 0u;  // (a collision makes the walk sequential)
        if (P.stream_res) P.stream_res[b] = res;
        if (sh.cross) atomicMin(&P.ctl[CTL_FIRST_CROSS], b);
    }
    __syncthreads();  // (sh.n_unk: k_walk reads it)
    return true;
}

// ------------------------------------------------------------ k_walk ---------------------
// The EXTRACT tokens of buffer b whose hash no resolved event supplied are hashed and entered
// into the declaration set (value = b<<32 | declaration position, min-merged); any such entry
// means the scan missed it: another round.  So are the declarations whose hash came from a later
// buffer's entry (tok_known 2): their min-merged value moves to this buffer.
__device__ __forceinline__ void decl_hash(const PlanDev &P, uint32_t b)
{
    const uint32_t l = lane_id();
    const uint8_t *base = P.in + P.buf_off[b];
    const uint32_t tb = P.tok_base[b], n = P.tok_cnt[b];
    for (uint32_t t0 = 0; t0 < n; t0 += 64u) {
        const uint32_t t = t0 + l;
        const bool unknown = t < n && P.tok_op[tb + t] == OP_EXTRACT && P.tok_known[tb + t] != 1u;
        for (uint64_t m = ballot(unknown); m; m &= m - 1) {
            const uint32_t tt = tb + t0 + (uint32_t)(__ffsll((unsigned long long)m) - 1);
            const uint32_t seg = uniform(P.tok_seg[tt]);
            const bool known = uniform(P.tok_known[tt]) != 0u;
            const uint64_t h = known ? ((uint64_t)uniform((uint32_t)(P.tok_h[tt] >> 32)) << 32) |
                                           uniform((uint32_t)P.tok_h[tt])
                                     : wave_window_hash(base + seg);
            if (P.anc_scan && !known) {
                // anchor-scanned: events are the windows equal to indexed segments, so a candidate
                // outside them was assumed a miss; a cache entry with its hash (other bytes: a
                // collision, xcodec_encoder.cc:129-137) makes the exact scan redo the sub-batch
                uint64_t v;
                if (set_find(P.cache, h, &v) && l == 0) atomicOr(&P.ctl[CTL_AFAIL], 2u);
            }
            if (l == 0) {
                P.tok_h[tt] = h;
                const uint64_t v = ((uint64_t)b << 32) | P.tok_dpos[tt];
                // (an anchor-scanned sub-batch's set is keys and values only: k_clear_set leaves its
                // filters and lo32 keys alone, so nothing may be added to them)
                if (P.anc_scan) {
                    uint32_t slot;
                    set_insert_kv(P.dset, h, v, &slot);
                } else {
                    set_insert(P.dset, h, v, true, nullptr, nullptr);
                }
                // not in the set the positions were scanned against: another round is needed
                if (__hip_atomic_load(&P.ctl[CTL_GREW], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u)
                    atomicOr(&P.ctl[CTL_GREW], 1u);
            }
        }
    }
}

// One wave per buffer: the first round tries the block-parallel walk, else (and in later rounds)
// the sequential walk; then the declarations whose hash is still unknown are hashed.
__global__ __launch_bounds__(64 * WALK_WAVES_MAX) void k_walk(WalkArgs a)
{
    if (aborted(a.P)) return;
    extern __shared__ uint64_t walk_lds[];
    __shared__ WalkShared sh;
    const uint32_t b = a.j0 + blockIdx.x;
    if (b >= a.j1) return;
    const bool blocks = !a.use_d && walk_blocks(a, b, sh);  // (every wave, or none: uniform per block)
    if (threadIdx.x >= 64u) return;  // the sequential walk and the declaration hashes: wave 0
    if (!blocks) walk_seq(a, b, walk_lds);
    // (a block walk whose every EXTRACT hash came from an event leaves decl_hash nothing to do)
    if (!blocks || sh.n_unk) decl_hash(a.P, b);
}

// Hash of every aligned 2048-byte block, one wave per group of <= BLK_GROUP consecutive blocks
// of one buffer (P.blk_grp; [a.j0, a.j1) is a range of groups), four waves per workgroup: a
// wave has all its loads in flight together.  Depends on the input only, so it runs ahead on a
// side stream.  (One-wave workgroups made this kernel dispatch-bound.)

// Block g (global index; block k of buffer b) with hash h: blocks absent from the cache are the
// predicted declarations (hit-free data declares exactly these, xcodec_encoder.cc:77-82); they
// enter the declaration set and the combined level-2 filter before the scan (and, on an
// anchor-scanned sub-batch, the declaration set's anchor table: akey).  Cached blocks are
// predicted REFs (REF shadows).
// Returns the prediction (blk_pref).
__device__ __forceinline__ uint32_t block_predict(const PlanDev &P, uint32_t g, uint32_t b, uint32_t k, uint64_t h,
                                                  uint64_t akey);

constexpr uint32_t ANC_LIST = 512;  // anchor list entries per pass (a multiple of 64)

// The anchors of a k_blockhash group: G of every position of its na blocks
// (w[i]: block i, lane l: bytes 32 l .. 32 l + 31) into tile (per wave: 32 rows of 64 values and a pad word, then the
// 32 values of the lane before lane 0), the block's anchors compacted into a position-ordered list
// (list: ANC_LIST entries per wave, in passes), then every input anchor into the group's records, 64 list entries
// at a time (runs of equal fingerprints at consecutive positions, at most 32 and within a 32-byte
// lane part, as one record); returns, in lane i, the anchor key of full block i (its last anchor at
// block offset >= 63; ANC_NONE: none).  drop: blocks whose records are not written (bit i: block i
// and the one before it are cached, so every proposal of its anchors falls on an aligned window or in
// the shadow of a predicted REF, which k_aprop skips anyway; the group's anchor record and gaps still
// count them).
__device__ __forceinline__ uint64_t group_anchors(const PlanDev &P, uint32_t g, uint32_t k0, uint32_t len,
                                                  uint32_t n, uint32_t na, const uint8_t *base,
                                                  const uint32_t (&w)[BLK_GROUP][8], uint32_t *tile,
                                                  uint16_t *list, uint32_t abl, uint32_t drop)
{
    const uint32_t l = lane_id();
    uint32_t *prev = tile + 32u * XC_TILE_ROW;
    auto wave_sync = []() {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    };
    // G at positions -32 .. -1 before the group (block 0's lane 0 takes G(p - 32) from there) and
    // at -1 (its G before its first position); a buffer's first group has no anchor below 63
    uint32_t first = 0;
    if (k0 > 0) {
        const uint4 *pp = (const uint4 *)(base + (size_t)k0 * XC_SEG - 64u);
        const uint4 x0 = pp[0], x1 = pp[1], x2 = pp[2], x3 = pp[3];
        const uint32_t lo[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
        const uint32_t hi[8] = {x2.x, x2.y, x2.z, x2.w, x3.x, x3.y, x3.z, x3.w};
        uint32_t gg = gear32(lo), mine = 0;  // G(-33), then G(-32 + t)
#pragma unroll
        for (int t = 0; t < 32; t++) {
            gg = (gg << 1) + ((hi[t >> 2] >> (8 * (t & 3))) & 0xffu);
            mine = l == (uint32_t)t ? gg : mine;
        }
        if (l < 32u) prev[l] = mine;
        first = gg;
    }
    uint32_t cnt = 0;
    uint64_t bkey = ANC_NONE;
    // the group's first and last input anchor and its gaps (anchors >= 1986 apart, group-relative
    // positions: k_aprop's gap windows)
    uint32_t firstp = NONE, lastp = NONE, ngap = 0;
#pragma unroll
    for (uint32_t i = 0; i < BLK_GROUP; i++) {
        if (i >= na) break;
        const uint32_t *wi = w[i];
        const uint32_t sf = gear32(wi);
        const uint32_t gi = gear_prev(sf, first);
        first = readlane(sf, 63);
        if (i > 0) {  // lane 0's G(p - 32): the last lane of the block before
            wave_sync();
            if (l < 32u) prev[l] = tile[l * XC_TILE_ROW + 63u];
            wave_sync();
        }
        const bool keep = !((drop >> i) & 1u);
        // (timing ablations, XC_ABL_BH: 8 = no G tile, 4 = no anchor list / records)
        uint32_t m = (abl & 8u) ? gear_mask<false>(wi, gi, nullptr) : gear_mask<true>(wi, gi, tile);
        if (abl & 12u) {
            if (l == i) bkey = m;  // (keeps the mask live)
            continue;
        }
        // buffer positions p0 + t: anchors need p >= 63 (the context in the buffer) and p < len
        const uint32_t p0 = (k0 + i) * XC_SEG + 32u * l;
        if (p0 < 63u) m &= p0 + 31u >= 63u ? ~0u >> (63u - p0) : 0u;  // bit 31 - t: t >= 63 - p0
        if (p0 + 32u > len) m &= p0 >= len ? 0u : ~(~0u >> (len - p0));  // t < len - p0
        if (!keep) {
            // a block whose records are dropped: only its first and last anchor (the group record)
            // and its key, from the masks and two tile reads (no list, no fingerprints); a block
            // whose anchors may hold a gap inside it takes the full pass below
            const uint64_t lanes = ballot(m != 0u);
            if (!lanes) {
                if (i < n && l == i) bkey = ANC_NONE;
                wave_sync();
                continue;
            }
            const int f = __ffsll((unsigned long long)lanes) - 1, L = 63 - __builtin_clzll(lanes);
            const uint32_t fbk = 32u * (uint32_t)f + (uint32_t)__builtin_clz(readlane(m, f));
            const uint32_t cpk = 32u * (uint32_t)L + 31u - (uint32_t)__builtin_ctz(readlane(m, L));
            if (cpk - fbk < XC_SEG - 62u) {
                const uint32_t gf = i * XC_SEG + fbk;
                if (firstp == NONE) firstp = gf;
                if (lastp != NONE && gf - lastp >= XC_SEG - 62u) {
                    if (l == 0 && ngap < AGAP_CAP) P.agap[g * AGAP_CAP + ngap] = make_uint2(lastp, gf);
                    ngap++;
                }
                lastp = i * XC_SEG + cpk;
                if (i < n) {
                    uint64_t key = ANC_NONE;
                    if (cpk >= 63u) {
                        wave_sync();  // (the gear pass's tile writes of the other lanes)
                        const uint32_t ln = cpk >> 5, t = cpk & 31u;
                        const uint32_t gv = tile[t * XC_TILE_ROW + ln];
                        const uint32_t g2 = ln ? tile[t * XC_TILE_ROW + ln - 1u] : prev[t];
                        key = anc_key(anc_fp(gv, g2), cpk);
                    }
                    if (l == i) bkey = key;
                }
                wave_sync();  // (the next block's tile overwrites this one)
                continue;
            }
        }
        // compaction: every anchor's block offset, in position order, ANC_LIST entries per pass (a
        // random block has ~32 anchors: one pass; a constant run can make every position one)
        const uint32_t k = (uint32_t)__popc(m), incl = wave_incl_scan(k);
        const uint32_t total = readlane(incl, 63);
        uint32_t cp = NONE;  // the previous list entry's offset and fingerprint (uniform)
        uint64_t cfp = 0;
        uint32_t fb = 0;  // the block's first anchor offset (uniform)
        for (uint32_t b0 = 0; b0 < total; b0 += 64u) {
            if (b0 % ANC_LIST == 0u) {  // the list's next pass: entries [b0, b0 + ANC_LIST)
                if (b0) wave_sync();    // (the last pass's readers are done)
                uint32_t o = incl - k, mm = m;
                for (; mm && o < b0 + ANC_LIST; o++) {
                    const uint32_t t = (uint32_t)__builtin_clz(mm);
                    mm &= ~(0x80000000u >> t);
                    if (o >= b0) list[o - b0] = (uint16_t)(32u * l + t);
                }
                wave_sync();
            }
            const uint32_t idx = b0 + l;
            const bool live = idx < total;
            const uint32_t p = live ? list[idx % ANC_LIST] : 0u;
            const uint32_t ln = p >> 5, t = p & 31u;
            const uint32_t gv = tile[t * XC_TILE_ROW + ln];
            const uint32_t g2 = ln ? tile[t * XC_TILE_ROW + ln - 1u] : prev[t];
            const uint64_t fp = anc_fp(gv, g2);
            // a run continues when the entry before has the position before (inside one lane's
            // 32 positions) and the same fingerprint
            // the entry before's position and fingerprint (lane l - 1: a DPP wave shift, no LDS)
            const uint32_t pp = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)p, 0x138, 0xf, 0xf, false);
            const uint32_t fl = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)fp, 0x138, 0xf, 0xf, false);
            const uint32_t fh = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(fp >> 32), 0x138, 0xf, 0xf, false);
            // (a run does not continue across 64 entries: a chunk's first entry is a head)
            const bool cont = live && l != 0u && (p & 31u) != 0u && pp + 1u == p && fl == (uint32_t)fp &&
                              fh == (uint32_t)(fp >> 32);
            if (b0 == 0u) fb = readlane(p, 0);
            const bool head = live && !cont;
            const uint64_t heads = ballot(head);
            const bool runs = ballot(cont) != 0ull;  // (every lane: a ballot inside the branch below sees heads only)
            if (keep) {
                if (head) {
                    // a run's length: up to the next head (without runs, the common case: 1)
                    uint32_t n1 = 1u;
                    if (runs) {
                        const uint64_t above = heads & (l == 63u ? 0ull : ~0ull << (l + 1u));
                        n1 = (above ? b0 + (uint32_t)__builtin_ctzll(above) : min(total, b0 + 64u)) - idx;
                    }
                    const uint32_t ri = cnt + mbcnt(heads);
                    if (ri < REC_CAP) P.rec[(size_t)g * REC_CAP + ri] = rec_make(fp, i * XC_SEG + p, n1);
                }
                cnt += (uint32_t)__popcll(heads);
            }
            const uint32_t last = min(total - b0, 64u) - 1u;
            cp = readlane(p, (int)last);
            cfp = readlane64(fp, (int)last);
        }
        if (total) {  // the group's anchor record (k_aprop's gap windows): anchors >= 1986 apart
            const uint32_t gf = i * XC_SEG + fb;
            if (firstp == NONE) firstp = gf;
            if (lastp != NONE && gf - lastp >= XC_SEG - 62u) {
                if (l == 0 && ngap < AGAP_CAP) P.agap[g * AGAP_CAP + ngap] = make_uint2(lastp, gf);
                ngap++;
            }
            if (cp - fb >= XC_SEG - 62u) {  // (rare: <= 62 anchors, one list pass, still in LDS)
                const uint32_t p = l < total ? list[l] : 0u;
                const uint32_t pp = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(4u * ((l + 63u) & 63u)), (int)p);
                for (uint64_t gm = ballot(l > 0u && l < total && p - pp >= XC_SEG - 62u); gm; gm &= gm - 1) {
                    const int f = __ffsll((unsigned long long)gm) - 1;
                    const uint32_t x = i * XC_SEG + readlane(pp, f), y = i * XC_SEG + readlane(p, f);
                    if (l == 0 && ngap < AGAP_CAP) P.agap[g * AGAP_CAP + ngap] = make_uint2(x, y);
                    ngap++;
                }
            }
            lastp = i * XC_SEG + cp;
        }
        if (i < n) {  // the block's anchor: its last one at offset >= 63 (none: block_predict and
                      // the emit take a later level's, seg_key_serial / wave_seg_anchor)
            const uint64_t key = total && cp >= 63u ? anc_key(cfp, cp) : ANC_NONE;
            if (l == i) bkey = key;
        }
        wave_sync();  // (the next block's tile and list overwrite these)
    }
    if (l == 0) {
        // REC_GAP: a gap (>= 1985 positions without an anchor) may touch this group: one inside it,
        // none at all, or 993 positions without one at its start or its end (a gap across the
        // boundary has that on one side at least); k_aprop reads the record of such groups only
        const uint32_t span = min(len - k0 * XC_SEG, na * XC_SEG);
        const bool chk = ngap || lastp == NONE || firstp >= 993u || span - 1u - lastp >= 993u;
        P.ainfo[g] = make_uint4(firstp, lastp, ngap, chk ? 1u : 0u);
        P.rec_cnt[g] = (cnt <= REC_CAP ? cnt : (REC_OVF | REC_CAP)) | (chk ? REC_GAP : 0u);
    }
    return bkey;
}

// predict: also the predictions of these blocks (the run's first sub-batch, hashed in line after
// the declaration set's clear: one kernel instead of two).  ANC: the group's anchors too (a run in
// anchor mode); groups then also cover a buffer's partial last block.
// (LDS 38 KB and <= 128 VGPRs: four workgroups, 16 waves, per CU; with a whole block's list, 49
// KB and 3 waves per SIMD, the side-stream hashing hid less of its latency: cfg5 A/B +2.3 %)
template <bool PREDICT, bool ANC>
__global__ __launch_bounds__(256, 4) void k_blockhash(DeclArgs a)
{
    __shared__ uint32_t tiles[ANC ? 4 : 1][ANC ? 32 * XC_TILE_ROW + 32 : 1];
    __shared__ uint16_t lists[ANC ? 4 : 1][ANC ? ANC_LIST : 1];
    const PlanDev &P = a.P;
    const uint32_t g = a.j0 + blockIdx.x * 4u + (threadIdx.x >> 6);
    if (g >= a.j1) return;
    const uint2 gr = P.blk_grp[g];
    const uint32_t b = gr.x, k0 = gr.y;
    const uint32_t len = P.buf_len[b];
    const uint8_t *base = P.in + P.buf_off[b];
    const uint32_t nfull = len / XC_SEG;
    const uint32_t n = nfull > k0 ? min(BLK_GROUP, nfull - k0) : 0u;
    const uint32_t na = ANC ? min(BLK_GROUP, (len + XC_SEG - 1u) / XC_SEG - k0) : n;
    uint32_t w[BLK_GROUP][8];  // (kept for the compares below)
    wave_load_blocks<BLK_GROUP>(base + (size_t)k0 * XC_SEG, na, w);
    const uint64_t h = block_group_hash<BLK_GROUP>(w);
    const uint32_t l = lane_id();
    const uint32_t gi = P.blk_base[b] + k0 + l;
    uint32_t cmp = 0;  // the cached slot + 1 to compare the block with (blk_cmp)
    if (!PREDICT && l < n && a.limit && !stream_carried(P, b)) {
        // (a concurrent k_alloc may be entering keys: only complete entries are compared)
        uint64_t v;
        if (set_find(P.cache, h, &v) && (uint32_t)v < min(*a.limit, a.limit_cap)) cmp = (uint32_t)v + 1u;
    }
    // blocks cached with the block before them cached too (entries complete at the run's start are
    // also found by k_blockpredict: these blocks are predicted REFs after a predicted REF)
    uint32_t drop = 0;
    if (ANC && !PREDICT && a.drop_shadowed) {
        const uint32_t m = (uint32_t)ballot(cmp != 0u);
        drop = m & (m << 1);
    }
    uint64_t akey = ANC_NONE;
    // XC_ABL_BH (timing ablations only: the results are wrong; in builds with -DXC_ABLATIONS=1):
    // 2 = no anchors at all
    const uint32_t abl = XC_ABLATIONS ? (uint32_t)a.nt : 0u;
    if (ANC && !(abl & 2u))
        akey = group_anchors(P, g, k0, len, n, na, base, w, tiles[(threadIdx.x >> 6) & (ANC ? 3 : 0)],
                             lists[(threadIdx.x >> 6) & (ANC ? 3 : 0)], abl, drop);
    if (l < n) {
        P.blk_h[gi] = h;
        if (ANC) P.blk_anc[gi] = akey;
        if (PREDICT) {
            const uint32_t pref = block_predict(P, gi, b, k0 + l, h, akey);
            if (blk_cached(pref)) cmp = pref;
        }
    }
    // the compares of a predicted REF's bytes, off k_resolve's critical path, against the block
    // words still in registers: four blocks per pass, their segments' loads all in flight
    uint32_t verdict = cmp;
    if (ballot(cmp != 0u)) {
#pragma unroll
        for (int g0 = 0; g0 < (int)BLK_GROUP; g0 += 4) {
            uint4 y[4][2];
            uint32_t slot[4];
#pragma unroll
            for (int i = 0; i < 4; i++) {
                slot[i] = readlane(cmp, g0 + i);
                if (slot[i]) {
                    const uint4 *yp = (const uint4 *)(seg_at(P.segs, slot[i] - 1u) + 32u * l);
                    y[i][0] = yp[0];
                    y[i][1] = yp[1];
                }
            }
#pragma unroll
            for (int i = 0; i < 4; i++) {
                if (!slot[i]) continue;
                const uint32_t *x = w[g0 + i];
                const uint32_t diff = (x[0] ^ y[i][0].x) | (x[1] ^ y[i][0].y) | (x[2] ^ y[i][0].z) | (x[3] ^ y[i][0].w) |
                                      (x[4] ^ y[i][1].x) | (x[5] ^ y[i][1].y) | (x[6] ^ y[i][1].z) | (x[7] ^ y[i][1].w);
                if (ballot(diff != 0u) && (int)l == g0 + i) verdict |= BC_DIFF;
            }
        }
    }
    if (l < n) P.blk_cmp[gi] = verdict;
}
template __global__ void k_blockhash<false, false>(DeclArgs);
template __global__ void k_blockhash<true, false>(DeclArgs);
template __global__ void k_blockhash<false, true>(DeclArgs);
template __global__ void k_blockhash<true, true>(DeclArgs);

// One lane per aligned block of buffers [j0, j1) (P.blk_buf maps a block to its buffer).
__global__ __launch_bounds__(256) void k_blockpredict(DeclArgs a)
{
    if (aborted(a.P)) return;
    const PlanDev &P = a.P;
    const uint32_t g = P.blk_base[a.j0] + blockIdx.x * 256u + threadIdx.x;
    if (g >= P.blk_base[a.j1]) return;
    const uint32_t b = P.blk_buf[g], k = g - P.blk_base[b];
    // a block the hashing found cached (an entry complete then, under the removal floor: still
    // there, at the same segment index) is a predicted REF without another probe of the cache
    const uint32_t cmp = P.blk_cmp[g] & ~BC_DIFF;
    if (cmp && !stream_carried(P, b)) {
        P.blk_pref[g] = cmp;
        return;
    }
    block_predict(P, g, b, k, P.blk_h[g], P.anc_scan ? P.blk_anc[g] : ANC_NONE);
}

__device__ __forceinline__ uint32_t block_predict(const PlanDev &P, uint32_t g, uint32_t b, uint32_t k, uint64_t h,
                                                  uint64_t akey)
{
    uint32_t pref = 0u;  // blocks relative to a carried source_: no predictions
    uint64_t v;
    if (stream_carried(P, b)) {
    } else if (set_find(P.cache, h, &v)) {
        pref = (uint32_t)v + 1u;  // (cache capacity <= 2^28: bit 31 stays free)
    } else {
        uint32_t slot;
        const uint64_t val = ((uint64_t)b << 32) | (k * XC_SEG + 2u * XC_SEG - 1u);
        if (P.anc_scan) {
            // an anchor-scanned sub-batch reads the set's keys and values only (k_aprop proposes
            // through the anchor table, k_resolve and k_walk look keys up); its filters and lo32
            // keys serve the exact scan, which a redo of the sub-batch runs after clearing the set
            set_insert_kv(P.dset, h, val, &slot);
        } else {
            // (the set's level-2 filter is P.l2mix, the combined filter the scan reads)
            set_insert(P.dset, h, val, true, &slot, nullptr);
            const uint32_t lo = (uint32_t)h;  // (the combined level-1 image the first scan loads)
            atomicOr(&P.fmix[filt_word_n(lo, XC_FILT_WORDS >> P.fmix_fold)], filt_mask(lo));
        }
        if (P.anc_scan) {
            // the anchor scan finds windows equal to this block through its anchor (a block
            // without a level-0 anchor: a later level's, found through the gap windows)
            if (akey == ANC_NONE) akey = seg_key_serial(P.in + P.buf_off[b] + (size_t)k * XC_SEG);
            if (akey == ANC_NONE) atomicOr(&P.ctl[CTL_AFAIL], 1u);
            else anc_insert(P.danc, akey);
        }
        pref = BP_DECL | slot;
    }
    P.blk_pref[g] = pref;
    return pref;
}

// -------------------------------------------------------------- k_emit ------------------
// One workgroup (4 waves) per buffer in [j0, j1): token sizes, offsets, wire bytes; every
// EXTRACT payload is entered in the cache (xcodec_encoder.cc:203-215).

constexpr uint32_t MAX_TOK = 2u * (MAX_BUF / XC_SEG) + 3u;

__device__ __forceinline__ uint32_t count_magic(const uint8_t *p, uint32_t n)
{
    uint32_t c = 0;
    for (uint32_t o = 4u * lane_id(); o < n; o += 256u) {
#pragma unroll
        for (uint32_t k = 0; k < 4; k++)
            if (o + k < n) c += p[o + k] == XC_MAGIC ? 1u : 0u;
    }
    return wave_sum(c);
}

// encode_escape (xcodec_encoder.cc:217-239): bytes, with F1 -> F1 00.  Returns bytes written.
__device__ __forceinline__ uint32_t write_escaped(uint8_t *dst, const uint8_t *p, uint32_t n)
{
    uint32_t o = 0;
    for (uint32_t x = 0; x < n; x += 256u) {
        const uint32_t s = x + 4u * lane_id();
        uint32_t v[4], cnt = 0;
#pragma unroll
        for (uint32_t k = 0; k < 4; k++) {
            v[k] = (s + k < n) ? p[s + k] : 0x100u;
            cnt += v[k] == 0x100u ? 0u : (v[k] == XC_MAGIC ? 2u : 1u);
        }
        const uint32_t inc = wave_incl_scan(cnt);
        uint32_t q = o + inc - cnt;
#pragma unroll
        for (uint32_t k = 0; k < 4; k++) {
            if (v[k] == 0x100u) continue;
            dst[q++] = (uint8_t)v[k];
            if (v[k] == XC_MAGIC) dst[q++] = 0;
        }
        o += readlane(inc, 63);
    }
    return o;
}


// Payloads a wave has in flight: 4 since the emit compiles without the anchor path and keeps 32 bytes
// per lane per payload (78 VGPRs; 2 before: cfg5 864 -> 876 GiB/s, cfg3 711 -> 717, one box,
// profiles/r06/ab/emit_pay_r6i.txt; round 3 measured 4 slower when the kernel had 84 VGPRs at 2)
#ifndef XC_EMIT_PAY
#define XC_EMIT_PAY 4
#endif
constexpr int EMIT_PAY = XC_EMIT_PAY;

// k_alloc's gate (a sub-batch that needs the host stops the device pipeline here).
__device__ __forceinline__ bool gate_stop(const EmitArgs &a)
{
    const uint32_t *ctl = a.P.ctl;
    return a.gate_sb != NONE &&
           (ctl[CTL_GREW] || ctl[CTL_SHADOW] || ctl[CTL_FIRST_CROSS] < a.j1 || ctl[CTL_ERROR] || ctl[CTL_AFAIL]);
}

__device__ __forceinline__ void gate_abort(const EmitArgs &a)
{
    a.P.ctl[CTL_ABORT_SB] = a.gate_sb;
    __threadfence();  // (an emit on its own stream reads the sub-batch after seeing the flag)
    a.P.ctl[CTL_ABORT] = 1u;
}

// The emit's stop: a pass stopped at this sub-batch or before it.  (An emit on its own stream may
// run after a later sub-batch's gate stopped the pass: its own sub-batch passed its gate, and its
// bytes are due.)
__device__ __forceinline__ bool emit_aborted(const EmitArgs &a)
{
    if (!aborted(a.P)) return false;
    if (a.gate_sb == NONE) return true;
    const uint32_t sb = __builtin_amdgcn_readfirstlane(
        (int)__atomic_load_n((const uint32_t *)&a.P.ctl[CTL_ABORT_SB], __ATOMIC_ACQUIRE));
    return sb <= a.gate_sb;
}

// The control words to the caller's mapped host buffer (one thread).
__device__ __forceinline__ void ctl_publish(const EmitArgs &a)
{
    if (!a.ctl_host) return;
    __threadfence();
    for (uint32_t i = 0; i + 1u < CTL_WORDS; i++) a.ctl_host[i] = __atomic_load_n(&a.P.ctl[i], __ATOMIC_RELAXED);
    // the last word (unused: 0) clears the host's sentinel only after the others are visible
    __threadfence_system();
    a.ctl_host[CTL_WORDS - 1] = __atomic_load_n(&a.P.ctl[CTL_WORDS - 1], __ATOMIC_RELAXED);
    __threadfence_system();
}

// XCodecMemoryCache::enter (xcodec_cache.h:182-188) of the EXTRACT token t of buffer b (ext) into
// cache slot idx, one lane per token, the whole wave present: the hash tables (undo record) and, on
// an anchor run, the anchor index (an aligned block's key from k_blockhash, any other segment's
// computed here, wave-wide, one at a time).
template <bool ANC>
__device__ __forceinline__ void enter_tokens(const PlanDev &P, uint32_t b, const uint8_t *base, uint32_t tb,
                                             uint32_t t, bool ext, uint32_t idx)
{
    const uint32_t l = lane_id();
    if (ANC && P.anc_run) {
        const uint32_t sg = ext ? P.tok_seg[tb + t] : 0u;
        uint64_t key = ext && (sg & (XC_SEG - 1u)) == 0u ? P.blk_anc[P.blk_base[b] + sg / XC_SEG] : ANC_NONE;
        // (an aligned block without a level-0 anchor too: its key of a later level)
        for (uint64_t m = ballot(ext && key == ANC_NONE); m; m &= m - 1) {
            const int f = __ffsll((unsigned long long)m) - 1;
            uint32_t wv[8];
            load32_window(base + readlane(sg, f) + 32u * l, wv);
            const uint64_t k2 = wave_seg_anchor(wv);
            if ((int)l == f) key = k2;
        }
        if (ext && idx < P.seg_cap) {
            P.anc_of[idx] = key;
            if (key != ANC_NONE) {
                P.aundo[idx] = anc_insert(P.canc, key);
            } else {
                P.aundo[idx] = NONE;
                atomicMax(P.anc_bad, ~idx);
            }
        }
    }
    if (ext && idx < P.seg_cap) {
        uint32_t s1, s2;
        if (set_insert(P.cache, P.tok_h[tb + t], idx, false, &s1, &s2) || s2 == XC_REVIVED) {
            P.undo[idx] = make_uint2(s1, s2);
        } else {
            // the hash is in the cache: a stateful stream's carried candidate declared after another
            // connection entered the hash (xc_memcache.cpp).  The table keeps the first entry
            // (nothing to undo); the host replays the run.
            P.undo[idx] = make_uint2(NONE, NONE);
            atomicAdd(&P.ctl[CTL_DUPS], 1u);
        }
    }
}

// The cache enters of buffers [j0, j1) (a sub-batch without in-emit slots), one wave per buffer, so
// that every insert of the sub-batch is in flight at once instead of on one wave of each emit
// workgroup (the emit's critical path): after k_alloc (its slots), before k_emit.
// ANC: the run indexes anchors (a run on the exact scan compiles without that path: 22 VGPRs, not 86)
template <bool ANC>
__global__ __launch_bounds__(256) void k_insert(EmitArgs a)
{
    if (aborted(a.P)) return;
    const PlanDev &P = a.P;
    const uint32_t b = a.j0 + blockIdx.x * 4u + (threadIdx.x >> 6);
    if (b >= a.j1) return;
    const uint32_t l = lane_id();
    const uint8_t *base = P.in + P.buf_off[b];
    const uint32_t tb = P.tok_base[b], n = min(P.tok_cnt[b], MAX_TOK);
    const uint32_t slot0 = P.buf_slot[b];
    uint32_t carry = 0;  // EXTRACT tokens before this chunk
    for (uint32_t t0 = 0; t0 < n; t0 += 64u) {
        const uint32_t t = t0 + l;
        const bool ext = t < n && P.tok_op[tb + t] == OP_EXTRACT;
        const uint64_t em = ballot(ext);
        enter_tokens<ANC>(P, b, base, tb, t, ext, slot0 + carry + mbcnt(em));
        carry += (uint32_t)__popcll(em);
    }
}
template __global__ void k_insert<false>(EmitArgs);
template __global__ void k_insert<true>(EmitArgs);

// SLOTS: k_alloc's work too (sub-batches of <= EMIT_SLOTS_MAX buffers), with no extra round trip
// on a workgroup's path: the gate words, the sub-batch's start count (P.sb_count, written by
// k_clear_set: the cache count does not change before this kernel) and every buffer's buf_next /
// buf_nref are loaded with the token metadata; this buffer's first slot is the start count plus
// the buf_next of the buffers before it, and workgroup 0 publishes the totals.
// INS: the cache enters in this kernel (0: none, k_insert ran before it; 1: enters; 2: enters and
// anchor keys).  The anchor path alone takes the kernel from 54 to 84 VGPRs (5 instead of 8
// workgroups of 4 waves per CU), so each launch compiles only what its run needs.
template <uint32_t EMIT_WAVES, bool SLOTS, int INS>
__global__ __launch_bounds__(64 * EMIT_WAVES) void k_emit(EmitArgs a)
{
    if (emit_aborted(a)) return;
    const uint32_t eabl = XC_ABLATIONS ? a.abl : 0u;  // (XC_ABL_EMIT timing ablations: -DXC_ABLATIONS=1 builds)
    __shared__ uint32_t sz[MAX_TOK];
    __shared__ uint32_t ord[MAX_TOK];
    __shared__ uint4 red[EMIT_WAVES];
    const PlanDev &P = a.P;
    const uint32_t b = a.j0 + blockIdx.x;
    if (b >= a.j1) return;
    const uint32_t wave = threadIdx.x >> 6, l = lane_id();
    uint32_t s_pre = 0, s_tot = 0, s_ref = 0, s_stop = 0, s_base = 0;
    if (SLOTS) {
        for (uint32_t i = a.j0 + threadIdx.x; i < a.j1; i += 64u * EMIT_WAVES) {
            const uint32_t v = P.buf_next[i];
            s_tot += v;
            s_ref += P.buf_nref[i];
            if (i < b) s_pre += v;
        }
        if (threadIdx.x == 0) {
            s_stop = gate_stop(a) ? 1u : 0u;
            s_base = *a.base;
        }
    }
    const uint8_t *base = P.in + P.buf_off[b];
    uint8_t *out = P.out + P.out_off[b];
    const uint32_t tb = P.tok_base[b], n = min(P.tok_cnt[b], MAX_TOK);

    // token sizes: escaped literal run + op bytes; EXTRACT ordinals for the cache slots
    for (uint32_t t0 = wave * 64u; t0 < n; t0 += 64u * EMIT_WAVES) {
        const uint32_t t = t0 + l;
        uint32_t lb = 0, le = 0, op = OP_END;
        if (t < n) { lb = P.tok_lb[tb + t]; le = P.tok_le[tb + t]; op = P.tok_op[tb + t]; }
        uint32_t esc = le - lb;
        if (ballot(le > lb)) {  // count F1 bytes of non-empty literal runs, one run at a time
            uint64_t m = ballot(le > lb);
            while (m) {
                const int f = __ffsll((unsigned long long)m) - 1;
                m &= m - 1;
                const uint32_t flb = readlane(lb, f), fle = readlane(le, f);
                const uint32_t c = count_magic(base + flb, fle - flb);
                if ((int)l == f) esc += c;
            }
        }
        if (t < n) {
            sz[t] = esc + (op == OP_EXTRACT ? 2u + XC_SEG : op == OP_REF ? 10u : 0u);
            ord[t] = op == OP_EXTRACT ? 1u : 0u;
        }
    }
    if (SLOTS) {
        const uint32_t x = wave_sum(s_pre), y = wave_sum(s_tot), z = wave_sum(s_ref);
        if (l == 0) red[wave] = make_uint4(x, y, z, wave == 0 ? (s_stop | (s_base << 1)) : 0u);
    }
    __syncthreads();
    if (SLOTS) {
        uint4 t = make_uint4(0, 0, 0, 0);
        for (uint32_t k = 0; k < EMIT_WAVES; k++) {
            t.x += red[k].x;
            t.y += red[k].y;
            t.z += red[k].z;
        }
        if (red[0].w & 1u) {  // the gate: every workgroup decides the same
            if (blockIdx.x == 0 && threadIdx.x == 0) {
                gate_abort(a);
                ctl_publish(a);
            }
            return;
        }
        s_base = red[0].w >> 1;
        s_pre = t.x;
        if (blockIdx.x == 0 && threadIdx.x == 0) {
            const uint32_t count = s_base + t.y;
            *P.seg_count = count;
            P.ctl[CTL_COUNT] = count;
            P.ctl[CTL_NEXTRACT] += t.y;
            P.ctl[CTL_NREF] += t.z;
            if (count > P.seg_cap) P.ctl[CTL_ERROR] |= ERR_CAPACITY;
            if (a.pub_final) ctl_publish(a);
        }
    }
    if (wave == 0) {
        uint32_t carry = 0, ocarry = 0;
        for (uint32_t t0 = 0; t0 < n; t0 += 64u) {
            const uint32_t t = t0 + l;
            const uint32_t v = t < n ? sz[t] : 0u, o = t < n ? ord[t] : 0u;
            const uint32_t inc = wave_incl_scan(v), oinc = wave_incl_scan(o);
            if (t < n) { sz[t] = carry + inc - v; ord[t] = ocarry + oinc - o; }
            carry += readlane(inc, 63);
            ocarry += readlane(oinc, 63);
        }
        if (l == 0) P.out_len[b] = carry;
    }
    __syncthreads();
    const uint32_t slot0 = SLOTS ? s_base + s_pre : P.buf_slot[b];
    if (SLOTS && threadIdx.x == 0) P.buf_slot[b] = slot0;  // (the tail check's visibility test)
    // XCodecMemoryCache::enter of this buffer's declarations (SLOTS, or k_insert not split off): the
    // wave with the smallest token group (wave 0 did the prefix), one lane per EXTRACT token
    if (INS && wave == EMIT_WAVES - 1u && !(eabl & 4u)) {
        for (uint32_t t0 = 0; t0 < n; t0 += 64u) {
            const uint32_t t = t0 + l;
            const bool ext = t < n && P.tok_op[tb + t] == OP_EXTRACT;
            enter_tokens<INS == 2>(P, b, base, tb, t, ext, ext ? slot0 + ord[t] : 0u);
        }
    }
    // wire bytes: wave w takes a contiguous group of tokens, one per lane, so the group's
    // metadata arrives in one round trip and two payloads are in flight at a time
    const uint32_t G = (n + EMIT_WAVES - 1u) / EMIT_WAVES;
    const uint32_t g_end = min(n, (wave + 1u) * G);
    for (uint32_t g0 = wave * G; g0 < g_end; g0 += 64u) {
        const uint32_t t = g0 + l;
        const bool live = t < g_end;
        uint32_t lb = 0, le = 0, op = OP_END, seg = 0, off = 0;
        uint64_t h = 0;
        if (live) {
            lb = P.tok_lb[tb + t];
            le = P.tok_le[tb + t];
            op = P.tok_op[tb + t];
            seg = P.tok_seg[tb + t];
            h = P.tok_h[tb + t];
            off = sz[t];
        }
        // literal runs, F1-escaped (wave-cooperative, one run at a time)
        for (uint64_t m = ballot(live && le > lb); m; m &= m - 1) {
            const int f = __ffsll((unsigned long long)m) - 1;
            const uint32_t flb = readlane(lb, f);
            const uint32_t len = write_escaped(out + readlane(off, f), base + flb, readlane(le, f) - flb);
            if ((int)l == f) off += len;
        }
        uint8_t *o = out + off;
        if (live && op == OP_REF) {
            o[0] = (uint8_t)XC_MAGIC;
            o[1] = (uint8_t)OP_REF;
#pragma unroll
            for (int k = 0; k < 8; k++) o[2 + k] = (uint8_t)(h >> (8 * (7 - k)));
        } else if (live && op == OP_EXTRACT) {
            o[0] = (uint8_t)XC_MAGIC;
            o[1] = (uint8_t)OP_EXTRACT;
        }
        // payloads to the wire and into the slots k_alloc reserved, EMIT_PAY at a time
        for (uint64_t m = ballot(live && op == OP_EXTRACT && !(eabl & 8u)); m;) {
            int f[EMIT_PAY];
            uint32_t ii[EMIT_PAY];
            uint8_t *d[EMIT_PAY];
            PayloadRegs r[EMIT_PAY];
#pragma unroll
            for (int g = 0; g < EMIT_PAY; g++) {
                f[g] = m ? __ffsll((unsigned long long)m) - 1 : -1;
                if (m) m &= m - 1;
                if (f[g] >= 0) {
                    ii[g] = slot0 + ord[g0 + (uint32_t)f[g]];
                    d[g] = out + readlane(off, f[g]) + 2u;
                    payload_load(base + readlane(seg, f[g]), d[g], r[g]);
                }
            }
#pragma unroll
            for (int g = 0; g < EMIT_PAY; g++)
                if (f[g] >= 0) {
                    uint8_t *sg = ii[g] < P.seg_cap && !(eabl & 1u) ? seg_at(P.segs, ii[g]) : nullptr;
                    if (eabl & 2u) {
                        if (sg) payload_store_seg(sg, r[g]);
                    } else {
                        payload_store(d[g], sg, r[g]);
                    }
                }
        }
    }
}

// The wire bytes of a wave's token group (one token per lane, `live`): F1-escaped literal runs from
// off (the token's wire offset), the op bytes, then the EXTRACT payloads to the wire and into their
// cache slots (the lane's `slot`), EMIT_PAY at a time.
__device__ __forceinline__ void emit_group(const PlanDev &P, uint8_t *out, const uint8_t *base, bool live, uint32_t lb,
                                           uint32_t le, uint32_t op, uint32_t seg, uint64_t h, uint32_t off,
                                           uint32_t slot, uint32_t eabl)
{
    const uint32_t l = lane_id();
    // literal runs, F1-escaped (wave-cooperative, one run at a time)
    for (uint64_t m = ballot(live && le > lb); m; m &= m - 1) {
        const int f = __ffsll((unsigned long long)m) - 1;
        const uint32_t flb = readlane(lb, f);
        const uint32_t len = write_escaped(out + readlane(off, f), base + flb, readlane(le, f) - flb);
        if ((int)l == f) off += len;
    }
    uint8_t *o = out + off;
    if (live && op == OP_REF) {
        o[0] = (uint8_t)XC_MAGIC;
        o[1] = (uint8_t)OP_REF;
#pragma unroll
        for (int k = 0; k < 8; k++) o[2 + k] = (uint8_t)(h >> (8 * (7 - k)));
    } else if (live && op == OP_EXTRACT) {
        o[0] = (uint8_t)XC_MAGIC;
        o[1] = (uint8_t)OP_EXTRACT;
    }
    // payloads to the wire and into the slots k_alloc reserved, EMIT_PAY at a time
    for (uint64_t m = ballot(live && op == OP_EXTRACT && !(eabl & 8u)); m;) {
        int f[EMIT_PAY];
        uint32_t ii[EMIT_PAY];
        uint8_t *d[EMIT_PAY];
        PayloadRegs r[EMIT_PAY];
#pragma unroll
        for (int g = 0; g < EMIT_PAY; g++) {
            f[g] = m ? __ffsll((unsigned long long)m) - 1 : -1;
            if (m) m &= m - 1;
            if (f[g] >= 0) {
                ii[g] = readlane(slot, f[g]);
                d[g] = out + readlane(off, f[g]) + 2u;
                payload_load(base + readlane(seg, f[g]), d[g], r[g]);
            }
        }
#pragma unroll
        for (int g = 0; g < EMIT_PAY; g++)
            if (f[g] >= 0) {
                uint8_t *sg = ii[g] < P.seg_cap && !(eabl & 1u) ? seg_at(P.segs, ii[g]) : nullptr;
                if (eabl & 2u) {
                    if (sg) payload_store_seg(sg, r[g]);
                } else {
                    payload_store(d[g], sg, r[g]);
                }
            }
    }
}

// k_emit's one-pass form, for plans whose buffers have at most 64 tokens per wave (the host's bound
// 2 len / 2048 + 3; every 64 KiB proxy read): wave w loads its contiguous token group once, sizes it
// (escaped literals + op bytes), scans it in registers, and after one barrier (the group totals and
// EXTRACT counts of the waves before it) enters its declarations and writes its bytes.  SLOTS / INS as
// for k_emit.
template <uint32_t EMIT_WAVES, bool SLOTS, int INS>
__global__ __launch_bounds__(64 * EMIT_WAVES) void k_emit1(EmitArgs a)
{
    if (emit_aborted(a)) return;
    const uint32_t eabl = XC_ABLATIONS ? a.abl : 0u;  // (XC_ABL_EMIT timing ablations: -DXC_ABLATIONS=1 builds)
    __shared__ uint4 red[EMIT_WAVES];
    __shared__ uint2 grp[EMIT_WAVES];  // (one pass: each wave's wire bytes and EXTRACT tokens)
    const PlanDev &P = a.P;
    const uint32_t b = a.j0 + blockIdx.x;
    if (b >= a.j1) return;
    const uint32_t wave = threadIdx.x >> 6, l = lane_id();
    uint32_t s_pre = 0, s_tot = 0, s_ref = 0, s_stop = 0, s_base = 0;
    if (SLOTS) {
        for (uint32_t i = a.j0 + threadIdx.x; i < a.j1; i += 64u * EMIT_WAVES) {
            const uint32_t v = P.buf_next[i];
            s_tot += v;
            s_ref += P.buf_nref[i];
            if (i < b) s_pre += v;
        }
        if (threadIdx.x == 0) {
            s_stop = gate_stop(a) ? 1u : 0u;
            s_base = *a.base;
        }
    }
    const uint8_t *base = P.in + P.buf_off[b];
    uint8_t *out = P.out + P.out_off[b];
    const uint32_t tb = P.tok_base[b], n = min(P.tok_cnt[b], MAX_TOK);
    const uint32_t G = (n + EMIT_WAVES - 1u) / EMIT_WAVES;
    const uint32_t g_end = min(n, (wave + 1u) * G);

    // this lane's token of the wave's group, kept in registers to the end
    uint32_t lb = 0, le = 0, op = OP_END, seg = 0;
    uint64_t h = 0;
    const uint32_t t = wave * G + l;
    const bool live = t < g_end;
    if (live) {
        lb = P.tok_lb[tb + t];
        le = P.tok_le[tb + t];
        op = P.tok_op[tb + t];
        seg = P.tok_seg[tb + t];
        h = P.tok_h[tb + t];
    }
    uint32_t esc = le - lb;
    for (uint64_t m = ballot(le > lb); m; m &= m - 1) {  // F1 bytes of non-empty literal runs
        const int f = __ffsll((unsigned long long)m) - 1;
        const uint32_t flb = readlane(lb, f), fle = readlane(le, f);
        const uint32_t c = count_magic(base + flb, fle - flb);
        if ((int)l == f) esc += c;
    }
    const uint32_t tsz = live ? esc + (op == OP_EXTRACT ? 2u + XC_SEG : op == OP_REF ? 10u : 0u) : 0u;
    const uint32_t inc = wave_incl_scan(tsz);
    const uint32_t nx = (uint32_t)__popcll(ballot(live && op == OP_EXTRACT));
    const uint32_t tot = readlane(inc, 63);
    if (l == 0) grp[wave] = make_uint2(tot, nx);
    if (SLOTS) {
        const uint32_t x = wave_sum(s_pre), y = wave_sum(s_tot), z = wave_sum(s_ref);
        if (l == 0) red[wave] = make_uint4(x, y, z, wave == 0 ? (s_stop | (s_base << 1)) : 0u);
    }
    __syncthreads();
    if (SLOTS) {
        uint4 t = make_uint4(0, 0, 0, 0);
        for (uint32_t k = 0; k < EMIT_WAVES; k++) {
            t.x += red[k].x;
            t.y += red[k].y;
            t.z += red[k].z;
        }
        if (red[0].w & 1u) {  // the gate: every workgroup decides the same
            if (blockIdx.x == 0 && threadIdx.x == 0) {
                gate_abort(a);
                ctl_publish(a);
            }
            return;
        }
        s_base = red[0].w >> 1;
        s_pre = t.x;
        if (blockIdx.x == 0 && threadIdx.x == 0) {
            const uint32_t count = s_base + t.y;
            *P.seg_count = count;
            P.ctl[CTL_COUNT] = count;
            P.ctl[CTL_NEXTRACT] += t.y;
            P.ctl[CTL_NREF] += t.z;
            if (count > P.seg_cap) P.ctl[CTL_ERROR] |= ERR_CAPACITY;
            if (a.pub_final) ctl_publish(a);
        }
    }
    const uint32_t slot0 = SLOTS ? s_base + s_pre : P.buf_slot[b];
    if (SLOTS && threadIdx.x == 0) P.buf_slot[b] = slot0;  // (the tail check's visibility test)
    uint32_t off = inc - tsz, xo = 0, total = 0;
    for (uint32_t k = 0; k < EMIT_WAVES; k++) {
        const uint2 gk = grp[k];
        total += gk.x;
        if (k < wave) {
            off += gk.x;
            xo += gk.y;
        }
    }
    if (threadIdx.x == 0) P.out_len[b] = total;
    const bool ext = live && op == OP_EXTRACT;
    const uint32_t slot = slot0 + xo + mbcnt(ballot(ext));
    // XCodecMemoryCache::enter of the group's declarations (xcodec_cache.h:182-188), every wave its own
    if (INS && !(eabl & 4u)) enter_tokens<INS == 2>(P, b, base, tb, wave * G + l, ext, ext ? slot : 0u);
    emit_group(P, out, base, live, lb, le, op, seg, h, off, slot, eabl);
}

template __global__ void k_emit<4, false, 0>(EmitArgs);
template __global__ void k_emit<16, false, 0>(EmitArgs);
template __global__ void k_emit<4, false, 1>(EmitArgs);
template __global__ void k_emit<16, false, 1>(EmitArgs);
template __global__ void k_emit<4, false, 2>(EmitArgs);
template __global__ void k_emit<16, false, 2>(EmitArgs);
template __global__ void k_emit<4, true, 1>(EmitArgs);
template __global__ void k_emit<16, true, 1>(EmitArgs);
template __global__ void k_emit<4, true, 2>(EmitArgs);
template __global__ void k_emit<16, true, 2>(EmitArgs);
template __global__ void k_emit1<4, false, 0>(EmitArgs);
template __global__ void k_emit1<4, false, 1>(EmitArgs);
template __global__ void k_emit1<4, false, 2>(EmitArgs);
template __global__ void k_emit1<4, true, 1>(EmitArgs);
template __global__ void k_emit1<4, true, 2>(EmitArgs);

// One workgroup: cache slots for the declarations of buffers [j0, j1) in buffer order
// (exclusive prefix of buf_next on top of the current segment count), plus run totals.
__global__ __launch_bounds__(1024) void k_alloc(EmitArgs a)
{
    if (aborted(a.P)) return;
    if (a.gate_sb != NONE) {
        // async pipeline gate: stop here (and every later launch) if sub-batch gate_sb needs
        // the host: declaration growth, a missed REF shadow, a cross-buffer conflict or an error
        __shared__ uint32_t stop;
        if (threadIdx.x == 0) {
            stop = gate_stop(a) ? 1u : 0u;
            if (stop) {
                gate_abort(a);
                ctl_publish(a);
            }
        }
        __syncthreads();
        if (stop) return;
    }
    __shared__ uint32_t wsum[16][2];
    __shared__ uint32_t carry[2];
    const PlanDev &P = a.P;
    const uint32_t wave = threadIdx.x >> 6, l = lane_id();
    if (threadIdx.x == 0) { carry[0] = *P.seg_count; carry[1] = 0; }
    __syncthreads();
    const uint32_t start = carry[0];
    uint32_t nref_tot = 0;
    for (uint32_t b0 = a.j0; b0 < a.j1; b0 += 1024u) {
        const uint32_t b = b0 + threadIdx.x;
        const uint32_t v = b < a.j1 ? P.buf_next[b] : 0u;
        const uint32_t r = b < a.j1 ? P.buf_nref[b] : 0u;
        const uint32_t inc = wave_incl_scan(v);
        const uint32_t rs = wave_sum(r);
        if (l == 63) { wsum[wave][0] = inc; wsum[wave][1] = rs; }
        __syncthreads();
        uint32_t off = carry[0];
        for (uint32_t k = 0; k < wave; k++) off += wsum[k][0];
        if (b < a.j1) P.buf_slot[b] = off + inc - v;
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t tot = 0, rt = 0;
            for (uint32_t k = 0; k < 16; k++) { tot += wsum[k][0]; rt += wsum[k][1]; }
            carry[0] += tot;
            carry[1] += rt;
        }
        __syncthreads();
    }
    (void)nref_tot;
    if (threadIdx.x == 0) {
        *P.seg_count = carry[0];
        P.ctl[CTL_COUNT] = carry[0];
        P.ctl[CTL_NEXTRACT] += carry[0] - start;
        P.ctl[CTL_NREF] += carry[1];
        if (carry[0] > P.seg_cap) P.ctl[CTL_ERROR] |= ERR_CAPACITY;
        if (a.pub_final) ctl_publish(a);  // (the pass's last sub-batch: its emit changes no word)
    }
}

// -------------------------------------------------------------- k_pack ------------------
// Packed offsets of buffers [j0, j1) after the running total (one workgroup), then one
// workgroup per buffer copies its encoded stream to dst + offset.  With dst in pinned host
// memory the copy is the device-to-host transfer, overlapping the next sub-batch's encode.

__global__ __launch_bounds__(1024) void k_pack_offsets(PackArgs a)
{
    if (aborted(a.P)) return;
    __shared__ uint64_t wsum[16];
    __shared__ uint64_t carry;
    const uint32_t wave = threadIdx.x >> 6, l = lane_id();
    if (threadIdx.x == 0) carry = a.j0 == 0u ? 0ull : *a.total;  // (the run's first buffers: from 0)
    __syncthreads();
    for (uint32_t b0 = a.j0; b0 < a.j1; b0 += 1024u) {
        const uint32_t b = b0 + threadIdx.x;
        const uint64_t v = b < a.j1 ? a.P.out_len[b] : 0u;
        // a buffer's stream is < 2^21 bytes, so 64 of them sum below 2^32
        const uint32_t lo = wave_incl_scan((uint32_t)v);
        if (l == 63) wsum[wave] = lo;
        __syncthreads();
        uint64_t off = carry;
        for (uint32_t k = 0; k < wave; k++) off += wsum[k];
        if (b < a.j1) a.pos[b] = off + lo - v;
        __syncthreads();
        if (threadIdx.x == 0) {
            uint64_t t = 0;
            for (uint32_t k = 0; k < 16; k++) t += wsum[k];
            carry += t;
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        *a.total = carry;
        if (carry > a.cap) atomicOr(&a.P.ctl[CTL_ERROR], ERR_PACK_CAP);
    }
}

__global__ __launch_bounds__(256) void k_pack_copy(PackArgs a)
{
    if (aborted(a.P)) return;
    const uint32_t b = a.j0 + blockIdx.x;
    if (b >= a.j1) return;
    const uint64_t n = a.P.out_len[b], o = a.pos[b];
    if (o + n > a.cap) return;  // flagged by k_pack_offsets
    const uint8_t *src = a.P.out + a.P.out_off[b];
    uint8_t *dst = a.dst + o;
    // four waves, each a contiguous quarter cut at a 16-byte boundary of dst
    const uint32_t wave = threadIdx.x >> 6;
    const uint64_t head = (16u - ((uintptr_t)dst & 15u)) & 15u;
    const uint64_t body = n > head ? (n - head) & ~15ull : 0u;
    const uint64_t q = (body / 64u) * 16u;  // 16-byte multiple per wave
    uint64_t s0 = wave == 0 ? 0 : head + q * wave, s1 = wave == 3 ? n : head + q * (wave + 1u);
    if (s1 > n) s1 = n;
    if (s0 < s1) wave_copy(dst + s0, src + s0, (uint32_t)(s1 - s0));
}

// ------------------------------------------------------------ utilities -----------------
__global__ __launch_bounds__(64) void k_hash_segments(const uint8_t *segs, uint64_t n, uint64_t *out)
{
    for (uint64_t i = blockIdx.x; i < n; i += gridDim.x) {
        const uint64_t h = wave_window_hash(segs + i * XC_SEG);
        if (lane_id() == 0) out[i] = h;
    }
}

// Plain per-position hashes (window ends p >= 2047) via the same block recurrence as k_scan.
__global__ __launch_bounds__(64) void k_window_hashes(const uint8_t *in, uint32_t n, uint64_t *out)
{
    const uint32_t l = lane_id();
    const uint32_t blk = blockIdx.x;  // window ends [2048*blk, 2048*blk + 2048)
    const uint32_t s = blk * XC_SEG;
    if (s >= n) return;
    if (blk == 0) {
        for (uint32_t i = l; i < min(n, XC_SEG - 1u); i += 64u) out[i] = 0;
        if (n >= XC_SEG) {
            const uint64_t h = wave_window_hash(in);
            if (l == 0) out[XC_SEG - 1u] = h;
        }
        return;
    }
    // full hash at the lane's window ending q-1, then roll 32 positions (both components)
    const uint32_t q = s + 32u * l;
    uint32_t w[8], pw[8];
    // padded reads are in bounds of the arena (caller pads by >= 64 bytes)
    load32_unaligned(in + q, w);
    load32_unaligned(in + q - XC_SEG, pw);
    // window sums ending at q-1: recompute directly (2048 bytes per lane; test utility only)
    uint32_t s1w = 0, s2w = 0, s1f = 0, s2f = 0;
    for (uint32_t i = 0; i < XC_SEG; i++) {
        const uint32_t by = in[q - XC_SEG + i];
        s1w += by + 1u;
        s2w += (XC_SEG - i) * (by + 1u);
        const uint32_t f = ffs8(by);
        s1f += f;
        s2f += (XC_SEG - i) * f;
    }
#pragma unroll
    for (int d = 0; d < 8; d++) {
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const uint32_t ib = (w[d] >> (8 * k)) & 0xffu, ob = (pw[d] >> (8 * k)) & 0xffu;
            const uint32_t fi = ffs8(ib), fo = ffs8(ob);
            s1w += ib - ob;
            s2w = s2w - XC_SEG * (ob + 1u) + s1w;
            s1f += fi - fo;
            s2f = s2f - XC_SEG * fo + s1f;
            const uint32_t p = q + (uint32_t)(d * 4 + k);
            if (p < n) {
                const uint32_t bytes_hash = (s1w << 20) + s2w, bits_hash = (s1f << 16) + s2f;
                out[p] = ((uint64_t)bits_hash << 36) + bytes_hash;
            }
        }
    }
}

// Clear a declaration set (all of its tables) and seed the combined level-2 filter with the
// cache's: one launch instead of a memset per table.
// With amix (an anchor-scanned sub-batch, whose set is keys and values only: block_predict) the
// filters, the lo32 keys and the combined level-1 / level-2 images are left alone.
__global__ void k_clear_set(DevSet s, uint32_t n_lo, uint32_t n_full, uint4 *l2mix, const uint4 *cache_l2,
                            uint32_t *fmix, const uint32_t *cache_filt, uint32_t fold, const uint32_t *count,
                            uint32_t *count_out, uint32_t *ctl_zero, AncSet danc, uint4 *amix, const uint4 *cache_afilt)
{
    const uint32_t stride = gridDim.x * blockDim.x;
    const uint32_t i0 = blockIdx.x * blockDim.x + threadIdx.x;
    if (count_out && i0 == 0) *count_out = *count;  // (the sub-batch's start count: P.sb_count)
    // the first scan's level-1 image starts as the cache's, folded
    if (fmix)
        for (uint32_t i = i0; i < (XC_FILT_WORDS >> fold); i += stride) {
            uint32_t v = 0;
            for (uint32_t j = 0; j < (1u << fold); j++) v |= cache_filt[(i << fold) + j];
            fmix[i] = v;
        }
    // a run's first sub-batch also clears the run's control words (nothing reads them before the
    // kernels after this one)
    if (ctl_zero && i0 < CTL_WORDS) ctl_zero[i0] = 0u;
    const uint4 z = make_uint4(0, 0, 0, 0), ones = make_uint4(~0u, ~0u, ~0u, ~0u);
    if (!amix) {
        for (uint32_t i = i0; i < XC_FILT_WORDS / 4; i += stride) ((uint4 *)s.filt)[i] = z;
        const bool own_l2 = (const void *)s.l2 != (const void *)l2mix;  // (plans alias the two)
        for (uint32_t i = i0; i < XC_L2_WORDS / 2; i += stride) {
            if (own_l2) ((uint4 *)s.l2)[i] = z;
            l2mix[i] = cache_l2[i];
        }
        for (uint32_t i = i0; i < n_lo / 4; i += stride) ((uint4 *)s.lo_keys)[i] = z;
        if (i0 == 0) *s.lo_zero = 0u;
    }
    for (uint32_t i = i0; i < n_full / 2; i += stride) {
        ((uint4 *)s.keys)[i] = ones;
        ((uint4 *)s.vals)[i] = ones;
    }
    // an anchor-scanned sub-batch: the declarations' anchor table empty, the combined anchor
    // filter seeded with the cache's
    if (amix) {
        for (uint32_t i = i0; i < ANC_FILT_WORDS / 4; i += stride) amix[i] = cache_afilt[i];
        for (uint32_t i = i0; i < (danc.mask + 1u) / 2; i += stride) ((uint4 *)danc.keys)[i] = ones;
    }
}

__global__ void k_or_words(uint4 *dst, const uint4 *a, const uint4 *b, uint32_t n)
{
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        uint4 x = a[i];
        if (b) {
            const uint4 y = b[i];
            x.x |= y.x; x.y |= y.y; x.z |= y.z; x.w |= y.w;
        }
        dst[i] = x;
    }
}

// Cache restore: clear every table slot entered after the snapshot.
__global__ void k_undo(DevSet cache, const uint2 *undo, uint32_t from, uint32_t to)
{
    for (uint32_t i = from + blockIdx.x * blockDim.x + threadIdx.x; i < to; i += gridDim.x * blockDim.x) {
        const uint2 u = undo[i];
        if (u.y == XC_REVIVED) {
            cache.vals[u.x] |= XC_DEAD;
            continue;
        }
        if (u.x != NONE) cache.keys[u.x] = XC_EMPTY64;
        if (u.y != NONE) cache.lo_keys[u.y] = 0u;
    }
}

// Same, reading the current count on the device (no host round trip).
__global__ void k_undo_dev(DevSet cache, const uint2 *undo, uint32_t from, const uint32_t *count, uint32_t cap,
                           const uint4 *snap_filt, const uint4 *snap_l2, const uint32_t *snap_lo_zero)
{
    // every table slot entered after the snapshot is cleared, the filters are copied back from
    // the snapshot (one launch for the whole restore; the count is restored after it)
    const uint32_t to = min(*count, cap);
    const uint32_t i0 = blockIdx.x * blockDim.x + threadIdx.x, stride = gridDim.x * blockDim.x;
    for (uint32_t i = from + i0; i < to; i += stride) {
        const uint2 u = undo[i];
        if (u.y == XC_REVIVED) {
            cache.vals[u.x] |= XC_DEAD;
            continue;
        }
        if (u.x != NONE) cache.keys[u.x] = XC_EMPTY64;
        if (u.y != NONE) cache.lo_keys[u.y] = 0u;
    }
    for (uint32_t i = i0; i < XC_FILT_WORDS / 4; i += stride) ((uint4 *)cache.filt)[i] = snap_filt[i];
    for (uint32_t i = i0; i < XC_L2_WORDS / 2; i += stride) ((uint4 *)cache.l2)[i] = snap_l2[i];
    if (i0 == 0) *cache.lo_zero = *snap_lo_zero;
}

// The same with the current count known on the host (to): nothing reads the count, so the
// restore writes the snapshot's count itself (one launch, no device-to-device copy).
__global__ void k_undo_known(DevSet cache, const uint2 *undo, uint32_t from, uint32_t to, uint32_t *count,
                             const uint4 *snap_filt, const uint4 *snap_l2, const uint32_t *snap_lo_zero)
{
    const uint32_t i0 = blockIdx.x * blockDim.x + threadIdx.x, stride = gridDim.x * blockDim.x;
    for (uint32_t i = from + i0; i < to; i += stride) {
        const uint2 u = undo[i];
        if (u.y == XC_REVIVED) {
            cache.vals[u.x] |= XC_DEAD;
            continue;
        }
        if (u.x != NONE) cache.keys[u.x] = XC_EMPTY64;
        if (u.y != NONE) cache.lo_keys[u.y] = 0u;
    }
    for (uint32_t i = i0; i < XC_FILT_WORDS / 4; i += stride) ((uint4 *)cache.filt)[i] = snap_filt[i];
    for (uint32_t i = i0; i < XC_L2_WORDS / 2; i += stride) ((uint4 *)cache.l2)[i] = snap_l2[i];
    if (i0 == 0) {
        *cache.lo_zero = *snap_lo_zero;
        *count = from;
    }
}

// Cache growth and truncation (xc_runtime.hip cache_rebuild): every entry of the old full table
// with a segment index below `keep` (live, with drop_dead) into the tables of `to`, its slots into the undo log at its segment index (the restore's record).  A lo32
// key shared by several entries belongs, in the undo log, to the oldest (smallest index) entry, as
// when they were entered in index order: lo_owner[slot] = that index (k_rehash_owner applies it).
// The filters depend on the keys only and are copied as they are.
__global__ void k_rehash(DevSet from, DevSet to, uint2 *undo, uint32_t *lo_owner, uint32_t keep, int drop_dead)
{
    const uint32_t n = from.mask + 1u;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const uint64_t h = from.keys[i];
        if (h == XC_EMPTY64) continue;
        const uint32_t v = (uint32_t)from.vals[i];
        if (v >= keep || (drop_dead && (from.vals[i] & XC_DEAD))) continue;
        uint32_t j = key_slot(h, to.mask);
        while (atomicCAS((unsigned long long *)&to.keys[j], (unsigned long long)XC_EMPTY64, (unsigned long long)h) !=
               XC_EMPTY64)
            j = (j + 1u) & to.mask;  // (keys are unique: every other key found here is another's)
        to.vals[j] = from.vals[i];   // (an evicted entry stays evicted)
        const uint32_t lo = (uint32_t)h;
        uint32_t ls = NONE;
        if (lo != 0u) {
            ls = lo_slot(lo, to.lo_mask);
            for (;;) {
                const uint32_t prev = atomicCAS(&to.lo_keys[ls], 0u, lo);
                if (prev == 0u || prev == lo) break;
                ls = (ls + 1u) & to.lo_mask;
            }
            atomicMin(&lo_owner[ls], v);
        }
        undo[v] = make_uint2(j, ls);
    }
}

__global__ void k_rehash_owner(uint2 *undo, uint32_t n, const uint32_t *lo_owner)
{
    for (uint32_t v = blockIdx.x * blockDim.x + threadIdx.x; v < n; v += gridDim.x * blockDim.x) {
        const uint2 u = undo[v];
        if (u.y != NONE && lo_owner[u.y] != v) undo[v].y = NONE;
    }
}

// Cache enter from the host API (single segment).
__global__ void k_enter_one(PlanDev P, uint64_t h, const uint8_t *seg)
{
    if (uniform(P.seg_count[0]) >= P.seg_cap) {
        if (lane_id() == 0) atomicOr(&P.ctl[CTL_ERROR], ERR_CAPACITY);
        return;
    }
    uint64_t v;
    if (set_find(P.cache, h, &v)) {  // release-build XCodecMemoryCache::enter overwrites
        wave_copy(seg_at(P.segs, v), seg, XC_SEG);
        return;
    }
    const uint32_t idx = uniform(P.seg_count[0]);
    wave_copy(seg_at(P.segs, idx), seg, XC_SEG);
    if (lane_id() == 0) {
        uint32_t s1, s2;
        set_insert(P.cache, h, idx, false, &s1, &s2);
        P.undo[idx] = make_uint2(s1, s2);
        P.seg_count[0] = idx + 1u;
    }
}

// Many host-API enters at once (the COSS tier's load of its index at open): one wave per segment,
// into slots first, first + 1, ... (the host has checked capacity and that the hashes are new).
__global__ void k_enter_bulk(PlanDev P, const uint64_t *h, const uint8_t *segs, uint32_t n, uint32_t first)
{
    const uint32_t i = blockIdx.x * 4u + (threadIdx.x >> 6);
    if (i >= n) return;
    const uint32_t idx = first + i;
    wave_copy(seg_at(P.segs, idx), segs + (size_t)i * XC_SEG, XC_SEG);
    if (lane_id() == 0) {
        uint32_t s1, s2;
        set_insert(P.cache, h[i], idx, false, &s1, &s2);
        P.undo[idx] = make_uint2(s1, s2);
    }
}

// A run's lookup hits for the recent window (xc_memcache.cpp), one wave per buffer: at
// out[tok_base[b] + b * (COLL_CAP + 1)] the count (bit 63: more collisions than were recorded), then
// the hashes in the reference's order: REF tokens (window end seg + 2047) and the recorded collision
// lookups, by position.  Without collision records (the common case) the REF tokens are compacted
// 64 at a time by ballot; with them, lane 0 merges the two lists.
__global__ __launch_bounds__(256) void k_hits(PlanDev P, uint64_t *out)
{
    const uint32_t b = blockIdx.x * 4u + (threadIdx.x >> 6), l = lane_id();
    if (b >= P.nb) return;
    uint64_t *o = out + P.hit_base[b];  // (room for every REF, len / 2048, and COLL_CAP collisions)
    const uint32_t tb = P.tok_base[b], n = min(P.tok_cnt[b], P.tok_base[b + 1] - tb), cc = P.coll_cnt[b];
    const uint32_t nc = min(cc, COLL_CAP);
    if (nc == 0u) {
        uint32_t k = 0;
        for (uint32_t t0 = 0; t0 < n; t0 += 64u) {
            const uint32_t t = t0 + l;
            const bool ref = t < n && P.tok_op[tb + t] == OP_REF;
            const uint64_t m = ballot(ref);
            if (ref) o[1u + k + mbcnt(m)] = P.tok_h[tb + t];
            k += (uint32_t)__popcll(m);
        }
        if (l == 0) o[0] = (uint64_t)k;
        return;
    }
    if (l != 0) return;
    uint32_t k = 0, ci = 0;
    for (uint32_t t = 0; t < n; t++) {
        if (P.tok_op[tb + t] != OP_REF) continue;
        const uint32_t q = P.tok_seg[tb + t] + (XC_SEG - 1u);
        for (; ci < nc && P.coll[b * COLL_CAP + ci].x < q; ci++) {
            const uint4 r = P.coll[b * COLL_CAP + ci];
            o[1 + k++] = ((uint64_t)r.z << 32) | r.y;
        }
        o[1 + k++] = P.tok_h[tb + t];
    }
    for (; ci < nc; ci++) {
        const uint4 r = P.coll[b * COLL_CAP + ci];
        o[1 + k++] = ((uint64_t)r.z << 32) | r.y;
    }
    o[0] = (uint64_t)k | (cc > COLL_CAP ? 1ull << 63 : 0ull);
}

// k_hits' output (device) into pinned host memory, only the words each buffer filled: one wave per
// buffer, a few workgroups (the writes cross PCIe; the kernel runs beside the next run).
__global__ void k_hits_out(const uint64_t *stage, uint64_t *host, const uint32_t *hit_base, uint32_t nb)
{
    const uint32_t waves = gridDim.x * (blockDim.x >> 6);
    for (uint32_t b = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); b < nb; b += waves) {
        const uint64_t off = hit_base[b];
        const uint32_t n = 1u + (uint32_t)(stage[off] & 0xFFFFFFFFu);
        for (uint32_t i = lane_id(); i < n; i += 64u) host[off + i] = stage[off + i];
    }
}

// The table values of n hashes (~0: absent or evicted), no side effects.
__global__ void k_find(DevSet cache, const uint64_t *h, uint64_t *val, uint32_t n)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint64_t v;
    val[i] = set_find(cache, h[i], &v) ? v : ~0ull;
}

// The table value of a present key (evicted or not), set.
__global__ void k_setval(DevSet cache, uint64_t h, uint64_t val)
{
    if (threadIdx.x != 0) return;
    uint32_t j = key_slot(h, cache.mask);
    for (;;) {
        const uint64_t x = cache.keys[j];
        if (x == h) {
            cache.vals[j] = val;
            return;
        }
        if (x == XC_EMPTY64) return;
        j = (j + 1u) & cache.mask;
    }
}

// Segments the COSS tier evicted (purge_stripe, xcodec_cache_coss.cc:347-377): absent to every
// later lookup until entered again.
__global__ void k_kill(DevSet cache, const uint64_t *h, uint32_t n)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t k = h[i];
    uint32_t j = key_slot(k, cache.mask);
    for (;;) {
        const uint64_t x = cache.keys[j];
        if (x == k) {
            cache.vals[j] |= XC_DEAD;
            return;
        }
        if (x == XC_EMPTY64) return;
        j = (j + 1u) & cache.mask;
    }
}

__global__ void k_lookup_one(PlanDev P, uint64_t h, uint8_t *out, uint32_t *found)
{
    uint64_t v;
    if (set_find(P.cache, h, &v)) {
        wave_copy(out, seg_at(P.segs, v), XC_SEG);
        if (lane_id() == 0) *found = 1u;
    } else if (lane_id() == 0) {
        *found = 0u;
    }
}

// Wave primitive self-test: scan against a serial loop, hash against the rolling form.
__global__ void k_selftest(uint32_t *err)
{
    const uint32_t l = lane_id();
    uint32_t x = l * 2654435761u + 12345u;
    const uint32_t inc = wave_incl_scan(x);
    uint32_t ref = 0;
    for (uint32_t k = 0; k <= l; k++) ref += k * 2654435761u + 12345u;
    if (inc != ref) atomicOr(err, 1u);
    const uint64_t m = ballot((l & 3) == 1);
    if (mbcnt(m) != (l + 2) / 4) atomicOr(err, 2u);
    for (uint32_t k = 0; k < 64; k++) {  // the scan's level-2 mix inverts
        const uint32_t v = (x ^ (k * 0x9E3779B9u)) * (k | 1u);
        if (l2_unmix(l2_mix(v)) != v) atomicOr(err, 4u);
    }
}

// ------------------------------------------------------------ anchor index upkeep --------
// Index the segments of slots [from, to) (entered by runs without anchors: while the cache was
// small, by a decoder, through the host API), one wave per slot.
__global__ __launch_bounds__(256) void k_anc_backfill(PlanDev P, uint32_t from, uint32_t to, uint32_t *ctl)
{
    const uint32_t l = lane_id();
    for (uint32_t s = from + blockIdx.x * 4u + (threadIdx.x >> 6); s < to; s += gridDim.x * 4u) {
        const uint4 *sp = (const uint4 *)(seg_at(P.segs, s) + 32u * l);
        const uint4 x = sp[0], y = sp[1];
        const uint32_t w[8] = {x.x, x.y, x.z, x.w, y.x, y.y, y.z, y.w};
        const uint64_t key = wave_seg_anchor(w);
        if (l == 0) {
            P.anc_of[s] = key;
            if (key != ANC_NONE) {
                P.aundo[s] = anc_insert(P.canc, key);
            } else {
                P.aundo[s] = NONE;
                atomicMax(&ctl[CTL_ANCLESS], ~s);
            }
        }
    }
}

// Restore: the anchor-table slots the segments [from, to) took are emptied (a snapshot's later
// entries are all removed together, so no probe chain of a kept key passes through them); the
// filter from the snapshot when snap is given.
// (word / value: the cache's anchorless word as of the snapshot, set here rather than by a 4-byte
// copy from pageable host memory: one API call less in the host's turn between two runs)
__global__ void k_anc_undo(AncSet s, const uint32_t *aundo, uint32_t from, uint32_t to, uint4 *filt, const uint4 *snap,
                           uint32_t *word, uint32_t value)
{
    const uint32_t i0 = blockIdx.x * blockDim.x + threadIdx.x, stride = gridDim.x * blockDim.x;
    if (word && i0 == 0) *word = value;
    for (uint32_t i = from + i0; i < to; i += stride) {
        const uint32_t a = aundo[i];
        if (a != NONE) s.keys[a] = XC_EMPTY64;
    }
    if (snap)
        for (uint32_t i = i0; i < ANC_FILT_WORDS / 4; i += stride) filt[i] = snap[i];
}

// Growth / truncation: the anchors of segments [0, n) into a new table in parallel; a key shared
// by several segments belongs (undo log) to the oldest, as when they were entered in order:
// owner[slot] = min segment, k_anc_owner writes aundo.
__global__ void k_anc_rehash(AncSet to, const uint64_t *anc_of, uint32_t n, uint32_t *aslot, uint32_t *owner)
{
    for (uint32_t v = blockIdx.x * blockDim.x + threadIdx.x; v < n; v += gridDim.x * blockDim.x) {
        const uint64_t key = anc_of[v];
        if (key == ANC_NONE) {
            aslot[v] = NONE;
            continue;
        }
        uint32_t k = anc_home(key >> 11, to.mask);
        for (;;) {
            const uint64_t prev = atomicCAS((unsigned long long *)&to.keys[k], (unsigned long long)XC_EMPTY64,
                                            (unsigned long long)key);
            if (prev == XC_EMPTY64 || prev == key) break;
            k = (k + 1u) & to.mask;
        }
        aslot[v] = k;
        atomicMin(&owner[k], v);
    }
}

__global__ void k_anc_owner(uint32_t *aundo, const uint32_t *aslot, uint32_t n, const uint32_t *owner)
{
    for (uint32_t v = blockIdx.x * blockDim.x + threadIdx.x; v < n; v += gridDim.x * blockDim.x) {
        const uint32_t a = aslot[v];
        aundo[v] = a != NONE && owner[a] == v ? a : NONE;
    }
}

// ------------------------------------------------------------ k_tailcheck ----------------
// After an anchor-scanned run.  The recent window (xcodec_cache.h:89-159,
// xc_memcache.cpp) remembers every lookup hit, collisions included; an anchor scan's events are
// the windows equal to indexed segments, and a collision where a candidate is pending changes
// nothing the walk decides, so those were not looked for.  The window's state after the run
// depends on its last 64 hits only: for the buffers that hold the run's last >= 64 recorded hits
// (REF tokens and recorded collisions), every collision lookup is found again here: each looked-up
// window end (not a REF, not in a REF's shadow) whose hash the cache held at that point (an entry
// before the buffer's, or one of its own declarations made before it) with other bytes; the
// buffer's collision records are replaced by them.  Persistent grid, a workgroup per buffer.

// Did buffer b's lookup at q see the entry in slot v (wave-uniform)?
__device__ __forceinline__ bool tail_visible(const PlanDev &P, uint32_t b, uint32_t q, uint32_t v)
{
    const uint32_t s0 = P.buf_slot[b];
    if (v < s0) return true;
    const uint32_t i = v - s0;
    if (i >= P.buf_next[b]) return false;
    const uint32_t l = lane_id();
    const uint32_t tb = P.tok_base[b], n = P.tok_cnt[b];
    uint32_t ord = 0;
    for (uint32_t t0 = 0; t0 < n; t0 += 64u) {
        const uint32_t t = t0 + l;
        const bool ext = t < n && P.tok_op[tb + t] == OP_EXTRACT;
        const uint32_t incl = wave_incl_scan(ext ? 1u : 0u);
        const uint64_t m = ballot(ext && ord + incl - 1u == i);
        if (m) {
            const uint32_t dpos = readlane(P.tok_dpos[tb + t0 + (uint32_t)(__ffsll((unsigned long long)m) - 1)], 0);
            return dpos != DPOS_FLUSH && dpos <= q;
        }
        ord += readlane(incl, 63);
    }
    return false;
}

// Window sums of the bits half (w = ffs(byte), xcodec_hash.h:93-135) before a lane's first position,
// as block_sums gives those of the bytes half.
__device__ __forceinline__ BlockSums block_sums_ffs(const uint32_t w[8], uint32_t l)
{
    uint32_t sf = 0, jf = 0;
#pragma unroll
    for (int d = 0; d < 8; d++) {
        const uint32_t wt = (uint32_t)(4 * d) * 0x01010101u + 0x03020100u;
        const uint32_t f = ffs_bytes(w[d]);
        sf = __builtin_amdgcn_udot4(f, 0x01010101u, sf, false);
        jf = __builtin_amdgcn_udot4(f, wt, jf, false);
    }
    const uint32_t A = sf, C = 32u * l * A + jf;
    const uint32_t ia = wave_incl_scan(A), ic = wave_incl_scan(C);
    BlockSums s;
    s.totA = readlane(ia, 63);
    s.totC = readlane(ic, 63);
    s.preA = ia - A;
    s.preC = ic - C;
    return s;
}

// The first buffer of the run's tail (its last buffers whose REF hits reach the window's 64, all of
// the run when fewer), wave-uniform.
__device__ __forceinline__ uint32_t tail_first(const PlanDev &P, uint32_t nb)
{
    const uint32_t l = lane_id();
    uint32_t acc = 0;
    for (uint32_t e = nb; e > 0; e = e > 64u ? e - 64u : 0u) {
        const bool ok = l < e;
        const uint32_t v = ok ? P.buf_nref[e - 1u - l] : 0u;
        const uint32_t incl = wave_incl_scan(v);
        const uint64_t m = ballot(ok && acc + incl >= 64u);
        if (m) return e - 1u - (uint32_t)(__ffsll((unsigned long long)m) - 1);
        acc += readlane(incl, 63);
    }
    return 0u;
}

// One wave per aligned block of the tail's buffers (window ends [s, s + 2048); block 0: the first
// window, 2047), all of them in flight across the chip: the low 32 bits of every full hash by the
// rolling recurrence of the bytes half (k_scan's), the looked-up ends (not a REF's, not in the 2047
// ends after one) tested in the cache's level-2 filter; only its few positives take the bits half
// and a probe of the full table; collisions into the buffer's scratch list (tcnt, tlist), which
// k_tailfinal sorts into its records.
// At most 96 VGPRs (5 waves per SIMD): the kernel runs behind the run's last emit while the next
// run's block hashing (128 VGPRs, 4 waves per SIMD) fills the chip on the side stream, and a wave
// that needs more registers than one block-hashing wave frees waited for the hashing's end (171
// VGPRs: 342 us per cfg5 step instead of 30, profiles/r05/step_timeline_r5fin.txt).
__global__ __launch_bounds__(256, 5) void k_tailcheck(PlanDev P, uint32_t nb, uint32_t *tcnt, uint4 *tlist)
{
    if (aborted(P)) return;  // (enqueued behind a pass that stopped: the host's redo runs it again)
    __shared__ uint32_t refs[4][4];
    const uint32_t wave = threadIdx.x >> 6, l = lane_id();
    const uint32_t j0 = tail_first(P, nb);
    const uint32_t g0 = P.buf_grp0[j0], g1 = P.buf_grp0[nb];
    for (uint32_t u = (g0 * BLK_GROUP) + blockIdx.x * 4u + wave; u < g1 * BLK_GROUP; u += gridDim.x * 4u) {
        const uint2 gr = P.blk_grp[u / BLK_GROUP];
        const uint32_t b = gr.x, k = gr.y + u % BLK_GROUP;
        const uint32_t len = P.buf_len[b], s = k * XC_SEG;
        if (s >= len || len < XC_SEG) continue;
        const uint8_t *base = P.in + P.buf_off[b];
        // the REF window ends e in [s - 2047, s + 2047] (at most two: REFs are >= 2048 apart)
        uint32_t nr = 0;
        {
            const uint32_t tb = P.tok_base[b], n = P.tok_cnt[b];
            for (uint32_t t0 = 0; t0 < n; t0 += 64u) {
                const uint32_t t = t0 + l;
                uint32_t e = 0;
                bool r = false;
                if (t < n && P.tok_op[tb + t] == OP_REF) {
                    e = P.tok_seg[tb + t] + (XC_SEG - 1u);
                    r = e + (XC_SEG - 1u) >= s && e < s + XC_SEG;
                }
                const uint64_t m = ballot(r);
                if (r && nr + mbcnt(m) < 4u) refs[wave][nr + mbcnt(m)] = e;
                nr += (uint32_t)__popcll(m);
            }
            nr = min(nr, 4u);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
        const uint32_t q0 = s + 32u * l;
        uint32_t shadow = 0;  // bit t: end q0 + t is not looked up
        for (uint32_t r = 0; r < nr; r++) {
            const uint32_t e = refs[wave][r];
            const uint32_t a = e > q0 ? e - q0 : 0u;
            const uint32_t z = e + (XC_SEG - 1u) >= q0 + 31u ? 32u : (e + XC_SEG > q0 ? e + XC_SEG - q0 : 0u);
            if (z > a && a < 32u) shadow |= (z - a >= 32u ? ~0u : ((1u << (z - a)) - 1u)) << a;
        }
        uint32_t live = ~0u;
        if (s == 0) live = l == 63u ? 0x80000000u : 0u;  // (block 0: its last end only)
        if (q0 + 32u > len) live &= q0 >= len ? 0u : (1u << (len - q0)) - 1u;
        live &= ~shadow;
        if (!ballot(live != 0u)) continue;
        uint32_t pw[8], w[8];
        if (s == 0) {  // the first window: block 0 after 2048 zero bytes (rolled out by its end)
            load32_aligned(base + 32u * l, w);
            for (int d = 0; d < 8; d++) pw[d] = 0u;
        } else {
            load32_aligned(base + s - XC_SEG + 32u * l, pw);
            load32_aligned(base + s + 32u * l, w);
        }
        // H = bits << 36 | bytes (xcodec_hash.h:155-174), both halves by k_scan's rolling recurrences,
        // 16 window ends at a time (registers: the kernel's 96-VGPR bound)
        const BlockSums ps = block_sums(pw, l), cs = block_sums(w, l);
        const BlockSums pf = block_sums_ffs(pw, l), cf = block_sums_ffs(w, l);
        const uint32_t sufA = ps.totA - ps.preA, sufC = ps.totC - ps.preC;
        uint32_t U = sufA + cs.preA - XC_SEG;
        uint32_t V = (XC_SEG + 32u * l) * sufA - sufC + 32u * l * cs.preA - cs.preC + 0x80000000u;
        const uint32_t fA = pf.totA - pf.preA, fC = pf.totC - pf.preC;
        uint32_t Uf = fA + cf.preA;
        uint32_t Vf = (XC_SEG + 32u * l) * fA - fC + 32u * l * cf.preA - cf.preC;
        uint32_t hit = 0;
#pragma unroll
        for (int h16 = 0; h16 < 2; h16++) {
            uint32_t lo[16], hb[16];
#pragma unroll
            for (int d = 0; d < 4; d++) {
#pragma unroll
                for (int kk = 0; kk < 4; kk++) {
                    const uint32_t ib = (w[4 * h16 + d] >> (8 * kk)) & 0xffu, ob = (pw[4 * h16 + d] >> (8 * kk)) & 0xffu;
                    U += ib - ob;
                    V += U + (uint32_t)__mul24((int)ob, -2048);
                    const uint32_t fi = ffs8(ib), fo = ffs8(ob);
                    Uf += fi - fo;
                    Vf += Uf - XC_SEG * fo;
                    lo[4 * d + kk] = (U << 20) + V;
                    hb[4 * d + kk] = (Uf << 16) + Vf;
                }
            }
            // the cache's level-2 filter first (2 MB, L2-resident: every key of the table has its bits,
            // set_insert), the table only for its few positives
            const uint32_t lv = live >> (16 * h16);
            uint32_t cand = 0;
#pragma unroll
            for (int t8 = 0; t8 < 16; t8 += 8) {
                uint32_t fw[8];
#pragma unroll
                for (int t = 0; t < 8; t++) fw[t] = P.cache.l2[(lv >> (t8 + t)) & 1u ? l2_word(l2_mix(lo[t8 + t])) : 0u];
#pragma unroll
                for (int t = 0; t < 8; t++)
                    if (((lv >> (t8 + t)) & 1u) && l2_test(fw[t], l2_mix(lo[t8 + t]))) cand |= 1u << (t8 + t);
            }
            while (cand) {
                const uint32_t t = (uint32_t)__builtin_ctz(cand);
                cand &= cand - 1u;
                uint32_t x = lo[0], y = hb[0];
#pragma unroll
                for (int tt = 1; tt < 16; tt++) {
                    x = t == (uint32_t)tt ? lo[tt] : x;
                    y = t == (uint32_t)tt ? hb[tt] : y;
                }
                uint64_t v;
                if (set_find(P.cache, ((uint64_t)y << 36) + x, &v)) hit |= 1u << (16u * h16 + t);
            }
        }
        for (;;) {
            const uint64_t m = ballot(hit != 0u);
            if (!m) break;
            const int f = __ffsll((unsigned long long)m) - 1;
            const uint32_t t = (uint32_t)__builtin_ctz(readlane(hit, f));
            if ((int)l == f) hit &= hit - 1u;
            const uint32_t q = readlane(q0, f) + t;
            const uint8_t *win = base + q - (XC_SEG - 1u);
            const uint64_t hh = wave_window_hash(win);  // (the hit's full hash again, wave-wide: rare)
            uint64_t v = 0;
            if (set_find(P.cache, hh, &v)) {
                const uint32_t vv = uniform((uint32_t)v);
                if (!tail_visible(P, b, q, vv)) continue;
                if (wave_equal2048(win, seg_at(P.segs, vv))) continue;  // (the walk's REF)
                if (l == 0) {
                    const uint32_t kq = atomicAdd(&tcnt[b], 1u);
                    if (kq < COLL_CAP) tlist[(size_t)b * COLL_CAP + kq] = make_uint4(q, (uint32_t)hh, (uint32_t)(hh >> 32), NONE);
                }
            }
        }
    }
}

// The tail's buffers: their collision lookups, sorted by window end, replace the walk's records
// (one wave per buffer); the scratch counts back to zero.
__global__ __launch_bounds__(64) void k_tailfinal(PlanDev P, uint32_t nb, uint32_t *tcnt, const uint4 *tlist)
{
    if (aborted(P)) return;
    const uint32_t l = lane_id();
    const uint32_t j0 = tail_first(P, nb);
    for (uint32_t b = j0 + blockIdx.x; b < nb; b += gridDim.x) {
        const uint32_t c = tcnt[b], n = min(c, COLL_CAP);
        const uint4 e = l < n ? tlist[(size_t)b * COLL_CAP + l] : make_uint4(NONE, 0u, 0u, NONE);
        uint32_t rank = 0;
        for (uint32_t k = 0; k < n; k++) rank += readlane(e.x, (int)k) < e.x ? 1u : 0u;
        if (l < n) P.coll[b * COLL_CAP + rank] = e;
        if (l == 0) {
            P.coll_cnt[b] = c;
            tcnt[b] = 0u;
        }
    }
}

}  // namespace xc
