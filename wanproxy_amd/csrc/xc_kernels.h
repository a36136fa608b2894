// xc_kernels.h — device-side data layout shared by the encode/decode kernels and the host runtime.
#pragma once
#include <stdint.h>

#include "xc_device.h"

namespace xc {

constexpr uint32_t EV_CAP = 64;          // sparse events per scan chunk before it turns dense
constexpr uint32_t EV_DENSE = 0x80000000u;
constexpr uint32_t Q_CAP = 128;          // per-wave LDS queue of level-1 filter positives
#ifndef XC_SCAN_WAVES
#define XC_SCAN_WAVES 16
#endif
constexpr uint32_t SCAN_WAVES = XC_SCAN_WAVES;  // waves per scan workgroup (one per CU: all of its LDS)
constexpr uint32_t CHUNK_BLOCKS = 8;     // most 2048-byte blocks per scan chunk (16 KiB; small plans use fewer)
constexpr uint32_t SCAN_UNIT = 4;        // most chunks a scan wave takes from the work counter at a time
constexpr uint32_t EMIT_WAVES = 4;       // k_emit waves per buffer (workgroup)
constexpr uint32_t SCAN_LDS = XC_FILT_WORDS * 4u + SCAN_WAVES * Q_CAP * 8u;
constexpr uint32_t MAX_BUF = 1u << 20;   // longest single buffer accepted (1 MiB)
constexpr uint32_t MAX_DECL = MAX_BUF / XC_SEG + 2u;
constexpr uint32_t NONE = 0xFFFFFFFFu;
constexpr uint32_t DPOS_FLUSH = 0xFFFFFFFEu;  // declared by flush()

// event status (resolve / walk)
constexpr uint32_t ST_MISS = 0;  // lo32 matched, full hash did not
constexpr uint32_t ST_EQUAL = 1; // cache: hash present, bytes equal -> REF
constexpr uint32_t ST_COLL = 2;  // cache: hash present, bytes differ -> collision
constexpr uint32_t ST_MATCH = 3; // declaration set: hash present (val = buf<<32 | decl pos)

// token ops
constexpr uint32_t OP_END = 0, OP_EXTRACT = 1, OP_REF = 2;

// ctl words
enum : uint32_t {
    CTL_GREW = 0,
    CTL_FIRST_CROSS = 1,
    CTL_ERROR = 2,
    CTL_DENSE = 3,
    CTL_NEXTRACT = 4,
    CTL_NREF = 5,
    CTL_UNDO = 6,
    CTL_ABORT = 7,     // set by k_gate: a sub-batch needs the host (growth, cross-buffer, error)
    CTL_ABORT_SB = 8,  // ... and which one; every later pipeline kernel exits at once
    CTL_SHADOW = 9,    // a walk did not emit a predicted REF whose shadow the scan skipped
    CTL_SCAN_NEXT = 10,  // k_scan work counter (chunks handed out); k_resolve resets it
    CTL_COUNT = 11,      // the cache's segment count after the last k_alloc (for the host)
    CTL_DUPS = 12,       // k_emit entered hashes the cache held (a duplicate enter: the host replays)
    CTL_AFAIL = 13,      // an anchor-scanned sub-batch needs the exact scan
    CTL_ANCLESS = 14,    // (the cache's scratch words: ~slot of its first segment without an anchor)
    CTL_COLLS = 15,      // some walk recorded a collision lookup (the run's hits are more than its REFs)
    CTL_WORDS = 17       // (the last word: the host's publication sentinel)
};
constexpr uint32_t ERR_CAPACITY = 1, ERR_TOKENS = 2, ERR_DECLS = 4;  // (ERR_PACK_CAP = 8 below)

// One scan layer: per chunk a sorted sparse list (cnt < EV_CAP) or a dense bitmask.
struct Layer {
    uint32_t *cnt;   // [nchunks]  count | EV_DENSE
    uint32_t *pos;   // [nchunks * EV_CAP]  positions (relative to the buffer)
    uint32_t *stat;  // [nchunks * EV_CAP]
    uint64_t *h;     // [nchunks * EV_CAP]  full hash (resolved)
    uint64_t *val;   // [nchunks * EV_CAP]  table value (resolved)
    uint32_t *bits;  // [nchunks * chunk_len/32]
};

// The segment store: slots below dev_cap in HBM; the rest, the spill tier of a cache grown past the
// device's share, in pinned host memory mapped into the device's address space, chunks of
// 2^SPILL_SHIFT slots (host[k]: chunk k's device address).  Segments are written once (enter) and
// read by the compares of lookups that hit them, so spilled ones cost PCIe reads, not failures.
constexpr uint32_t SPILL_SHIFT = 16;
struct SegStore {
    uint8_t *dev;
    uint8_t *const *host;
    uint32_t dev_cap;
};

__device__ __forceinline__ uint8_t *seg_at(const SegStore &s, uint64_t i)
{
    if (i < s.dev_cap) return s.dev + i * XC_SEG;
    const uint64_t r = i - s.dev_cap;
    return s.host[r >> SPILL_SHIFT] + (r & ((1u << SPILL_SHIFT) - 1u)) * XC_SEG;
}

struct PlanDev {
    const uint8_t *in;
    const uint64_t *buf_off;
    const uint32_t *buf_len;
    uint32_t nb;
    const uint2 *chunks;       // (buffer, first position) per chunk
    const uint4 *chunk_desc;   // (first position, end position | more<<31 | more2<<30, arena offset lo, hi)
    const uint32_t *buf_chunk0;  // [nb+1]
    uint32_t chunk_len;
    Layer S, D;
    DevSet cache;
    SegStore segs;
    uint32_t *seg_count;
    uint32_t seg_cap;
    uint2 *undo;               // [seg_cap] (full slot, lo slot) of every enter()
    DevSet dset;
    const uint32_t *tok_base;  // [nb + 1]
    const uint32_t *hit_base;  // [nb + 1] k_hits' records: buffer b's at hit_base[b], len / 2048 + 1 + COLL_CAP + 1 words
    uint32_t *tok_cnt;
    uint32_t *tok_lb, *tok_le, *tok_seg, *tok_op, *tok_dpos;
    uint32_t *tok_known;       // EXTRACT hash known from a resolved event (no rehash needed)
    const uint32_t *blk_base;  // [nb + 1] first aligned-block index of the buffer
    const uint32_t *blk_buf;   // [blocks] buffer of every aligned block
    const uint2 *blk_grp;      // [groups] (buffer, first block) of every k_blockhash group
    uint64_t *blk_h;           // hash of every aligned 2048-byte block (k_blockhash)
    uint64_t *tok_h;
    uint32_t *buf_next;   // [nb] EXTRACT tokens of the buffer (walk)
    uint32_t *buf_nref;   // [nb] REF tokens of the buffer (walk)
    uint32_t *buf_slot;   // [nb] first cache slot of the buffer's declarations (k_alloc)
    uint8_t *out;
    const uint64_t *out_off;
    uint64_t *out_len;
    uint32_t *ctl;
    uint32_t *l2mix;  // level-2 filter of cache | predicted declarations (combined scan)
    // level-1 filter of cache | predicted declarations for the first round's scan, folded
    // (XC_FILT_WORDS >> fmix_fold words: word w is the OR of words w << fold .. (w + 1) << fold - 1
    // of the full filter, which is the word filt_word_n gives for the folded count) so that
    // small batches load a small image (k_clear_set builds it from the cache, block_predict adds)
    uint32_t *fmix;
    uint32_t fmix_fold;
    // k_blockpredict's verdict on aligned block g (global index), see blk_cached():
    //   cached slot + 1 (positive as int32): the block is in the cache, so the window ending at
    //     its last byte is a predicted REF.  REF shadows: the reference looks nothing up in the
    //     2047 positions after a REF (xcodec_encoder.cc:111-118 resets the hash), so the scan may
    //     skip the next block's windows and the walk verifies that the REF happened;
    //   0x80000000 | D slot: a predicted declaration, entered in D at that slot;
    //   0: no prediction (carried stream state).
    // k_resolve's first round takes the aligned windows' cache and D slots from here.
    uint32_t *blk_pref;
    // The block hashing's verdict on aligned block g against the cache of the time (entries below
    // the sub-batch's start count only: complete, and unchanged during the run): 0 none, else
    // (cached slot + 1) | (0x80000000 when the bytes differ).  k_resolve skips the 2048-byte
    // compare of a predicted REF whose slot it names.
    uint32_t *blk_cmp;
    uint32_t *sb_count;         // [sub-batches] the cache's count when the sub-batch started
    const uint32_t *chunk_blk;  // [nchunks] global index of the chunk's buffer's block 0
    // Stateful streams (xc_encode / xc_flush, xcodec_encoder.cc:60-201 across calls), or null
    // when every buffer is a fresh encoder's encode + flush.  stream_st[b] = {start, cand0,
    // flags, 0}: the buffer is the encoder's pending source_ (start bytes, whose window ends
    // were looked up by earlier calls, pending candidate cand0 or NONE) followed by the new
    // input; flags & SF_NOFLUSH: encode() only, the trailing candidate and literals stay
    // pending.  stream_res[b] = {base, cand}: the new source_ starts at base, the candidate.
    const uint4 *stream_st;
    uint2 *stream_res;
    // Lookups that hit the cache with different bytes (collisions, xcodec_encoder.cc:129-137), per
    // buffer, for the COSS tier's replay of lookup side effects (xc_coss.cpp), or null:
    // coll[b * COLL_CAP + i] = {window end, hash lo, hash hi, 0}, coll_cnt[b] = count (may exceed
    // COLL_CAP: then the host cannot replay the buffer).
    uint4 *coll;
    uint32_t *coll_cnt;
    // Anchor index.  anc_run: the run hashes anchors (k_blockhash: records and
    // block anchors) and indexes every segment it enters (k_emit); anc_scan: this sub-batch's
    // first-round scan takes its events from the index (k_ascan) instead of testing every window
    // end (k_scan).
    uint32_t anc_run, anc_scan;
    AncSet canc;               // the cache's anchor table (its filter: the cache's)
    AncSet danc;               // the declaration set's (its filter: amix)
    uint32_t *amix;            // anchor filter of cache | predicted declarations
    uint64_t *anc_of;          // [seg_cap] anchor key of every indexed segment (ANC_NONE: anchorless)
    uint32_t *aundo;           // [seg_cap] the anchor-table slot its insert took (NONE: none)
    uint64_t *blk_anc;         // [blocks] anchor key of every aligned block (k_blockhash)
    uint64_t *rec;             // [groups * REC_CAP] input anchors: fp << 19 | group position << 5 | run - 1
    uint32_t *rec_cnt;         // [groups] records (| REC_OVF: more than REC_CAP)
    uint4 *ainfo;              // [groups] first and last input anchor (group-relative, NONE: none), gaps
    uint2 *agap;               // [groups * AGAP_CAP] anchors >= 1986 apart inside the group (k_aprop's gaps)
    const uint32_t *buf_grp0;  // [nb + 1] first k_blockhash group of every buffer
    // the cache's word: ~slot of its first segment entered without an anchor (0: none; kept on
    // the device, as the emits after a run's early publication set it: k_ascan reads it)
    uint32_t *anc_bad;
};
constexpr uint32_t COLL_CAP = 16;
#ifndef XC_APROP_GROUPS
#define XC_APROP_GROUPS 2
#endif
constexpr uint32_t APROP_GROUPS = XC_APROP_GROUPS;  // k_aprop: block groups per workgroup
constexpr uint32_t BLK_GROUP = 8;    // aligned blocks per k_blockhash group (one wave)
constexpr uint32_t REC_CAP = 1024;  // anchor records per k_blockhash group (16 KiB; random data: ~256)
constexpr uint32_t REC_OVF = 0x80000000u;
constexpr uint32_t REC_GAP = 0x40000000u;  // the group may border a gap (k_aprop looks at its anchor record)
constexpr uint32_t AGAP_CAP = 4;   // gaps a k_blockhash group records (more: the exact scan)
constexpr uint32_t PROP_CAP = 64;  // anchor proposals a chunk keeps (more: the exact scan redoes the sub-batch)
__device__ __forceinline__ uint64_t rec_make(uint64_t fp, uint32_t pos, uint32_t n)
{
    return (fp << 19) | ((uint64_t)pos << 5) | (uint64_t)(n - 1u);
}
constexpr uint32_t SF_NOFLUSH = 1u;
constexpr uint32_t BP_DECL = 0x80000000u;  // blk_pref: predicted declaration | D slot
constexpr uint32_t BC_DIFF = 0x80000000u;  // blk_cmp: the block differs from the cached segment
__device__ __forceinline__ bool blk_cached(uint32_t pref) { return (int32_t)pref > 0; }
// A buffer with carried-over state (earlier positions already looked up, or a pending
// candidate): the aligned-block predictions and REF shadows do not apply to it.
__device__ __forceinline__ bool stream_carried(const PlanDev &P, uint32_t b)
{
    if (!P.stream_st) return false;
    const uint4 st = P.stream_st[b];
    return st.x != 0u || st.y != NONE;
}
// A buffer with no carried-over state: a fresh encoder's call, flushed at its end or not.
__device__ __forceinline__ bool stream_plain(const PlanDev &P, uint32_t b)
{
    if (!P.stream_st) return true;
    const uint4 st = P.stream_st[b];
    return st.x == 0u && st.y == NONE;
}
__device__ __forceinline__ bool stream_noflush(const PlanDev &P, uint32_t b)
{
    return P.stream_st && (P.stream_st[b].z & SF_NOFLUSH);
}

// kernel argument blocks (shared by xc_encode.hip and xc_runtime.hip)
// Pipeline kernels exit at once when the async sub-batch pipeline has been stopped.
__device__ __forceinline__ bool aborted(const PlanDev &P)
{
    return __builtin_amdgcn_readfirstlane((int)*(volatile const uint32_t *)&P.ctl[CTL_ABORT]) != 0;
}

struct ScanArgs {
    PlanDev P;
    Layer L;
    DevSet set;
    uint32_t ck_lo, ck_hi;
    uint32_t mode;  // ablation (timing only): 0 full, 1 no filter test, 2 loads + block sums only
    DevSet set2;    // optional second set tested in the same pass (predicted declarations)
    int has2;
    const uint32_t *l2;  // level-2 filter of set (| set2): one 4-byte L2 read per level-1 positive
    int shadow;       // skip the windows in the shadow of predicted REFs (P.blk_pref)
    uint32_t unit;    // chunks per work unit (the plan's scan granularity, <= SCAN_UNIT)
    const uint32_t *filt;  // level-1 image (set's filter, or P.fmix for set | set2), filt_words words
    uint32_t filt_words;
};
// k_ascan: one wave per chunk of [ck_lo, ck_hi), events from the anchor records
struct AScanArgs {
    PlanDev P;
    Layer L;
    uint32_t ck_lo, ck_hi;
    int shadow;
    uint32_t g_lo, g_hi;  // the sub-batch's k_blockhash groups (k_aprop)
    uint32_t *pcnt;       // [nchunks] proposals per chunk (zero between sub-batches)
    uint32_t *pq;         // [nchunks * PROP_CAP] their window ends
};
struct ResolveArgs {
    PlanDev P;
    Layer L;
    int dmode;  // 0: cache layer, 1: declaration layer, 2: cache + predicted declarations
    uint32_t ck_lo, ck_hi;
};
struct WalkArgs {
    PlanDev P;
    uint32_t j0, j1;
    int use_d;  // 0 on the first round (no declaration layer yet)
    int shadow; // the scan skipped predicted-REF shadows: verify every such REF was emitted
    uint32_t max_decl;  // >= declarations of any buffer (longest buffer / 2048 + 2)
    uint32_t waves;     // waves per buffer (workgroup) sharing the block-parallel walk's chunks
};
constexpr uint32_t WALK_WAVES_MAX = 4;
#ifndef XC_RES_WAVES
#define XC_RES_WAVES 1
#endif
constexpr uint32_t RES_WAVES = XC_RES_WAVES;  // k_resolve: chunks (waves) per workgroup
constexpr uint32_t MIX_FOLD_MAX = 4;  // (XC_FILT_WORDS >> 4 = 2304 words: still a multiple of 4)
// dynamic LDS of k_walk
__host__ __device__ constexpr uint32_t walk_lds_bytes(uint32_t max_decl) { return max_decl * 16u + 8u * (max_decl / 32u + 1u); }
struct DeclArgs {
    PlanDev P;
    uint32_t j0, j1;
    // k_blockhash on the side stream: the cache count below which entries are complete while it
    // runs (P.sb_count of the sub-batch the main stream is in); null: no block compares
    const uint32_t *limit;
    int nt;  // k_blockhash: the XC_ABL_BH timing-ablation bits (-DXC_ABLATIONS builds; 0 otherwise)
    // k_blockhash<false, true> with compares (limit): no anchor records for a block whose block and
    // the one before are cached (every proposal of them would fall on an aligned window or in a
    // predicted REF's shadow; the async pass's shadows are on: xc_plan.shadow)
    int drop_shadowed;
    // ... and below this count too (the early hashing of a run's first sub-batch: entries at or above
    // it were removed by a restore or truncation that the hashing may run before)
    uint32_t limit_cap;
};
struct EmitArgs {
    PlanDev P;
    uint32_t j0, j1;
    uint32_t gate_sb;  // k_alloc: async-pipeline gate for sub-batch gate_sb (NONE: no gate)
    // k_alloc / k_emit<.., true>: the control words also go here (mapped pinned host memory;
    // null: not wanted) when the gate stops the pass, and, on the pass's last sub-batch
    // (pub_final), once they are final
    uint32_t *ctl_host;
    const uint32_t *base;  // k_emit<.., true>: the cache count at the sub-batch's start (P.sb_count)
    uint32_t pub_final;
    uint32_t abl;  // timing ablations (XC_ABL_EMIT, diagnostics only: results are wrong): 1 no segment
                   // store, 2 no payload wire copy, 4 no cache inserts, 8 no payload loads or stores
    uint32_t split_ins;  // k_emit<.., false>: the cache enters ran in k_insert before it
};
// Sub-batches of at most this many buffers take k_alloc's work inside k_emit (every workgroup
// sums the buf_next of the buffers before it): one launch less on small batches.
#ifndef XC_EMIT_SLOTS_MAX
#define XC_EMIT_SLOTS_MAX 1024
#endif
constexpr uint32_t EMIT_SLOTS_MAX = XC_EMIT_SLOTS_MAX;
#ifndef XC_INSERT_SPLIT_MIN
#define XC_INSERT_SPLIT_MIN 8192
#endif
constexpr uint32_t INSERT_SPLIT_MIN = XC_INSERT_SPLIT_MIN;  // sub-batches of at least this many buffers enter the cache in k_insert

// Packing a sub-batch's encoded streams, in buffer order, into one caller buffer (pinned host
// memory written over PCIe by the kernel, or device memory): the end-to-end host path.
struct PackArgs {
    PlanDev P;
    uint32_t j0, j1;
    uint8_t *dst;        // device-visible pointer of the packed output
    uint64_t cap;        // its capacity
    uint64_t *total;     // running packed length (device)
    uint64_t *pos;       // [nb] packed offset of every buffer (device)
};
constexpr uint32_t ERR_PACK_CAP = 8;

template <int MODE> __global__ void k_scan(ScanArgs a);
template <uint32_t NW, bool SLOTS, int INS> __global__ void k_emit(EmitArgs a);
template <uint32_t NW, bool SLOTS, int INS> __global__ void k_emit1(EmitArgs a);
__global__ void k_pack_offsets(PackArgs a);
__global__ void k_pack_copy(PackArgs a);
__global__ void k_resolve(ResolveArgs a);
__global__ void k_walk(WalkArgs a);
template <bool PREDICT, bool ANC> __global__ void k_blockhash(DeclArgs a);
__global__ void k_aprop(AScanArgs a);
__global__ void k_aevents(AScanArgs a);
__global__ void k_anc_backfill(PlanDev P, uint32_t from, uint32_t to, uint32_t *ctl);
__global__ void k_anc_undo(AncSet s, const uint32_t *aundo, uint32_t from, uint32_t to, uint4 *filt, const uint4 *snap,
                           uint32_t *word, uint32_t value);
__global__ void k_anc_rehash(AncSet to, const uint64_t *anc_of, uint32_t n, uint32_t *aslot, uint32_t *owner);
__global__ void k_anc_owner(uint32_t *aundo, const uint32_t *aslot, uint32_t n, const uint32_t *owner);
__global__ void k_tailcheck(PlanDev P, uint32_t nb, uint32_t *tcnt, uint4 *tlist);
__global__ void k_tailfinal(PlanDev P, uint32_t nb, uint32_t *tcnt, const uint4 *tlist);
__global__ void k_blockpredict(DeclArgs a);
__global__ void k_or_words(uint4 *dst, const uint4 *a, const uint4 *b, uint32_t n);
__global__ void k_alloc(EmitArgs a);
template <bool ANC> __global__ void k_insert(EmitArgs a);
__global__ void k_clear_set(DevSet s, uint32_t n_lo, uint32_t n_full, uint4 *l2mix, const uint4 *cache_l2,
                            uint32_t *fmix, const uint32_t *cache_filt, uint32_t fold, const uint32_t *count,
                            uint32_t *count_out, uint32_t *ctl_zero, AncSet danc, uint4 *amix, const uint4 *cache_afilt);
__global__ void k_hash_segments(const uint8_t *segs, uint64_t n, uint64_t *out);
__global__ void k_window_hashes(const uint8_t *in, uint32_t n, uint64_t *out);
__global__ void k_undo(DevSet cache, const uint2 *undo, uint32_t from, uint32_t to);
__global__ void k_undo_dev(DevSet cache, const uint2 *undo, uint32_t from, const uint32_t *count, uint32_t cap,
                           const uint4 *snap_filt, const uint4 *snap_l2, const uint32_t *snap_lo_zero);
__global__ void k_undo_known(DevSet cache, const uint2 *undo, uint32_t from, uint32_t to, uint32_t *count,
                             const uint4 *snap_filt, const uint4 *snap_l2, const uint32_t *snap_lo_zero);
__global__ void k_rehash(DevSet from, DevSet to, uint2 *undo, uint32_t *lo_owner, uint32_t keep, int drop_dead);
__global__ void k_rehash_owner(uint2 *undo, uint32_t n, const uint32_t *lo_owner);
__global__ void k_enter_one(PlanDev P, uint64_t h, const uint8_t *seg);
__global__ void k_enter_bulk(PlanDev P, const uint64_t *h, const uint8_t *segs, uint32_t n, uint32_t first);
__global__ void k_kill(DevSet cache, const uint64_t *h, uint32_t n);
__global__ void k_find(DevSet cache, const uint64_t *h, uint64_t *val, uint32_t n);
__global__ void k_hits(PlanDev P, uint64_t *out);
__global__ void k_hits_out(const uint64_t *stage, uint64_t *host, const uint32_t *hit_base, uint32_t nb);
__global__ void k_setval(DevSet cache, uint64_t h, uint64_t val);
__global__ void k_lookup_one(PlanDev P, uint64_t h, uint8_t *out, uint32_t *found);
__global__ void k_selftest(uint32_t *err);

}  // namespace xc
