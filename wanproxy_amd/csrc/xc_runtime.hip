// xc_runtime.hip — host runtime behind include/xcodec_hip.h.
//
// Owns device contexts, the device-resident segment cache (XCodecMemoryCache,
// xcodec/xcodec_cache.h:162-211) and batch plans, and sequences the encode pipeline of
// xc_encode.hip.  The reference's order semantics (one cache shared by buffers fed in
// index order, xcodec/xcodec_filter.cc:146-157) are kept by committing a batch prefix
// only after every buffer in it is known not to depend on an earlier buffer's new
// declarations (see DESIGN.md "Sequential semantics").
#include <hip/hip_runtime.h>

#include <sched.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <chrono>
#include <cstring>
#include <deque>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/xcodec_hip.h"
#include "xc_kernels.h"
#include "xc_env.h"


using namespace xc;

static thread_local std::string g_err;

static int fail(int code, const std::string &msg)
{
    g_err = msg;
    return code;
}

#define HIPCHK(x)                                                                           \
    do {                                                                                    \
        hipError_t e_ = (x);                                                                \
        if (e_ != hipSuccess)                                                               \
            return fail(XC_EDEVICE, std::string(#x) + ": " + hipGetErrorString(e_));       \
    } while (0)

extern "C" const char *xc_last_error(void) { return g_err.c_str(); }

// ------------------------------------------------------------------ allocation ----------
// Caching allocator for device and pinned host memory.  Plans, declaration sets and the
// host-to-host entry points allocate and free dozens of arrays per call; hipMalloc/hipFree (and
// hipHostMalloc for staging) cost far more than the work of a small call.  Freed blocks are kept
// per (device, kind) in a best-fit pool (a block serves requests down to half its size) and
// reused; they go back to HIP only at process exit.
namespace {
struct Pool {
    std::mutex mu;
    std::multimap<std::pair<int, size_t>, void *> free_;  // (device | host flag, size) -> block
    std::unordered_map<void *, std::pair<int, size_t>> size_;
};
Pool &pool()
{
    static Pool *p = new Pool();  // never destroyed: blocks may be released after static teardown
    return *p;
}
size_t size_class(size_t n)
{
    if (n <= 4096) return 4096;
    if (n <= (64u << 20)) {
        size_t c = 4096;
        while (c < n) c <<= 1;
        return c;
    }
    return (n + (2u << 20) - 1) & ~(size_t)((2u << 20) - 1);
}
constexpr int HOST_KIND = 1 << 20;  // pinned host blocks share the pool under this key
}  // namespace

static hipError_t pool_alloc(void **out, size_t n, bool host)
{
    int dev = 0;
    if (!host && hipGetDevice(&dev) != hipSuccess) return hipErrorInvalidDevice;
    const int kind = host ? HOST_KIND : dev;
    const size_t c = size_class(std::max<size_t>(n, 1));
    Pool &P = pool();
    {
        std::lock_guard<std::mutex> g(P.mu);
        auto it = P.free_.lower_bound({kind, c});
        if (it != P.free_.end() && it->first.first == kind && it->first.second <= 2 * c) {
            *out = it->second;
            P.free_.erase(it);
            return hipSuccess;
        }
    }
    void *ptr = nullptr;
    hipError_t e = host ? hipHostMalloc(&ptr, c, hipHostMallocMapped) : hipMalloc(&ptr, c);
    if (e != hipSuccess) {
        // release cached blocks of this kind and retry once
        std::vector<void *> drop;
        {
            std::lock_guard<std::mutex> g(P.mu);
            for (auto it = P.free_.begin(); it != P.free_.end();) {
                if (it->first.first == kind) {
                    drop.push_back(it->second);
                    P.size_.erase(it->second);
                    it = P.free_.erase(it);
                } else {
                    ++it;
                }
            }
        }
        for (void *q : drop) host ? (void)hipHostFree(q) : (void)hipFree(q);
        e = host ? hipHostMalloc(&ptr, c, hipHostMallocMapped) : hipMalloc(&ptr, c);
        if (e != hipSuccess) return e;
    }
    std::lock_guard<std::mutex> g(P.mu);
    P.size_[ptr] = {kind, c};
    *out = ptr;
    return hipSuccess;
}

static void pool_free(void *ptr)
{
    if (!ptr) return;
    Pool &P = pool();
    std::lock_guard<std::mutex> g(P.mu);
    auto it = P.size_.find(ptr);
    if (it == P.size_.end()) return;  // not from the pool
    P.free_.insert({it->second, ptr});
}

// Device / pinned-host arrays of T (the pool's hipMalloc / hipFree).
template <class T>
static hipError_t dmalloc(T **p, size_t bytes)
{
    return pool_alloc((void **)p, bytes, false);
}
static hipError_t dfree(void *p)
{
    pool_free(p);
    return hipSuccess;
}
static hipError_t hmalloc(void **p, size_t bytes) { return pool_alloc(p, bytes, true); }

// Host copies into / out of the pinned arenas, split over a few threads when a batch is large (one
// core's memcpy, ~10 GB/s, would otherwise bound a turn's batch of connections).
struct HostCopy {
    uint8_t *dst;
    const uint8_t *src;
    uint64_t n;
};
static void host_copies(const std::vector<HostCopy> &cp)
{
    uint64_t total = 0;
    for (const HostCopy &c : cp) total += c.n;
    const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
    const unsigned nt = (unsigned)std::min<uint64_t>({8, hw, total >> 21});  // >= 2 MiB a thread
    if (nt <= 1) {
        for (const HostCopy &c : cp)
            if (c.n) memcpy(c.dst, c.src, c.n);
        return;
    }
    // contiguous byte ranges of the concatenated copies, one a thread
    auto work = [&](unsigned t) {
        const uint64_t lo = total * t / nt, hi = total * (t + 1) / nt;
        uint64_t at = 0;
        for (const HostCopy &c : cp) {
            const uint64_t a = std::max(lo, at), b = std::min(hi, at + c.n);
            if (a < b) memcpy(c.dst + (a - at), c.src + (a - at), b - a);
            at += c.n;
            if (at >= hi) break;
        }
    };
    std::vector<std::thread> th;
    for (unsigned t = 1; t < nt; t++) th.emplace_back(work, t);
    work(0);
    for (std::thread &x : th) x.join();
}

// For xc_decode.hip.
extern "C" int xc__dalloc(void **p, uint64_t bytes)
{
    return pool_alloc(p, bytes, false) == hipSuccess ? XC_OK : fail(XC_ENOMEM, "device allocation failed");
}
extern "C" int xc__halloc(void **p, uint64_t bytes)
{
    return pool_alloc(p, bytes, true) == hipSuccess ? XC_OK : fail(XC_ENOMEM, "pinned allocation failed");
}
extern "C" void xc__pfree(void *p) { pool_free(p); }


// ------------------------------------------------------------------ context ----------
struct xc_ctx {
    int dev;
    hipStream_t stream;
    hipStream_t side = nullptr;  // block hashing ahead of the scans (shared by the plans)
    hipStream_t copy = nullptr;  // host-path input copies
    int n_cu;
    uint32_t *d_scratch;  // small device scratch (flags)
    uint8_t *d_seg;       // one segment of device scratch
};

static int set_dev(xc_ctx *ctx)
{
    HIPCHK(hipSetDevice(ctx->dev));
    return XC_OK;
}

extern "C" int xc_device_count(int *n)
{
    if (!n) return fail(XC_EINVAL, "null");
    HIPCHK(hipGetDeviceCount(n));
    return XC_OK;
}

extern "C" int xc_ctx_create(int dev, xc_ctx **out)
{
    if (!out) return fail(XC_EINVAL, "null");
    int n = 0;
    HIPCHK(hipGetDeviceCount(&n));
    if (dev < 0 || dev >= n) return fail(XC_EINVAL, "no such device");
    HIPCHK(hipSetDevice(dev));
    xc_ctx *c = new xc_ctx();
    c->dev = dev;
    // (at the default priority: the context stream high and the side stream low starved the block
    // hashing, cfg5 -7.5 %)
    HIPCHK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    hipDeviceProp_t prop;
    HIPCHK(hipGetDeviceProperties(&prop, dev));
    c->n_cu = prop.multiProcessorCount;
    HIPCHK(dmalloc(&c->d_scratch, 4096));
    HIPCHK(dmalloc(&c->d_seg, 4096));
    *out = c;
    return XC_OK;
}

extern "C" int xc_ctx_destroy(xc_ctx *ctx)
{
    if (!ctx) return XC_OK;
    hipSetDevice(ctx->dev);
    hipStreamSynchronize(ctx->stream);
    dfree(ctx->d_scratch);
    dfree(ctx->d_seg);
    if (ctx->side) { hipStreamSynchronize(ctx->side); hipStreamDestroy(ctx->side); }
    if (ctx->copy) { hipStreamSynchronize(ctx->copy); hipStreamDestroy(ctx->copy); }
    hipStreamDestroy(ctx->stream);
    delete ctx;
    return XC_OK;
}

extern "C" void *xc_ctx_stream(xc_ctx *ctx) { return ctx ? (void *)ctx->stream : nullptr; }

extern "C" int xc_ctx_device(xc_ctx *ctx, int *dev)
{
    if (!ctx || !dev) return fail(XC_EINVAL, "null");
    *dev = ctx->dev;
    return XC_OK;
}

extern "C" int xc_ctx_sync(xc_ctx *ctx)
{
    if (!ctx) return fail(XC_EINVAL, "null");
    HIPCHK(hipSetDevice(ctx->dev));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    return XC_OK;
}

// ------------------------------------------------------------------ sets ----------
static uint32_t pow2_at_least(uint64_t x, uint32_t minimum)
{
    uint64_t p = minimum;
    while (p < x) p <<= 1;
    return (uint32_t)p;
}

struct HostSet {
    DevSet d{};
    AncSet a{};  // the anchor table: keys sized like the full table; a cache's
                 // own filter, a declaration set's the plan's combined one (amix)
    uint32_t n_lo = 0, n_full = 0;
    int alloc(uint64_t entries, bool own_afilt)
    {
        n_full = pow2_at_least(entries * 2, 1024);
        n_lo = pow2_at_least(entries * 4, 1024);
        // (slot hashes use 27 bits: lo_slot / key_slot in xc_device.h)
        if (n_full > (1u << 27) || n_lo > (1u << 27)) return fail(XC_EINVAL, "set too large");
        HIPCHK(dmalloc(&d.filt, XC_FILT_WORDS * 4));
        HIPCHK(dmalloc(&d.l2, (size_t)XC_L2_WORDS * 8));
        HIPCHK(dmalloc(&d.lo_keys, (size_t)n_lo * 4));
        HIPCHK(dmalloc(&d.lo_zero, 4));
        HIPCHK(dmalloc(&d.keys, (size_t)n_full * 8));
        HIPCHK(dmalloc(&d.vals, (size_t)n_full * 8));
        d.lo_mask = n_lo - 1;
        d.mask = n_full - 1;
        HIPCHK(dmalloc(&a.keys, (size_t)n_full * 8));
        if (own_afilt) HIPCHK(dmalloc(&a.filt, (size_t)ANC_FILT_WORDS * 4));
        a.mask = n_full - 1;
        return XC_OK;
    }
    int clear(hipStream_t s)
    {
        HIPCHK(hipMemsetAsync(d.filt, 0, XC_FILT_WORDS * 4, s));
        HIPCHK(hipMemsetAsync(d.l2, 0, (size_t)XC_L2_WORDS * 8, s));
        HIPCHK(hipMemsetAsync(d.lo_keys, 0, (size_t)n_lo * 4, s));
        HIPCHK(hipMemsetAsync(d.lo_zero, 0, 4, s));
        HIPCHK(hipMemsetAsync(d.keys, 0xFF, (size_t)n_full * 8, s));
        HIPCHK(hipMemsetAsync(d.vals, 0xFF, (size_t)n_full * 8, s));
        HIPCHK(hipMemsetAsync(a.keys, 0xFF, (size_t)n_full * 8, s));
        if (a.filt) HIPCHK(hipMemsetAsync(a.filt, 0, (size_t)ANC_FILT_WORDS * 4, s));
        return XC_OK;
    }
    void release(bool own_afilt)
    {
        dfree(d.filt);
        dfree(d.l2);
        dfree(d.lo_keys);
        dfree(d.lo_zero);
        dfree(d.keys);
        dfree(d.vals);
        dfree(a.keys);
        if (own_afilt) dfree(a.filt);
        d = DevSet{};
        a = AncSet{};
    }
};

// ------------------------------------------------------------------ cache ----------
// The memory cache's recent window and duplicate enters (xc_memcache.cpp).
struct xc_memmodel;
extern "C" xc_memmodel *xc__mem_new(xc_cache *c, xc_ctx *ctx);
extern "C" void xc__mem_free(xc_memmodel *m);
extern "C" xc_memmodel *xc__mem_clone(const xc_memmodel *m);
extern "C" int xc__mem_restore(xc_memmodel *m, const xc_memmodel *snap);
extern "C" void xc__mem_hits(xc_memmodel *m, const uint64_t *h, uint64_t n, int complete);
extern "C" void xc__mem_hits_run(xc_memmodel *m, const uint64_t *h, const uint32_t *tok_base, uint32_t stride,
                                 uint32_t nb);
extern "C" int xc__mem_live(const xc_memmodel *m);
extern "C" uint64_t xc__mem_extra(const xc_memmodel *m);
extern "C" int xc__mem_encode_batch(xc_memmodel *m, const uint8_t *in, const uint64_t *in_off, const uint64_t *in_len,
                                    uint64_t nbuf, uint8_t *out, const uint64_t *out_off, const uint64_t *out_cap,
                                    uint64_t *out_len);
extern "C" int xc__mem_encode_gather(xc_memmodel *m, uint64_t nbuf, const uint8_t *const *head,
                                     const uint64_t *head_len, const uint8_t *const *tail, const uint64_t *tail_len,
                                     const uint64_t *start, const int64_t *cand, const uint32_t *flags,
                                     uint64_t *rbase, int64_t *rcand,
                                     int (*take)(void *ctx, uint64_t i, const uint8_t *out, uint64_t out_len,
                                                 const uint8_t *in),
                                     void *ctx);
extern "C" int xc__mem_lookup(xc_memmodel *m, uint64_t h, uint8_t *out, int *found);
extern "C" int xc__mem_enter(xc_memmodel *m, uint64_t h, const uint8_t *seg, int *dup);
// decode plans (xc_decode.hip): a finished run's lookup hits, in the reference's order
extern "C" int xc__dplan_hits(void *dplan, uint64_t **hits, uint64_t *n, int *complete);
// A run on the memory cache needs the replay engine (xc_memcache.cpp): a duplicated hash may
// answer with other bytes than the device holds, or the run entered a hash twice.
constexpr int XC__SLOW = -1000;

struct xc_cache {
    xc_ctx *ctx;
    uint64_t cap;      // segment slots (the tables are sized for them)
    // the lowest count a removal (a restore, a truncation, an eviction) left since the last run's
    // submit: a plan's next early hashing compares only with entries below it (they survived)
    uint32_t removed_floor = 0xFFFFFFFFu;
    // host-path plans of small batches kept for the next call with the same buffer lengths (a
    // proxy's one-read consume, xcodec_filter.cc:146-157: its plan's ~15 uploads and allocations
    // cost more than the encode); plan_acquire / plan_release, oldest dropped past PLAN_POOL_MAX
    std::vector<xc_plan *> plan_pool;
    HostSet set;
    uint8_t *segs;     // device: the first dev_cap slots
    uint64_t dev_cap = 0;
    uint64_t dev_limit = 0;           // the device's share of the slots (SEG_DEV_MAX; a test hook lowers it)
    std::vector<uint8_t *> spill;     // the spill tier: pinned host chunks of 2^SPILL_SHIFT slots
    uint8_t **d_spill = nullptr;      // device: their device addresses
    uint32_t *count;   // device
    uint2 *undo;       // device [cap]
    uint32_t *ctl;     // device scratch ctl for single-op kernels
    // snapshot
    bool has_snap = false;
    uint32_t snap_count = 0;
    uint32_t snap_gen = 0;  // gen at the snapshot: a rebuild since re-placed its keys
    uint32_t *snap_filt = nullptr;
    uint32_t *snap_lo_zero = nullptr;
    uint32_t *snap_count_dev = nullptr;
    uint32_t *snap_l2 = nullptr;
    // the device's segment count as the host last learned it (a run's control words), or -1:
    // lets a restore write the count itself instead of copying it on the device
    int64_t host_count = -1;
    uint32_t gen = 0;  // bumped when the cache grows (its arrays move): plans refresh their copies
    const void *busy = nullptr;  // the plan whose submitted run is in flight on this cache
    // the plan whose run was the last thing to change the cache (nothing else wrote segments or
    // tables since): its next run may hash its first sub-batch ahead (xc_plan_set_input_ready)
    const void *last_plan = nullptr;
    // the reference's recent window and duplicate enters (null: a COSS tier's mirror, whose Store
    // has its own), its copy at the snapshot, the run whose lookup hits it has not replayed yet
    // (one encode or decode plan: consumed before the next operation that needs the order, dropped
    // by a restore), and whether the replay engine drives the cache (no hooks then)
    xc_memmodel *mem = nullptr;
    xc_memmodel *mem_snap = nullptr;
    void *pend_dec = nullptr;
    // The encoder runs' lookup hits for the window model, in run order: k_hits
    // packs a finished run's hits into a device slot behind the run on the context stream,
    // k_hits_out copies them into the slot's pinned memory on hl_stream, and the host replays them
    // while the next run works (its wait) or before the next operation whose answer depends on the
    // window (cache_settle); a restore drops them.  Two slots: the next run packs into the other.
    struct HitSlot {
        uint64_t *d = nullptr;   // device: buffer b's record at rec_base[b] (the plan's hit_base), count first
        uint64_t *h = nullptr;   // pinned host copy (same layout), hd its device address
        uint64_t *hd = nullptr;
        uint32_t *dtb = nullptr;  // device copy of the run's hit_base (the copy outlives the plan)
        size_t cap = 0, tb_cap = 0;
        hipEvent_t ev = nullptr;  // the copy into h is complete
        std::vector<uint32_t> rec_base;
        uint32_t nb = 0;
        uint32_t next_b = 0;  // replay progress: the first buffer not replayed yet
        uint64_t serial = 0;  // the plan whose layout dtb / rec_base hold
        bool copying = false;    // an asynchronous copy into h was issued and not seen complete
        bool host_sync = false;  // written into h on the context stream: complete once it is synchronised
    } hl[2];
    std::deque<int> hl_fifo;  // slots whose hits are not replayed yet, oldest first
    // a finished run whose hits are not packed yet: packed (k_hits, its copy) at the next operation
    // on the cache, before anything can overwrite its token arrays; a restore drops it unpacked
    // (the bench's restore-per-step headline then pays nothing for the window)
    xc_plan *hl_pend = nullptr;
    int hl_next = 0;
    hipStream_t hl_stream = nullptr;
    hipEvent_t hl_packed = nullptr;
    uint64_t hl_runs = 0, hl_hits = 0;
    double hl_sec = 0;  // host time spent replaying
    int engine = 0;
    // anchor index: segments [0, anc_upto) are in it (runs without anchors and
    // other enter paths append behind it: a backfill catches up before an anchor run); anc_bad:
    // the first segment without an anchor (NONE: none), which keeps the cache on the exact scan
    uint64_t *anc_of = nullptr;  // device [cap]
    uint32_t *aundo = nullptr;   // device [cap]
    uint32_t anc_upto = 0, anc_bad = NONE;
    uint32_t *snap_afilt = nullptr;
    uint32_t snap_anc_upto = 0;
    bool anc_dirty = false;  // entries indexed since the snapshot (a restore takes them out)
    uint32_t anc_bad_word = 0;  // (host source of the device word's reset)
};

static int cache_settle(xc_cache *c);
static int hits_flush(xc_cache *c);

// A run submitted on the cache and not finished (xc_encode_submit without poll/wait): every other
// operation on the cache would read a partial count, or move the arrays that run's kernels (and
// its host-side redo) still use.
static int cache_busy(const xc_cache *c, const void *owner = nullptr)
{
    if (c && c->busy && c->busy != owner)
        return fail(XC_EBUSY, "a run on this cache is in flight (xc_encode_poll / xc_encode_wait first)");
    return XC_OK;
}

// The reference's memory cache is unbounded (xcodec/xcodec_cache.h:164,182-188).  The device cache
// starts at the capacity it was created with and grows (cache_reserve) before any run that could
// exceed it.  Its tables (keys, lo32 set, undo log) stay in HBM for up to CAP_MAX segments; the
// segment bytes fill SEG_DEV_MAX slots of HBM (64 GiB) and then spill to pinned host memory
// (SegStore, xc_kernels.h), so a cache outgrows the device's share instead of failing.
static const uint64_t CAP_MAX = 1ull << 28;      // 512 GiB of segments: tables of ~12 GB
static const uint64_t SEG_DEV_MAX = 1ull << 25;  // segment slots in HBM
static const uint64_t SPILL_CHUNK = 1ull << SPILL_SHIFT;

static SegStore cache_segstore(const xc_cache *c)
{
    return SegStore{c->segs, c->d_spill, (uint32_t)c->dev_cap};
}

// Spill chunks for every slot from `base` (the device part's size: it never changes once chunks
// exist) up to ncap (pinned, mapped into the device's address space; device addresses in d_spill).
static int cache_spill_to(xc_cache *c, uint64_t base, uint64_t ncap)
{
    if (!c->spill.empty() && base != c->dev_cap) return fail(XC_EDEVICE, "spill tier moved");
    const uint64_t need = ncap > base ? (ncap - base + SPILL_CHUNK - 1) / SPILL_CHUNK : 0;
    if (need <= c->spill.size()) return XC_OK;
    if (!c->d_spill && dmalloc(&c->d_spill, (size_t)(CAP_MAX / SPILL_CHUNK) * sizeof(uint8_t *)) != hipSuccess)
        return fail(XC_ENOMEM, "device allocation failed");
    std::vector<uint8_t *> dptr;
    for (uint64_t k = c->spill.size(); k < need; k++) {
        void *h = nullptr, *d = nullptr;
        if (hipHostMalloc(&h, SPILL_CHUNK * XC_SEG + 4096, hipHostMallocMapped) != hipSuccess)
            return fail(XC_ENOMEM, "host memory for the cache's spill tier exhausted");
        if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess) {
            hipHostFree(h);
            return fail(XC_EDEVICE, "spill chunk not mapped");
        }
        c->spill.push_back((uint8_t *)h);
        dptr.push_back((uint8_t *)d);
    }
    const size_t k0 = c->spill.size() - dptr.size();
    HIPCHK(hipMemcpy(c->d_spill + k0, dptr.data(), dptr.size() * sizeof(uint8_t *), hipMemcpyHostToDevice));
    return XC_OK;
}

// (tests) The device's share of the segment slots: later growth spills past max(n, the current
// device part) to host memory.
extern "C" int xc__cache_set_dev_limit(xc_cache *c, uint64_t n)
{
    if (!c || n == 0) return fail(XC_EINVAL, "bad device limit");
    c->dev_limit = std::min<uint64_t>(n, SEG_DEV_MAX);
    return XC_OK;
}

// (tests) The segment slots in HBM and in the spill tier.
extern "C" int xc__cache_tiers(xc_cache *c, uint64_t *dev_slots, uint64_t *spill_slots)
{
    if (!c || !dev_slots || !spill_slots) return fail(XC_EINVAL, "null");
    *dev_slots = c->dev_cap;
    *spill_slots = c->spill.size() * SPILL_CHUNK;
    return XC_OK;
}

extern "C" void xc__cache_count_unknown(xc_cache *c)
{
    if (c) c->host_count = -1;
}
// The host's copy of the count (-1: unknown), and setting it after a run that knows it.
extern "C" int64_t xc__cache_host_count(xc_cache *c) { return c ? c->host_count : -1; }
extern "C" void xc__cache_set_host_count(xc_cache *c, int64_t n)
{
    if (c) c->host_count = n;
}

static PlanDev cache_plandev(xc_cache *c)
{
    PlanDev P{};
    P.cache = c->set.d;
    P.segs = cache_segstore(c);
    P.seg_count = c->count;
    P.seg_cap = (uint32_t)c->cap;
    P.undo = c->undo;
    P.ctl = c->ctl;
    P.canc = c->set.a;
    P.anc_of = c->anc_of;
    P.aundo = c->aundo;
    P.anc_bad = c->ctl + CTL_ANCLESS;
    return P;
}

extern "C" int xc_cache_create(xc_ctx *ctx, uint64_t cap, xc_cache **out)
{
    if (!ctx || !out || cap == 0 || cap > CAP_MAX) return fail(XC_EINVAL, "bad cache capacity");
    int rc = set_dev(ctx);
    if (rc) return rc;
    xc_cache *c = new xc_cache();
    c->ctx = ctx;
    c->cap = cap;
    c->dev_limit = SEG_DEV_MAX;
    c->dev_cap = std::min(cap, c->dev_limit);
    if ((rc = c->set.alloc(cap, true))) return rc;
    HIPCHK(dmalloc(&c->segs, (size_t)c->dev_cap * XC_SEG + 4096));
    if ((rc = cache_spill_to(c, c->dev_cap, cap))) return rc;
    HIPCHK(dmalloc(&c->count, 4));
    HIPCHK(dmalloc(&c->undo, (size_t)cap * sizeof(uint2)));
    HIPCHK(dmalloc(&c->anc_of, (size_t)cap * 8));
    HIPCHK(dmalloc(&c->aundo, (size_t)cap * 4));
    HIPCHK(dmalloc(&c->snap_afilt, (size_t)ANC_FILT_WORDS * 4));
    HIPCHK(dmalloc(&c->ctl, CTL_WORDS * 4));
    HIPCHK(dmalloc(&c->snap_filt, XC_FILT_WORDS * 4));
    HIPCHK(dmalloc(&c->snap_lo_zero, 4));
    HIPCHK(dmalloc(&c->snap_count_dev, 4));
    HIPCHK(dmalloc(&c->snap_l2, (size_t)XC_L2_WORDS * 8));
    if ((rc = c->set.clear(ctx->stream))) return rc;
    HIPCHK(hipMemsetAsync(c->count, 0, 4, ctx->stream));
    HIPCHK(hipMemsetAsync(c->ctl, 0, CTL_WORDS * 4, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    if (!(c->mem = xc__mem_new(c, ctx))) return fail(XC_ENOMEM, "host allocation failed");
    *out = c;
    return XC_OK;
}

// A COSS tier's device mirror (xc_coss.cpp): its Store replays every lookup, recent window included.
extern "C" void xc__cache_untracked(xc_cache *c)
{
    if (!c) return;
    xc__mem_free(c->mem);
    c->mem = nullptr;
}

// The replay engine drives the cache (xc_memcache.cpp): the hooks stand aside.
extern "C" void xc__cache_engine(xc_cache *c, int on)
{
    if (c) {
        c->engine = on;
        c->last_plan = nullptr;
    }
}

static void plan_pool_drain(xc_cache *c);

extern "C" int xc_cache_destroy(xc_cache *c)
{
    if (!c) return XC_OK;
    hipSetDevice(c->ctx->dev);
    plan_pool_drain(c);
    hipDeviceSynchronize();  // pooled memory is reused at once: every stream must be done with it
    c->set.release(true);
    dfree(c->anc_of);
    dfree(c->aundo);
    dfree(c->snap_afilt);
    dfree(c->segs);
    for (uint8_t *h : c->spill) hipHostFree(h);
    dfree(c->d_spill);
    dfree(c->count);
    dfree(c->undo);
    dfree(c->ctl);
    dfree(c->snap_filt);
    dfree(c->snap_lo_zero);
    dfree(c->snap_count_dev);
    dfree(c->snap_l2);
    xc__mem_free(c->mem);
    xc__mem_free(c->mem_snap);
    for (auto &sl : c->hl) {
        dfree(sl.d);
        dfree(sl.dtb);
        pool_free(sl.h);
        if (sl.ev) hipEventDestroy(sl.ev);
    }
    if (c->hl_packed) hipEventDestroy(c->hl_packed);
    if (c->hl_stream) hipStreamDestroy(c->hl_stream);
    delete c;
    return XC_OK;
}

static int cache_count_host(xc_cache *c, uint32_t *n)
{
    HIPCHK(hipMemcpyAsync(n, c->count, 4, hipMemcpyDeviceToHost, c->ctx->stream));
    HIPCHK(hipStreamSynchronize(c->ctx->stream));
    return XC_OK;
}

// The anchor index serves a memory cache (a COSS mirror's lookups all go through
// its Store); its segments without an anchor (anc_bad) are found through the gap windows.
static bool cache_anc_ok(const xc_cache *c) { return c->mem && !c->engine; }

// Index the segments entered since the index last caught up (the count known on the host).
static int cache_anc_catch_up(xc_cache *c)
{
    const uint32_t cnt = (uint32_t)std::min<int64_t>(c->host_count, (int64_t)c->cap);
    if (c->host_count < 0 || c->anc_upto >= cnt) return XC_OK;
    hipStream_t s = c->ctx->stream;
    const uint32_t n = cnt - c->anc_upto;
    hipLaunchKernelGGL(k_anc_backfill, dim3(std::min<uint32_t>((n + 3) / 4, 8192)), dim3(256), 0, s, cache_plandev(c),
                       c->anc_upto, cnt, c->ctl);
    HIPCHK(hipGetLastError());
    uint32_t bad = 0;
    HIPCHK(hipMemcpyAsync(&bad, c->ctl + CTL_ANCLESS, 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    if (bad) c->anc_bad = std::min(c->anc_bad, ~bad);
    c->anc_upto = cnt;
    c->anc_dirty = true;
    return XC_OK;
}

// After a restore: the device's anchorless word as of the snapshot (a segment without an anchor
// below the snapshot's count was learned by the snapshot's catch-up).  copy: written by a copy here,
// else by the k_anc_undo launched with the value.
static int cache_anc_bad_reset(xc_cache *c, bool copy = true)
{
    if (c->anc_bad >= c->snap_count) c->anc_bad = NONE;
    c->anc_bad_word = c->anc_bad == NONE ? 0u : ~c->anc_bad;
    if (copy) HIPCHK(hipMemcpyAsync(c->ctl + CTL_ANCLESS, &c->anc_bad_word, 4, hipMemcpyHostToDevice, c->ctx->stream));
    return XC_OK;
}

// A restore's part of the anchor index: the keys of the segments indexed since the snapshot out,
// its filter back (enqueued).
static int cache_anc_restore(xc_cache *c)
{
    if (!c->anc_dirty) return XC_OK;
    hipStream_t s = c->ctx->stream;
    const uint32_t to = std::max(c->anc_upto, c->snap_count);
    const uint32_t n = std::max<uint32_t>(to - c->snap_count, ANC_FILT_WORDS / 4);
    cache_anc_bad_reset(c, false);
    hipLaunchKernelGGL(k_anc_undo, dim3(std::min<uint32_t>((n + 255) / 256, 2048)), dim3(256), 0, s, c->set.a,
                       (const uint32_t *)c->aundo, c->snap_count, to, (uint4 *)c->set.a.filt, (const uint4 *)c->snap_afilt,
                       c->ctl + CTL_ANCLESS, c->anc_bad_word);
    HIPCHK(hipGetLastError());
    c->anc_upto = std::min(c->anc_upto, c->snap_anc_upto);
    c->anc_dirty = false;
    return XC_OK;
}

// Rebuild the cache's tables for `ncap` segments, keeping the entries with a segment index below
// `keep` (and, with drop_dead, only the live ones): the undo log is rewritten for the new slots and
// the segment store copied when the capacity changes; the filters depend on the keys only and are
// copied.  Snapshots stay valid: the rebuilt undo log records the new slots.
static int cache_rebuild(xc_cache *c, uint64_t ncap, uint32_t keep, bool drop_dead)
{
    c->removed_floor = std::min(c->removed_floor, keep);
    hipStream_t s = c->ctx->stream;
    HIPCHK(hipDeviceSynchronize());  // (plans' side streams too: nothing may use the old arrays)
    uint32_t count = 0;
    int rc = cache_count_host(c, &count);
    if (rc) return rc;
    {   // the device's record of an anchorless segment (an anchor run's emit) joins the host's
        uint32_t bad = 0;
        HIPCHK(hipMemcpy(&bad, c->ctl + CTL_ANCLESS, 4, hipMemcpyDeviceToHost));
        if (bad) c->anc_bad = std::min(c->anc_bad, ~bad);
    }
    count = std::min<uint32_t>(count, (uint32_t)c->cap);
    const uint32_t kept = std::min(count, keep);
    // the device part of the segment store grows up to the device's share, the spill tier after it
    const uint64_t ndev = std::max(c->dev_cap, std::min(ncap, c->dev_limit));
    const bool move_segs = ndev != c->dev_cap;
    if (ncap > ndev && (rc = cache_spill_to(c, ndev, ncap))) return rc;
    HostSet ns;
    uint8_t *segs = nullptr;
    uint2 *undo = nullptr;
    uint32_t *owner = nullptr, *aundo = nullptr, *aslot = nullptr, *aowner = nullptr;
    uint64_t *anc_of = nullptr;
    const uint32_t akept = std::min(kept, c->anc_upto);  // segments whose anchors move along
    if ((rc = ns.alloc(ncap, true))) return rc;
    if ((move_segs && dmalloc(&segs, (size_t)ndev * XC_SEG + 4096) != hipSuccess) ||
        dmalloc(&undo, (size_t)ncap * sizeof(uint2)) != hipSuccess || dmalloc(&owner, (size_t)ns.n_lo * 4) != hipSuccess ||
        dmalloc(&anc_of, (size_t)ncap * 8) != hipSuccess || dmalloc(&aundo, (size_t)ncap * 4) != hipSuccess ||
        dmalloc(&aslot, (size_t)std::max<uint32_t>(akept, 1) * 4) != hipSuccess ||
        dmalloc(&aowner, (size_t)ns.n_full * 4) != hipSuccess) {
        ns.release(true);
        dfree(segs);
        dfree(undo);
        dfree(owner);
        dfree(anc_of);
        dfree(aundo);
        dfree(aslot);
        dfree(aowner);
        return fail(XC_ENOSPC, "device cache capacity exhausted (device memory)");
    }
    HIPCHK(hipMemcpyAsync(ns.d.filt, c->set.d.filt, XC_FILT_WORDS * 4, hipMemcpyDeviceToDevice, s));
    HIPCHK(hipMemcpyAsync(ns.d.l2, c->set.d.l2, (size_t)XC_L2_WORDS * 8, hipMemcpyDeviceToDevice, s));
    HIPCHK(hipMemcpyAsync(ns.d.lo_zero, c->set.d.lo_zero, 4, hipMemcpyDeviceToDevice, s));
    HIPCHK(hipMemsetAsync(ns.d.lo_keys, 0, (size_t)ns.n_lo * 4, s));
    HIPCHK(hipMemsetAsync(ns.d.keys, 0xFF, (size_t)ns.n_full * 8, s));
    HIPCHK(hipMemsetAsync(ns.d.vals, 0xFF, (size_t)ns.n_full * 8, s));
    HIPCHK(hipMemsetAsync(undo, 0xFF, (size_t)ncap * sizeof(uint2), s));
    HIPCHK(hipMemsetAsync(owner, 0xFF, (size_t)ns.n_lo * 4, s));
    if (move_segs && kept)
        HIPCHK(hipMemcpyAsync(segs, c->segs, (size_t)std::min<uint64_t>(kept, c->dev_cap) * XC_SEG,
                              hipMemcpyDeviceToDevice, s));
    const uint32_t blocks = std::min<uint32_t>((c->set.n_full + 255) / 256, 8192);
    hipLaunchKernelGGL(k_rehash, dim3(blocks), dim3(256), 0, s, c->set.d, ns.d, undo, owner, keep, (int)drop_dead);
    HIPCHK(hipGetLastError());
    if (kept) {
        hipLaunchKernelGGL(k_rehash_owner, dim3(std::min<uint32_t>((kept + 255) / 256, 8192)), dim3(256), 0, s,
                           undo, kept, (const uint32_t *)owner);
        HIPCHK(hipGetLastError());
    }
    // the anchor index: the kept segments' keys into the new table (the filter depends on the
    // keys only and is copied), the undo slots to their oldest owners
    HIPCHK(hipMemsetAsync(ns.a.keys, 0xFF, (size_t)ns.n_full * 8, s));
    HIPCHK(hipMemcpyAsync(ns.a.filt, c->set.a.filt, (size_t)ANC_FILT_WORDS * 4, hipMemcpyDeviceToDevice, s));
    if (akept) {
        HIPCHK(hipMemcpyAsync(anc_of, c->anc_of, (size_t)akept * 8, hipMemcpyDeviceToDevice, s));
        HIPCHK(hipMemsetAsync(aowner, 0xFF, (size_t)ns.n_full * 4, s));
        const uint32_t ab = std::min<uint32_t>((akept + 255) / 256, 8192);
        hipLaunchKernelGGL(k_anc_rehash, dim3(ab), dim3(256), 0, s, ns.a, (const uint64_t *)anc_of, akept, aslot, aowner);
        HIPCHK(hipGetLastError());
        hipLaunchKernelGGL(k_anc_owner, dim3(ab), dim3(256), 0, s, aundo, (const uint32_t *)aslot, akept,
                           (const uint32_t *)aowner);
        HIPCHK(hipGetLastError());
    }
    if (kept != count) HIPCHK(hipMemcpyAsync(c->count, &kept, 4, hipMemcpyHostToDevice, s));
    HIPCHK(hipStreamSynchronize(s));
    dfree(aslot);
    dfree(aowner);
    dfree(c->anc_of);
    dfree(c->aundo);
    c->anc_of = anc_of;
    c->aundo = aundo;
    c->anc_upto = akept;
    if (c->anc_bad >= kept) c->anc_bad = NONE;
    // the device word follows (a stale one would send every later anchor run to the exact scan)
    c->anc_bad_word = c->anc_bad == NONE ? 0u : ~c->anc_bad;
    HIPCHK(hipMemcpy(c->ctl + CTL_ANCLESS, &c->anc_bad_word, 4, hipMemcpyHostToDevice));
    c->set.release(true);
    if (move_segs) {
        dfree(c->segs);
        c->segs = segs;
        c->dev_cap = ndev;
    }
    dfree(c->undo);
    dfree(owner);
    c->set = ns;
    c->undo = undo;
    c->cap = ncap;
    c->host_count = kept;
    c->gen++;
    c->last_plan = nullptr;
    return XC_OK;
}

// Move the cache into arrays for `need` segments (or twice the capacity).
static int cache_grow(xc_cache *c, uint64_t need)
{
    if (need > CAP_MAX) return fail(XC_ENOSPC, "cache capacity exhausted (2^28 segments)");
    const uint64_t ncap = std::min<uint64_t>(CAP_MAX, std::max<uint64_t>(need + need / 4, 2 * c->cap));
    return cache_rebuild(c, ncap, 0xFFFFFFFFu, false);
}

// Room for `extra` more segments: grow first when the count could pass the capacity.
static int cache_reserve(xc_cache *c, uint64_t extra)
{
    if (int rc = cache_busy(c)) return rc;
    if (c->host_count < 0) {
        uint32_t v = 0;
        int rc = cache_count_host(c, &v);
        if (rc) return rc;
        c->host_count = v;
    }
    if ((uint64_t)c->host_count + extra <= c->cap) return XC_OK;
    return cache_grow(c, (uint64_t)c->host_count + extra);
}

// For the COSS tier (xc_coss.cpp): the segments entered after the first `keep` are taken out again,
// evicted ones too.  The tables are rebuilt rather than the later slots cleared: a batch's inserts
// run in parallel, so an entry kept can sit past one taken out on its probe chain.
extern "C" int xc__cache_truncate(xc_cache *c, uint64_t keep)
{
    int rc = set_dev(c->ctx);
    if (!rc) rc = cache_busy(c);
    if (rc) return rc;
    return cache_rebuild(c, c->cap, (uint32_t)std::min<uint64_t>(keep, 0xFFFFFFFFu), true);
}

// Evicted segments (host hashes): absent to every lookup until entered again.
extern "C" int xc__cache_kill(xc_cache *c, const uint64_t *h, uint64_t n)
{
    if (!n) return XC_OK;
    c->removed_floor = 0;  // (evicted entries of any age)
    c->last_plan = nullptr;
    int rc = set_dev(c->ctx);
    if (!rc) rc = cache_busy(c);
    if (rc) return rc;
    hipStream_t s = c->ctx->stream;
    uint64_t *d = nullptr;
    HIPCHK(dmalloc(&d, n * 8));
    HIPCHK(hipMemcpyAsync(d, h, n * 8, hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(k_kill, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, s, c->set.d, (const uint64_t *)d,
                       (uint32_t)n);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(s));
    dfree(d);
    return XC_OK;
}

// n new (hash, segment) pairs from host memory at once (the hashes absent from the cache).
extern "C" int xc__cache_enter_bulk(xc_cache *c, const uint64_t *h, const uint8_t *segs, uint64_t n)
{
    if (!n) return XC_OK;
    c->last_plan = nullptr;
    int rc = set_dev(c->ctx);
    if (!rc) rc = cache_busy(c);
    if (rc) return rc;
    if ((rc = cache_reserve(c, n))) return rc;
    hipStream_t s = c->ctx->stream;
    const uint32_t first = (uint32_t)c->host_count;
    uint64_t *dh = nullptr;
    uint8_t *ds = nullptr;
    HIPCHK(dmalloc(&dh, n * 8));
    HIPCHK(dmalloc(&ds, n * XC_SEG));
    HIPCHK(hipMemcpyAsync(dh, h, n * 8, hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(ds, segs, n * XC_SEG, hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(k_enter_bulk, dim3((uint32_t)((n + 3) / 4)), dim3(256), 0, s, cache_plandev(c),
                       (const uint64_t *)dh, (const uint8_t *)ds, (uint32_t)n, first);
    HIPCHK(hipGetLastError());
    const uint32_t cnt = first + (uint32_t)n;
    HIPCHK(hipMemcpyAsync(c->count, &cnt, 4, hipMemcpyHostToDevice, s));
    HIPCHK(hipStreamSynchronize(s));
    c->host_count = cnt;
    dfree(dh);
    dfree(ds);
    return XC_OK;
}

extern "C" int xc__cache_reserve(xc_cache *c, uint64_t extra)
{
    int rc = set_dev(c->ctx);
    return rc ? rc : cache_reserve(c, extra);
}
extern "C" uint32_t xc__cache_gen(xc_cache *c) { return c->gen; }

extern "C" int xc_cache_capacity(xc_cache *c, uint64_t *cap)
{
    if (!c || !cap) return fail(XC_EINVAL, "null");
    *cap = c->cap;
    return XC_OK;
}

extern "C" int xc_cache_count(xc_cache *c, uint64_t *n)
{
    if (!c || !n) return fail(XC_EINVAL, "null");
    int rc = set_dev(c->ctx);
    if (rc) return rc;
    uint32_t v = 0;
    if ((rc = cache_count_host(c, &v))) return rc;
    // (the reference's map holds a hash entered twice once; the device keeps both segments)
    *n = std::min<uint64_t>(v, c->cap) - std::min<uint64_t>(xc__mem_extra(c->mem), std::min<uint64_t>(v, c->cap));
    return XC_OK;
}

// The device's segment count (the replay engine's truncation points).
extern "C" int xc__cache_count_raw(xc_cache *c, uint64_t *n)
{
    int rc = set_dev(c->ctx);
    if (rc) return rc;
    uint32_t v = 0;
    if ((rc = cache_count_host(c, &v))) return rc;
    *n = std::min<uint64_t>(v, c->cap);
    return XC_OK;
}

extern "C" int xc_cache_snapshot(xc_cache *c)
{
    if (!c) return fail(XC_EINVAL, "null");
    int rc = set_dev(c->ctx);
    if (!rc) rc = cache_busy(c);
    if (!rc) rc = cache_settle(c);
    if (rc) return rc;
    if (c->mem) {
        xc__mem_free(c->mem_snap);
        if (!(c->mem_snap = xc__mem_clone(c->mem))) return fail(XC_ENOMEM, "host allocation failed");
    }
    if ((rc = cache_count_host(c, &c->snap_count))) return rc;
    c->host_count = c->snap_count;
    // (the snapshot includes the anchor index: a restore then leaves nothing to backfill)
    if (cache_anc_ok(c) && (rc = cache_anc_catch_up(c))) return rc;
    hipStream_t s = c->ctx->stream;
    HIPCHK(hipMemcpyAsync(c->snap_afilt, c->set.a.filt, (size_t)ANC_FILT_WORDS * 4, hipMemcpyDeviceToDevice, s));
    c->snap_anc_upto = std::min(c->anc_upto, c->snap_count);
    c->anc_dirty = false;
    HIPCHK(hipMemcpyAsync(c->snap_filt, c->set.d.filt, XC_FILT_WORDS * 4, hipMemcpyDeviceToDevice, s));
    HIPCHK(hipMemcpyAsync(c->snap_lo_zero, c->set.d.lo_zero, 4, hipMemcpyDeviceToDevice, s));
    HIPCHK(hipMemcpyAsync(c->snap_count_dev, c->count, 4, hipMemcpyDeviceToDevice, s));
    HIPCHK(hipMemcpyAsync(c->snap_l2, c->set.d.l2, (size_t)XC_L2_WORDS * 8, hipMemcpyDeviceToDevice, s));
    HIPCHK(hipStreamSynchronize(s));
    c->has_snap = true;
    c->snap_gen = c->gen;
    return XC_OK;
}

// A restore across a rebuild (the cache grew since the snapshot): the rebuild inserted every key
// in parallel, so a key entered after the snapshot can sit before an older one on its probe chain,
// and clearing it (the undo log) would cut the chain.  The tables are rebuilt again from the
// snapshot's entries instead, and take the snapshot's filters; later restores use the undo log.
static int cache_restore_rebuilt(xc_cache *c)
{
    int rc = cache_rebuild(c, c->cap, c->snap_count, false);
    if (rc) return rc;
    hipStream_t s = c->ctx->stream;
    HIPCHK(hipMemcpyAsync(c->set.d.filt, c->snap_filt, XC_FILT_WORDS * 4, hipMemcpyDeviceToDevice, s));
    HIPCHK(hipMemcpyAsync(c->set.d.lo_zero, c->snap_lo_zero, 4, hipMemcpyDeviceToDevice, s));
    HIPCHK(hipMemcpyAsync(c->set.d.l2, c->snap_l2, (size_t)XC_L2_WORDS * 8, hipMemcpyDeviceToDevice, s));
    HIPCHK(hipMemcpyAsync(c->set.a.filt, c->snap_afilt, (size_t)ANC_FILT_WORDS * 4, hipMemcpyDeviceToDevice, s));
    HIPCHK(hipMemcpyAsync(c->count, &c->snap_count, 4, hipMemcpyHostToDevice, s));
    HIPCHK(hipStreamSynchronize(s));
    c->anc_upto = std::min(c->anc_upto, c->snap_anc_upto);
    c->anc_dirty = false;
    if ((rc = cache_anc_bad_reset(c))) return rc;
    HIPCHK(hipStreamSynchronize(s));
    c->snap_gen = c->gen;
    c->host_count = c->snap_count;
    return XC_OK;
}

// Enqueue the restore on the context stream (no host sync): for timed loops.
static int cache_restore_async(xc_cache *c, uint32_t cur_count)
{
    c->removed_floor = std::min(c->removed_floor, c->snap_count);
    hipStream_t s = c->ctx->stream;
    uint32_t to = std::min<uint32_t>(cur_count, (uint32_t)c->cap);
    if (to > c->snap_count) {
        uint32_t n = to - c->snap_count;
        uint32_t blocks = std::min<uint32_t>((n + 255) / 256, 4096);
        hipLaunchKernelGGL(k_undo, dim3(blocks), dim3(256), 0, s, c->set.d, (const uint2 *)c->undo,
                           c->snap_count, to);
        HIPCHK(hipGetLastError());
    }
    HIPCHK(hipMemcpyAsync(c->set.d.filt, c->snap_filt, XC_FILT_WORDS * 4, hipMemcpyDeviceToDevice, s));
    HIPCHK(hipMemcpyAsync(c->set.d.lo_zero, c->snap_lo_zero, 4, hipMemcpyDeviceToDevice, s));
    HIPCHK(hipMemcpyAsync(c->count, &c->snap_count, 4, hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(c->set.d.l2, c->snap_l2, (size_t)XC_L2_WORDS * 8, hipMemcpyDeviceToDevice, s));
    return cache_anc_restore(c);
}

// The model as it was at the snapshot (the runs since are undone: their lookups are not replayed).
static int mem_restore(xc_cache *c)
{
    c->hl_fifo.clear();
    c->hl_pend = nullptr;
    c->pend_dec = nullptr;
    return c->mem && c->mem_snap ? xc__mem_restore(c->mem, c->mem_snap) : XC_OK;
}

extern "C" int xc_cache_restore_async(xc_cache *c)
{
    if (!c) return fail(XC_EINVAL, "null");
    if (!c->has_snap) return fail(XC_EINVAL, "no snapshot");
    int rc = set_dev(c->ctx);
    if (!rc) rc = cache_busy(c);
    if (rc) return rc;
    struct MemAfter {  // (after the device restore is enqueued: a mirror's fix-up follows it)
        xc_cache *c;
        ~MemAfter() { mem_restore(c); }
    } mem_after{c};
    if (c->gen != c->snap_gen) return cache_restore_rebuilt(c);
    c->removed_floor = std::min(c->removed_floor, c->snap_count);
    hipStream_t s = c->ctx->stream;
    if (c->host_count >= 0) {
        // one kernel: table slots entered since the snapshot, filters and count from the snapshot
        const uint32_t to = (uint32_t)std::min<int64_t>(c->host_count, (int64_t)c->cap);
        const uint32_t n = std::max<uint32_t>(to > c->snap_count ? to - c->snap_count : 0u, XC_L2_WORDS / 2);
        const uint32_t blocks = std::min<uint32_t>((n + 255) / 256, 2048);
        hipLaunchKernelGGL(k_undo_known, dim3(blocks), dim3(256), 0, s, c->set.d, (const uint2 *)c->undo,
                           c->snap_count, to, c->count, (const uint4 *)c->snap_filt, (const uint4 *)c->snap_l2,
                           (const uint32_t *)c->snap_lo_zero);
        HIPCHK(hipGetLastError());
        c->host_count = c->snap_count;
        return cache_anc_restore(c);
    }
    // one kernel: table slots entered since the snapshot, filters copied back; then the count
    const uint32_t n = (uint32_t)std::max<uint64_t>(c->cap - c->snap_count, XC_L2_WORDS / 2);
    const uint32_t blocks = std::min<uint32_t>((n + 255) / 256, 2048);
    hipLaunchKernelGGL(k_undo_dev, dim3(blocks), dim3(256), 0, s, c->set.d, (const uint2 *)c->undo, c->snap_count,
                       (const uint32_t *)c->count, (uint32_t)c->cap, (const uint4 *)c->snap_filt,
                       (const uint4 *)c->snap_l2, (const uint32_t *)c->snap_lo_zero);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(c->count, c->snap_count_dev, 4, hipMemcpyDeviceToDevice, s));
    c->host_count = c->snap_count;
    return cache_anc_restore(c);
}

extern "C" int xc_cache_restore(xc_cache *c)
{
    if (!c) return fail(XC_EINVAL, "null");
    if (!c->has_snap) return fail(XC_EINVAL, "no snapshot");
    int rc = set_dev(c->ctx);
    if (!rc) rc = cache_busy(c);
    if (rc) return rc;
    if (c->gen != c->snap_gen) {
        if ((rc = cache_restore_rebuilt(c))) return rc;
        return mem_restore(c);
    }
    uint32_t cur = 0;
    if ((rc = cache_count_host(c, &cur))) return rc;
    if ((rc = cache_restore_async(c, cur))) return rc;
    HIPCHK(hipStreamSynchronize(c->ctx->stream));
    c->host_count = c->snap_count;
    return mem_restore(c);
}

// Lookup without side effects (the device's bytes for the hash).
extern "C" int xc__cache_read(xc_cache *c, uint64_t h, uint8_t *out, int *found)
{
    int rc = set_dev(c->ctx);
    if (rc) return rc;
    hipStream_t s = c->ctx->stream;
    uint32_t *d_found = c->ctx->d_scratch;
    hipLaunchKernelGGL(k_lookup_one, dim3(1), dim3(64), 0, s, cache_plandev(c), h, c->ctx->d_seg, d_found);
    HIPCHK(hipGetLastError());
    uint32_t f = 0;
    HIPCHK(hipMemcpyAsync(&f, d_found, 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(out, c->ctx->d_seg, XC_SEG, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    *found = (int)f;
    return XC_OK;
}

// XCodecMemoryCache::lookup (xcodec_cache.h:190-210): the recent window decides the bytes of a
// hash entered twice, and remembers a map hit.
extern "C" int xc_cache_lookup(xc_cache *c, uint64_t h, uint8_t *out, int *found)
{
    if (!c || !out || !found) return fail(XC_EINVAL, "null");
    int rc = set_dev(c->ctx);
    if (!rc) rc = cache_busy(c);
    if (!rc) rc = cache_settle(c);
    if (rc) return rc;
    return c->mem && !c->engine ? xc__mem_lookup(c->mem, h, out, found) : xc__cache_read(c, h, out, found);
}

// Diagnostic: the false-positive rates a random window end sees in the cache's level-1 (LDS) and
// level-2 (L2) filters, from their word occupancy (k = 2 bits in one word: the mean of (bits set /
// 32)^2 over the words).
extern "C" int xc_cache_filter_stats(xc_cache *c, double *l1_fp, double *l2_fp)
{
    if (!c || !l1_fp || !l2_fp) return fail(XC_EINVAL, "null");
    int rc = set_dev(c->ctx);
    if (!rc) rc = cache_busy(c);
    if (rc) return rc;
    std::vector<uint32_t> f(XC_FILT_WORDS), l2((size_t)XC_L2_WORDS * 2);
    HIPCHK(hipMemcpyAsync(f.data(), c->set.d.filt, f.size() * 4, hipMemcpyDeviceToHost, c->ctx->stream));
    HIPCHK(hipMemcpyAsync(l2.data(), c->set.d.l2, l2.size() * 4, hipMemcpyDeviceToHost, c->ctx->stream));
    HIPCHK(hipStreamSynchronize(c->ctx->stream));
    auto fp = [](const std::vector<uint32_t> &w) {
        double a = 0;
        for (uint32_t x : w) {
            const double b = __builtin_popcount(x) / 32.0;
            a += b * b;
        }
        return a / (double)w.size();
    };
    *l1_fp = fp(f);
    *l2_fp = fp(l2);
    return XC_OK;
}

// Device values of n hashes (~0: absent), no side effects.
extern "C" int xc__cache_find(xc_cache *c, const uint64_t *h, uint64_t n, uint64_t *val)
{
    if (!n) return XC_OK;
    int rc = set_dev(c->ctx);
    if (rc) return rc;
    hipStream_t s = c->ctx->stream;
    uint64_t *d = nullptr;
    HIPCHK(dmalloc(&d, n * 16));
    HIPCHK(hipMemcpyAsync(d, h, n * 8, hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(k_find, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, s, c->set.d, (const uint64_t *)d,
                       d + n, (uint32_t)n);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(val, d + n, n * 8, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    dfree(d);
    return XC_OK;
}

// The table value of a present hash, set (a restore puts back what a mirror replaced).
extern "C" int xc__cache_set_value(xc_cache *c, uint64_t h, uint64_t val)
{
    c->last_plan = nullptr;
    int rc = set_dev(c->ctx);
    if (rc) return rc;
    hipLaunchKernelGGL(k_setval, dim3(1), dim3(64), 0, c->ctx->stream, c->set.d, h, val);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(c->ctx->stream));
    return XC_OK;
}

// XCodecMemoryCache::enter (xcodec_cache.h:182-188); a hash entered again with other bytes takes
// the release build's semantics (xc_memcache.cpp).
extern "C" int xc_cache_enter(xc_cache *c, uint64_t h, const uint8_t *seg)
{
    if (!c || !seg) return fail(XC_EINVAL, "null");
    int rc = set_dev(c->ctx);
    if (!rc) rc = cache_busy(c);
    if (!rc) rc = cache_settle(c);
    if (rc) return rc;
    if (c->mem && !c->engine) {
        int dup = 0;
        if ((rc = xc__mem_enter(c->mem, h, seg, &dup)) || dup) return rc;
    }
    hipStream_t s = c->ctx->stream;
    if ((rc = cache_reserve(c, 1))) return rc;
    c->host_count = -1;
    c->last_plan = nullptr;  // (an enter of a present hash rewrites its segment's bytes)
    HIPCHK(hipMemcpyAsync(c->ctx->d_seg, seg, XC_SEG, hipMemcpyHostToDevice, s));
    // only the word k_enter_one reports: CTL_ANCLESS is the device's record of an anchorless
    // segment an anchor run entered, which the host may not have learned yet
    HIPCHK(hipMemsetAsync(c->ctl + CTL_ERROR, 0, 4, s));
    hipLaunchKernelGGL(k_enter_one, dim3(1), dim3(64), 0, s, cache_plandev(c), h, (const uint8_t *)c->ctx->d_seg);
    HIPCHK(hipGetLastError());
    uint32_t ctl[CTL_WORDS];
    HIPCHK(hipMemcpyAsync(ctl, c->ctl, sizeof ctl, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    if (ctl[CTL_ERROR] & ERR_CAPACITY) return fail(XC_ENOSPC, "cache full");
    return XC_OK;
}

extern "C" int xc_hash_segments(xc_ctx *ctx, const uint8_t *d_segs, uint64_t n, uint64_t *d_out, void *stream)
{
    if (!ctx) return fail(XC_EINVAL, "null");
    if (n == 0) return XC_OK;
    int rc = set_dev(ctx);
    if (rc) return rc;
    hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
    uint32_t blocks = (uint32_t)std::min<uint64_t>(n, 65536);
    hipLaunchKernelGGL(k_hash_segments, dim3(blocks), dim3(64), 0, s, d_segs, n, d_out);
    HIPCHK(hipGetLastError());
    return XC_OK;
}

extern "C" int xc_hash_segments_host(xc_ctx *ctx, const uint8_t *segs, uint64_t n, uint64_t *out);
extern "C" int xc__hash_segments_host_raw(xc_ctx *ctx, const uint8_t *segs, uint64_t n, uint64_t *out)
{
    return xc_hash_segments_host(ctx, segs, n, out);
}
extern "C" int xc_hash_segments_host(xc_ctx *ctx, const uint8_t *segs, uint64_t n, uint64_t *out)
{
    if (!ctx || (n && (!segs || !out))) return fail(XC_EINVAL, "null");
    if (n == 0) return XC_OK;
    int rc = set_dev(ctx);
    if (rc) return rc;
    hipStream_t s = ctx->stream;
    uint8_t *d_segs = nullptr;
    uint64_t *d_out = nullptr;
    if ((rc = xc__dalloc((void **)&d_segs, n * XC_SEG))) return rc;
    if ((rc = xc__dalloc((void **)&d_out, n * 8))) return rc;
    HIPCHK(hipMemcpyAsync(d_segs, segs, n * XC_SEG, hipMemcpyHostToDevice, s));
    if ((rc = xc_hash_segments(ctx, d_segs, n, d_out, s))) return rc;
    HIPCHK(hipMemcpyAsync(out, d_out, n * 8, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    xc__pfree(d_segs);
    xc__pfree(d_out);
    return XC_OK;
}

extern "C" int xc_window_hashes(xc_ctx *ctx, const uint8_t *d_in, uint64_t n, uint64_t *d_out, void *stream)
{
    if (!ctx) return fail(XC_EINVAL, "null");
    if (n == 0) return XC_OK;
    if (n > 0xFFFFFFF0ull) return fail(XC_EINVAL, "too long");
    int rc = set_dev(ctx);
    if (rc) return rc;
    hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
    uint32_t blocks = (uint32_t)((n + XC_SEG - 1) / XC_SEG);
    hipLaunchKernelGGL(k_window_hashes, dim3(blocks), dim3(64), 0, s, d_in, (uint32_t)n, d_out);
    HIPCHK(hipGetLastError());
    return XC_OK;
}

// ------------------------------------------------------------------ plan ----------
static const uint32_t CHUNK_LEN = 16384;  // the longest scan chunk (plans of small batches use shorter ones)
static_assert(CHUNK_LEN == CHUNK_BLOCKS * XC_SEG, "k_scan loads a chunk's shadow flags in one wave load");
static const uint64_t HOST_SUB_BYTES = 256ull << 20;      // ... of plans run from host memory (copies pipelined)
static const uint64_t SUB_BYTES_DEFAULT = 512ull << 20;  // sub-batch: bound on input bytes (tuned on cfg5)
static const uint32_t SUB_BUFS = 32768;                  // sub-batch: bound on buffers

static const uint64_t SUB_BYTES_MAX = 1024ull << 20;    // ... grown up to this while the run keeps two
// The sub-batch byte bound of a run of `total` input bytes: half the run, between 256 MiB and 1 GiB,
// so that a large run has two sub-batches or more (its later sub-batches hashed on the side stream
// beside the earlier ones) and as few as that allows: per sub-batch, each of the ~9 dependent kernels
// of the main stream pays its ramp-down (cfg5, 2 GiB: A/B 512 MiB 845-847 / 768 MiB 848-853 /
// 1 GiB 856-858 GiB/s, profiles/r05/ab/sub_batch_size_r5j.txt).  XC_SUB_MB overrides it (tests,
// tuning experiments).
// Runs of 512 MiB to 1 GiB take two halves too (at least 256 MiB each): the N=4 rank's 512 MiB shard
// of cfg5 722-732 -> 756 GiB/s with two, its hashing of the second beside the first's main-stream
// kernels (profiles/r05/ab/rank_sub_batches_r5ab.txt); below 512 MiB one sub-batch (cfg3 and the
// N=8 rank's 256 MiB: two of 128 MiB 596 against 686, shard8_sub_batches_r5o.txt).
static const uint64_t SUB_BYTES_MIN = 256ull << 20;
static uint64_t sub_bytes(uint64_t total, uint64_t bound)
{
    const char *e = getenv("XC_SUB_MB");
    const long v = e ? atol(e) : 0;
    if (v > 0) return (uint64_t)v << 20;
    if (bound) return bound;
    if (total < 2 * SUB_BYTES_MIN) return SUB_BYTES_DEFAULT;
    const uint64_t half = ((total / 2 + (1u << 20) - 1) >> 20) << 20;
    return std::min(SUB_BYTES_MAX, std::max(SUB_BYTES_MIN, half));
}
static const uint32_t MAX_ROUNDS = 64;

struct HostLayer {
    Layer d{};
    int alloc(uint32_t nchunks, uint32_t chunk_len)
    {
        size_t n = std::max<uint32_t>(nchunks, 1);
        HIPCHK(dmalloc(&d.cnt, n * 4));
        HIPCHK(dmalloc(&d.pos, n * EV_CAP * 4));
        HIPCHK(dmalloc(&d.stat, n * EV_CAP * 4));
        HIPCHK(dmalloc(&d.h, n * EV_CAP * 8));
        HIPCHK(dmalloc(&d.val, n * EV_CAP * 8));
        HIPCHK(dmalloc(&d.bits, n * (chunk_len / 32) * 4));
        return XC_OK;
    }
    void release()
    {
        dfree(d.cnt);
        dfree(d.pos);
        dfree(d.stat);
        dfree(d.h);
        dfree(d.val);
        dfree(d.bits);
    }
};

static std::atomic<uint64_t> g_plan_serial{0};

struct xc_plan {
    uint64_t serial = ++g_plan_serial;  // (never reused, unlike the plan's address)
    xc_cache *cache;
    uint32_t nb;
    std::vector<uint64_t> len, in_off, out_off;
    uint64_t in_bytes, out_bytes;
    std::vector<uint32_t> chunk0;   // host copy of buf_chunk0
    std::vector<uint32_t> sub;      // sub-batch boundaries (buffer indices), sub.back() = nb
    uint32_t nchunks;
    PlanDev P{};
    HostLayer S, D;
    HostSet dset;
    // device arrays owned
    uint64_t *d_buf_off, *d_out_off;
    uint32_t *d_buf_len, *d_chunk0, *d_tok_base;
    uint2 *d_chunks;
    uint4 *d_desc;
    uint32_t *d_blk_base, *d_blk_buf = nullptr;
    std::vector<uint32_t> blk_base;  // host copy [nb + 1]
    uint2 *d_blk_grp = nullptr;      // k_blockhash groups
    std::vector<uint32_t> grp_base;  // [nb + 1] first group of every buffer
    uint32_t *d_l2mix;  // level-2 filter of cache | declaration set for the combined scan
    uint32_t *d_fmix;   // level-1 image of cache | declaration set for the first scan (folded)
    xc_run_stats stats{};
    // per-kernel HIP-event timing: 0 off, XC_TIMING_ALL every kernel, XC_TIMING_SCAN the scans only
    // (each recorded event pair costs the stream a few microseconds between dependent launches)
    int timing = 0;
    std::vector<hipEvent_t> ev_pool;
    std::vector<std::pair<int, std::pair<hipEvent_t, hipEvent_t>>> ev_live;
    xc_kernel_times ktimes{};
    std::vector<uint64_t> chunk_bytes;  // prefix of input bytes covered by chunks
    // block hashing runs ahead on a side stream (it reads only the input), overlapping the
    // scans; sub-batch k's prediction step waits for ev_hash[k]
    hipStream_t hs = nullptr;
    hipEvent_t ev_start = nullptr;
    uint32_t *h_ctl = nullptr;  // pinned copy of the control words (read_ctl)
    uint32_t *d_hctl = nullptr;  // its device address (k_emit<.., true> publishes the words there)
    uint32_t *emit_ctl_host = nullptr;  // set while a pass that publishes its control words is enqueued
    uint32_t emit_pub_final = 0;        // ... on its last sub-batch
    bool g_publish = false;      // the captured graph's emit publishes the control words
    bool pass_published = false;  // the in-flight first pass publishes them (else a copy)
    int completion = XC_COMPLETE_RUN;  // xc_plan_set_completion
    bool inflight = false;        // xc_encode_submit enqueued a run not finished yet
    // xc_cache_quiesce finished the run for another caller: its status, for the submitter's poll/wait
    bool parked = false;
    int parked_rc = XC_OK;
    std::string parked_msg;
    hipEvent_t ev_ctl = nullptr;
    std::vector<hipEvent_t> ev_hash, ev_go;
    // xc_plan_set_input_ready: the input is complete when a run is submitted, so the run's first
    // sub-batch is hashed on the side stream at once, beside the previous run's last kernels
    // (early_ok: the previous run of this plan went through the asynchronous pass unchanged;
    // ev_sb0: after its first sub-batch's last kernel that reads the block arrays; ev_last: after its
    // last sub-batch's emit, the last reader of every later sub-batch's block arrays)
    bool input_ready = false, early_ok = false;
    bool rec_sb0 = false;  // (this run records ev_sb0 and ev_last: only a plan of several sub-batches with its input ready uses them)
    hipEvent_t ev_sb0 = nullptr, ev_last = nullptr;
    // The emit of a large sub-batch (its wire bytes and segment-store copies) runs on its own stream
    // es, beside the next sub-batch's predictions and anchor scan; the main stream joins it before
    // the next resolve (the first reader of the new segments' bytes) and at the pass's end.
    // ev_ins: after the sub-batch's cache inserts; ev_emit: after its emit; emit_open: an emit
    // the main stream has not joined yet.
    hipStream_t es = nullptr;
    hipEvent_t ev_ins = nullptr, ev_emit = nullptr;
    bool emit_open = false;
    uint64_t early_runs = 0;
    uint32_t next_hash = 0;  // first sub-batch not yet enqueued for hashing in this run
    // end-to-end host path (xc_encode_run_host): per-sub-batch H2D on a copy stream, packing
    // kernels after every emitted sub-batch
    bool host_path = false;
    hipStream_t cs = nullptr;
    std::vector<hipEvent_t> ev_h2d;
    uint8_t *e_in = nullptr, *e_out = nullptr;
    // (one block: lengths, packed positions, stream results; one copy back)
    uint64_t *e_len = nullptr, *e_pos = nullptr, *e_total = nullptr;
    uint2 *e_res = nullptr;
    bool h2d_inline = false;  // a one-sub-batch host-path run copies its input on the context stream
    uint8_t *pack_dst = nullptr;
    uint64_t *h_lenpos = nullptr;  // pinned: the host path's lengths, positions and stream results (xc_encode_run_host)
    bool res_staged = false;       // the last host-path run's stream results are in h_lenpos + 2 nb
    std::vector<uint4> st_dev;     // the stream states d_stream_st holds (set_streams skips an equal upload)
    uint4 *h_st = nullptr;         // pinned staging of their upload
    bool cand_carried = false;     // a stream state carries a candidate (a hash may be entered twice)
    uint64_t pack_cap = 0;
    int shadow = 1;          // REF shadows in the async pass (XC_NO_SHADOW=1 disables)
    uint32_t max_decl = 2;   // longest buffer / 2048 + 2 (k_walk's LDS)
    uint32_t walk_waves = 1; // waves per buffer in k_walk (the block-parallel walk's chunk groups)
    uint64_t runs_done = 0;  // completed xc_encode_run calls (timing ablations)
    uint32_t *d_chunk_blk = nullptr;
    // scan granularity: chunk length (a multiple of 2048 up to CHUNK_LEN) and chunks per work
    // unit, chosen so that the largest sub-batch gives every SIMD of the chip a unit
    uint32_t chunk_len = CHUNK_LEN, scan_unit = SCAN_UNIT;
    uint4 *d_stream_st = nullptr;  // stateful streams (xc_plan_set_streams), else null
    uint2 *d_stream_res = nullptr;
    // The asynchronous pass of a run (every sub-batch's kernels and the control-word readback) as
    // a HIP graph: one launch instead of ~10 host launches per sub-batch, which bound small batches
    // (the host enqueues slower than the device runs their kernels).  Captured on the first run
    // with given arenas, replayed while they stay the same.
    hipGraphExec_t gexec = nullptr;
    const void *g_in = nullptr, *g_out = nullptr, *g_len = nullptr;
    const void *g_stream = nullptr;  // P.stream_st the graph was captured with
    xc_run_stats g_stats{};          // host-side counters of the captured pass
    bool g_off = false;              // capture failed (or XC_NO_GRAPH): enqueue directly
    bool zero_ctl = false;           // the next k_clear_set also clears the run's control words
    uint32_t cache_gen = 0;          // the cache arrays P holds (xc_cache::gen)
    uint4 *d_coll = nullptr;         // collision records of every buffer (COLL_CAP each)
    uint32_t *d_coll_cnt = nullptr;
    std::vector<uint32_t> tok_base;  // host copy [nb + 1]
    std::vector<uint32_t> hit_base;  // host copy [nb + 1] (k_hits' layout)
    uint32_t *d_hit_base = nullptr;
    int64_t count0 = -1;             // the cache's count before a run that may enter a hash twice
    uint64_t max_new = 0;            // most segments a run can enter (sum of len / 2048 + 1)
    // anchor index: xc_plan_set_scan's mode; this run hashes anchors (anc_run),
    // its remaining sub-batches scan through the index (anc_scan_on), some did (anc_any)
    int scan_mode = XC_SCAN_AUTO;
    bool anc_run = false, anc_scan_on = false, anc_any = false, g_anc = false;
    bool tail_enqueued = false;  // the first pass enqueued the tail check behind itself
    uint64_t ngroups = 0, nblocks = 0;
    uint32_t *d_buf_grp0 = nullptr;
    uint64_t *d_rec = nullptr, *d_blk_anc = nullptr;
    uint32_t *d_rec_cnt = nullptr, *d_amix = nullptr;
    uint4 *d_ainfo = nullptr;
    uint2 *d_agap = nullptr;
    uint32_t *d_tcnt = nullptr;  // the tail check's collision lists (k_tailcheck / k_tailfinal)
    uint32_t *d_pcnt = nullptr, *d_pq = nullptr;  // the anchor scan's proposals per chunk
    uint4 *d_tlist = nullptr;
};

static hipEvent_t ev_get(xc_plan *p)
{
    if (p->ev_pool.empty()) {
        hipEvent_t e;
        if (hipEventCreate(&e) != hipSuccess) return nullptr;
        return e;
    }
    hipEvent_t e = p->ev_pool.back();
    p->ev_pool.pop_back();
    return e;
}

struct KSpan {
    xc_plan *p;
    int k;
    hipEvent_t a = nullptr, b = nullptr;
    hipStream_t st;
    KSpan(xc_plan *p_, int k_, hipStream_t s_ = nullptr) : p(p_), k(k_), st(s_ ? s_ : p_->cache->ctx->stream)
    {
        if (!p->timing || (p->timing == XC_TIMING_SCAN && k != XC_K_SCAN)) return;
        a = ev_get(p);
        b = ev_get(p);
        if (a) hipEventRecord(a, st);
    }
    ~KSpan()
    {
        if (!a || !b) return;
        hipEventRecord(b, st);
        p->ev_live.push_back({k, {a, b}});
    }
};

// After a stream sync: fold the recorded spans into ktimes.
static void ev_collect(xc_plan *p)
{
    for (auto &x : p->ev_live) {
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, x.second.first, x.second.second) == hipSuccess) {
            p->ktimes.ms[x.first] += ms;
            p->ktimes.launches[x.first] += 1;
        }
        p->ev_pool.push_back(x.second.first);
        p->ev_pool.push_back(x.second.second);
    }
    p->ev_live.clear();
}

extern "C" int xc_encode_plan_create(xc_cache *c, const uint64_t *lengths, uint64_t nbuf, xc_plan **out)
{
    return xc_encode_plan_create_sub(c, lengths, nbuf, 0, out);
}

extern "C" int xc_encode_plan_create_sub(xc_cache *c, const uint64_t *lengths, uint64_t nbuf, uint64_t sub_bytes_max,
                                         xc_plan **out)
{
    if (!c || !out || (!lengths && nbuf)) return fail(XC_EINVAL, "null");
    if (nbuf > (1u << 24)) return fail(XC_EINVAL, "too many buffers");
    if (sub_bytes_max && sub_bytes_max < MAX_BUF) return fail(XC_EINVAL, "sub-batch bound below 1 MiB");
    int rc = set_dev(c->ctx);
    if (rc) return rc;
    xc_plan *p = new xc_plan();
    p->cache = c;
    p->nb = (uint32_t)nbuf;
    p->len.assign(lengths, lengths + nbuf);
    p->in_off.resize(nbuf);
    p->out_off.resize(nbuf);
    // sub-batches (bounded input bytes and buffers, in index order)
    p->sub.push_back(0);
    uint64_t max_sub_blocks = 0;
    {
        uint64_t bytes = 0, blocks = 0;
        uint32_t cnt = 0;
        uint64_t decl = 0, maxdecl = 0;
        uint64_t total = 0;
        for (uint32_t i = 0; i < nbuf; i++) total += lengths[i];
        uint64_t sub_max = sub_bytes(total, sub_bytes_max);
        // (XC_FIRST_PCT=p, -DXC_ABLATIONS builds: two sub-batches, the first p % of the run)
        uint64_t first_max = sub_max;
        if (const char *fp = abl_env("XC_FIRST_PCT"); fp && atoi(fp) > 0 && atoi(fp) < 100) {
            first_max = ((total * (uint64_t)atoi(fp) / 100 + (1u << 20) - 1) >> 20) << 20;
            sub_max = std::max<uint64_t>(total - first_max, 1u << 20);
        }
        for (uint32_t i = 0; i < nbuf; i++) {
            if (lengths[i] > MAX_BUF) return fail(XC_EINVAL, "buffer longer than 1 MiB");
            if (cnt && (bytes + lengths[i] > (p->sub.size() == 1 ? first_max : sub_max) || cnt >= SUB_BUFS)) {
                p->sub.push_back(i);
                maxdecl = std::max(maxdecl, decl);
                max_sub_blocks = std::max(max_sub_blocks, blocks);
                bytes = 0;
                cnt = 0;
                decl = 0;
                blocks = 0;
            }
            bytes += lengths[i];
            blocks += lengths[i] >= XC_SEG ? (lengths[i] + XC_SEG - 1) / XC_SEG : 0;
            cnt++;
            decl += lengths[i] / XC_SEG + 1;
        }
        maxdecl = std::max(maxdecl, decl);
        max_sub_blocks = std::max(max_sub_blocks, blocks);
        if (p->sub.back() != nbuf) p->sub.push_back((uint32_t)nbuf);
        if ((rc = p->dset.alloc(std::max<uint64_t>(maxdecl, 64), false))) return rc;
    }
    // scan granularity: the longest chunks and units that still give every SIMD of the chip a
    // work unit in the largest sub-batch (a 16 MiB batch would otherwise keep 16 of 256 CUs busy)
    {
        const uint64_t waves = (uint64_t)c->ctx->n_cu * SCAN_WAVES;
        static const uint32_t opts[][2] = {{8, 4}, {8, 2}, {8, 1}, {4, 1}, {2, 1}, {1, 1}};  // blocks, unit
        for (const auto &o : opts) {
            p->chunk_len = o[0] * XC_SEG;
            p->scan_unit = o[1];
            if (max_sub_blocks / ((uint64_t)o[0] * o[1]) >= waves) break;
        }
        const char *e = getenv("XC_CHUNK_BLOCKS");  // (deployment tuning: force a chunk length, unit 1)
        if (e && atoi(e) >= 1 && atoi(e) <= (int)CHUNK_BLOCKS) {
            p->chunk_len = (uint32_t)atoi(e) * XC_SEG;
            p->scan_unit = 1;
        }
    }
    const uint32_t chunk_len = p->chunk_len;
    std::vector<uint32_t> blen(nbuf), chunk0(nbuf + 1), tok_base(nbuf + 1), blk_base(nbuf + 1), hit_base(nbuf + 1);
    uint64_t hits = 0;
    uint64_t nblk = 0;
    std::vector<uint2> chunks;
    std::vector<uint4> descs;
    uint64_t io = 0, oo = 0;
    uint64_t toks = 0;
    for (uint64_t i = 0; i < nbuf; i++) {
        uint64_t n = lengths[i];
        blen[i] = (uint32_t)n;
        p->in_off[i] = io;
        io += (n + 255) / 256 * 256;
        p->out_off[i] = oo;
        oo += (2 * n + 16 + 255) / 256 * 256;
        chunk0[i] = (uint32_t)chunks.size();
        if (n >= XC_SEG)
            for (uint32_t s = 0; s < n; s += chunk_len) {
                chunks.push_back(make_uint2((uint32_t)i, s));
                // bit 31 of the end position: the next chunk continues this buffer; bit 30: and
                // it reaches past its first block (the scan's 2-deep prefetch ring needs to know)
                const uint32_t more = (s + chunk_len < n ? 0x80000000u : 0u) |
                                      (s + chunk_len + XC_SEG < n ? 0x40000000u : 0u);
                descs.push_back(make_uint4(s, (uint32_t)std::min<uint64_t>(s + chunk_len, n) | more,
                                           (uint32_t)p->in_off[i], (uint32_t)(p->in_off[i] >> 32)));
            }
        p->max_decl = std::max<uint32_t>(p->max_decl, (uint32_t)(n / XC_SEG) + 2u);
        tok_base[i] = (uint32_t)toks;
        hit_base[i] = (uint32_t)hits;
        hits += n / XC_SEG + 1 + COLL_CAP + 1;
        blk_base[i] = (uint32_t)nblk;
        nblk += n / XC_SEG;
        toks += 2 * (n / XC_SEG) + 3;
    }
    chunk0[nbuf] = (uint32_t)chunks.size();
    blk_base[nbuf] = (uint32_t)nblk;
    {   // a wave per 4 chunks of the longest buffer, up to WALK_WAVES_MAX: short chunks (small
        // batches) would leave the block walk one memory round trip per 4 chunks on one wave
        uint32_t maxc = 0;
        for (uint64_t i = 0; i < nbuf; i++) maxc = std::max(maxc, chunk0[i + 1] - chunk0[i]);
        p->walk_waves = std::min<uint32_t>(WALK_WAVES_MAX, std::max<uint32_t>(1u, (maxc + 3u) / 4u));
    }
    if (toks > 0xFFFFFFF0ull) return fail(XC_EINVAL, "batch too large");
    p->in_bytes = io + 8192;  // slack: the scan prefetches up to two blocks past a buffer
    p->out_bytes = oo + 256;
    p->nchunks = (uint32_t)chunks.size();
    p->chunk0 = chunk0;
    tok_base[nbuf] = (uint32_t)toks;
    p->tok_base = tok_base;
    if (hits > 0xFFFFFFF0ull) return fail(XC_EINVAL, "batch too large");
    hit_base[nbuf] = (uint32_t)hits;
    p->hit_base = hit_base;
    p->chunk_bytes.assign(chunks.size() + 1, 0);
    for (size_t k = 0; k < chunks.size(); k++) {
        uint64_t n = lengths[chunks[k].x];
        uint64_t e = std::min<uint64_t>(chunks[k].y + chunk_len, n);
        p->chunk_bytes[k + 1] = p->chunk_bytes[k] + (e - chunks[k].y);
    }
    if ((rc = p->S.alloc(p->nchunks, chunk_len))) return rc;
    if ((rc = p->D.alloc(p->nchunks, chunk_len))) return rc;

    size_t nb1 = std::max<uint64_t>(nbuf, 1);
    HIPCHK(dmalloc(&p->d_buf_off, nb1 * 8));
    HIPCHK(dmalloc(&p->d_out_off, nb1 * 8));
    HIPCHK(dmalloc(&p->d_buf_len, nb1 * 4));
    HIPCHK(dmalloc(&p->d_chunk0, (nbuf + 1) * 4));
    HIPCHK(dmalloc(&p->d_tok_base, (nbuf + 1) * 4));
    HIPCHK(dmalloc(&p->d_hit_base, (nbuf + 1) * 4));
    HIPCHK(dmalloc(&p->d_chunks, std::max<size_t>(chunks.size(), 1) * sizeof(uint2)));
    HIPCHK(dmalloc(&p->d_desc, std::max<size_t>(chunks.size(), 1) * sizeof(uint4)));
    hipStream_t s = c->ctx->stream;
    if (nbuf) {
        HIPCHK(hipMemcpyAsync(p->d_buf_off, p->in_off.data(), nbuf * 8, hipMemcpyHostToDevice, s));
        HIPCHK(hipMemcpyAsync(p->d_out_off, p->out_off.data(), nbuf * 8, hipMemcpyHostToDevice, s));
        HIPCHK(hipMemcpyAsync(p->d_buf_len, blen.data(), nbuf * 4, hipMemcpyHostToDevice, s));
        HIPCHK(hipMemcpyAsync(p->d_tok_base, tok_base.data(), (nbuf + 1) * 4, hipMemcpyHostToDevice, s));
    }
    HIPCHK(hipMemcpyAsync(p->d_chunk0, chunk0.data(), (nbuf + 1) * 4, hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(p->d_hit_base, hit_base.data(), (nbuf + 1) * 4, hipMemcpyHostToDevice, s));
    if (!chunks.empty()) {
        HIPCHK(hipMemcpyAsync(p->d_chunks, chunks.data(), chunks.size() * sizeof(uint2), hipMemcpyHostToDevice, s));
        HIPCHK(hipMemcpyAsync(p->d_desc, descs.data(), descs.size() * sizeof(uint4), hipMemcpyHostToDevice, s));
    }

    PlanDev &P = p->P;
    P = cache_plandev(c);
    p->cache_gen = c->gen;
    for (uint64_t i = 0; i < nbuf; i++) p->max_new += lengths[i] / XC_SEG + 1;
    P.buf_off = p->d_buf_off;
    P.buf_len = p->d_buf_len;
    P.nb = (uint32_t)nbuf;
    P.chunks = p->d_chunks;
    P.chunk_desc = p->d_desc;
    P.buf_chunk0 = p->d_chunk0;
    P.chunk_len = chunk_len;
    P.S = p->S.d;
    P.D = p->D.d;
    P.dset = p->dset.d;
    P.tok_base = p->d_tok_base;
    P.hit_base = p->d_hit_base;
    size_t nt = std::max<uint64_t>(toks, 1);
    HIPCHK(dmalloc(&P.tok_cnt, nb1 * 4));
    HIPCHK(dmalloc(&P.tok_lb, nt * 4));
    HIPCHK(dmalloc(&P.tok_le, nt * 4));
    HIPCHK(dmalloc(&P.tok_seg, nt * 4));
    HIPCHK(dmalloc(&P.tok_op, nt * 4));
    HIPCHK(dmalloc(&P.tok_dpos, nt * 4));
    HIPCHK(dmalloc(&P.tok_h, nt * 8));
    HIPCHK(dmalloc(&P.tok_known, nt * 4));
    // every lookup that hits with other bytes (xcodec_encoder.cc:129-137): the recent window's
    // replay (xc_memcache.cpp) and the COSS tier's (xc_coss.cpp)
    HIPCHK(dmalloc(&p->d_coll, nb1 * COLL_CAP * sizeof(uint4)));
    HIPCHK(dmalloc(&p->d_coll_cnt, nb1 * 4));
    HIPCHK(hipMemsetAsync(p->d_coll_cnt, 0, nb1 * 4, s));
    P.coll = p->d_coll;
    P.coll_cnt = p->d_coll_cnt;
    HIPCHK(dmalloc(&P.blk_h, std::max<uint64_t>(nblk, 1) * 8));
    HIPCHK(dmalloc(&P.blk_pref, std::max<uint64_t>(nblk, 1) * 4));
    HIPCHK(hipMemsetAsync(P.blk_pref, 0, std::max<uint64_t>(nblk, 1) * 4, s));
    HIPCHK(dmalloc(&P.blk_cmp, std::max<uint64_t>(nblk, 1) * 4));
    HIPCHK(hipMemsetAsync(P.blk_cmp, 0, std::max<uint64_t>(nblk, 1) * 4, s));
    HIPCHK(dmalloc(&P.sb_count, p->sub.size() * 4));
    HIPCHK(hipMemsetAsync(P.sb_count, 0, p->sub.size() * 4, s));
    {
        std::vector<uint32_t> cb(std::max<size_t>(chunks.size(), 1), 0);
        for (size_t k = 0; k < chunks.size(); k++) cb[k] = blk_base[chunks[k].x];
        HIPCHK(dmalloc(&p->d_chunk_blk, cb.size() * 4));
        HIPCHK(hipMemcpyAsync(p->d_chunk_blk, cb.data(), cb.size() * 4, hipMemcpyHostToDevice, s));
        P.chunk_blk = p->d_chunk_blk;
        const char *e = getenv("XC_NO_SHADOW");
        p->shadow = (e && atoi(e)) ? 0 : 1;
    }
    HIPCHK(dmalloc(&p->d_blk_base, (nbuf + 1) * 4));
    {
        std::vector<uint32_t> bb(std::max<uint64_t>(nblk, 1), 0);
        for (uint64_t i = 0; i < nbuf; i++)
            for (uint32_t g = blk_base[i]; g < blk_base[i + 1]; g++) bb[g] = (uint32_t)i;
        HIPCHK(dmalloc(&p->d_blk_buf, bb.size() * 4));
        HIPCHK(hipMemcpyAsync(p->d_blk_buf, bb.data(), bb.size() * 4, hipMemcpyHostToDevice, s));
        P.blk_buf = p->d_blk_buf;
        p->blk_base = blk_base;
        // block-hash groups: up to 8 consecutive blocks of one buffer
        std::vector<uint2> grp;
        p->grp_base.assign(nbuf + 1, 0);
        for (uint64_t i = 0; i < nbuf; i++) {
            p->grp_base[i] = (uint32_t)grp.size();
            // (a partial last block too: the anchor records cover every position)
            const uint32_t nbk = lengths[i] >= XC_SEG ? (uint32_t)((lengths[i] + XC_SEG - 1) / XC_SEG) : 0u;
            for (uint32_t k0 = 0; k0 < nbk; k0 += 8) grp.push_back(make_uint2((uint32_t)i, k0));
        }
        p->grp_base[nbuf] = (uint32_t)grp.size();
        HIPCHK(dmalloc(&p->d_blk_grp, std::max<size_t>(grp.size(), 1) * sizeof(uint2)));
        if (!grp.empty())
            HIPCHK(hipMemcpyAsync(p->d_blk_grp, grp.data(), grp.size() * sizeof(uint2), hipMemcpyHostToDevice, s));
        P.blk_grp = p->d_blk_grp;
        p->ngroups = grp.size();
        p->nblocks = nblk;
        HIPCHK(dmalloc(&p->d_buf_grp0, (nbuf + 1) * 4));
        HIPCHK(hipMemcpyAsync(p->d_buf_grp0, p->grp_base.data(), (nbuf + 1) * 4, hipMemcpyHostToDevice, s));
        P.buf_grp0 = p->d_buf_grp0;
    }
    HIPCHK(dmalloc(&p->d_l2mix, (size_t)XC_L2_WORDS * 8));
    P.l2mix = p->d_l2mix;
    HIPCHK(dmalloc(&p->d_fmix, (size_t)XC_FILT_WORDS * 4));
    P.fmix = p->d_fmix;
    P.fmix_fold = 0;
    // the declaration set's level-2 filter is the combined one (cache | declarations): every
    // declaration insert lands there directly, and the declaration-layer scans test a superset
    P.dset.l2 = p->d_l2mix;
    // (the side stream at the default priority too: at the highest, cfg5 869-870 -> 874-875 GiB/s but
    // the decoder's streams ran slower beside it, cfg4 1370 -> 826, profiles/r05/ab/side_priority_r5s.txt)
    if (!c->ctx->side) HIPCHK(hipStreamCreateWithFlags(&c->ctx->side, hipStreamNonBlocking));
    p->hs = c->ctx->side;
    HIPCHK(hipEventCreateWithFlags(&p->ev_start, hipEventDisableTiming));
    p->ev_hash.assign(p->sub.size(), nullptr);
    p->ev_go.assign(p->sub.size(), nullptr);
    for (auto &e : p->ev_hash) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    for (auto &e : p->ev_go) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&p->ev_sb0, hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&p->ev_last, hipEventDisableTiming));
    HIPCHK(hipMemcpyAsync(p->d_blk_base, blk_base.data(), (nbuf + 1) * 4, hipMemcpyHostToDevice, s));
    P.blk_base = p->d_blk_base;
    HIPCHK(dmalloc(&P.buf_next, nb1 * 4));
    HIPCHK(dmalloc(&P.buf_nref, nb1 * 4));
    HIPCHK(dmalloc(&P.buf_slot, nb1 * 4));
    HIPCHK(dmalloc(&P.ctl, CTL_WORDS * 4));
    HIPCHK(hipMemsetAsync(P.ctl, 0, CTL_WORDS * 4, s));
    P.out_off = p->d_out_off;
    HIPCHK(hipStreamSynchronize(s));
    *out = p;
    return XC_OK;
}

static hipError_t spin_wait(hipEvent_t ev);

// Replay the oldest slot's hits into the window model (per buffer, in the reference's order: its
// REF tokens and its recorded collision lookups, by position; bit 63 of the count: more collisions
// than were recorded).  block = false: only when its copy is complete (*done = 0 otherwise).
// max_b: at most that many buffers of it (a host waiting for the device replays in steps, checking
// the device between them; progress is kept in the slot).
static int hits_replay_front(xc_cache *c, bool block, bool *done, uint32_t max_b = 0xFFFFFFFFu)
{
    xc_cache::HitSlot &sl = c->hl[c->hl_fifo.front()];
    if (sl.host_sync) {  // (a host-path run's host synchronises behind it: normally done already)
        HIPCHK(hipStreamSynchronize(c->ctx->stream));
        sl.host_sync = false;
    }
    hipError_t e = sl.copying ? hipEventQuery(sl.ev) : hipSuccess;
    *done = false;
    if (e == hipErrorNotReady) {
        if (!block) return XC_OK;
        e = spin_wait(sl.ev);
    }
    if (e != hipSuccess) return fail(XC_EDEVICE, std::string("lookup hits: ") + hipGetErrorString(e));
    sl.copying = false;
    const auto t0 = std::chrono::steady_clock::now();
    uint64_t n = 0;
    uint32_t end = block ? sl.nb : (uint32_t)std::min<uint64_t>(sl.nb, (uint64_t)sl.next_b + max_b);
    if (sl.next_b == 0 && !xc__mem_live(c->mem)) {
        // no hash entered twice: the whole run at once, chunks of it simulated ahead on helper
        // threads (a fraction of a millisecond for a cfg5 batch)
        xc__mem_hits_run(c->mem, sl.h, sl.rec_base.data(), 0u, sl.nb);
        for (uint32_t b = 0; b < sl.nb; b++) n += sl.h[sl.rec_base[b]] & 0xFFFFFFFFu;
        end = sl.next_b = sl.nb;
    }
    for (uint32_t b = sl.next_b; b < end; b++) {
        const uint64_t *r = sl.h + sl.rec_base[b];
        const uint64_t k = r[0] & 0xFFFFFFFFu;
        xc__mem_hits(c->mem, r + 1, k, (r[0] >> 63) ? 0 : 1);
        n += k;
    }
    sl.next_b = end;
    c->hl_hits += n;
    c->hl_sec += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (end == sl.nb) {
        c->hl_fifo.pop_front();
        c->hl_runs++;
        *done = true;
    }
    return XC_OK;
}

// Every pending run's hits that are ready (block: all of them, waiting for their copies).
static int hits_replay(xc_cache *c, bool block)
{
    while (!c->hl_fifo.empty()) {
        bool done = false;
        if (int rc = hits_replay_front(c, block, &done)) return rc;
        if (!done) break;
    }
    return XC_OK;
}

// A finished run's hits into the next slot (enqueued behind the run: tokens and collision records
// are final, the tail check's included).
// The host paths' plan pools (plan_acquire): at most this many plans of at most this many buffers.
static const size_t PLAN_POOL_MAX = 8;
static const uint64_t PLAN_POOL_NBUF = 64;

// The next slot for run p's hits: its older hits replayed first (the FIFO keeps the runs' order),
// buffers of the run's size.
static int hits_slot(xc_plan *p, int *slot)
{
    xc_cache *c = p->cache;
    const int si = *slot = c->hl_next;
    while (std::find(c->hl_fifo.begin(), c->hl_fifo.end(), si) != c->hl_fifo.end()) {
        bool done = false;
        if (int rc = hits_replay_front(c, true, &done)) return rc;
    }
    xc_cache::HitSlot &sl = c->hl[si];
    if (!sl.ev) HIPCHK(hipEventCreateWithFlags(&sl.ev, hipEventDisableTiming));
    const size_t words = p->hit_base[p->nb];
    if (sl.cap < words || sl.tb_cap < (size_t)p->nb + 1) {
        HIPCHK(hipEventSynchronize(sl.ev));  // (a dropped slot's copy may still run)
        dfree(sl.d);
        dfree(sl.dtb);
        pool_free(sl.h);
        sl.d = nullptr;
        sl.h = nullptr;
        sl.dtb = nullptr;
        sl.cap = sl.tb_cap = 0;
        sl.serial = 0;
        const size_t cap = words + words / 4, tbc = (size_t)p->nb + 1 + p->nb / 4;
        if (dmalloc(&sl.d, cap * 8) != hipSuccess || dmalloc(&sl.dtb, tbc * 4) != hipSuccess ||
            hmalloc((void **)&sl.h, cap * 8) != hipSuccess)
            return fail(XC_ENOMEM, "lookup-hit buffers: allocation failed");
        void *dp = nullptr;
        HIPCHK(hipHostGetDevicePointer(&dp, sl.h, 0));
        sl.hd = (uint64_t *)dp;
        sl.cap = cap;
        sl.tb_cap = tbc;
        sl.copying = false;
    }
    return XC_OK;
}

// A host-path run's hits (its host synchronises the context stream right after the run): k_hits
// writes them straight into the slot's pinned memory behind the run, with no copy, stream or event.
static int hits_enqueue_direct(xc_plan *p)
{
    xc_cache *c = p->cache;
    if (!p->nb) return XC_OK;
    int si = 0;
    if (int rc = hits_slot(p, &si)) return rc;
    xc_cache::HitSlot &sl = c->hl[si];
    if (sl.copying) {  // (a dropped slot's copy may still run into h)
        HIPCHK(hipEventSynchronize(sl.ev));
        sl.copying = false;
    }
    hipLaunchKernelGGL(k_hits, dim3((p->nb + 3) / 4), dim3(256), 0, c->ctx->stream, p->P, sl.hd);
    HIPCHK(hipGetLastError());
    sl.rec_base = p->hit_base;
    sl.serial = 0;  // (dtb does not hold this layout)
    sl.nb = p->nb;
    sl.next_b = 0;
    sl.host_sync = true;
    c->hl_fifo.push_back(si);
    c->hl_next = si ^ 1;
    return XC_OK;
}

// A finished run's hits into the next slot (enqueued behind the run: tokens and collision records
// are final, the tail check's included), copied to the host on the hit-log stream.
static int hits_enqueue(xc_plan *p)
{
    xc_cache *c = p->cache;
    if (!p->nb) return XC_OK;
    int si = 0;
    if (int rc = hits_slot(p, &si)) return rc;
    xc_cache::HitSlot &sl = c->hl[si];
    hipStream_t m = c->ctx->stream;
    if (!c->hl_stream) {
        HIPCHK(hipStreamCreateWithFlags(&c->hl_stream, hipStreamNonBlocking));
        HIPCHK(hipEventCreateWithFlags(&c->hl_packed, hipEventDisableTiming));
    }
    HIPCHK(hipStreamWaitEvent(m, sl.ev, 0));  // the slot's previous copy has read d
    if (sl.serial != p->serial) {  // (the layout of another plan: its hit_base)
        HIPCHK(hipMemcpyAsync(sl.dtb, p->d_hit_base, ((size_t)p->nb + 1) * 4, hipMemcpyDeviceToDevice, m));
        sl.rec_base = p->hit_base;
        sl.serial = p->serial;
    }
    hipLaunchKernelGGL(k_hits, dim3((p->nb + 3) / 4), dim3(256), 0, m, p->P, sl.d);
    HIPCHK(hipGetLastError());
    HIPCHK(hipEventRecord(c->hl_packed, m));
    HIPCHK(hipStreamWaitEvent(c->hl_stream, c->hl_packed, 0));
    // the slot to pinned memory by the copy engine (no compute units: a kernel writing only the
    // filled words across PCIe took ~250 us of CU slots beside the next run, cfg5)
    HIPCHK(hipMemcpyAsync(sl.h, sl.d, (size_t)p->hit_base[p->nb] * 8, hipMemcpyDeviceToHost, c->hl_stream));
    HIPCHK(hipEventRecord(sl.ev, c->hl_stream));
    sl.copying = true;
    sl.host_sync = false;
    sl.nb = p->nb;
    sl.next_b = 0;
    c->hl_fifo.push_back(si);
    c->hl_next = si ^ 1;
    return XC_OK;
}

// The pending run's hits packed and on their way to the host (hit log).
static int hits_flush(xc_cache *c)
{
    xc_plan *p = c->hl_pend;
    if (!p) return XC_OK;
    c->hl_pend = nullptr;
    return hits_enqueue(p);
}

// A pending decode run's hits into the recent window (before anything that comes after it).
static int cache_settle_dec(xc_cache *c)
{
    if (!c->mem || c->engine || !c->pend_dec) return XC_OK;
    void *d = c->pend_dec;
    c->pend_dec = nullptr;
    uint64_t *h = nullptr, n = 0;
    int complete = 1;
    if (int rc = xc__dplan_hits(d, &h, &n, &complete)) return rc;
    xc__mem_hits(c->mem, h, n, complete);
    free(h);
    return XC_OK;
}

// The pending runs' lookup hits into the recent window (before anything that comes after them).
static int cache_settle(xc_cache *c)
{
    if (!c->mem || c->engine) return XC_OK;
    if (int rc = set_dev(c->ctx)) return rc;
    if (int rc = hits_flush(c)) return rc;
    if (int rc = hits_replay(c, true)) return rc;
    return cache_settle_dec(c);
}

// For the replay engine (xc_memcache.cpp): the window is complete before it reads it.
extern "C" int xc__cache_settle(xc_cache *c) { return c ? cache_settle(c) : XC_OK; }

// (bench) runs replayed into the window, their hits, host seconds spent.
extern "C" int xc__cache_hit_stats(xc_cache *c, uint64_t *runs, uint64_t *hits, double *sec)
{
    if (!c || !runs || !hits || !sec) return fail(XC_EINVAL, "null");
    *runs = c->hl_runs;
    *hits = c->hl_hits;
    *sec = c->hl_sec;
    return XC_OK;
}

// For xc_decode.hip: a decode run on the memory cache starts (the pending run is replayed first;
// *slow: the replay engine must run it) / has finished (its hits are the pending ones now) / its
// plan is destroyed.
extern "C" int xc__cache_run_start(xc_cache *c, int *slow)
{
    *slow = 0;
    c->last_plan = nullptr;  // (a decode run writes segments and tables)
    int rc = cache_settle(c);
    if (!rc && c->mem && !c->engine) *slow = xc__mem_live(c->mem);
    return rc;
}
extern "C" void xc__cache_run_done_dec(xc_cache *c, void *dplan)
{
    if (c->mem && !c->engine) c->pend_dec = dplan;
}
extern "C" void xc__cache_plan_gone_dec(xc_cache *c, void *dplan)
{
    if (c->pend_dec == dplan) cache_settle(c);
}
extern "C" int xc__mem_decode_batch(xc_memmodel *m, const uint8_t *in, const uint64_t *in_off,
                                    const uint64_t *in_len, uint64_t nbuf, uint8_t *out, const uint64_t *out_off,
                                    const uint64_t *out_cap, uint64_t *out_len, uint64_t *consumed, int32_t *status,
                                    uint64_t *unknown, int32_t *has_unknown);
extern "C" xc_memmodel *xc__cache_mem(xc_cache *c) { return c->mem; }

extern "C" int xc_plan_destroy(xc_plan *p)
{
    if (!p) return XC_OK;
    hipSetDevice(p->cache->ctx->dev);
    if (p->cache->hl_pend == p) hits_flush(p->cache);  // (its hits, before its arrays go)
    // pooled memory goes back for reuse at once: nothing may still read or write it
    hipStreamSynchronize(p->cache->ctx->stream);
    if (p->hs) hipStreamSynchronize(p->hs);
    if (p->cs) hipStreamSynchronize(p->cs);
    if (p->es) hipStreamSynchronize(p->es);
    p->S.release();
    p->D.release();
    p->dset.release(false);
    dfree(p->d_buf_grp0);
    dfree(p->d_rec);
    dfree(p->d_rec_cnt);
    dfree(p->d_ainfo);
    dfree(p->d_agap);
    dfree(p->d_tcnt);
    dfree(p->d_pcnt);
    dfree(p->d_pq);
    dfree(p->d_tlist);
    dfree(p->d_blk_anc);
    dfree(p->d_amix);
    dfree(p->d_buf_off);
    dfree(p->d_out_off);
    dfree(p->d_buf_len);
    dfree(p->d_chunk0);
    dfree(p->d_tok_base);
    dfree(p->d_hit_base);
    dfree(p->d_chunks);
    dfree(p->d_desc);
    dfree(p->P.tok_cnt);
    dfree(p->P.tok_lb);
    dfree(p->P.tok_le);
    dfree(p->P.tok_seg);
    dfree(p->P.tok_op);
    dfree(p->P.tok_dpos);
    dfree(p->P.tok_h);
    dfree(p->P.tok_known);
    dfree(p->P.blk_h);
    dfree(p->P.blk_pref);
    dfree(p->P.blk_cmp);
    dfree(p->P.sb_count);
    dfree(p->d_chunk_blk);
    dfree(p->d_blk_base);
    dfree(p->d_blk_buf);
    dfree(p->d_blk_grp);
    dfree(p->d_l2mix);
    dfree(p->d_fmix);
    dfree(p->P.buf_next);
    dfree(p->P.buf_nref);
    dfree(p->P.buf_slot);
    dfree(p->P.ctl);
    dfree(p->d_stream_st);
    dfree(p->d_stream_res);
    dfree(p->d_coll);
    dfree(p->d_coll_cnt);
    for (auto &x : p->ev_live) { hipEventDestroy(x.second.first); hipEventDestroy(x.second.second); }
    for (auto e : p->ev_pool) hipEventDestroy(e);
    if (p->hs) {
        hipStreamSynchronize(p->hs);  // (the context's side stream: kept)
    }
    if (p->gexec) hipGraphExecDestroy(p->gexec);
    if (p->ev_start) hipEventDestroy(p->ev_start);
    if (p->ev_ctl) hipEventDestroy(p->ev_ctl);
    if (p->h_ctl) pool_free(p->h_ctl);
    if (p->cs) {
        hipStreamSynchronize(p->cs);  // (the context's copy stream: kept)
    }
    for (auto e : p->ev_h2d)
        if (e) hipEventDestroy(e);
    dfree(p->e_in);
    dfree(p->e_out);
    dfree(p->e_len);
    dfree(p->e_total);
    for (auto e : p->ev_hash)
        if (e) hipEventDestroy(e);
    for (auto e : p->ev_go)
        if (e) hipEventDestroy(e);
    if (p->ev_sb0) hipEventDestroy(p->ev_sb0);
    if (p->ev_last) hipEventDestroy(p->ev_last);
    pool_free(p->h_lenpos);
    pool_free(p->h_st);
    if (p->es) {
        hipStreamSynchronize(p->es);
        hipStreamDestroy(p->es);
    }
    if (p->ev_ins) hipEventDestroy(p->ev_ins);
    if (p->ev_emit) hipEventDestroy(p->ev_emit);
    if (p->cache->last_plan == p) p->cache->last_plan = nullptr;
    delete p;
    return XC_OK;
}

extern "C" int xc_plan_layout(xc_plan *p, uint64_t *in_off, uint64_t *out_off, uint64_t *in_bytes,
                              uint64_t *out_bytes)
{
    if (!p) return fail(XC_EINVAL, "null");
    if (in_off) std::copy(p->in_off.begin(), p->in_off.end(), in_off);
    if (out_off) std::copy(p->out_off.begin(), p->out_off.end(), out_off);
    if (in_bytes) *in_bytes = p->in_bytes;
    if (out_bytes) *out_bytes = p->out_bytes;
    return XC_OK;
}

extern "C" int xc_plan_set_timing(xc_plan *p, int enable)
{
    if (!p) return fail(XC_EINVAL, "null");
    p->timing = enable == XC_TIMING_SCAN ? XC_TIMING_SCAN : enable ? XC_TIMING_ALL : 0;
    return XC_OK;
}

extern "C" int xc_plan_kernel_times(xc_plan *p, xc_kernel_times *out, int reset)
{
    if (!p) return fail(XC_EINVAL, "null");
    if (out) *out = p->ktimes;
    if (reset) p->ktimes = xc_kernel_times{};
    return XC_OK;
}

extern "C" int xc_plan_stats(xc_plan *p, xc_run_stats *st)
{
    if (!p || !st) return fail(XC_EINVAL, "null");
    *st = p->stats;
    return XC_OK;
}

extern "C" int xc_plan_set_scan(xc_plan *p, int mode)
{
    if (!p || mode < XC_SCAN_AUTO || mode > XC_SCAN_ANCHOR) return fail(XC_EINVAL, "scan mode");
    if (p->inflight) return fail(XC_EBUSY, "a run of this plan is in flight");
    p->scan_mode = mode;
    return XC_OK;
}

// XC_ANCHOR_MIN_KEYS (default): the cached + new segments from which the anchor index replaces the
// exact scan in XC_SCAN_AUTO (below it the exact scan's level-1 filter still sorts out nearly
// every window end and the anchors' hashing costs more than it saves: cfg5-shaped runs of 4096 /
// 8192 / 16384 buffers, 143 k / 278 k / 549 k keys, exact 628 / 650 / 626, anchor 565 / 667 / 701
// GiB/s, profiles/r03/crossover_r3p.txt).  The environment XC_SCAN=exact|anchor overrides a plan's
// AUTO mode (tests).
static const uint64_t ANCHOR_MIN_KEYS = 200000;
static uint64_t anc_min_keys()
{
    const char *e = getenv("XC_ANCHOR_MIN_KEYS");
    return e ? (uint64_t)atoll(e) : ANCHOR_MIN_KEYS;
}
static int scan_mode_of(const xc_plan *p)
{
    if (p->scan_mode != XC_SCAN_AUTO) return p->scan_mode;
    const char *e = getenv("XC_SCAN");
    if (e && !strcmp(e, "exact")) return XC_SCAN_EXACT;
    if (e && !strcmp(e, "anchor")) return XC_SCAN_ANCHOR;
    return XC_SCAN_AUTO;
}

// Decide whether a run uses the anchor index (the cache's count known on the host): its arrays on
// first use, the index caught up with segments entered without it.
static int plan_anchor_setup(xc_plan *p)
{
    xc_cache *c = p->cache;
    p->anc_run = false;
    const int mode = scan_mode_of(p);
    if (mode != XC_SCAN_EXACT && cache_anc_ok(c) && !p->P.stream_st && p->nb && c->host_count >= 0) {
        const uint64_t keys = (uint64_t)c->host_count + p->max_new;
        p->anc_run = mode == XC_SCAN_ANCHOR || keys >= anc_min_keys();
    }
    if (p->anc_run) {
        hipStream_t s = c->ctx->stream;
        if (!p->d_rec) {
            HIPCHK(dmalloc(&p->d_rec, std::max<uint64_t>(p->ngroups, 1) * REC_CAP * 8));
            HIPCHK(dmalloc(&p->d_rec_cnt, std::max<uint64_t>(p->ngroups, 1) * 4));
            HIPCHK(dmalloc(&p->d_ainfo, std::max<uint64_t>(p->ngroups, 1) * sizeof(uint4)));
            HIPCHK(dmalloc(&p->d_agap, std::max<uint64_t>(p->ngroups, 1) * AGAP_CAP * sizeof(uint2)));
            HIPCHK(dmalloc(&p->d_tcnt, std::max<uint64_t>(p->nb, 1) * 4));
            HIPCHK(hipMemsetAsync(p->d_tcnt, 0, std::max<uint64_t>(p->nb, 1) * 4, s));
            HIPCHK(dmalloc(&p->d_tlist, std::max<uint64_t>(p->nb, 1) * COLL_CAP * sizeof(uint4)));
            HIPCHK(dmalloc(&p->d_pcnt, std::max<uint64_t>(p->nchunks, 1) * 4));
            HIPCHK(hipMemsetAsync(p->d_pcnt, 0, std::max<uint64_t>(p->nchunks, 1) * 4, s));
            HIPCHK(dmalloc(&p->d_pq, std::max<uint64_t>(p->nchunks, 1) * PROP_CAP * 4));
            HIPCHK(dmalloc(&p->d_blk_anc, std::max<uint64_t>(p->nblocks, 1) * 8));
            HIPCHK(dmalloc(&p->d_amix, (size_t)ANC_FILT_WORDS * 4));
            HIPCHK(hipMemsetAsync(p->d_rec_cnt, 0, std::max<uint64_t>(p->ngroups, 1) * 4, s));
            p->dset.a.filt = p->d_amix;
            p->P.rec = p->d_rec;
            p->P.rec_cnt = p->d_rec_cnt;
            p->P.ainfo = p->d_ainfo;
            p->P.agap = p->d_agap;
            p->P.blk_anc = p->d_blk_anc;
            p->P.amix = p->d_amix;
            p->P.danc = p->dset.a;
        }
        int rc = cache_anc_catch_up(c);
        if (rc) return rc;
    }
    p->P.anc_run = p->anc_run ? 1u : 0u;
    p->P.anc_scan = 0;
    p->anc_scan_on = p->anc_run;
    p->anc_any = false;
    if (p->anc_run) c->anc_dirty = true;
    return XC_OK;
}

extern "C" int xc_plan_set_streams(xc_plan *p, const uint64_t *start, const int64_t *cand, const uint32_t *flags)
{
    if (!p) return fail(XC_EINVAL, "null");
    int rc = set_dev(p->cache->ctx);
    if (rc) return rc;
    hipStream_t s = p->cache->ctx->stream;
    if (!start && !cand && !flags) {  // back to fresh encode + flush per buffer
        p->P.stream_st = nullptr;
        p->P.stream_res = nullptr;
        return XC_OK;
    }
    if (p->inflight) return fail(XC_EBUSY, "a run of this plan is in flight (xc_encode_poll / xc_encode_wait)");
    std::vector<uint4> st(p->nb);
    bool carried = false;
    for (uint32_t i = 0; i < p->nb; i++) {
        const uint64_t n = p->len[i], a = start ? start[i] : 0;
        const int64_t c = cand ? cand[i] : -1;
        // the reference's invariants between calls: the carried candidate's window is complete
        // (c + 2048 <= start) and was not yet due for declaration (c + 4095 >= start)
        if (a > n || (c >= 0 && ((uint64_t)c + XC_SEG > a || (uint64_t)c + 2 * XC_SEG - 1 < a)) || c < -1)
            return fail(XC_EINVAL, "invalid stream state for buffer " + std::to_string(i));
        st[i] = make_uint4((uint32_t)a, c < 0 ? NONE : (uint32_t)c, flags ? flags[i] & SF_NOFLUSH : 0u, 0u);
        carried |= c >= 0;
    }
    const size_t nb1 = std::max<uint32_t>(p->nb, 1);
    if (!p->d_stream_st) {
        HIPCHK(dmalloc(&p->d_stream_st, nb1 * sizeof(uint4)));
        HIPCHK(dmalloc(&p->d_stream_res, nb1 * sizeof(uint2)));
        if (hmalloc((void **)&p->h_st, nb1 * sizeof(uint4)) != hipSuccess) return fail(XC_ENOMEM, "pinned allocation failed");
    }
    // (the same states as the device holds, e.g. a pooled plan of one connection's calls: no copy;
    // else through pinned staging, ordered before the run on the context stream: no host wait.
    // The staging is rewritten only here, after the plan's last run, which the copy preceded)
    const bool same = p->st_dev.size() == st.size() &&
                      std::equal(st.begin(), st.end(), p->st_dev.begin(), [](const uint4 &x, const uint4 &y) {
                          return x.x == y.x && x.y == y.y && x.z == y.z && x.w == y.w;
                      });
    if (p->nb && !same) {
        HIPCHK(hipStreamSynchronize(s));  // (an earlier upload from the staging has been done)
        std::copy(st.begin(), st.end(), p->h_st);
        HIPCHK(hipMemcpyAsync(p->d_stream_st, p->h_st, p->nb * sizeof(uint4), hipMemcpyHostToDevice, s));
        p->st_dev = st;
    }
    p->cand_carried = carried;
    p->P.stream_st = p->d_stream_st;
    p->P.stream_res = p->d_stream_res;
    return XC_OK;
}

extern "C" int xc_plan_stream_results(xc_plan *p, uint64_t *base, int64_t *cand)
{
    if (!p || (p->nb && (!base || !cand))) return fail(XC_EINVAL, "null");
    if (!p->P.stream_res) return fail(XC_EINVAL, "plan has no stream state (xc_plan_set_streams)");
    int rc = set_dev(p->cache->ctx);
    if (rc) return rc;
    std::vector<uint2> r(p->nb);
    if (p->res_staged && p->nb) memcpy(r.data(), p->h_lenpos + 2 * (size_t)p->nb, p->nb * sizeof(uint2));  // (nb >= 1)
    else if (p->nb) HIPCHK(hipMemcpy(r.data(), p->d_stream_res, p->nb * sizeof(uint2), hipMemcpyDeviceToHost));
    for (uint32_t i = 0; i < p->nb; i++) {
        base[i] = r[i].x;
        cand[i] = r[i].y == NONE ? -1 : (int64_t)r[i].y;
    }
    return XC_OK;
}

// The run's one host wait: the control words through a pinned buffer, then a spin on an event
// (returns within a few us of the copy; a blocking stream synchronize wakes up later).
// Wait for an event: poll it (a blocking wait wakes up tens of microseconds late), yielding the
// core to other threads of the process (a proxy's event loop) after the first ~20 us.
static hipError_t spin_wait(hipEvent_t ev)
{
    hipError_t e;
    for (int i = 0; (e = hipEventQuery(ev)) == hipErrorNotReady; i++)
        if (i >= 64) sched_yield();
    return e;
}
extern "C" hipError_t xc__spin_wait(hipEvent_t ev) { return spin_wait(ev); }

static int ctl_buffers(xc_plan *p)
{
    if (!p->h_ctl) {
        if (hmalloc((void **)&p->h_ctl, CTL_WORDS * 4) != hipSuccess) return fail(XC_ENOMEM, "pinned allocation failed");
        void *dp = nullptr;
        HIPCHK(hipHostGetDevicePointer(&dp, p->h_ctl, 0));
        p->d_hctl = (uint32_t *)dp;
        HIPCHK(hipEventCreateWithFlags(&p->ev_ctl, hipEventDisableTiming));
    }
    return XC_OK;
}

// XC_COMPLETE_STREAM: a published first pass is decided once the emit's publication has cleared
// the sentinel in the last control word (it is written last); the event covers a pass that
// published nothing (the caller then reads the words).
static bool published(const xc_plan *p)
{
    if (*(volatile const uint32_t *)(p->h_ctl + CTL_WORDS - 1) != 0u) return false;
    __atomic_thread_fence(__ATOMIC_ACQUIRE);
    return true;
}

static bool early_done(const xc_plan *p)
{
    return p->completion == XC_COMPLETE_STREAM && p->pass_published;
}

// Not published yet: has the stream drained (the pass ended without publishing: the caller reads
// the words), or failed?
static hipError_t pass_state(xc_plan *p)
{
    return published(p) ? hipSuccess : hipStreamQuery(p->cache->ctx->stream);
}

// A publication poll asks the stream whether it drained only after 2000 us without a
// publication (checked every 256 polls): hipStreamQuery on a stream with kernels in flight enqueues
// a marker behind them, whose release leaves the device idle for ~6 us before the next kernel (the
// decoder's emit -> the next restore, cfg4).  A pass that publishes nothing still ends the poll.
extern "C" bool xc__query_due(int64_t *t0)
{
    static const int64_t lim = abl_env("XC_QUERY_US") ? atoll(abl_env("XC_QUERY_US")) * 1000 : 2000000;
    const int64_t t = std::chrono::duration_cast<std::chrono::nanoseconds>(
                          std::chrono::steady_clock::now().time_since_epoch()).count();
    if (*t0 == 0) *t0 = t;
    return t - *t0 >= lim;
}

// While the device works: the earlier runs' lookup hits whose copies are complete go to the window.
static void replay_while_waiting(xc_plan *p)
{
    xc_cache *c = p->cache;
    if (c->hl_fifo.empty() || !c->mem || c->engine) return;
    bool done = false;
    hits_replay_front(c, false, &done, 1024);  // (~0.1 ms of host work; an error shows at the settle)
}

static hipError_t wait_decided(xc_plan *p)
{
    if (!early_done(p)) {
        for (int i = 0;; i++) {
            const hipError_t e = hipEventQuery(p->ev_ctl);
            if (e != hipErrorNotReady) return e;
            replay_while_waiting(p);
            if (i >= 64) sched_yield();
        }
    }
    int64_t t0 = 0;
    for (int i = 0;; i++) {
        if (published(p)) return hipSuccess;
        replay_while_waiting(p);
        if ((i & 255) == 255) {
            if (xc__query_due(&t0)) {
                const hipError_t e = pass_state(p);
                if (e != hipErrorNotReady) return e;
            }
            if (i >= 4096) sched_yield();
        }
    }
}

// Wait for the copy of the control words enqueued before ev_ctl.
static int wait_ctl(xc_plan *p, uint32_t *ctl);

static int read_ctl(xc_plan *p, uint32_t *ctl)
{
    hipStream_t s = p->cache->ctx->stream;
    int rc = ctl_buffers(p);
    if (rc) return rc;
    HIPCHK(hipMemcpyAsync(p->h_ctl, p->P.ctl, CTL_WORDS * 4, hipMemcpyDeviceToHost, s));
    return wait_ctl(p, ctl);
}

static int wait_ctl(xc_plan *p, uint32_t *ctl)
{
    hipStream_t s = p->cache->ctx->stream;
    HIPCHK(hipEventRecord(p->ev_ctl, s));
    HIPCHK(spin_wait(p->ev_ctl));
    memcpy(ctl, p->h_ctl, CTL_WORDS * 4);
    ev_collect(p);
    return XC_OK;
}

static int launch_scan(xc_plan *p, const Layer &L, const DevSet &set, uint32_t ck_lo, uint32_t ck_hi,
                       const DevSet *set2 = nullptr, int shadow = 0)
{
    if (ck_hi <= ck_lo) return XC_OK;
    xc_ctx *ctx = p->cache->ctx;
    ScanArgs a{p->P, L, set, ck_lo, ck_hi, 0, DevSet{}, 0, (const uint32_t *)set.l2, shadow, p->scan_unit,
               set.filt, XC_FILT_WORDS};
    if (set2) {
        a.set2 = *set2;
        a.has2 = 1;
        a.l2 = (const uint32_t *)p->d_l2mix;  // cache | set2, built by k_clear_set + k_blockhash
        a.filt = p->d_fmix;               // the same for level 1, folded
        a.filt_words = XC_FILT_WORDS >> p->P.fmix_fold;
    }
    KSpan span(p, XC_K_SCAN);
    if (p->timing) p->ktimes.scan_bytes += p->chunk_bytes[ck_hi] - p->chunk_bytes[ck_lo];
    uint32_t need = (ck_hi - ck_lo + SCAN_WAVES * p->scan_unit - 1) / (SCAN_WAVES * p->scan_unit);
    uint32_t grid = std::min<uint32_t>(need, (uint32_t)ctx->n_cu);
    // XC_SCAN_GRID=n (-DXC_ABLATIONS builds): at most n scan workgroups, the other CUs left to the
    // kernels of other streams
    static const uint32_t grid_cap = abl_env("XC_SCAN_GRID") ? (uint32_t)atoi(abl_env("XC_SCAN_GRID")) : 0u;
    if (grid_cap) grid = std::min(grid, grid_cap);
    // XC_SCAN_ABLATION=m (-DXC_ABLATIONS builds, timing only: results are wrong) runs k_scan<m>
    static const int abl = abl_env("XC_SCAN_ABLATION") ? atoi(abl_env("XC_SCAN_ABLATION")) : 0;
    auto kern = abl == 1 ? k_scan<1> : abl == 2 ? k_scan<2> : abl == 3 ? k_scan<3> : abl == 4 ? k_scan<4>
              : abl == 5 ? k_scan<5> : k_scan<0>;
    if (abl) a.mode = (uint32_t)abl;
    hipLaunchKernelGGL(kern, dim3(grid), dim3(64 * SCAN_WAVES), 0, ctx->stream, a);
    HIPCHK(hipGetLastError());
    return XC_OK;
}

// The anchor scan of buffers [j0, s1) (chunks [ck_lo, ck_hi)) into layer S.
static int launch_ascan(xc_plan *p, uint32_t j0, uint32_t s1, uint32_t ck_lo, uint32_t ck_hi, int shadow)
{
    if (ck_hi <= ck_lo) return XC_OK;
    const uint32_t g_lo = p->grp_base[j0], g_hi = p->grp_base[s1];
    AScanArgs a{p->P, p->P.S, ck_lo, ck_hi, shadow, g_lo, g_hi, p->d_pcnt, p->d_pq};
    KSpan span(p, XC_K_SCAN);
    if (p->timing) p->ktimes.scan_bytes += p->chunk_bytes[ck_hi] - p->chunk_bytes[ck_lo];
    hipStream_t s = p->cache->ctx->stream;
    if (g_hi > g_lo) {
        hipLaunchKernelGGL(k_aprop, dim3((g_hi - g_lo + APROP_GROUPS - 1) / APROP_GROUPS), dim3(256), 0, s, a);
        HIPCHK(hipGetLastError());
    }
    hipLaunchKernelGGL(k_aevents, dim3((ck_hi - ck_lo + 255) / 256), dim3(256), 0, s, a);
    HIPCHK(hipGetLastError());
    return XC_OK;
}

static int launch_resolve(xc_plan *p, const Layer &L, int dmode, uint32_t ck_lo, uint32_t ck_hi)
{
    ResolveArgs a{p->P, L, dmode, ck_lo, ck_hi};
    KSpan span(p, XC_K_RESOLVE);
    hipLaunchKernelGGL(k_resolve, dim3(std::max<uint32_t>(1u, (ck_hi - ck_lo + RES_WAVES - 1) / RES_WAVES)),
                       dim3(64 * RES_WAVES), 0,
                       p->cache->ctx->stream, a);
    HIPCHK(hipGetLastError());
    return XC_OK;
}

static int launch_walk_round(xc_plan *p, uint32_t j0, uint32_t j1, int use_d, int shadow = 0)
{
    hipStream_t s = p->cache->ctx->stream;
    // (k_resolve, always launched just before, reset GREW / FIRST_CROSS / SHADOW)
    // one wave per buffer: the block-parallel walk on the first round where it applies, else
    // the sequential walk (every buffer on the declaration-layer rounds), then the hashes of
    // declarations no event supplied
    const uint32_t nw = use_d ? 1u : p->walk_waves;  // (later rounds walk sequentially: one wave)
    WalkArgs w{p->P, j0, j1, use_d, shadow, p->max_decl, nw};
    {
        KSpan span(p, XC_K_WALK);
        hipLaunchKernelGGL(k_walk, dim3(j1 - j0), dim3(64 * nw), walk_lds_bytes(p->max_decl), s, w);
        HIPCHK(hipGetLastError());
    }
    p->stats.walk_rounds++;
    return XC_OK;
}

static int launch_emit(xc_plan *p, uint32_t sb, uint32_t j0, uint32_t jc, uint32_t gate_sb = NONE)
{
    hipStream_t s = p->cache->ctx->stream;
    // few buffers: the slots inside the emit (one launch less)
    const bool slots = jc > j0 && jc - j0 <= EMIT_SLOTS_MAX;
    // (the pass's last sub-batch publishes the control words: from the emit when it takes the
    // slots, else from k_alloc; the non-slot emit never reads ctl_host)
    // (XC_ABL_EMIT, -DXC_ABLATIONS builds: read per launch, a diagnostic run sets it late)
    const char *abl = abl_env("XC_ABL_EMIT");
    const uint32_t ab = abl ? (uint32_t)atoi(abl) : 0u;
    // one workgroup per buffer: 4 waves when the buffers alone fill the chip, 16 for few buffers
    const bool wide = (uint64_t)(jc - j0) * EMIT_WAVES < (uint64_t)p->cache->ctx->n_cu * 16u;
    // (one pass: the plan's longest buffer has at most 64 tokens per emit wave, 2 len / 2048 + 3; for
    // the 4-wave emit only: cfg5 872-873 -> 877-879 GiB/s, cfg3 +-0, but the 16-wave one of a few
    // buffers 222-225 -> 215 (cfg2), profiles/r06/ab/emit_one_pass_r6q.txt)
    const bool one = !wide && 2u * p->max_decl - 1u <= 64u * EMIT_WAVES;
    // the two-pass emit's cache enters go to k_insert for large sub-batches (cfg5's 8192 buffers: A/B
    // 751 -> 766 GiB/s; below that the launch cost more than it saved, cfg3's 4096: 650 -> 634): there
    // one wave per workgroup enters the whole buffer; the one-pass emit spreads them over its waves and
    // keeps them (cfg5 875-880 -> 884-886 GiB/s against k_insert, profiles/r06/ab/emit_inserts_r6s.txt)
    EmitArgs e{p->P, j0, jc, gate_sb, p->emit_ctl_host, p->P.sb_count + sb, p->emit_pub_final, ab,
               !slots && !one && jc - j0 >= INSERT_SPLIT_MIN ? 1u : 0u};
    if (!slots) {
        hipLaunchKernelGGL(k_alloc, dim3(1), dim3(1024), 0, s, e);
        HIPCHK(hipGetLastError());
    }
    if (jc <= j0) return XC_OK;
    KSpan span(p, XC_K_EMIT);
    if (e.split_ins && !(ab & 4u)) {
        hipLaunchKernelGGL(p->P.anc_run ? k_insert<true> : k_insert<false>, dim3((jc - j0 + 3) / 4), dim3(256), 0, s, e);
        HIPCHK(hipGetLastError());
    }
    // (the cache enters: in k_insert, or here with or without the anchor index)
    const int ins = e.split_ins && !(ab & 4u) ? 0 : p->P.anc_run ? 2 : 1;
#define XC_EMIT_PICK(K, W)                                                                                       \
    (slots ? (ins == 2 ? K<W, true, 2> : K<W, true, 1>) : (ins == 0 ? K<W, false, 0> : ins == 2 ? K<W, false, 2> : K<W, false, 1>))
    auto kern = wide ? XC_EMIT_PICK(k_emit, 16) : one ? XC_EMIT_PICK(k_emit1, EMIT_WAVES) : XC_EMIT_PICK(k_emit, EMIT_WAVES);
#undef XC_EMIT_PICK
    // (in the context stream's order: on a stream of its own, beside the next sub-batch's predictions
    // and anchor scan, cfg5 measured -1.3 %)
    hipLaunchKernelGGL(kern, dim3(jc - j0), dim3(64 * (wide ? 16 : EMIT_WAVES)), 0, s, e);
    HIPCHK(hipGetLastError());
    return XC_OK;
}

// Predicted declarations (aligned blocks absent from the cache), then one scan of every
// position of buffers [j0, s1) against cache + predictions, resolve, first walk round.
// Hash sub-batch k's aligned blocks on the side stream once `after` (an event of the main
// stream) has passed; ev_hash[k] marks completion.
// On the main stream (st == nullptr: the run's first sub-batch, nothing to overlap with) no
// events are needed.
static int enqueue_block_hash(xc_plan *p, uint32_t k, hipEvent_t after, hipStream_t st, bool predict = false,
                              const uint32_t *limit = nullptr, uint32_t limit_cap = 0xFFFFFFFFu)
{
    const bool side = st == p->hs;
    if (after) HIPCHK(hipStreamWaitEvent(st, after, 0));
    if (p->host_path && !p->h2d_inline) HIPCHK(hipStreamWaitEvent(st, p->ev_h2d[k], 0));  // its input has landed
    const uint32_t g0 = p->grp_base[p->sub[k]], g1 = p->grp_base[p->sub[k + 1]];
    // a range of block groups; on the side stream (sub-batch k - 1 on the main stream) the block
    // compares against the entries complete when k - 1 started
    // (chained hashing may run while the main stream is several sub-batches behind: its compares
    // take the entries complete at the run's start)
    // XC_ABL_BH=m (-DXC_ABLATIONS builds: timing ablations of the block hashing, read per launch,
    // bench.py --diag-env sets it for the diagnostic steps only; the results are wrong): 2 no anchors,
    // 4 no records, 8 no G tile
    const char *abl_bh = abl_env("XC_ABL_BH");
    const int nt_abl = abl_bh ? atoi(abl_bh) & ~1 : 0;
    DeclArgs d{p->P, g0, g1, limit ? limit : side && k > 0 ? p->P.sb_count : nullptr,
               nt_abl, p->shadow, limit_cap};
    // XC_ABL_SKIP_BLOCKHASH=1 (-DXC_ABLATIONS builds, timing only, valid when every run reads the same input):
    // the side stream's block hashing after the plan's first run is skipped
    static const bool skip = abl_flag("XC_ABL_SKIP_BLOCKHASH");
    if (g1 > g0 && !(skip && side && p->runs_done > 0)) {
        KSpan span(p, XC_K_BLOCKHASH, st);
        auto kern = predict ? (p->anc_run ? k_blockhash<true, true> : k_blockhash<true, false>)
                            : (p->anc_run ? k_blockhash<false, true> : k_blockhash<false, false>);
        hipLaunchKernelGGL(kern, dim3((g1 - g0 + 3) / 4), dim3(256), 0, st, d);
        HIPCHK(hipGetLastError());
    }
    if (side) HIPCHK(hipEventRecord(p->ev_hash[k], st));
    p->next_hash = k + 1;
    return XC_OK;
}

// shadow: skip the windows in predicted-REF shadows (async pass; the step-by-step redo of a
// sub-batch scans every position).
static int launch_first_round(xc_plan *p, uint32_t sb, uint32_t j0, uint32_t s1, int shadow)
{
    hipStream_t s = p->cache->ctx->stream;
    int rc;
    const uint32_t ck_lo = p->chunk0[j0], ck_hi = p->chunk0[s1];
    p->stats.outer_rounds++;
    // the set's clear (and, first in a run, the control words' clear)
    const bool anc = p->P.anc_scan != 0;
    hipLaunchKernelGGL(k_clear_set, dim3(1024), dim3(256), 0, s, p->P.dset, p->dset.n_lo, p->dset.n_full,
                       (uint4 *)p->d_l2mix, (const uint4 *)p->P.cache.l2, anc ? nullptr : p->d_fmix,
                       (const uint32_t *)p->P.cache.filt,
                       p->P.fmix_fold, p->P.seg_count, p->P.sb_count + sb, p->zero_ctl ? p->P.ctl : nullptr,
                       p->dset.a, anc ? (uint4 *)p->d_amix : nullptr, (const uint4 *)p->P.canc.filt);
    HIPCHK(hipGetLastError());
    p->zero_ctl = false;
    const bool inline_hash = p->next_hash <= sb;
    // a run whose first sub-batch was hashed ahead: the later sub-batches' hashing may start once the
    // set is cleared (their compares read the cache count k_clear_set noted), not after this
    // sub-batch's predictions: sub-batch 1 then no longer waits for its hashes (the production trace's
    // 35 us, profiles/r04/gaps; cfg5 A/B 762-764 -> 771-773 GiB/s, profiles/r05/ab/go_early_r5.txt).
    // Nothing sub-batch 0's predictions write is read by the side stream's hashing (the declaration
    // set and the combined filters are not; block hashes and records are per sub-batch).
    const bool chain = p->next_hash == sb + 1 && sb + 2 < p->sub.size();
    const bool go_early = chain && !inline_hash;
    if (go_early) HIPCHK(hipEventRecord(p->ev_go[sb], s));
    if (inline_hash) {
        // first sub-batch of the run: nothing to overlap with, its blocks are hashed in line
        // (after whatever the caller enqueued on the context stream to fill the input), and
        // predicted by the same kernel
        if ((rc = enqueue_block_hash(p, sb, nullptr, s, true))) return rc;
    } else {
        HIPCHK(hipStreamWaitEvent(s, p->ev_hash[sb], 0));  // hashed ahead on the side stream
    }
    if (!inline_hash || j0 != p->sub[sb]) {
        DeclArgs d{p->P, j0, s1};
        KSpan span(p, XC_K_DECLHASH);
        const uint32_t nblk = p->blk_base[s1] - p->blk_base[j0];
        hipLaunchKernelGGL(k_blockpredict, dim3(std::max<uint32_t>(1u, (nblk + 255) / 256)), dim3(256), 0, s, d);
        HIPCHK(hipGetLastError());
    }
    // the next sub-batch's block hashes run beside this scan (memory-bound beside LDS/L2-bound)
    // every later sub-batch's blocks back to back on the side stream, the first after this
    // sub-batch's predictions: the side stream never waits for the main one, whose sub-batch k then
    // rarely waits for k's hashes (round 2 hashed one sub-batch ahead, beside the scan before it)
    if (chain) {
        if (!go_early) HIPCHK(hipEventRecord(p->ev_go[sb], s));
        const uint32_t last = (uint32_t)p->sub.size() - 2;
        for (uint32_t k = sb + 1; k <= last; k++)
            if ((rc = enqueue_block_hash(p, k, k == sb + 1 ? p->ev_go[sb] : nullptr, p->hs))) return rc;
    }
    if (anc) {
        if ((rc = launch_ascan(p, j0, s1, ck_lo, ck_hi, shadow))) return rc;
    } else if ((rc = launch_scan(p, p->P.S, p->P.cache, ck_lo, ck_hi, &p->P.dset, shadow))) {
        return rc;
    }
    // (the previous sub-batch's emit, earlier in the stream, wrote the segments this resolve may compare)
    if ((rc = launch_resolve(p, p->P.S, 2, ck_lo, ck_hi))) return rc;
    return launch_walk_round(p, j0, s1, 0, shadow);
}

// Host path: pack buffers [j0, j1) (emitted) to the caller's buffer.
static int launch_pack(xc_plan *p, uint32_t j0, uint32_t j1)
{
    if (!p->host_path || j1 <= j0) return XC_OK;
    hipStream_t s = p->cache->ctx->stream;
    PackArgs a{p->P, j0, j1, p->pack_dst, p->pack_cap, p->e_total, p->e_pos};
    hipLaunchKernelGGL(k_pack_offsets, dim3(1), dim3(1024), 0, s, a);
    HIPCHK(hipGetLastError());
    hipLaunchKernelGGL(k_pack_copy, dim3(j1 - j0), dim3(256), 0, s, a);
    HIPCHK(hipGetLastError());
    return XC_OK;
}

// Sub-batch sb with no host synchronisation: first round, gate, emit of the whole sub-batch.
static int encode_sub_async(xc_plan *p, uint32_t sb)
{
    const uint32_t j0 = p->sub[sb], s1 = p->sub[sb + 1];
    int rc;
    p->stats.sub_batches++;
    p->P.anc_scan = p->anc_scan_on ? 1u : 0u;
    if (p->anc_scan_on) {
        p->anc_any = true;
        p->stats.anchor_scans++;
    }
    if ((rc = launch_first_round(p, sb, j0, s1, p->shadow))) return rc;
    if ((rc = launch_emit(p, sb, j0, s1, sb))) return rc;
    // (an event recorded between two kernels leaves the device idle ~6 us: only when a next run uses it)
    if (sb == 0 && p->rec_sb0) HIPCHK(hipEventRecord(p->ev_sb0, p->cache->ctx->stream));
    return launch_pack(p, j0, s1);
}

// Sub-batch sb step by step: declaration-growth rounds until D is closed, then emit up to the
// first buffer whose lookups an earlier buffer's new declarations would change, and repeat
// from there (outer rounds).
static int encode_sub_sync(xc_plan *p, uint32_t sb, uint32_t *ctl)
{
    const uint32_t s1 = p->sub[sb + 1];
    uint32_t j0 = p->sub[sb];
    int rc;
    p->P.anc_scan = 0;  // (the exact scan: every window end against the cache)
    while (j0 < s1) {
        const uint32_t ck_lo = p->chunk0[j0], ck_hi = p->chunk0[s1];
        if ((rc = launch_first_round(p, sb, j0, s1, 0))) return rc;
        if ((rc = read_ctl(p, ctl))) return rc;
        uint32_t rounds = 0;
        while (!ctl[CTL_ERROR] && ctl[CTL_GREW]) {
            // a walk declared hashes nobody predicted: match every position against the
            // whole declaration set and walk again
            if (++rounds > MAX_ROUNDS) return fail(XC_EDEVICE, "declaration rounds did not converge");
            if ((rc = launch_scan(p, p->P.D, p->P.dset, ck_lo, ck_hi))) return rc;
            if ((rc = launch_resolve(p, p->P.D, 1, ck_lo, ck_hi))) return rc;
            if ((rc = launch_walk_round(p, j0, s1, 1))) return rc;
            if ((rc = read_ctl(p, ctl))) return rc;
        }
        if (ctl[CTL_ERROR]) return XC_OK;
        uint32_t jc = std::min<uint32_t>(ctl[CTL_FIRST_CROSS], s1);
        if (jc <= j0) jc = j0 + 1;  // cannot happen (buffer j0 has no earlier buffer); progress guard
        if ((rc = launch_emit(p, sb, j0, jc))) return rc;
        j0 = jc;
    }
    return XC_OK;
}

// The graph path applies to device-resident single-sub-batch runs without per-kernel timing
// events.  (With several sub-batches the graph loses the side stream's block hashing beside the
// scans: cfg5 A/B on one box, graph 489-507 GiB/s against 515-525 enqueued directly; the host's
// launches are hidden behind the long kernels there anyway.)
// A HIP graph of a one-sub-batch run's launches: no longer the default (ROCm 7.2: hipGraphLaunch
// starts its first node ~15-20 us after the call, where seven direct launches keep the host ahead
// of the device after the first: cfg2 A/B 187-188 -> 204-206 GiB/s, cfg3 678-682 -> 695-696,
// profiles/r05/ab/graph_vs_direct_r5s.txt).  XC_GRAPH=1 replays the graph (experiments).
static bool use_graph(xc_plan *p)
{
    const char *e = getenv("XC_GRAPH");  // (read per run: tests switch it)
    const bool on = e && atoi(e);
    // (nor for stateful streams: a duplicate enter is counted by the emit, after the graph's
    // published control words)
    return on && !p->g_off && !p->timing && !p->host_path && p->sub.size() == 2 && !p->P.stream_st;
}

// Record ev_ctl after the control words' copy to h_ctl (enqueued by the caller or published by
// the emit): the host reads them once it has passed.
static int record_ctl(xc_plan *p)
{
    // a stream-ordered published pass needs no event (its marker costs ~4 us between passes):
    // every outcome of the gate is published, and a stream query covers the rest
    if (early_done(p)) return XC_OK;
    HIPCHK(hipEventRecord(p->ev_ctl, p->cache->ctx->stream));
    return XC_OK;
}

// The first asynchronous pass of a run (the ctl words were cleared before it) as a graph launch,
// then ev_ctl; nothing waits.  (Re)captured when the arenas differ from the captured ones.
static int graph_launch(xc_plan *p)
{
    hipStream_t s = p->cache->ctx->stream;
    int rc = ctl_buffers(p);
    if (rc) return rc;
    const size_t nsub = p->sub.size() - 1;
    if (!p->gexec || p->g_in != p->P.in || p->g_out != p->P.out || p->g_len != p->P.out_len ||
        p->g_stream != p->P.stream_st || p->g_anc != p->anc_run) {
        if (p->gexec) {
            HIPCHK(hipGraphExecDestroy(p->gexec));
            p->gexec = nullptr;
        }
        // capture on the context stream (work the caller enqueued before it stays outside)
        // a one-sub-batch graph whose emit takes the slots also publishes the control words
        // (no copy launch after it)
        const uint32_t nlast = p->sub[nsub] - p->sub[nsub - 1];
        const bool publish = nsub == 1 && nlast > 0 && !p->host_path;
        HIPCHK(hipStreamBeginCapture(s, hipStreamCaptureModeRelaxed));
        const xc_run_stats st0 = p->stats;
        p->emit_ctl_host = publish ? p->d_hctl : nullptr;
        for (size_t k = 0; k < nsub && !rc; k++) {
            p->emit_pub_final = k + 1 == nsub;
            rc = encode_sub_async(p, (uint32_t)k);
        }
        p->emit_ctl_host = nullptr;
        p->emit_pub_final = 0;
        if (!rc && !publish && hipMemcpyAsync(p->h_ctl, p->P.ctl, CTL_WORDS * 4, hipMemcpyDeviceToHost, s) != hipSuccess)
            rc = fail(XC_EDEVICE, "graph capture: control-word copy");
        hipGraph_t g = nullptr;
        const hipError_t ce = hipStreamEndCapture(s, &g);
        if (!rc && ce == hipSuccess && g && hipGraphInstantiate(&p->gexec, g, nullptr, nullptr, 0) == hipSuccess) {
            p->g_stats = p->stats;
            p->g_stats.sub_batches -= st0.sub_batches;
            p->g_stats.outer_rounds -= st0.outer_rounds;
            p->g_stats.walk_rounds -= st0.walk_rounds;
            p->g_stats.anchor_scans -= st0.anchor_scans;
            p->g_in = p->P.in;
            p->g_out = p->P.out;
            p->g_len = p->P.out_len;
            p->g_stream = p->P.stream_st;
            p->g_anc = p->anc_run;
            p->g_publish = publish;
        } else {
            p->gexec = nullptr;
        }
        if (g) hipGraphDestroy(g);
        (void)hipGetLastError();
        p->stats = st0;
        if (!p->gexec) {  // not capturable here: enqueue directly from now on
            p->g_off = true;
            p->next_hash = 0;
            p->pass_published = false;
            for (size_t k = 0; k < nsub; k++)
                if ((rc = encode_sub_async(p, (uint32_t)k))) return rc;
            HIPCHK(hipMemcpyAsync(p->h_ctl, p->P.ctl, CTL_WORDS * 4, hipMemcpyDeviceToHost, s));
            return record_ctl(p);
        }
    }
    // (a sentinel in the unused last word: the emit's publication clears it)
    if (p->g_publish) p->h_ctl[CTL_WORDS - 1] = 0xFFFFFFFFu;
    HIPCHK(hipGraphLaunch(p->gexec, s));
    p->stats.sub_batches += p->g_stats.sub_batches;
    p->stats.outer_rounds += p->g_stats.outer_rounds;
    p->stats.walk_rounds += p->g_stats.walk_rounds;
    p->stats.anchor_scans += p->g_stats.anchor_scans;
    p->anc_any = p->g_stats.anchor_scans != 0;
    p->next_hash = (uint32_t)nsub;  // (the graph hashed every sub-batch's blocks)
    p->pass_published = p->g_publish;
    return record_ctl(p);
}

static int launch_tailcheck(xc_plan *p);

// Everything of a run up to its first asynchronous pass, which is enqueued with ev_ctl after it.
static int encode_submit(xc_plan *p, const uint8_t *d_in, uint8_t *d_out, uint64_t *d_out_len)
{
    if (p && p->inflight) return fail(XC_EBUSY, "a run of this plan is in flight (xc_encode_poll / xc_encode_wait)");
    // (a run another caller finished, xc_cache_quiesce: its status waits for the submitter's poll /
    // wait, which alone clears it, so that no failure of it is dropped)
    if (p && p->parked)
        return fail(XC_EBUSY, "a finished run's status waits for xc_encode_poll / xc_encode_wait");
    if (!p || (!d_in && p->nb) || (!d_out && p->nb) || (!d_out_len && p->nb)) return fail(XC_EINVAL, "null");
    int rc = set_dev(p->cache->ctx);
    if (rc) return rc;
    hipStream_t s = p->cache->ctx->stream;
    // room for every segment this run can declare (the reference's cache never fills)
    xc_cache *c = p->cache;
    // (a decode's hits go first; earlier encode runs' hits are replayed while this one works)
    if ((rc = cache_busy(c, p)) || (rc = hits_flush(c)) || (rc = cache_settle_dec(c)) || (rc = hits_replay(c, false)))
        return rc;
    if (c->mem && !c->engine) {
        // a hash entered twice may answer with other bytes than the device holds: the host paths
        // replay such runs (xc_memcache.cpp)
        if (xc__mem_live(c->mem)) return fail(XC__SLOW, "a hash entered twice is in the recent window");
        // (XC_FORCE_REPLAY=1, tests only, read per run: a device-resident run takes the replay, so that
        // its results can be compared with the device path's on the same state)
        const char *fr = getenv("XC_FORCE_REPLAY");
        if (fr && atoi(fr) && !p->host_path) return fail(XC__SLOW, "replay forced");
        p->count0 = -1;
        if (p->P.stream_st && p->cand_carried) {  // (only a carried candidate can enter a hash twice)
            uint32_t n = 0;
            if (c->host_count >= 0) n = (uint32_t)c->host_count;
            else if ((rc = cache_count_host(c, &n))) return rc;
            p->count0 = n;
        }
    }
    if ((rc = cache_reserve(c, p->max_new))) return rc;
    if (p->cache_gen != c->gen) {  // the cache grew: its arrays moved
        const PlanDev cp = cache_plandev(c);
        p->P.cache = cp.cache;
        p->P.segs = cp.segs;
        p->P.seg_count = cp.seg_count;
        p->P.seg_cap = cp.seg_cap;
        p->P.undo = cp.undo;
        p->P.canc = cp.canc;
        p->P.anc_of = cp.anc_of;
        p->P.aundo = cp.aundo;
        p->P.anc_bad = cp.anc_bad;
        p->cache_gen = c->gen;
        if (p->gexec) {
            HIPCHK(hipGraphExecDestroy(p->gexec));
            p->gexec = nullptr;
        }
    }
    p->P.in = d_in;
    p->P.out = d_out;
    p->P.out_len = d_out_len;
    p->stats = xc_run_stats{};
    p->tail_enqueued = false;
    p->res_staged = false;
    {   // the first scans' level-1 image: folded while it keeps >= 16 bits per key (the keys of
        // the cache at the start, when known, and every segment this run can enter)
        const uint64_t keys = (p->cache->host_count >= 0 ? (uint64_t)p->cache->host_count : p->cache->cap) + p->max_new;
        uint32_t f = 0;
        while (f < MIX_FOLD_MAX && ((uint64_t)XC_FILT_WORDS * 32u >> (f + 1)) >= 16u * keys) f++;
        p->P.fmix_fold = f;
    }
    if ((rc = plan_anchor_setup(p))) return rc;
    // the first sub-batch's blocks hashed ahead on the side stream (their compares take the entries
    // complete when the previous run's last sub-batch started: immutable since, nothing else having
    // written the cache; a restore in between only unmaps later entries, which the predictions then
    // do not name)
    const bool early = p->input_ready && p->early_ok && c->last_plan == p && p->sub.size() > 2 &&
                       !p->P.stream_st && !p->host_path && !use_graph(p) && !p->timing;
    static const bool dbg_early = abl_flag("XC_DEBUG_EARLY");
    if (dbg_early)
        fprintf(stderr, "early=%d input_ready=%d early_ok=%d last=%d nsub=%zu stream=%d host=%d graph=%d timing=%d\n",
                (int)early, (int)p->input_ready, (int)p->early_ok, (int)(c->last_plan == p), p->sub.size() - 1,
                (int)(p->P.stream_st != nullptr), (int)p->host_path, (int)use_graph(p), p->timing);
    if (c->last_plan != p) c->last_plan = nullptr;
    p->early_ok = false;
    // (a restore or a truncation since the last run removed the entries from its floor up, and the
    // hashing below may run before it on the side stream: only the entries under it are compared,
    // which k_blockpredict, after it, finds too)
    const uint32_t floor = c->removed_floor;
    c->removed_floor = 0xFFFFFFFFu;
    uint32_t hashed = 0;
    if (early) {
        // every sub-batch's blocks ahead, back to back on the side stream (their compares take the
        // same entries: complete when the previous run's last sub-batch started, under the floor);
        // the main stream then records no start event for them (an event between two of its
        // kernels idles the device ~6 us) and sub-batch 1's hashing starts as soon as 0's ends
        const uint32_t *lim = p->P.sb_count + (p->sub.size() - 2);
        const uint32_t upto = (uint32_t)p->sub.size() - 1;
        for (uint32_t k = 0; k < upto; k++)
            // (sub-batch 0 after the previous run's sub-batch 0 emit; the later ones, chained behind it,
            // after the previous run's last emit: its k_insert / k_emit read those block arrays after the
            // stream-ordered completion let the host return)
            if ((rc = enqueue_block_hash(p, k, k == 0 ? p->ev_sb0 : k == 1 ? p->ev_last : nullptr, p->hs, false, lim,
                                         floor)))
                return rc;
        hashed = upto;
        p->early_runs++;
        p->stats.early_hashed = 1;
    }
    p->cache->host_count = -1;
    if (p->sub.size() > 1) p->zero_ctl = true;  // (the first k_clear_set clears the control words)
    else HIPCHK(hipMemsetAsync(p->P.ctl, 0, CTL_WORDS * 4, s));
    p->next_hash = hashed;  // (sub-batches hashed ahead: their predictions wait for ev_hash[k])
    const size_t nsub = p->sub.size() - 1;
    if ((rc = ctl_buffers(p))) return rc;
    p->rec_sb0 = p->input_ready && p->sub.size() > 2;
    if (use_graph(p)) {
        if ((rc = graph_launch(p))) return rc;
    } else {
        // stream-ordered completion: the last sub-batch's k_alloc (or slot-taking emit) publishes
        // the control words, so the host returns before the last emit has finished (no copy of
        // the words after it: a copy landing after the host re-armed the sentinel would clear it)
        const bool pub = p->completion == XC_COMPLETE_STREAM && !p->timing && !p->host_path && nsub > 0 &&
                         p->sub[nsub] > p->sub[nsub - 1] && !p->P.stream_st;
        if (pub) p->h_ctl[CTL_WORDS - 1] = 0xFFFFFFFFu;
        p->pass_published = pub;
        for (size_t k = 0; k < nsub; k++) {
            p->emit_ctl_host = pub ? p->d_hctl : nullptr;
            p->emit_pub_final = k + 1 == nsub;
            rc = encode_sub_async(p, (uint32_t)k);
            p->emit_ctl_host = nullptr;
            p->emit_pub_final = 0;
            if (rc) return rc;
        }
        if (p->rec_sb0) HIPCHK(hipEventRecord(p->ev_last, s));  // (the next run's early hashing of sub-batches >= 1)
        if (!pub) HIPCHK(hipMemcpyAsync(p->h_ctl, p->P.ctl, CTL_WORDS * 4, hipMemcpyDeviceToHost, s));
        if ((rc = record_ctl(p))) return rc;
        // the tail check right behind the pass (after its event: the host's wait does not cover it),
        // so that it does not wait for the host's turn
        if ((rc = launch_tailcheck(p))) return rc;
        p->tail_enqueued = true;
    }
    p->inflight = true;
    c->busy = p;
    return XC_OK;
}

// The recent window's collision lookups that the anchor scans did not look for (enqueued: the
// run's lookup hits are replayed after it).  Both kernels stand down behind a stopped pass.
static int launch_tailcheck(xc_plan *p)
{
    xc_cache *c = p->cache;
    if (!(p->anc_any && c->mem && !c->engine && p->nb)) return XC_OK;
    hipStream_t s = c->ctx->stream;
    // a small grid (the tail is a few buffers: ~100 blocks on cfg5): the next run's early block hashing
    // fills the CUs meanwhile, and each workgroup of a wide grid waits for a slot, even one with
    // nothing to do (1024 workgroups: 340 us per cfg5 step instead of 30)
    // (XC_TAIL_GRID, -DXC_ABLATIONS builds: another grid)
    static const uint32_t grid = abl_env("XC_TAIL_GRID") ? (uint32_t)atoi(abl_env("XC_TAIL_GRID")) : 64u;
    hipLaunchKernelGGL(k_tailcheck, dim3(std::max(1u, grid)), dim3(256), 0, s, p->P, p->nb, p->d_tcnt, p->d_tlist);
    HIPCHK(hipGetLastError());
    hipLaunchKernelGGL(k_tailfinal, dim3(std::min<uint32_t>(p->nb, std::max(1u, grid))), dim3(64), 0, s, p->P, p->nb,
                       p->d_tcnt, (const uint4 *)p->d_tlist);
    HIPCHK(hipGetLastError());
    return XC_OK;
}

static bool dbg_finish()
{
    static const bool d = abl_flag("XC_DEBUG_EARLY");
    return d;
}

// After the first pass's ev_ctl: its control words, then the sub-batches that need the host
// (step by step) and further asynchronous passes, then the run's totals.
static int encode_finish(xc_plan *p)
{
    p->inflight = false;
    p->cache->busy = nullptr;
    int rc = XC_OK;
    hipStream_t s = p->cache->ctx->stream;
    uint32_t ctl[CTL_WORDS];
    memcpy(ctl, p->h_ctl, CTL_WORDS * 4);
    ev_collect(p);
    if (p->pass_published && ctl[CTL_WORDS - 1] != 0u && (rc = read_ctl(p, ctl))) return rc;  // (not published)
    const size_t nsub = p->sub.size() - 1;
    bool fresh = true;  // ctl was read after the last launch
    bool redone = false;
    while (ctl[CTL_ABORT]) {
        fresh = false;
        redone = true;
        size_t si = ctl[CTL_ABORT_SB];
        HIPCHK(hipMemsetAsync(p->P.ctl + CTL_ABORT, 0, 4, s));
        if (ctl[CTL_ERROR]) break;
        p->stats.redone++;
        if (ctl[CTL_AFAIL]) {
            static const bool dbg_af = abl_flag("XC_DEBUG_AFAIL");
            if (dbg_af) fprintf(stderr, "anchor fallback: sub-batch %zu, flags %u\n", si, ctl[CTL_AFAIL]);
            // the anchor index cannot decide this sub-batch: the exact scan redoes it, and the
            // rest of the run (a collision or an anchorless segment may concern later ones too)
            HIPCHK(hipMemsetAsync(p->P.ctl + CTL_AFAIL, 0, 4, s));
            p->anc_scan_on = false;
            p->stats.anchor_fallbacks++;
        }
        if (ctl[CTL_SHADOW]) p->stats.shadow_misses++;
        // that sub-batch, step by step (its pipeline state is discarded and redone)
        if ((rc = encode_sub_sync(p, (uint32_t)si, ctl))) return rc;
        if (ctl[CTL_ERROR]) break;
        if ((rc = launch_pack(p, p->sub[si], p->sub[si + 1]))) return rc;
        if (++si >= nsub) break;
        // the rest asynchronously again: k_alloc's gate stops at the next sub-batch needing the host
        for (size_t k = si; k < nsub; k++)
            if ((rc = encode_sub_async(p, (uint32_t)k))) return rc;
        if ((rc = read_ctl(p, ctl))) return rc;
        fresh = true;
    }
    if (!fresh && (rc = read_ctl(p, ctl))) return rc;
    for (uint64_t i = 0; i < p->nb; i++) p->stats.in_bytes += p->len[i];
    p->stats.n_extract = ctl[CTL_NEXTRACT];
    p->stats.n_ref = ctl[CTL_NREF];
    p->stats.dense_chunks = ctl[CTL_DENSE];
    if (!ctl[CTL_ERROR] && p->sub.size() > 1) p->cache->host_count = ctl[CTL_COUNT];
    p->runs_done++;
    if (ctl[CTL_ERROR] & ERR_CAPACITY) {
        uint32_t cap = (uint32_t)p->cache->cap;
        hipMemcpyAsync(p->cache->count, &cap, 4, hipMemcpyHostToDevice, s);
        hipStreamSynchronize(s);
        return fail(XC_ENOSPC, "device cache capacity exhausted");
    }
    if (ctl[CTL_ERROR] & ERR_PACK_CAP) return fail(XC_EINVAL, "packed output capacity too small");
    if (ctl[CTL_ERROR]) return fail(XC_EDEVICE, "internal encode error " + std::to_string(ctl[CTL_ERROR]));
    xc_cache *c = p->cache;
    if (p->anc_run) {
        // every segment of the run is indexed; one without an anchor keeps the cache exact (the
        // emit flags it on the device after the run's early publication: a later anchor scan
        // falls back, and the host learns it from there)
        if (p->sub.size() > 1) c->anc_upto = ctl[CTL_COUNT];
        if (p->stats.anchor_fallbacks) {
            uint32_t bad = 0;
            HIPCHK(hipMemcpyAsync(&bad, c->ctl + CTL_ANCLESS, 4, hipMemcpyDeviceToHost, s));
            HIPCHK(hipStreamSynchronize(s));
            if (bad) c->anc_bad = std::min(c->anc_bad, ~bad);
            static const bool dbg_anc = abl_flag("XC_DEBUG_ANC");
            if (dbg_anc && bad && ~bad < c->dev_cap) {
                std::vector<uint8_t> sb(XC_SEG);
                uint64_t key = 0;
                HIPCHK(hipMemcpy(sb.data(), c->segs + (size_t)~bad * XC_SEG, XC_SEG, hipMemcpyDeviceToHost));
                HIPCHK(hipMemcpy(&key, c->anc_of + ~bad, 8, hipMemcpyDeviceToHost));
                fprintf(stderr, "anchorless segment %u key %016llx bytes ", ~bad, (unsigned long long)key);
                for (uint8_t v : sb) fprintf(stderr, "%02x", v);
                fprintf(stderr, "\n");
            }
        }
    }
    // (the first pass enqueued it behind itself unless a sub-batch was redone since)
    if (!(p->tail_enqueued && !redone) && (rc = launch_tailcheck(p))) return rc;
    p->early_ok = !redone && p->sub.size() > 2 && p->rec_sb0;
    if (dbg_finish()) fprintf(stderr, "finish redone=%d nsub=%zu\n", (int)redone, p->sub.size() - 1);
    c->last_plan = p;
    if (c->mem && !c->engine) {
        if (ctl[CTL_DUPS]) {
            // a carried candidate entered a hash the cache held: undone, the host replays the run
            if (p->count0 < 0) return fail(XC_EDEVICE, "duplicate enter in a run without stream state");
            if ((rc = cache_rebuild(c, c->cap, (uint32_t)p->count0, true))) return rc;
            c->host_count = p->count0;
            return fail(XC__SLOW, "a hash entered twice");
        }
        // its lookup hits, for the recent window (none: no REF, no collision recorded, no tail
        // check behind the run that could record one)
        // (XC_NO_HITS=1, -DXC_ABLATIONS builds: none at all, a timing diagnostic only: the window model
        // is then wrong)
        static const bool no_hits = abl_flag("XC_NO_HITS");
        if (!no_hits && (ctl[CTL_NREF] || ctl[CTL_COLLS] || p->anc_any)) {
            if ((rc = hits_flush(c))) return rc;
            // (a small host-path run: into pinned memory now, its host's synchronisation follows)
            if (p->host_path && p->nb <= PLAN_POOL_NBUF) rc = hits_enqueue_direct(p);
            else c->hl_pend = p;  // (packed at the next operation on the cache)
            if (rc) return rc;
        }
    }
    return XC_OK;
}

// A run xc_cache_quiesce finished: its status, once, to its submitter.
static int take_parked(xc_plan *p)
{
    p->parked = false;
    return p->parked_rc ? fail(p->parked_rc, p->parked_msg) : XC_OK;
}

static int encode_poll(xc_plan *p, int *done)
{
    if (!p || !done) return fail(XC_EINVAL, "null");
    if (!p->inflight && p->parked) {
        *done = 1;
        return take_parked(p);
    }
    if (!p->inflight) return fail(XC_EINVAL, "no run in flight");
    int rc = set_dev(p->cache->ctx);
    if (rc) return rc;
    const hipError_t e = early_done(p) ? pass_state(p) : hipEventQuery(p->ev_ctl);
    if (e == hipErrorNotReady) {
        *done = 0;
        return XC_OK;
    }
    *done = 1;
    if (e != hipSuccess) {
        p->inflight = false;
        p->cache->busy = nullptr;
        return fail(XC_EDEVICE, std::string("run: ") + hipGetErrorString(e));
    }
    return encode_finish(p);
}

static int encode_wait(xc_plan *p)
{
    if (!p) return fail(XC_EINVAL, "null");
    if (!p->inflight && p->parked) return take_parked(p);
    if (!p->inflight) return fail(XC_EINVAL, "no run in flight");
    int rc = set_dev(p->cache->ctx);
    if (rc) return rc;
    const hipError_t e = wait_decided(p);
    if (e != hipSuccess) {
        p->inflight = false;
        p->cache->busy = nullptr;
        return fail(XC_EDEVICE, std::string("run: ") + hipGetErrorString(e));
    }
    return encode_finish(p);
}

extern "C" int xc_plan_set_input_ready(xc_plan *p, int ready)
{
    if (!p) return fail(XC_EINVAL, "null");
    if (p->inflight) return fail(XC_EBUSY, "a run of this plan is in flight");
    p->input_ready = ready != 0;
    return XC_OK;
}

extern "C" int xc_plan_set_completion(xc_plan *p, int mode)
{
    if (!p || (mode != XC_COMPLETE_RUN && mode != XC_COMPLETE_STREAM)) return fail(XC_EINVAL, "completion mode");
    if (p->inflight) return fail(XC_EBUSY, "a run of this plan is in flight");
    p->completion = mode;
    return XC_OK;
}

struct ReplayOut {
    const xc_plan *p;
    std::vector<uint8_t> *out;
    std::vector<uint64_t> *len;
};

static int replay_take(void *ctx, uint64_t i, const uint8_t *o, uint64_t n, const uint8_t *)
{
    ReplayOut &r = *(ReplayOut *)ctx;
    if (n > 2 * r.p->len[i] + 16) return fail(XC_EDEVICE, "replayed stream longer than its slot");
    if (n) memcpy(r.out->data() + r.p->out_off[i], o, n);
    (*r.len)[i] = n;
    return XC_OK;
}

// A device-resident run the device path hands back (XC__SLOW: a hash entered twice by a stateful
// stream is in the recent window, or the run entered one; the cache is as before the run): the
// recent window's replay (xc_memcache.cpp, the host paths' engine) over the run's input arena, its
// streams and lengths (and stream results) written where the device run puts them.  Rare: only a
// stateful connection's carried candidate enters a hash twice (xcodec_cache.h:182-188).
static int replay_device_run(xc_plan *p, const uint8_t *d_in, uint8_t *d_out, uint64_t *d_out_len)
{
    xc_cache *c = p->cache;
    const uint32_t nb = p->nb;
    if (!c->mem) return fail(XC_EDEVICE, "replay without a memory cache");
    int rc = set_dev(c->ctx);
    if (rc) return rc;
    HIPCHK(hipStreamSynchronize(c->ctx->stream));
    if (nb == 0) return XC_OK;
    std::vector<uint8_t> in(p->in_bytes);
    HIPCHK(hipMemcpy(in.data(), d_in, p->in_bytes, hipMemcpyDeviceToHost));
    std::vector<const uint8_t *> head(nb), tail(nb, in.data());
    std::vector<uint64_t> hl(nb), tl(nb, 0), start(nb, 0), rbase(nb, 0), olen(nb, 0);
    std::vector<int64_t> cand(nb, -1), rcand(nb, -1);
    std::vector<uint32_t> flags(nb, 0);
    const bool streams = p->P.stream_st != nullptr;
    for (uint32_t i = 0; i < nb; i++) {
        head[i] = in.data() + p->in_off[i];
        hl[i] = p->len[i];
        if (streams) {  // (the states xc_plan_set_streams uploaded)
            const uint4 &s = p->st_dev[i];
            start[i] = s.x;
            cand[i] = s.y == NONE ? -1 : (int64_t)s.y;
            flags[i] = s.z;
        }
    }
    const uint64_t extent = p->out_off[nb - 1] + 2 * p->len[nb - 1] + 16;
    std::vector<uint8_t> out(extent, 0);
    ReplayOut r{p, &out, &olen};
    rc = xc__mem_encode_gather(c->mem, nb, head.data(), hl.data(), tail.data(), tl.data(), start.data(), cand.data(),
                               flags.data(), rbase.data(), rcand.data(), replay_take, &r);
    if (rc) return rc;
    HIPCHK(hipMemcpy(d_out, out.data(), extent, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(d_out_len, olen.data(), nb * 8, hipMemcpyHostToDevice));
    if (streams) {
        std::vector<uint2> res(nb);
        for (uint32_t i = 0; i < nb; i++)
            res[i] = make_uint2((uint32_t)rbase[i], rcand[i] < 0 ? NONE : (uint32_t)rcand[i]);
        HIPCHK(hipMemcpy(p->d_stream_res, res.data(), nb * sizeof(uint2), hipMemcpyHostToDevice));
        p->res_staged = false;
    }
    return XC_OK;
}

// The library's host paths take an XC__SLOW run to the replay engine themselves; a device-resident
// run is replayed here, into its arenas.
static int public_rc(xc_plan *p, int rc, const uint8_t *d_in, uint8_t *d_out, uint64_t *d_out_len)
{
    if (rc == XC__SLOW && p && !p->host_path) return replay_device_run(p, d_in, d_out, d_out_len);
    return rc;
}

static int public_rc(xc_plan *p, int rc)
{
    return p ? public_rc(p, rc, p->P.in, p->P.out, p->P.out_len) : rc;
}

extern "C" int xc_encode_submit(xc_plan *p, const uint8_t *d_in, uint8_t *d_out, uint64_t *d_out_len)
{
    const int rc = encode_submit(p, d_in, d_out, d_out_len);
    if (rc != XC__SLOW || !p || p->host_path) return rc;
    // (refused before any launch: replayed now, its status for the poll / wait that finishes it)
    const int r = public_rc(p, rc, d_in, d_out, d_out_len);
    p->parked = true;
    p->parked_rc = r;
    p->parked_msg = r ? g_err : std::string();
    return XC_OK;
}

extern "C" int xc_encode_poll(xc_plan *p, int *done)
{
    return public_rc(p, encode_poll(p, done));
}

extern "C" int xc_encode_wait(xc_plan *p)
{
    return public_rc(p, encode_wait(p));
}

// Finish the run in flight on the cache (another caller's submit): a synchronous call that met
// XC_EBUSY can then go ahead; the submitter's next poll / wait returns that run's status.
extern "C" int xc_cache_quiesce(xc_cache *c)
{
    if (!c) return fail(XC_EINVAL, "null");
    int rc = set_dev(c->ctx);
    if (rc || !c->busy) return rc;
    xc_plan *p = (xc_plan *)c->busy;
    const int r = public_rc(p, encode_wait(p));
    p->parked = true;
    p->parked_rc = r;
    p->parked_msg = r ? g_err : std::string();
    return XC_OK;
}

extern "C" int xc_encode_run(xc_plan *p, const uint8_t *d_in, uint8_t *d_out, uint64_t *d_out_len)
{
    int rc = encode_submit(p, d_in, d_out, d_out_len);
    if (!rc) rc = encode_wait(p);
    return public_rc(p, rc, d_in, d_out, d_out_len);
}

extern "C" int xc_host_alloc(xc_ctx *ctx, uint64_t bytes, void **out)
{
    if (!ctx || !out) return fail(XC_EINVAL, "null");
    int rc = set_dev(ctx);
    if (rc) return rc;
    HIPCHK(hipHostMalloc(out, std::max<uint64_t>(bytes, 1), hipHostMallocMapped | hipHostMallocPortable));
    return XC_OK;
}

extern "C" int xc_host_free(void *ptr)
{
    if (ptr) HIPCHK(hipHostFree(ptr));
    return XC_OK;
}

extern "C" int xc_encode_run_host(xc_plan *p, const uint8_t *h_in, uint8_t *h_out, uint64_t h_out_cap,
                                  uint64_t *h_len, uint64_t *h_pos)
{
    if (!p || (p->nb && (!h_in || !h_out || !h_len))) return fail(XC_EINVAL, "null");
    int rc = set_dev(p->cache->ctx);
    if (rc) return rc;
    hipStream_t s = p->cache->ctx->stream;
    if (!p->e_in) {  // device arenas and the copy stream, kept for later runs
        HIPCHK(dmalloc(&p->e_in, p->in_bytes));
        HIPCHK(dmalloc(&p->e_out, p->out_bytes));
        const uint64_t nb1 = std::max<uint64_t>(p->nb, 1);
        HIPCHK(dmalloc(&p->e_len, nb1 * 24));
        p->e_pos = p->e_len + nb1;
        p->e_res = (uint2 *)(p->e_len + 2 * nb1);
        HIPCHK(dmalloc(&p->e_total, 8));
        if (!p->cache->ctx->copy) HIPCHK(hipStreamCreateWithFlags(&p->cache->ctx->copy, hipStreamNonBlocking));
        p->cs = p->cache->ctx->copy;
        p->ev_h2d.assign(p->sub.size(), nullptr);
        for (auto &e : p->ev_h2d) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    }
    void *dev_out = nullptr;
    if (hipHostGetDevicePointer(&dev_out, h_out, 0) != hipSuccess || !dev_out)
        return fail(XC_EINVAL, "h_out is not pinned host memory (use xc_host_alloc)");
    // every sub-batch's input on the copy stream, in order; sub-batch k's block hashing (the
    // first kernel to read it) waits for its event.  A run of one sub-batch has nothing to overlap
    // the copy with: on the context stream, no events (a cross-stream wait idles the device ~6 us)
    p->h2d_inline = p->sub.size() <= 2;
    if (p->h2d_inline) {
        if (p->in_bytes) HIPCHK(hipMemcpyAsync(p->e_in, h_in, p->in_bytes, hipMemcpyHostToDevice, s));
    } else {
        HIPCHK(hipEventRecord(p->ev_start, s));
        HIPCHK(hipStreamWaitEvent(p->cs, p->ev_start, 0));
        for (size_t k = 0; k + 1 < p->sub.size(); k++) {
            const uint64_t a = p->nb ? p->in_off[p->sub[k]] : 0;
            const uint64_t b = p->sub[k + 1] < p->nb ? p->in_off[p->sub[k + 1]] : p->in_bytes;
            if (b > a) HIPCHK(hipMemcpyAsync(p->e_in + a, h_in + a, b - a, hipMemcpyHostToDevice, p->cs));
            HIPCHK(hipEventRecord(p->ev_h2d[k], p->cs));
        }
    }
    // (the packed total starts at 0 with the run's first buffers: k_pack_offsets)
    p->host_path = true;
    p->pack_dst = (uint8_t *)dev_out;
    p->pack_cap = h_out_cap;
    uint2 *const res_dev = p->P.stream_res;  // (the run's stream results into the same block)
    if (res_dev) p->P.stream_res = p->e_res;
    rc = xc_encode_run(p, p->e_in, p->e_out, p->e_len);
    p->P.stream_res = res_dev;
    p->host_path = false;
    if (rc) {
        hipStreamSynchronize(p->cs);
        hipStreamSynchronize(s);
        return rc;
    }
    if (p->nb) {  // (through the plan's pinned copy of them: pageable copies stage synchronously)
        const uint64_t nb1 = std::max<uint64_t>(p->nb, 1);
        if (!p->h_lenpos && hmalloc((void **)&p->h_lenpos, (size_t)nb1 * 24) != hipSuccess)
            return fail(XC_ENOMEM, "pinned allocation failed");
        // lengths, positions and (xc_plan_stream_results reads them from here) stream results
        HIPCHK(hipMemcpyAsync(p->h_lenpos, p->e_len, nb1 * (res_dev ? 24 : 16), hipMemcpyDeviceToHost, s));
        p->res_staged = res_dev != nullptr;
    }
    // (the run's lookup hits go to the recent window through the cache's hit log, hits_enqueue)
    HIPCHK(hipStreamSynchronize(s));
    for (auto &sl : p->cache->hl) sl.host_sync = false;  // (written behind the run: complete now)
    if (p->nb) {
        memcpy(h_len, p->h_lenpos, p->nb * 8);
        if (h_pos) memcpy(h_pos, p->h_lenpos + p->nb, p->nb * 8);
    }
    return XC_OK;
}

// Host-to-host batch, optionally with stream state (xc_stream.hip): start / cand / flags as in
// xc_plan_set_streams, the resulting source_ base / candidate to rbase / rcand.
// Host-to-host batch with stream state (xc_stream.cpp) and, when coll_cnt is given, every buffer's
// collision lookups (the COSS tier's replay, xc_coss.cpp): coll_cnt[i] records in
// coll[i * COLL_CAP * 4 ..] as {window end, hash lo, hash hi, 0} (at most COLL_CAP kept).
// The host paths' plans (xc__encode_batch_host_coll, xc__encode_gather): a plan of these exact
// lengths from the cache's pool, else a new one; released plans go back (small batches only: a
// pooled plan holds its device workspace).
static int plan_acquire(xc_cache *c, const uint64_t *len, uint64_t nbuf, xc_plan **out)
{
    for (size_t k = c->plan_pool.size(); k-- > 0;) {
        xc_plan *p = c->plan_pool[k];
        if (p->nb == nbuf && std::equal(p->len.begin(), p->len.end(), len)) {
            c->plan_pool.erase(c->plan_pool.begin() + (ptrdiff_t)k);
            *out = p;
            return XC_OK;
        }
    }
    // (host-path plans: sub-batches of 256 MiB pipeline the copies, xc_encode_plan_create_sub)
    return xc_encode_plan_create_sub(c, len, nbuf, HOST_SUB_BYTES, out);
}
static void plan_release(xc_cache *c, xc_plan *p)
{
    if (!p) return;
    if (p->nb > PLAN_POOL_NBUF || p->inflight || xc_plan_set_streams(p, nullptr, nullptr, nullptr) != XC_OK) {
        xc_plan_destroy(p);
        return;
    }
    c->plan_pool.push_back(p);
    if (c->plan_pool.size() > PLAN_POOL_MAX) {
        xc_plan *old = c->plan_pool.front();
        c->plan_pool.erase(c->plan_pool.begin());
        xc_plan_destroy(old);
    }
}
static void plan_pool_drain(xc_cache *c)
{
    std::vector<xc_plan *> v;
    v.swap(c->plan_pool);
    for (xc_plan *p : v) xc_plan_destroy(p);
}

extern "C" int xc__encode_batch_host_coll(xc_cache *c, const uint8_t *in, const uint64_t *in_off,
                                          const uint64_t *in_len, uint64_t nbuf, uint8_t *out,
                                          const uint64_t *out_off, const uint64_t *out_cap, uint64_t *out_len,
                                          const uint64_t *start, const int64_t *cand, const uint32_t *flags,
                                          uint64_t *rbase, int64_t *rcand, uint32_t *coll_cnt, uint32_t *coll)
{
    if (!c || (nbuf && (!in || !in_off || !in_len || !out || !out_off || !out_cap || !out_len)))
        return fail(XC_EINVAL, "null");
    xc_plan *p = nullptr;
    int rc = plan_acquire(c, in_len, nbuf, &p);
    if (rc) return rc;
    const bool streams = start || cand || flags;
    if (streams && (rc = xc_plan_set_streams(p, start, cand, flags))) {
        xc_plan_destroy(p);
        return rc;
    }
    // the end-to-end path (xc_encode_run_host): per-sub-batch input copies overlapping the
    // encode, the encoded streams packed into pinned memory by a kernel; the input arena needs no
    // clearing (bytes past a buffer's end are read but never used)
    uint8_t *h_in = nullptr, *h_out = nullptr;
    uint64_t cap_total = 0;
    for (uint64_t i = 0; i < nbuf; i++) cap_total += 2 * in_len[i] + 16;
    std::vector<uint64_t> lens(std::max<uint64_t>(nbuf, 1)), pos(std::max<uint64_t>(nbuf, 1));
    if (hmalloc((void **)&h_in, p->in_bytes) != hipSuccess || hmalloc((void **)&h_out, cap_total + 16) != hipSuccess) {
        pool_free(h_in);
        xc_plan_destroy(p);
        return fail(XC_ENOMEM, "pinned allocation failed");
    }
    {
        std::vector<HostCopy> cp(nbuf);
        for (uint64_t i = 0; i < nbuf; i++) cp[i] = {h_in + p->in_off[i], in + in_off[i], in_len[i]};
        host_copies(cp);
    }
    rc = xc_encode_run_host(p, h_in, h_out, cap_total + 16, lens.data(), pos.data());
    if (!rc) {
        std::vector<HostCopy> cp;
        cp.reserve(nbuf);
        for (uint64_t i = 0; i < nbuf; i++) {
            out_len[i] = lens[i];
            if (lens[i] > out_cap[i]) { rc = fail(XC_EINVAL, "output capacity too small"); continue; }
            cp.push_back({out + out_off[i], h_out + pos[i], lens[i]});
        }
        host_copies(cp);
        if (!rc && streams && rbase && rcand) rc = xc_plan_stream_results(p, rbase, rcand);
        if (!rc && coll_cnt && nbuf) {
            if (hipMemcpy(coll_cnt, p->d_coll_cnt, nbuf * 4, hipMemcpyDeviceToHost) != hipSuccess ||
                hipMemcpy(coll, p->d_coll, (size_t)nbuf * COLL_CAP * sizeof(uint4), hipMemcpyDeviceToHost) != hipSuccess)
                rc = fail(XC_EDEVICE, "collision records copy");
        }
    }
    // (nothing of the run may still touch the pinned buffers when they return to the pool)
    if (hipStreamSynchronize(c->ctx->stream) != hipSuccess && !rc) rc = fail(XC_EDEVICE, "stream synchronize");
    if (rc) xc_plan_destroy(p);
    else plan_release(c, p);
    pool_free(h_in);
    pool_free(h_out);
    return rc;
}

// Internal (xc_stream.cpp): the host batch with each item gathered from two host pieces (an
// encoder's pending source_ and its new input) straight into the pinned input arena, and each
// item's encoded bytes handed to `take` from pinned memory together with the item's input (from
// which the caller keeps the new source_), after the stream results are in rbase / rcand: no
// intermediate host arenas.
extern "C" int xc__encode_gather(xc_cache *c, uint64_t nbuf, const uint8_t *const *head, const uint64_t *head_len,
                                 const uint8_t *const *tail, const uint64_t *tail_len, const uint64_t *start,
                                 const int64_t *cand, const uint32_t *flags, uint64_t *rbase, int64_t *rcand,
                                 int (*take)(void *ctx, uint64_t i, const uint8_t *out, uint64_t out_len,
                                             const uint8_t *in),
                                 void *ctx)
{
    if (!c || (nbuf && (!head || !head_len || !tail || !tail_len || !rbase || !rcand || !take)))
        return fail(XC_EINVAL, "null");
    if (nbuf == 0) return XC_OK;
    std::vector<uint64_t> len(nbuf);
    for (uint64_t i = 0; i < nbuf; i++) len[i] = head_len[i] + tail_len[i];
    xc_plan *p = nullptr;
    int rc = plan_acquire(c, len.data(), nbuf, &p);
    if (rc) return rc;
    if ((rc = xc_plan_set_streams(p, start, cand, flags))) {
        xc_plan_destroy(p);
        return rc;
    }
    uint8_t *h_in = nullptr, *h_out = nullptr;
    uint64_t cap_total = 0;
    for (uint64_t i = 0; i < nbuf; i++) cap_total += 2 * len[i] + 16;
    std::vector<uint64_t> lens(nbuf), pos(nbuf);
    if (hmalloc((void **)&h_in, p->in_bytes) != hipSuccess || hmalloc((void **)&h_out, cap_total + 16) != hipSuccess) {
        pool_free(h_in);
        xc_plan_destroy(p);
        return fail(XC_ENOMEM, "pinned allocation failed");
    }
    {
        std::vector<HostCopy> cp;
        cp.reserve(2 * nbuf);
        for (uint64_t i = 0; i < nbuf; i++) {
            cp.push_back({h_in + p->in_off[i], head[i], head_len[i]});
            cp.push_back({h_in + p->in_off[i] + head_len[i], tail[i], tail_len[i]});
        }
        host_copies(cp);
    }
    rc = xc_encode_run_host(p, h_in, h_out, cap_total + 16, lens.data(), pos.data());
    if (!rc) rc = xc_plan_stream_results(p, rbase, rcand);
    for (uint64_t i = 0; i < nbuf && !rc; i++) rc = take(ctx, i, h_out + pos[i], lens[i], h_in + p->in_off[i]);
    if (hipStreamSynchronize(c->ctx->stream) != hipSuccess && !rc) rc = fail(XC_EDEVICE, "stream synchronize");
    if (rc) xc_plan_destroy(p);
    else plan_release(c, p);
    pool_free(h_in);
    pool_free(h_out);
    if (rc == XC__SLOW)  // a hash entered twice: the recent window's replay (xc_memcache.cpp)
        rc = xc__mem_encode_gather(c->mem, nbuf, head, head_len, tail, tail_len, start, cand, flags, rbase, rcand,
                                   take, ctx);
    return rc;
}

extern "C" int xc__encode_batch_host_ex(xc_cache *c, const uint8_t *in, const uint64_t *in_off,
                                        const uint64_t *in_len, uint64_t nbuf, uint8_t *out,
                                        const uint64_t *out_off, const uint64_t *out_cap, uint64_t *out_len,
                                        const uint64_t *start, const int64_t *cand, const uint32_t *flags,
                                        uint64_t *rbase, int64_t *rcand)
{
    int rc = xc__encode_batch_host_coll(c, in, in_off, in_len, nbuf, out, out_off, out_cap, out_len, start, cand,
                                        flags, rbase, rcand, nullptr, nullptr);
    if (rc == XC__SLOW && !start && !cand && !flags)
        rc = xc__mem_encode_batch(c->mem, in, in_off, in_len, nbuf, out, out_off, out_cap, out_len);
    else if (rc == XC__SLOW)
        rc = fail(XC_EINVAL, "stream state through the host batch with a hash entered twice: use xc_encode_streams");
    return rc;
}

extern "C" int xc_encode_batch_host(xc_cache *c, const uint8_t *in, const uint64_t *in_off, const uint64_t *in_len,
                                    uint64_t nbuf, uint8_t *out, const uint64_t *out_off, const uint64_t *out_cap,
                                    uint64_t *out_len)
{
    return xc__encode_batch_host_ex(c, in, in_off, in_len, nbuf, out, out_off, out_cap, out_len, nullptr, nullptr,
                                    nullptr, nullptr, nullptr);
}

// Internal accessors for xc_decode.hip (not part of the public header).
extern "C" int xc__cache_devset(xc_cache *c, void *devset, SegStore *segs, uint32_t **count, uint32_t *cap,
                                uint2 **undo, void **stream, int *dev)
{
    if (!c) return fail(XC_EINVAL, "null");
    *(DevSet *)devset = c->set.d;
    *segs = cache_segstore(c);
    *count = c->count;
    *cap = (uint32_t)c->cap;
    *undo = c->undo;
    *stream = (void *)c->ctx->stream;
    *dev = c->ctx->dev;
    return XC_OK;
}

extern "C" int xc__set_error(int code, const char *msg) { return fail(code, msg); }

// Internal: time `iters` launches of the scan of the whole plan against the cache set in an
// ablation mode (ScanArgs::mode); returns microseconds per launch.  Needs P.in set by a run.
extern "C" double xc__scan_ablation(xc_plan *p, const uint8_t *d_in, int mode, int iters)
{
    xc_ctx *ctx = p->cache->ctx;
    hipSetDevice(ctx->dev);
    p->P.in = d_in;
    ScanArgs a{p->P, p->P.S, p->P.cache, 0, p->nchunks, (uint32_t)mode, DevSet{}, 0, (const uint32_t *)p->P.cache.l2, 0,
               p->scan_unit, p->P.cache.filt, XC_FILT_WORDS};
    uint32_t need = (p->nchunks + SCAN_WAVES * p->scan_unit - 1) / (SCAN_WAVES * p->scan_unit);
    uint32_t grid = std::min<uint32_t>(need, (uint32_t)ctx->n_cu);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto kern = mode == 0 ? k_scan<0> : mode == 1 ? k_scan<1> : mode == 2 ? k_scan<2> : mode == 3 ? k_scan<3> : mode == 4 ? k_scan<4> : k_scan<5>;
    hipMemsetAsync(p->P.ctl + CTL_SCAN_NEXT, 0, 4, ctx->stream);
    hipLaunchKernelGGL(kern, dim3(grid), dim3(64 * SCAN_WAVES), 0, ctx->stream, a);
    hipEventRecord(e0, ctx->stream);
    for (int i = 0; i < iters; i++) {
        hipMemsetAsync(p->P.ctl + CTL_SCAN_NEXT, 0, 4, ctx->stream);
        hipLaunchKernelGGL(kern, dim3(grid), dim3(64 * SCAN_WAVES), 0, ctx->stream, a);
    }
    hipEventRecord(e1, ctx->stream);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    hipEventDestroy(e0);
    hipEventDestroy(e1);
    return 1000.0 * ms / iters;
}

extern "C" int xc_selftest(xc_ctx *ctx)
{
    if (!ctx) return fail(XC_EINVAL, "null");
    int rc = set_dev(ctx);
    if (rc) return rc;
    hipStream_t s = ctx->stream;
    HIPCHK(hipMemsetAsync(ctx->d_scratch, 0, 4, s));
    hipLaunchKernelGGL(k_selftest, dim3(1), dim3(64), 0, s, ctx->d_scratch);
    HIPCHK(hipGetLastError());
    uint32_t err = 0;
    HIPCHK(hipMemcpyAsync(&err, ctx->d_scratch, 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    if (err) return fail(XC_EDEVICE, "selftest failed: " + std::to_string(err));
    return XC_OK;
}


