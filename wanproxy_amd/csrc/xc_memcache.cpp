// xc_memcache.cpp — XCodecMemoryCache's recent window and duplicate enters, on the host.
//
// Reference (xcodec/xcodec_cache.h:89-211): lookup() first scans a 64-entry window of the (hash,
// data pointer) pairs its last map hits remembered (find_recent, :137-147, the first entry with the
// hash), then the map, remembering a map hit in the next window slot (:130-135, cursor round
// robin).  enter() asserts that the hash is new (:184); a release build overwrites the map value
// and leaves the old data alive, so after a second enter of a hash with other bytes the window
// keeps returning the old bytes until 64 later remembers push its entry out, and the map returns
// the new ones.  The only way an encoder gets there is a stateful connection whose candidate was
// looked up (a miss) in one call and is declared in a later one after another connection entered a
// different segment with the same hash (xcodec_encoder.cc:77-82,203-215; the hash is weak enough to
// build such pairs).
//
// Without such a duplicate the window never changes what a lookup returns (it caches map
// pointers), so the device cache has no window: a run's lookup hits (the REF tokens and the
// collisions its walk records; the decoder's executed tokens) are replayed here afterwards, lazily
// (runtime: the cache's pending run, consumed before the next operation on the cache that needs the
// order, dropped by a restore).  A duplicate enter (k_emit finds the key, CTL_DUPS) or a run while
// a duplicated hash may still answer with other bytes than the device holds goes through the replay
// engine of xc_replay.h with the Store below: the device cache then mirrors, for every hash, the
// bytes the reference's lookup returns, following each change the window makes.
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
#include <mutex>
#include <new>
#include <thread>
#include <vector>

#include "xc_replay.h"

extern "C" int xc__cache_find(xc_cache *c, const uint64_t *h, uint64_t n, uint64_t *val);  // ~0: absent
extern "C" int xc__cache_read(xc_cache *c, uint64_t h, uint8_t *out, int *found);            // no side effects
extern "C" int xc__cache_set_value(xc_cache *c, uint64_t h, uint64_t val);
extern "C" void xc__cache_engine(xc_cache *c, int on);
extern "C" int xc__cache_settle(xc_cache *c);  // the earlier runs' lookup hits into the window first

namespace {
using replay::SEG;
using replay::Touch;
constexpr int WINDOW = 64;  // XCODEC_WINDOW_COUNT, xcodec_cache.h:48

// The memory cache as the reference's lookups see it.
class MemStore {
public:
    xc_cache *cache = nullptr;
    // the recent window: hash and the version of the bytes it remembered (-1: never used, no data),
    // slot by slot (the replay's inner loop reads the hashes alone)
    uint64_t wh[WINDOW] = {};
    int32_t wv[WINDOW];
    uint32_t cursor = 0;
    // window slots per bucket(hash), the unused ones (hash 0) included: a run's hits are replayed
    // here one by one (half a million per cfg5 step), and almost none is in the window
    uint8_t wcnt[16384] = {};
    static uint32_t bucket(uint64_t h) { return (uint32_t)(h ^ (h >> 29)) & 16383u; }
    // hashes entered again with other bytes: every version (ver[0] the first), cur = the map's
    struct Dup {
        std::vector<std::vector<uint8_t>> ver;
        uint32_t cur = 0;
    };
    std::unordered_map<uint64_t, Dup> dups;
    // per replay pass: in the cache before the pass (device), first enters of the pass
    std::unordered_set<uint64_t> present;
    std::unordered_map<uint64_t, const uint8_t *> inpass;
    bool last_dup = false;  // the last enter() found the hash present
    int err = XC_OK;

    MemStore()
    {
        for (auto &v : wv) v = -1;
        wcnt[bucket(0)] = WINDOW;
    }

    // find_recent: the first slot with the hash (hash 0 matches the unused slots, whose data is
    // null: not found)
    int find_recent(uint64_t h) const
    {
        if (h == 0) {
            for (int i = 0; i < WINDOW; i++)
                if (wh[i] == 0) return wv[i] >= 0 ? i : -1;
            return -1;
        }
        if (!wcnt[bucket(h)]) return -1;
        for (int i = 0; i < WINDOW; i++)  // (a hash is in the window once at most)
            if (wh[i] == h) return i;
        return -1;
    }

    const uint8_t *bytes(uint64_t h, int32_t v) const
    {
        static const uint8_t any[SEG] = {};
        if (dups.empty()) return any;
        auto it = dups.find(h);
        return it == dups.end() ? any : it->second.ver[(size_t)v].data();
    }
    int32_t curver(uint64_t h) const
    {
        if (dups.empty()) return 0;  // (the common case: no hash entered twice, no map probe)
        auto it = dups.find(h);
        return it == dups.end() ? 0 : (int32_t)it->second.cur;
    }
    bool is_present(uint64_t h) const { return dups.count(h) || present.count(h) || inpass.count(h); }

    // remember (xcodec_cache.h:130-135); an evicted entry of a duplicated hash may change what a
    // lookup of that hash returns
    void remember(uint64_t h, int32_t v, Touch *t)
    {
        const uint64_t o = wh[cursor];
        if (t && wv[cursor] >= 0 && o && dups.count(o)) t->hs.push_back(o);
        wcnt[bucket(o)]--;
        wh[cursor] = h;
        wv[cursor] = v;
        wcnt[bucket(h)]++;
        cursor = (cursor + 1) & (WINDOW - 1);
    }

    // XCodecMemoryCache::lookup (:190-210)
    const uint8_t *lookup(uint64_t h, Touch *t)
    {
        const int s = find_recent(h);
        if (s >= 0) return bytes(h, wv[s]);
        if (!is_present(h)) return nullptr;
        const int32_t v = curver(h);
        remember(h, v, t);
        return bytes(h, v);
    }

    // a lookup the device found (a run's hit): the window only
    void hit(uint64_t h)
    {
        if (find_recent(h) < 0) remember(h, curver(h), nullptr);
    }
    // a run's hits in order (the replay's inner loop: half a million per cfg5 batch)
    void hits(const uint64_t *h, uint64_t n)
    {
        if (!dups.empty()) {
            for (uint64_t i = 0; i < n; i++) hit(h[i]);
            return;
        }
        uint32_t c = cursor;
        for (uint64_t i = 0; i < n; i++) {
            const uint64_t x = h[i];
            const uint32_t bx = bucket(x);
            if (__builtin_expect(wcnt[bx] != 0, 0)) {  // (maybe in the window)
                if (x == 0) {
                    cursor = c;
                    hit(x);
                    c = cursor;
                    continue;
                }
                bool in = false;
                for (int j = 0; j < WINDOW; j++) in |= wh[j] == x;
                if (in) continue;
            }
            // not in the window: remembered, version 0
            wcnt[bucket(wh[c])]--;
            wh[c] = x;
            wv[c] = 0;
            wcnt[bx]++;
            c = (c + 1) & (WINDOW - 1);
        }
        cursor = c;
    }

    // ---- a run's hits on several threads (no hash entered twice) ----
    // Whatever the window held, after a stretch of hits that inserted 64 hashes it holds those 64,
    // in that order.  So a chunk of a run's hits is simulated ahead from an empty window (its
    // insert decisions recorded), and the exact simulation from the true window, run over the chunk
    // afterwards, stops as soon as the two decided alike on a stretch with 64 insertions: from there
    // on they are the same simulation, and the chunk's end state is the ahead run's.
    struct Spec {
        std::vector<uint64_t> dec;  // bit i: hit i of the chunk inserted
        uint64_t win[WINDOW];
        uint32_t cur = 0;
        uint64_t nins = 0;
        bool ok = false;  // false: a hash 0 in the chunk (the window's unused slots): no shortcut
    };
    // A run's packed hits: buffer b's record at h + tok_base[b] + b * stride (count in the low word
    // of its first entry, the hashes after it).
    struct Run {
        const uint64_t *h;
        const uint32_t *tok_base;
        uint32_t stride;
        const uint64_t *rec(uint32_t b) const { return h + tok_base[b] + (uint64_t)b * stride; }
    };

    static void spec_sim(const Run &R, uint32_t b0, uint32_t b1, Spec &o)
    {
        uint64_t n = 0;
        for (uint32_t b = b0; b < b1; b++) n += R.rec(b)[0] & 0xFFFFFFFFu;
        o.dec.assign((n + 63) / 64, 0);
        o.ok = false;
        uint64_t w[WINDOW] = {};
        uint8_t cnt[16384] = {};
        cnt[bucket(0)] = WINDOW;
        uint32_t c = 0;
        uint64_t i = 0, nins = 0;
        for (uint32_t b = b0; b < b1; b++) {
            const uint64_t *r = R.rec(b);
            const uint64_t k = r[0] & 0xFFFFFFFFu;
            for (uint64_t j = 0; j < k; j++, i++) {
                const uint64_t x = r[1 + j];
                if (!x) return;
                const uint32_t bx = bucket(x);
                if (__builtin_expect(cnt[bx] != 0, 0)) {
                    bool in = false;
                    for (int s = 0; s < WINDOW; s++) in |= w[s] == x;
                    if (in) continue;
                }
                cnt[bucket(w[c])]--;
                w[c] = x;
                cnt[bx]++;
                c = (c + 1) & (WINDOW - 1);
                nins++;
                o.dec[i >> 6] |= 1ull << (i & 63);
            }
        }
        std::memcpy(o.win, w, sizeof w);
        o.cur = c;
        o.nins = nins;
        o.ok = true;
    }

    // The exact simulation of chunk [b0, b1) from the window as it is, taking o's end state once
    // they agree (o: spec_sim of the same chunk).
    void hits_fixup(const Run &R, uint32_t b0, uint32_t b1, const Spec &o)
    {
        if (!o.ok || !dups.empty()) {
            for (uint32_t b = b0; b < b1; b++) {
                const uint64_t *r = R.rec(b);
                hits(r + 1, r[0] & 0xFFFFFFFFu);
            }
            return;
        }
        uint32_t c = cursor, agree = 0;
        uint64_t i = 0, sins = 0;
        for (uint32_t b = b0; b < b1; b++) {
            const uint64_t *r = R.rec(b);
            const uint64_t k = r[0] & 0xFFFFFFFFu;
            for (uint64_t j = 0; j < k; j++, i++) {
                const uint64_t x = r[1 + j];  // (non-zero: o.ok)
                const uint32_t bx = bucket(x);
                bool ins = true;
                if (wcnt[bx]) {
                    bool in = false;
                    for (int s = 0; s < WINDOW; s++) in |= wh[s] == x;
                    ins = !in;
                }
                if (ins) {
                    wcnt[bucket(wh[c])]--;
                    wh[c] = x;
                    wv[c] = 0;
                    wcnt[bx]++;
                    c = (c + 1) & (WINDOW - 1);
                }
                const bool sd = (o.dec[i >> 6] >> (i & 63)) & 1u;
                sins += sd;
                if (ins != sd) {
                    agree = 0;
                } else if (ins && ++agree == WINDOW) {
                    // the same 64 insertions: the windows are equal; the rest of the chunk is o's
                    const uint32_t cf = (uint32_t)((c + (o.nins - sins)) & (WINDOW - 1));
                    for (int s = 0; s < WINDOW; s++) wcnt[bucket(wh[s])]--;
                    for (int s = 0; s < WINDOW; s++) {
                        wh[(cf + s) & (WINDOW - 1)] = o.win[(o.cur + s) & (WINDOW - 1)];
                        wv[s] = 0;
                    }
                    for (int s = 0; s < WINDOW; s++) wcnt[bucket(wh[s])]++;
                    cursor = cf;
                    return;
                }
            }
        }
        cursor = c;
    }

    // XCodecMemoryCache::enter (:182-188), release semantics
    void enter(uint64_t h, const uint8_t *seg, Touch *t)
    {
        last_dup = is_present(h);
        if (!last_dup) {
            inpass.emplace(h, seg);
            return;
        }
        auto d = dups.find(h);
        const uint8_t *cur = nullptr;
        std::vector<uint8_t> dev;
        if (d != dups.end()) {
            cur = d->second.ver[d->second.cur].data();
        } else if (inpass.count(h)) {
            cur = inpass[h];
        } else {
            dev.resize(SEG);
            int found = 0;
            if ((err = xc__cache_read(cache, h, dev.data(), &found)) == XC_OK && !found)
                err = xc__set_error(XC_EDEVICE, "memory cache: a present hash is not on the device");
            if (err) return;
            cur = dev.data();
        }
        if (std::memcmp(cur, seg, SEG) == 0) return;  // the same bytes again: nothing a lookup sees
        Dup &x = dups[h];
        if (x.ver.empty()) x.ver.emplace_back(cur, cur + SEG);
        x.ver.emplace_back(seg, seg + SEG);
        x.cur = (uint32_t)x.ver.size() - 1;
        if (t) t->hs.push_back(h);
    }

    int peek(uint64_t h, const uint8_t **p, replay::Loc *, uint64_t *) const
    {
        const int s = find_recent(h);
        if (s >= 0) {
            *p = bytes(h, wv[s]);
            return replay::FOUND;
        }
        if (!is_present(h)) return replay::ABSENT;
        *p = bytes(h, curver(h));
        return replay::FOUND;
    }
    bool read_segment(const replay::Loc &, uint8_t *) const { return false; }
    bool copy_bytes(const uint8_t *p, uint8_t *out) const
    {
        std::memcpy(out, p, SEG);
        return true;
    }
    void owners(uint64_t, std::vector<uint64_t> &) const {}
    template <class F>
    void peek_owners(uint64_t, F) const {}  // (no stripe ranges)
    void window_in_slot(int, std::vector<uint64_t> &) const {}
    void count_misses(uint64_t) {}
};
}  // namespace

// A memory cache's model (xc_replay.h's context).
struct xc_memmodel {
    xc_cache *cache = nullptr;
    xc_ctx *ctx = nullptr;
    MemStore st;
    std::unordered_map<uint64_t, uint64_t> known;  // the device's bytes (fingerprint) of duplicated hashes
    std::unordered_set<uint64_t> load_miss;         // (none: a memory-cache miss has no side effect)
    bool valid = true;  // false: some run's lookups were not all recorded (the window is unknown)
    uint64_t extra = 0;  // device segments that are no map entry (a duplicate enter's, a mirror's)
    // mirrors (hash, the device value before): a restore puts them back
    std::vector<std::pair<uint64_t, uint64_t>> mirror_log;

    void entered(uint64_t h, const uint8_t *)
    {
        if (!st.last_dup) return;
        extra++;  // (the device took a slot for the declaration; the map has the hash once)
        if (st.dups.count(h) && !known.count(h)) {
            // what the device answers for the hash now (its first insert of the batch won)
            uint8_t b[SEG];
            int found = 0;
            if (!st.err && (st.err = xc__cache_read(cache, h, b, &found)) == XC_OK && found)
                known[h] = replay::fingerprint(b);
        }
    }
    void mirrored(const replay::Change &ch) { extra += ch.added.size(); }
    int unmirrorable()
    {
        if (st.err) return st.err;
        if (!valid && !st.dups.empty())
            return xc__set_error(XC_EINVAL, "memory cache: the recent window's state was lost (more than 16 hash "
                                            "collisions in one buffer) and a hash was entered twice");
        return XC_OK;
    }
    // the pass's device batch has run: the entries below count0 were there before it (the
    // batch's own are seen through inpass, in the reference's order)
    int begin_pass(const std::vector<uint64_t> &hs, uint64_t count0)
    {
        st.inpass.clear();
        st.present.clear();
        std::vector<uint64_t> q;
        for (uint64_t h : hs)
            if (!st.dups.count(h)) q.push_back(h);
        std::sort(q.begin(), q.end());
        q.erase(std::unique(q.begin(), q.end()), q.end());
        if (q.empty()) return XC_OK;
        std::vector<uint64_t> v(q.size());
        int rc = xc__cache_find(cache, q.data(), q.size(), v.data());
        if (rc) return rc;
        for (size_t i = 0; i < q.size(); i++)
            if (v[i] != ~0ull && v[i] < count0) st.present.insert(q[i]);
        return XC_OK;
    }
    int end_pass()
    {
        if (st.err) return st.err;
        // a duplicated hash whose every window entry and the device answer with the map's bytes
        // is an ordinary entry again
        for (auto it = st.dups.begin(); it != st.dups.end();) {
            const uint64_t h = it->first;
            const int s = st.find_recent(h);
            const int32_t cur = (int32_t)it->second.cur;
            const auto k = known.find(h);
            if ((s < 0 || st.wv[s] == cur) && k != known.end() &&
                k->second == replay::fingerprint(it->second.ver[(size_t)cur].data())) {
                if (s >= 0) st.wv[s] = 0;
                known.erase(k);
                it = st.dups.erase(it);
            } else {
                ++it;
            }
        }
        st.inpass.clear();
        st.present.clear();
        return XC_OK;
    }
};

namespace {
// The engine's device passes: the runtime's hooks stand aside while it runs.
struct Engine {
    xc_memmodel *m;
    explicit Engine(xc_memmodel *mm) : m(mm) { xc__cache_engine(mm->cache, 1); }
    ~Engine() { xc__cache_engine(m->cache, 0); }
};
}  // namespace

extern "C" xc_memmodel *xc__mem_new(xc_cache *c, xc_ctx *ctx)
{
    xc_memmodel *m = new (std::nothrow) xc_memmodel();
    if (!m) return nullptr;
    m->cache = c;
    m->ctx = ctx;
    m->st.cache = c;
    return m;
}

extern "C" void xc__mem_free(xc_memmodel *m) { delete m; }

extern "C" xc_memmodel *xc__mem_clone(const xc_memmodel *m)
{
    if (!m) return nullptr;
    try {
        return new xc_memmodel(*m);
    } catch (...) {
        return nullptr;
    }
}

// A restore: the model as it was at the snapshot; the device values the mirrors since replaced
// are put back (the undo log revived or evicted their keys).
extern "C" int xc__mem_restore(xc_memmodel *m, const xc_memmodel *snap)
{
    if (!m || !snap) return XC_OK;
    int rc = XC_OK;
    for (size_t i = m->mirror_log.size(); i-- > snap->mirror_log.size() && !rc;)
        rc = xc__cache_set_value(m->cache, m->mirror_log[i].first, m->mirror_log[i].second);
    try {
        *m = *snap;
    } catch (...) {
        return xc__set_error(XC_ENOMEM, "host allocation failed");
    }
    return rc;
}

// A run's lookup hits in the reference's order (complete = 0: some were not recorded).
extern "C" void xc__mem_hits(xc_memmodel *m, const uint64_t *h, uint64_t n, int complete)
{
    if (!m) return;
    m->st.hits(h, n);
    if (!complete) m->valid = false;
}

namespace {
// Helper threads for the chunks simulated ahead (XC_REPLAY_THREADS, default 6; 0: none).  Made
// at the first use and never joined (they wait on the pool's condition between runs).
class ReplayPool {
public:
    static ReplayPool *get()
    {
        static ReplayPool *p = [] {
            const char *e = getenv("XC_REPLAY_THREADS");
            const int n = e ? std::max(0, std::min(32, atoi(e))) : 6;
            ReplayPool *q = new (std::nothrow) ReplayPool();
            if (q && !q->start(n)) q->nthreads = 0;
            return q;
        }();
        return p;
    }
    int threads() const { return nthreads; }
    // One run at a time owns the helpers (caches of different contexts may be driven from different
    // host threads): xc__mem_hits_run holds this from its launch until every job it launched is done.
    std::mutex &owner() { return own; }
    // run job(j) for j in [0, n) on the helpers; done[j] is set (release) as each finishes
    void launch(uint32_t n, std::function<void(uint32_t)> job, std::atomic<int> *done)
    {
        std::lock_guard<std::mutex> g(mu);
        fn = std::move(job);
        flags = done;
        njobs = n;
        gen++;
        next.store(gen << 32);
        cv.notify_all();
    }

private:
    bool start(int n)
    {
        try {
            for (int i = 0; i < n; i++) std::thread([this] { loop(); }).detach();
        } catch (...) {
            return false;
        }
        nthreads = n;
        return true;
    }
    void loop()
    {
        uint64_t seen = 0;
        for (;;) {
            std::function<void(uint32_t)> f;
            std::atomic<int> *d;
            uint32_t n;
            {
                std::unique_lock<std::mutex> g(mu);
                cv.wait(g, [&] { return gen != seen; });
                seen = gen;
                f = fn;
                d = flags;
                n = njobs;
            }
            // (the job counter carries its generation: a helper that wakes late takes no job of a
            // later launch with this one's function)
            for (;;) {
                uint64_t v = next.load();
                if ((v >> 32) != seen || (uint32_t)v >= n) break;
                if (!next.compare_exchange_weak(v, v + 1)) continue;
                f((uint32_t)v);
                d[(uint32_t)v].store(1, std::memory_order_release);
            }
        }
    }
    std::mutex mu, own;
    std::condition_variable cv;
    std::function<void(uint32_t)> fn;
    std::atomic<int> *flags = nullptr;
    uint32_t njobs = 0;
    std::atomic<uint64_t> next{0};  // generation << 32 | the next job
    uint64_t gen = 0;
    int nthreads = 0;
};
}  // namespace

// A run's packed lookup hits, buffers [0, nb) (record of buffer b at h + tok_base[b] + b * stride,
// bit 63 of its count: more than were recorded), in order.  With no hash entered twice and enough
// of them, chunks of buffers are simulated ahead on the helper threads while this thread replays
// the first exactly, then each next one exactly until it agrees with its ahead run.
extern "C" void xc__mem_hits_run(xc_memmodel *m, const uint64_t *h, const uint32_t *tok_base, uint32_t stride,
                                 uint32_t nb)
{
    if (!m || !nb) return;
    const MemStore::Run R{h, tok_base, stride};
    for (uint32_t b = 0; b < nb; b++)
        if (R.rec(b)[0] >> 63) m->valid = false;
    ReplayPool *pool = m->st.dups.empty() && nb >= 1024 ? ReplayPool::get() : nullptr;
    // (another cache's replay holds the helpers: this one runs on the calling thread alone)
    std::unique_lock<std::mutex> own;
    if (pool) own = std::unique_lock<std::mutex>(pool->owner(), std::try_to_lock);
    const uint32_t nt = pool && own.owns_lock() ? (uint32_t)pool->threads() : 0u;
    if (!nt) {
        for (uint32_t b = 0; b < nb; b++) {
            const uint64_t *r = R.rec(b);
            m->st.hits(r + 1, r[0] & 0xFFFFFFFFu);
        }
        return;
    }
    const uint32_t nc = nt + 1;  // chunk 0 here, 1 .. nt ahead
    std::vector<uint32_t> cut(nc + 1);
    for (uint32_t j = 0; j <= nc; j++) cut[j] = (uint32_t)((uint64_t)nb * j / nc);
    std::vector<MemStore::Spec> spec(nc);
    std::unique_ptr<std::atomic<int>[]> done(new std::atomic<int>[nc]);
    for (uint32_t j = 0; j < nc; j++) done[j].store(0);
    pool->launch(nt, [&](uint32_t j) { MemStore::spec_sim(R, cut[j + 1], cut[j + 2], spec[j + 1]); }, done.get() + 1);
    for (uint32_t b = cut[0]; b < cut[1]; b++) {
        const uint64_t *r = R.rec(b);
        m->st.hits(r + 1, r[0] & 0xFFFFFFFFu);
    }
    for (uint32_t j = 1; j < nc; j++) {
        while (!done[j].load(std::memory_order_acquire)) std::this_thread::yield();
        m->st.hits_fixup(R, cut[j], cut[j + 1], spec[j]);
    }
}

// Does a run need the replay engine (a duplicated hash that may answer other bytes)?
extern "C" int xc__mem_live(const xc_memmodel *m) { return m && !m->st.dups.empty() ? 1 : 0; }

// Device segments that are no entry of the reference's map.
extern "C" uint64_t xc__mem_extra(const xc_memmodel *m) { return m ? m->extra : 0; }

namespace {
struct Ctx {
    xc_memmodel *m;
    xc_cache *cache;
    xc_ctx *ctx;
    MemStore &st;
    std::unordered_map<uint64_t, uint64_t> &known;
    std::unordered_set<uint64_t> &load_miss;
    explicit Ctx(xc_memmodel *mm)
        : m(mm), cache(mm->cache), ctx(mm->ctx), st(mm->st), known(mm->known), load_miss(mm->load_miss) {}
    void entered(uint64_t h, const uint8_t *seg) { m->entered(h, seg); }
    // what a mirror replaces (a restore puts it back)
    int before_mirror(const replay::Change &ch)
    {
        if (ch.added.empty()) return XC_OK;
        std::vector<uint64_t> v(ch.added.size());
        int rc = xc__cache_find(cache, ch.added.data(), ch.added.size(), v.data());
        for (size_t i = 0; i < ch.added.size() && !rc; i++) m->mirror_log.push_back({ch.added[i], v[i]});
        return rc;
    }
    void mirrored(const replay::Change &ch) { m->mirrored(ch); }
    int unmirrorable() { return m->unmirrorable(); }
    // (the memory cache's bytes have no place to version: every settle fingerprints)
    bool same_bytes(uint64_t, const uint64_t *) const { return false; }
    void note_bytes(uint64_t, const uint64_t *) {}
    void move_id(const replay::IdMove &) {}
    int begin_pass(const std::vector<uint64_t> &hs, uint64_t count0) { return m->begin_pass(hs, count0); }
    int end_pass() { return m->end_pass(); }
};

int bad_alloc() { return xc__set_error(XC_ENOMEM, "host allocation failed"); }
}  // namespace

// Host batch of fresh encoders (xc_encode_batch_host's semantics) through the engine.
extern "C" int xc__mem_encode_batch(xc_memmodel *m, const uint8_t *in, const uint64_t *in_off, const uint64_t *in_len,
                                    uint64_t nbuf, uint8_t *out, const uint64_t *out_off, const uint64_t *out_cap,
                                    uint64_t *out_len)
{
    if (int rc = xc__cache_settle(m->cache)) return rc;
    try {
        Engine e(m);
        Ctx c(m);
        std::vector<replay::CItem> items;
        for (uint64_t i = 0; i < nbuf; i++) {
            items.push_back({i, in + in_off[i], in_len[i], 0, -1, 0, false});
            out_len[i] = 0;
        }
        std::vector<uint64_t> rb(nbuf);
        std::vector<int64_t> rc(nbuf);
        return replay::encode(&c, std::move(items), out, out_off, out_cap, out_len, rb.data(), rc.data());
    } catch (const std::bad_alloc &) {
        return bad_alloc();
    }
}

// Stream items (xc__encode_gather's contract, xc_stream.cpp) through the engine.
extern "C" int xc__mem_encode_gather(xc_memmodel *m, uint64_t nbuf, const uint8_t *const *head,
                                     const uint64_t *head_len, const uint8_t *const *tail, const uint64_t *tail_len,
                                     const uint64_t *start, const int64_t *cand, const uint32_t *flags,
                                     uint64_t *rbase, int64_t *rcand,
                                     int (*take)(void *ctx, uint64_t i, const uint8_t *out, uint64_t out_len,
                                                 const uint8_t *in),
                                     void *ctx)
{
    if (int rc = xc__cache_settle(m->cache)) return rc;
    try {
        Engine e(m);
        Ctx c(m);
        std::vector<std::vector<uint8_t>> data(nbuf);
        std::vector<uint64_t> ooff(nbuf), ocap(nbuf), olen(nbuf, 0);
        std::vector<replay::CItem> items;
        uint64_t osz = 0;
        for (uint64_t i = 0; i < nbuf; i++) {
            data[i].resize(head_len[i] + tail_len[i]);
            if (head_len[i]) std::memcpy(data[i].data(), head[i], head_len[i]);
            if (tail_len[i]) std::memcpy(data[i].data() + head_len[i], tail[i], tail_len[i]);
            ooff[i] = osz;
            ocap[i] = 2 * data[i].size() + 16;
            osz += ocap[i];
            items.push_back({i, data[i].data(), data[i].size(), start[i], cand[i], 0, (flags[i] & 1u) != 0});
        }
        std::vector<uint8_t> obuf(std::max<uint64_t>(osz, 1));
        int rc = replay::encode(&c, std::move(items), obuf.data(), ooff.data(), ocap.data(), olen.data(), rbase, rcand);
        for (uint64_t i = 0; i < nbuf && !rc; i++) rc = take(ctx, i, obuf.data() + ooff[i], olen[i], data[i].data());
        return rc;
    } catch (const std::bad_alloc &) {
        return bad_alloc();
    }
}

// Decoder batch (xc_decode_batch_host's semantics) through the engine.
extern "C" int xc__mem_decode_batch(xc_memmodel *m, const uint8_t *in, const uint64_t *in_off, const uint64_t *in_len,
                                    uint64_t nbuf, uint8_t *out, const uint64_t *out_off, const uint64_t *out_cap,
                                    uint64_t *out_len, uint64_t *consumed, int32_t *status, uint64_t *unknown,
                                    int32_t *has_unknown)
{
    if (int rc = xc__cache_settle(m->cache)) return rc;
    try {
        Engine e(m);
        Ctx c(m);
        return replay::decode(&c, in, in_off, in_len, nbuf, out, out_off, out_cap, out_len, consumed, status, unknown,
                              has_unknown);
    } catch (const std::bad_alloc &) {
        return bad_alloc();
    }
}

// XCodecMemoryCache::lookup (the <ASK> handler's, xcodec_filter.cc:296): found on the device, then
// the window decides the bytes and remembers a map hit.
extern "C" int xc__mem_lookup(xc_memmodel *m, uint64_t h, uint8_t *out, int *found)
{
    if (int rc = xc__cache_settle(m->cache)) return rc;
    try {
        Ctx c(m);
        uint64_t v = 0;
        int rc = m->st.dups.count(h) ? XC_OK : xc__cache_find(m->cache, &h, 1, &v);
        if (rc) return rc;
        if (!m->st.dups.count(h) && v != ~0ull) m->st.present.insert(h);
        replay::Touch t;
        const uint8_t *d = m->st.lookup(h, &t);
        m->st.present.clear();
        *found = d ? 1 : 0;
        if (d && m->st.dups.count(h)) {
            std::memcpy(out, d, SEG);
        } else if (d) {
            int f = 0;
            if ((rc = xc__cache_read(m->cache, h, out, &f))) return rc;
        }
        if ((rc = replay::follow(&c, t))) return rc;
        return m->end_pass();
    } catch (const std::bad_alloc &) {
        return bad_alloc();
    }
}

// XCodecMemoryCache::enter of a hash the cache holds (release semantics: the map takes the bytes).
// *dup = 0: the hash is absent, the caller enters it on the device.
extern "C" int xc__mem_enter(xc_memmodel *m, uint64_t h, const uint8_t *seg, int *dup)
{
    if (int rc = xc__cache_settle(m->cache)) return rc;
    try {
        Ctx c(m);
        uint64_t v = 0;
        int rc = m->st.dups.count(h) ? XC_OK : xc__cache_find(m->cache, &h, 1, &v);
        if (rc) return rc;
        *dup = m->st.dups.count(h) || v != ~0ull;
        if (!*dup) return XC_OK;
        if (!m->st.dups.count(h)) m->st.present.insert(h);
        replay::Touch t;
        m->st.enter(h, seg, &t);
        m->st.present.clear();
        if (m->st.err) return m->st.err;
        if (m->st.dups.count(h) && !m->known.count(h)) {  // the device holds the first bytes
            uint8_t b[SEG];
            int f = 0;
            if ((rc = xc__cache_read(m->cache, h, b, &f))) return rc;
            m->known[h] = replay::fingerprint(b);
        }
        if ((rc = replay::follow(&c, t))) return rc;
        return m->end_pass();
    } catch (const std::bad_alloc &) {
        return bad_alloc();
    }
}

// The window's hashes, oldest first (tests).
extern "C" void xc__mem_window(const xc_memmodel *m, uint64_t *out)
{
    for (int s = 0; s < WINDOW; s++) out[s] = m ? m->st.wh[(m->st.cursor + s) & (WINDOW - 1)] : 0;
}
