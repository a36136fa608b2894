// xc_replay.h — the device codec over a host state machine that decides what a lookup finds.
//
// Two caches of the reference have lookups whose answers depend on history the device tables do not
// hold: XCodecCacheCOSS (stripe loads, purges and the recent window, xcodec/cache/coss/
// xcodec_cache_coss.cc:163-377) and XCodecMemoryCache once a hash was entered twice with different
// bytes (the map takes the new bytes while the recent window keeps returning the old ones,
// xcodec/xcodec_cache.h:130-147,182-188).  For both, the device cache is a mirror that holds, for
// every hash, the bytes a lookup would return; a host Store restates the reference's state machine.
// A batch runs on the device, then its cache events are replayed into the Store in the reference's
// order (every EXTRACT's enter at its declaration point, every REF's lookup at its window end, every
// collision lookup the walk records; the decoder's tokens).  Each Store operation reports what it
// touched; those hashes are looked up again without side effects (Store::peek) and compared with
// the mirror.  When a change happens inside a batch and a later event depends on it, the device cache
// is rolled back to that event, follows the change, and the rest of the batch runs again from there.
//
// A context C (xc_coss, or the memory cache's model) provides: cache, ctx, st (the Store), known
// (hash -> fingerprint of the mirror's bytes for the hashes the Store tracks), load_miss,
// unmirrorable(), entered(h, seg) (the device entered a declared segment), before_mirror(change) /
// mirrored(change), begin_pass(hashes of the pass's events, the cache count before its device
// batch) and end_pass().  The Store provides enter, lookup, peek, read_segment, owners, window_in_slot and
// count_misses.
#pragma once
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <unordered_map>
#include <unordered_set>
#include <memory>
#include <vector>

#include "../../include/xcodec_hip.h"
#include "xc_env.h"

extern "C" int xc__set_error(int code, const char *msg);
extern "C" int xc__encode_batch_host_coll(xc_cache *c, const uint8_t *in, const uint64_t *in_off,
                                          const uint64_t *in_len, uint64_t nbuf, uint8_t *out,
                                          const uint64_t *out_off, const uint64_t *out_cap, uint64_t *out_len,
                                          const uint64_t *start, const int64_t *cand, const uint32_t *flags,
                                          uint64_t *rbase, int64_t *rcand, uint32_t *coll_cnt, uint32_t *coll);
extern "C" int xc__decode_batch_host_raw(xc_cache *c, const uint8_t *in, const uint64_t *in_off,
                                         const uint64_t *in_len, uint64_t nbuf, uint8_t *out,
                                         const uint64_t *out_off, const uint64_t *out_cap, uint64_t *out_len,
                                         uint64_t *consumed, int32_t *status, uint64_t *unknown,
                                         int32_t *has_unknown);
extern "C" int xc__hash_segments_host_raw(xc_ctx *ctx, const uint8_t *segs, uint64_t n, uint64_t *out);
extern "C" int xc__cache_truncate(xc_cache *c, uint64_t keep);
extern "C" int xc__cache_kill(xc_cache *c, const uint64_t *h, uint64_t n);
extern "C" int xc__cache_enter_bulk(xc_cache *c, const uint64_t *h, const uint8_t *segs, uint64_t n);
extern "C" int xc__cache_count_raw(xc_cache *c, uint64_t *n);

namespace replay {

constexpr uint32_t SEG = XC_SEGMENT_LENGTH;
constexpr uint32_t COLL_CAP = 16;  // xc_kernels.h

// A place in a COSS file (stripe range, position); unused by the memory cache.
struct Loc {
    uint64_t range;
    uint32_t pos;
};

// What a Store operation touched: the hashes and stripe ranges whose lookup result may have
// changed, and the slots whose bytes were replaced (recent-window entries point into them).
// moves: ids (Store::peek's versions of bytes) that name the same bytes as others now -- a full store of
// a stripe slot writes the slot's bytes to the file, so every position's slot (or earlier file) id and
// its new file id name the same bytes -- so that the settle does not read and fingerprint them again.
struct IdMove {
    uint64_t h;             // the hash stored at the position when its bytes were written
    uint64_t from[2], to[2];
};
struct Touch {
    std::vector<uint64_t> hs, ranges;
    std::vector<int> slots;
    std::vector<IdMove> moves;
    void clear()
    {
        hs.clear();
        ranges.clear();
        slots.clear();
        moves.clear();
    }
};

// Store::peek results: FOUND (*p: the bytes), IN_FILE (the stripe is loaded from the file first,
// *l: where the bytes are), ABSENT, or LOAD_MISS (not found, after loading a stripe: a miss with
// side effects).
enum { ABSENT, FOUND, IN_FILE, LOAD_MISS };

// What a Store operation did to the set of segments a lookup finds (the device mirror's contents).
struct Change {
    std::vector<uint64_t> removed;  // no longer found
    std::vector<uint64_t> added;    // found now, or found with other bytes
    std::vector<uint8_t> bytes;     // their bytes, SEG each
    bool new_lm = false;            // a hash became a LOAD_MISS one (a later miss of it has side effects)
    bool any() const { return !removed.empty() || !added.empty(); }
    void clear()
    {
        removed.clear();
        added.clear();
        bytes.clear();
        new_lm = false;
    }
};

// A hash map keyed by 64-bit hashes: open addressing, linear probing, backward-shift deletion, at
// most half full.  The COSS replay's settle looks up ~a million hashes per 64 MiB batch (the owners
// of every touched stripe range), and a node-based std::unordered_map spent most of that time in
// cache misses.  The subset of std::unordered_map's interface the replay uses: find (an entry
// pointer, end() = null), count, operator[], emplace, erase, size, clear, for_each.  Inserts and
// erases invalidate entry pointers.
template <class V>
class FlatMap {
public:
    struct Entry {
        uint64_t first;
        V second;
    };
    Entry *end() const { return nullptr; }
    const Entry *find(uint64_t k) const { return const_cast<FlatMap *>(this)->find(k); }
    Entry *find(uint64_t k)
    {
        if (k == 0) return has0_ ? &zero_ : nullptr;
        if (!n_) return nullptr;
        for (size_t i = home(k);; i = (i + 1) & mask_) {
            if (t_[i].first == k) return &t_[i];
            if (t_[i].first == 0) return nullptr;
        }
    }
    size_t count(uint64_t k) const { return find(k) ? 1 : 0; }
    V &operator[](uint64_t k) { return emplace(k, V{}).first->second; }
    std::pair<Entry *, bool> emplace(uint64_t k, const V &v)
    {
        if (k == 0) {
            if (has0_) return {&zero_, false};
            has0_ = true;
            zero_ = Entry{0, v};
            return {&zero_, true};
        }
        if (2 * (n_ + 1) > cap()) grow();
        size_t i = home(k);
        for (; t_[i].first != 0; i = (i + 1) & mask_)
            if (t_[i].first == k) return {&t_[i], false};
        t_[i] = Entry{k, v};
        n_++;
        return {&t_[i], true};
    }
    size_t erase(uint64_t k)
    {
        Entry *e = find(k);
        if (!e) return 0;
        erase(e);
        return 1;
    }
    void erase(Entry *e)
    {
        if (e == &zero_) {
            has0_ = false;
            return;
        }
        size_t i = (size_t)(e - t_.data());
        for (size_t j = (i + 1) & mask_; t_[j].first != 0; j = (j + 1) & mask_) {
            // an entry may fill the hole when the hole lies between its home and its slot
            if (((j - home(t_[j].first)) & mask_) >= ((j - i) & mask_)) {
                t_[i] = t_[j];
                i = j;
            }
        }
        t_[i].first = 0;
        n_--;
    }
    size_t size() const { return n_ + (has0_ ? 1 : 0); }
    void reserve(size_t n)
    {
        while (2 * n > cap()) grow();
    }
    bool empty() const { return size() == 0; }
    void clear()
    {
        std::fill(t_.begin(), t_.end(), Entry{0, V{}});
        n_ = 0;
        has0_ = false;
    }
    template <class F>
    void for_each(F f) const
    {
        if (has0_) f(zero_);
        for (const Entry &e : t_)
            if (e.first != 0) f(e);
    }

private:
    size_t cap() const { return t_.size(); }
    size_t home(uint64_t k) const { return (size_t)((k * 0x9E3779B97F4A7C15ull) >> shift_); }
    void grow()
    {
        std::vector<Entry> old;
        old.swap(t_);
        const size_t c = old.empty() ? 64 : 2 * old.size();
        t_.assign(c, Entry{0, V{}});
        mask_ = c - 1;
        shift_ = 64u - (unsigned)__builtin_ctzll(c);
        n_ = 0;
        for (const Entry &e : old)
            if (e.first != 0) emplace(e.first, e.second);
    }
    std::vector<Entry> t_;
    size_t mask_ = 0, n_ = 0;
    unsigned shift_ = 64;
    bool has0_ = false;
    Entry zero_{0, V{}};
};

// (four independent chains over interleaved words, then combined: the chain's multiply latency,
// not its throughput, bounded one chain; the replay fingerprints every entered segment)
inline uint64_t fingerprint(const uint8_t *p)
{
    uint64_t h[4] = {0x9E3779B97F4A7C15ull, 0xC2B2AE3D27D4EB4Full, 0x165667B19E3779F9ull, 0x27D4EB2F165667C5ull};
    for (uint32_t i = 0; i < SEG; i += 32) {
        uint64_t w[4];
        std::memcpy(w, p + i, 32);
        for (int k = 0; k < 4; k++) {
            h[k] = (h[k] ^ w[k]) * 0x100000001B3ull;
            h[k] ^= h[k] >> 29;
        }
    }
    uint64_t r = h[0];
    for (int k = 1; k < 4; k++) {
        r = (r ^ h[k]) * 0x100000001B3ull;
        r ^= r >> 29;
    }
    return r;
}

// The hashes an operation touched, looked up again without side effects: those the device holds
// and a lookup no longer finds, and those a lookup finds that the device lacks or holds with other
// bytes, go into ch (and `known` follows).
// Grow-only byte scratch, not value-initialised: a COSS batch's arenas (64 MiB in, 128 MiB out, 32
// MiB of payloads per 1024 x 64 KiB) as fresh std::vectors cost more in zeroing and first-touch page
// faults than the device's encode of them.  One per purpose and thread (the engine runs on the
// caller's thread).
struct Scratch {
    std::unique_ptr<uint8_t[]> p;
    size_t n = 0;
    uint8_t *get(size_t m)
    {
        m = std::max<size_t>(m, 1);
        if (m > n) {
            p.reset(new uint8_t[m]);
            n = m;
        }
        return p.get();
    }
};

struct SettleStats {  // (XC_REPLAY_PROF)
    uint64_t calls = 0, cand = 0, same = 0, reads = 0, copies = 0, ranges = 0;
};
inline SettleStats g_settle;

template <class C>
int settle(C *c, const Touch &t, Change &ch)
{
    // the touched hashes and window entries (few: sorted, deduplicated), then the owners of the
    // touched ranges (each hash owns one place: no duplicates among them; the COSS replay settles
    // ~a million per batch, whose sort dominated)
    for (const IdMove &m : t.moves) c->move_id(m);
    static thread_local std::vector<uint64_t> cand;  // (one settle at a time per thread: no allocation)
    cand.assign(t.hs.begin(), t.hs.end());
    for (int s : t.slots) c->st.window_in_slot(s, cand);
    std::sort(cand.begin(), cand.end());
    cand.erase(std::unique(cand.begin(), cand.end()), cand.end());
    g_settle.calls++;
    g_settle.cand += cand.size();
    g_settle.ranges += t.ranges.size();
    uint8_t buf[SEG];
    int rc = XC_OK;
    // one candidate h, peeked: r, p, l, id (where the bytes are, and their version there; 0: unknown)
    auto one = [&](uint64_t h, int r, const uint8_t *p, const Loc &l, const uint64_t *id) -> int {
        if (r == LOAD_MISS) ch.new_lm |= c->load_miss.insert(h).second;
        else if (!c->load_miss.empty()) c->load_miss.erase(h);
        // the same bytes as when the mirror last took this hash's (no read, no fingerprint): the
        // common case after a stripe load, whose 1024 hashes are all looked at
        if ((r == FOUND || r == IN_FILE) && id[0] && c->same_bytes(h, id)) {
            g_settle.same++;
            return XC_OK;
        }
        if (r == IN_FILE) {
            g_settle.reads++;
            if (!c->st.read_segment(l, buf)) return xc__set_error(XC_EDEVICE, "COSS: cannot read the cache file");
            p = buf;
        } else if (r == FOUND) {  // (a slot whose data stayed in the file: its bytes from there)
            g_settle.copies++;
            if (!c->st.copy_bytes(p, buf)) return xc__set_error(XC_EDEVICE, "COSS: cannot read the cache file");
            p = buf;
        }
        if (r != FOUND && r != IN_FILE) {
            c->note_bytes(h, nullptr);
            if (c->known.erase(h)) ch.removed.push_back(h);
            return XC_OK;
        }
        const uint64_t fp = fingerprint(p);
        c->note_bytes(h, id);
        auto it = c->known.find(h);
        if (it != c->known.end() && it->second == fp) return XC_OK;
        c->known[h] = fp;
        ch.added.push_back(h);
        ch.bytes.insert(ch.bytes.end(), p, p + SEG);
        return XC_OK;
    };
    for (uint64_t h : cand) {
        if (!h) continue;
        const uint8_t *p = nullptr;
        Loc l{0, 0};
        uint64_t id[2] = {0, 0};
        const int r = c->st.peek(h, &p, &l, id);
        if ((rc = one(h, r, p, l, id))) return rc;
    }
    if (!t.ranges.empty()) {
        // then the owners of the touched ranges not among them, range by range (each hash owns one
        // place: no duplicates among them)
        std::vector<uint64_t> rs(t.ranges);
        std::sort(rs.begin(), rs.end());
        rs.erase(std::unique(rs.begin(), rs.end()), rs.end());
        for (uint64_t rg : rs)
            c->st.peek_owners(rg, [&](uint64_t h, int r, const uint8_t *p, const Loc &l, const uint64_t *id) {
                if (rc || std::binary_search(cand.begin(), cand.end(), h)) return;
                g_settle.cand++;
                rc = one(h, r, p, l, id);
            });
    }
    return rc;
}

// The device mirror follows a change.
template <class C>
int mirror(C *c, const Change &ch)
{
    int rc = c->before_mirror(ch);
    if (!rc && !ch.removed.empty()) rc = xc__cache_kill(c->cache, ch.removed.data(), ch.removed.size());
    if (!rc && !ch.added.empty() && !(rc = xc__cache_kill(c->cache, ch.added.data(), ch.added.size())))
        rc = xc__cache_enter_bulk(c->cache, ch.added.data(), ch.bytes.data(), ch.added.size());
    if (!rc) c->mirrored(ch);
    return rc;
}

// A store operation outside a batch: the device follows at once.
template <class C>
int follow(C *c, const Touch &t)
{
    if (!c->cache) return XC_OK;
    Change ch;
    int rc = settle(c, t, ch);
    return rc ? rc : (ch.any() ? mirror(c, ch) : XC_OK);
}

// One cache event of an encoder item, in the reference's order (xcodec_encoder.cc:72-171).
struct EncEvent {
    uint64_t pos;       // window end of the lookup / declaration point (~0: flush's declaration)
    int kind;           // 0 enter (EXTRACT), 1 lookup hit (REF), 2 lookup hit (collision),
                        // 3 lookup miss with side effects (LOAD_MISS)
    uint64_t hash;
    uint64_t out_end;   // output bytes up to the end of this event's token (0 for a collision)
    uint64_t base;      // source_ start after the event (REF / EXTRACT), or at it (kinds 2, 3)
    int64_t cand;       // kinds 2, 3: the candidate pending after the lookup (-1 none)
    const uint8_t *seg; // EXTRACT payload
};

inline int64_t get_be64(const uint8_t *p)
{
    uint64_t v = 0;
    for (int i = 0; i < 8; i++) v = (v << 8) | p[i];
    return (int64_t)v;
}

// The encoder's lookup calls (xcodec_encoder.cc:111) at window ends [lo, hi) of an item, whose REF
// events are ev[0..n): every window end once the window is full, except the 2047 after a REF (the
// hash restarts, :117-127).  Minus its hits (the replay's Store::lookup counted those): its misses.
inline uint64_t enc_misses(uint64_t lo, uint64_t hi, const std::vector<EncEvent> &ev, size_t n)
{
    uint64_t calls = 0, hits = 0, cur = lo;
    for (size_t i = 0; i < n; i++) {
        const EncEvent &e = ev[i];
        if (e.kind == 0 || e.pos >= hi) continue;
        hits++;
        if (e.kind != 1) continue;
        if (e.pos >= cur) calls += e.pos + 1 - cur;
        cur = std::max(cur, e.pos + SEG);
    }
    if (hi > cur) calls += hi - cur;
    return calls > hits ? calls - hits : 0;
}

// XCodecHash (xcodec/xcodec_hash.h:31-174) over a sliding 2048-byte window: the hash of the window
// ending at each byte, as the encoder's rolling hash gives it (the value depends on the window's
// bytes only).  The device reports every lookup whose answer is a segment; the host needs the
// hashes of lookups that miss only in the one COSS state where a miss has side effects (below).
struct WindowHash {
    uint32_t s1w = 0, s2w = 0, s1b = 0, s2b = 0;
    uint64_t n = 0;
    const uint8_t *d;
    explicit WindowHash(const uint8_t *data) : d(data) {}
    static uint32_t bit(uint8_t c) { return c ? (uint32_t)__builtin_ctz(c) + 1u : 0u; }  // ffs()
    void push()  // the next byte d[n]
    {
        const uint8_t c = d[n];
        if (n >= SEG) {  // roll (:57-71): the byte leaving the window
            const uint8_t o = d[n - SEG];
            s1w -= o + 1u;
            s2w -= (o + 1u) * SEG;
            s1b -= bit(o);
            s2b -= bit(o) * SEG;
        }
        s1w += c + 1u;
        s2w += s1w;
        s1b += bit(c);
        s2b += s1b;
        n++;
    }
    uint64_t mix() const  // (:153-164: 32-bit sums and shifts)
    {
        const uint32_t bits = (s1b << 16) + s2b, bytes = (s1w << 20) + s2w;
        return ((uint64_t)bits << 36) + bytes;
    }
};

// An encoder batch item: `data` (len bytes) is an encoder's pending source_ followed by its new
// input, window ends below `start` already looked up, candidate `cand` (or -1), encode() only when
// `noflush`.  `off`: where data lies in the caller's item (restarts move it).
struct CItem {
    uint64_t buf;
    const uint8_t *data;
    uint64_t len, start;
    int64_t cand;
    uint64_t off;
    bool noflush;
};

// The lookups of item `it` that miss with side effects (Store::peek's LOAD_MISS: a COSS index entry
// whose stripe is not loaded and whose header in the file disagrees; xcodec_cache_coss.cc:200-220):
// every window end the encoder looks up (from max(2047, start); not the 2047 after a REF,
// xcodec_encoder.cc:111-127) whose hash is such a hash, as kind-3 events; then ev is sorted and each
// kind-3 event gets the state a restart after it needs (the candidate pending after the miss, the
// source_ start and output offset of the tokens before it).  The device treated them as the plain
// misses they are; the Store replays their side effects.
// A bit per 2^20 buckets of the load-miss hashes: almost every window end is rejected by one
// L2-resident load before the set's probe.
struct LmFilter {
    std::vector<uint64_t> bits;
    explicit LmFilter(const std::unordered_set<uint64_t> &lm) : bits(1u << 14, 0)
    {
        for (uint64_t h : lm) bits[bucket(h) >> 6] |= 1ull << (bucket(h) & 63);
    }
    static uint32_t bucket(uint64_t h) { return (uint32_t)((h ^ (h >> 31)) * 0x9E3779B97F4A7C15ull >> 44); }
    bool maybe(uint64_t h) const { return (bits[bucket(h) >> 6] >> (bucket(h) & 63)) & 1u; }
};

template <class Item>
void add_load_miss_lookups(const std::unordered_set<uint64_t> &lm, const LmFilter &f, const Item &it,
                           std::vector<EncEvent> &ev)
{
    std::vector<uint64_t> refs;
    for (const EncEvent &e : ev)
        if (e.kind == 1) refs.push_back(e.pos);
    std::sort(refs.begin(), refs.end());
    uint64_t resume = std::max<uint64_t>(SEG - 1, it.start);
    size_t ri = 0;
    WindowHash w(it.data);
    for (uint64_t p = 0; p < it.len; p++) {
        w.push();
        if (p < SEG - 1) continue;
        while (ri < refs.size() && refs[ri] < p) resume = std::max(resume, refs[ri++] + SEG);
        if (p < resume || (ri < refs.size() && refs[ri] == p)) continue;
        const uint64_t h = w.mix();
        if (f.maybe(h) && lm.count(h)) ev.push_back({p, 3, h, 0, 0, -1, nullptr});
    }
}

// After the sort: each kind-3 event's candidate (the first miss after the last REF / declaration
// sets it, collisions do not, xcodec_encoder.cc:96-170), source_ start and output offset.
inline void load_miss_state(std::vector<EncEvent> &ev, int64_t cand, uint64_t start)
{
    uint64_t a = std::max<uint64_t>(SEG - 1, start), base = 0, oe = 0;  // a: the next lookup
    for (EncEvent &e : ev) {
        if (e.pos == ~0ull) break;
        if (cand < 0 && a < e.pos) cand = (int64_t)(a - (SEG - 1));  // a miss before this event
        switch (e.kind) {
        case 0:  // a declaration at e.pos, whose own lookup follows
            cand = -1;
            a = e.pos;
            base = e.base;
            oe = e.out_end;
            break;
        case 1:  // REF: the hash restarts
            cand = -1;
            a = e.pos + SEG;
            base = e.base;
            oe = e.out_end;
            break;
        case 2:  // a collision is no candidate
            if (cand < 0) a = e.pos + 1;
            break;
        default:  // a miss
            if (cand < 0) cand = (int64_t)(e.pos - (SEG - 1));
            a = e.pos + 1;
            e.cand = cand;
            e.base = base;
            e.out_end = oe;
        }
    }
}

// The batch on the device, its cache events replayed into the Store in the reference's order
// (items in order), restarting the rest after a change a later event depends on.  Outputs append
// at out + out_off[buf]; res_base / res_cand: the new source_ start and candidate of each buffer,
// relative to its first item's data.
template <class C>
int encode(C *c, std::vector<CItem> items, uint8_t *out, const uint64_t *out_off, const uint64_t *out_cap,
           uint64_t *out_len, uint64_t *res_base, int64_t *res_cand)
{
    // (XC_REPLAY_PROF=1: passes, their items and the time of each phase, to stderr)
    static const bool prof = xc::abl_flag("XC_REPLAY_PROF");  // (-DXC_ABLATIONS builds)
    using clk = std::chrono::steady_clock;
    double t_dev = 0, t_ev = 0, t_rep = 0, t_set = 0, t_mir = 0;
    uint64_t n_set = 0, n_mir = 0, n_held = 0;
    uint64_t passes = 0, items0 = items.size(), items_run = 0;
    const auto t_all = clk::now();
    struct Report {
        bool on;
        const double &a, &b, &d, &e;
        const uint64_t &p, &i0, &ir;
        clk::time_point t0;
        ~Report()
        {
            if (on)
                fprintf(stderr, "replay: %llu items, %llu passes over %llu items; device %.1f ms, events %.1f ms, "
                                "store %.1f ms, total %.1f ms\n",
                        (unsigned long long)i0, (unsigned long long)p, (unsigned long long)ir, a * 1e3, b * 1e3,
                        d * 1e3, std::chrono::duration<double>(clk::now() - t0).count() * 1e3);
        }
    } report{prof, t_dev, t_ev, t_rep, t_rep, passes, items0, items_run, t_all};
    struct Report2 {
        bool on;
        const double &s, &mi;
        const uint64_t &ns, &nm, &nh;
        ~Report2()
        {
            if (on)
                fprintf(stderr, "replay store: settle %.1f ms (%llu with changes), mirror %.1f ms (%llu), held %llu; "
                                "settles %llu, candidates %llu, same %llu, reads %llu, copies %llu, ranges %llu\n",
                        s * 1e3, (unsigned long long)ns, mi * 1e3, (unsigned long long)nm, (unsigned long long)nh,
                        (unsigned long long)g_settle.calls, (unsigned long long)g_settle.cand,
                        (unsigned long long)g_settle.same, (unsigned long long)g_settle.reads,
                        (unsigned long long)g_settle.copies, (unsigned long long)g_settle.ranges);
            g_settle = SettleStats{};
        }
    } report2{prof, t_set, t_mir, n_set, n_mir, n_held};
    while (!items.empty()) {
        const uint64_t m = items.size();
        passes++;
        items_run += m;
        auto t0 = clk::now();
        uint64_t count0 = 0;
        int rc = xc__cache_count_raw(c->cache, &count0);
        if (rc) return rc;
        // the device batch
        std::vector<uint64_t> ioff(m), ilen(m), start(m), ooff(m), ocap(m), olen(m), rbase(m);
        std::vector<int64_t> cand(m), rcand(m);
        std::vector<uint32_t> fl(m, 0u), ccnt(m);
        for (uint64_t k = 0; k < m; k++) fl[k] = items[k].noflush ? 1u : 0u;  // (SF_NOFLUSH)
        std::vector<uint32_t> coll(m * COLL_CAP * 4);
        uint64_t isz = 0, osz = 0;
        for (uint64_t k = 0; k < m; k++) {
            ioff[k] = isz;
            ilen[k] = items[k].len;
            isz += items[k].len;
            ooff[k] = osz;
            ocap[k] = 2 * items[k].len + 16;
            osz += ocap[k];
            start[k] = items[k].start;
            cand[k] = items[k].cand;
        }
        static thread_local Scratch s_arena, s_obuf;
        uint8_t *const arena = s_arena.get(isz), *const obuf = s_obuf.get(osz);
        for (uint64_t k = 0; k < m; k++)
            if (items[k].len) std::memcpy(&arena[ioff[k]], items[k].data, items[k].len);
        rc = xc__encode_batch_host_coll(c->cache, arena, ioff.data(), ilen.data(), m, obuf, ooff.data(),
                                        ocap.data(), olen.data(), start.data(), cand.data(), fl.data(), rbase.data(),
                                        rcand.data(), ccnt.data(), coll.data());
        if (rc) return rc;
        t_dev += std::chrono::duration<double>(clk::now() - t0).count();
        t0 = clk::now();
        // the batch's cache events, item by item in the reference's order
        std::vector<std::vector<EncEvent>> ev(m);
        std::vector<const uint8_t *> payloads;
        for (uint64_t k = 0; k < m; k++) {
            if (ccnt[k] > COLL_CAP)
                return xc__set_error(XC_EINVAL, "too many hash collisions in one buffer to replay its cache events");
            const uint8_t *o = &obuf[ooff[k]];
            const uint64_t n = olen[k], len = items[k].len;
            uint64_t x = 0, t = 0;  // input offset, output offset
            while (t < n) {
                if (o[t] != 0xF1) { t++; x++; continue; }
                const uint8_t op = o[t + 1];
                if (op == 0x00) { t += 2; x++; continue; }
                if (op == 0x01) {  // EXTRACT: declared at cand + 4095, or by flush()
                    const uint64_t pos = x + 2 * SEG - 1 < len ? x + 2 * SEG - 1 : ~0ull;
                    ev[k].push_back({pos, 0, 0, t + 2 + SEG, x + SEG, -1, o + t + 2});
                    payloads.push_back(o + t + 2);
                    t += 2 + SEG;
                    x += SEG;
                } else {  // REF at the window's end
                    ev[k].push_back({x + SEG - 1, 1, (uint64_t)get_be64(o + t + 2), t + 10, x + SEG, -1, nullptr});
                    t += 10;
                    x += SEG;
                }
            }
            for (uint32_t i = 0; i < ccnt[k]; i++) {
                const uint32_t *r = &coll[(k * COLL_CAP + i) * 4];
                const uint64_t q = r[0];
                // source_ start at q: after the last token before it
                uint64_t base = 0, oe = 0;
                for (const EncEvent &e : ev[k])
                    if (e.kind != 2 && e.pos <= q) base = e.base, oe = e.out_end;
                ev[k].push_back({q, 2, ((uint64_t)r[2] << 32) | r[1], oe, base,
                                 r[3] == 0xFFFFFFFFu ? -1 : (int64_t)r[3], nullptr});
            }
        }
        // the lookups that miss with side effects: a host pass of the rolling hash over every item,
        // items over up to 16 threads (independent: each writes its own events)
        const bool lm = !c->load_miss.empty();
        if (lm) {
            const LmFilter f(c->load_miss);
            uint64_t total = 0;
            for (uint64_t k = 0; k < m; k++) total += items[k].len;
            const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
            const unsigned nt = (unsigned)std::min<uint64_t>({16, hw, m, std::max<uint64_t>(total >> 20, 1)});
            std::atomic<uint64_t> next{0};
            auto work = [&]() {
                for (uint64_t k; (k = next.fetch_add(1)) < m;) add_load_miss_lookups(c->load_miss, f, items[k], ev[k]);
            };
            std::vector<std::thread> th;
            try {
                for (unsigned t = 1; t < nt; t++) th.emplace_back(work);
            } catch (...) {
            }
            work();
            for (std::thread &x : th) x.join();
        }
        for (uint64_t k = 0; k < m; k++) {
            // (a declaration precedes the lookup at the same position; flush's comes last)
            std::stable_sort(ev[k].begin(), ev[k].end(), [](const EncEvent &a, const EncEvent &b) {
                return a.pos != b.pos ? a.pos < b.pos : a.kind < b.kind;
            });
            if (lm) load_miss_state(ev[k], items[k].cand, items[k].start);
        }
        // EXTRACT hashes (XCodecHash::hash of the payloads) on the device, one call
        std::vector<uint64_t> ph(payloads.size());
        if (!payloads.empty()) {
            static thread_local Scratch s_segs;
            uint8_t *const segs = s_segs.get(payloads.size() * (size_t)SEG);
            for (size_t i = 0; i < payloads.size(); i++) std::memcpy(&segs[i * SEG], payloads[i], SEG);
            if ((rc = xc__hash_segments_host_raw(c->ctx, segs, payloads.size(), ph.data()))) return rc;
        }
        {
            size_t pi = 0;
            for (uint64_t k = 0; k < m; k++) {
                // (payload order = EXTRACT order in the output; events were sorted stably)
                std::vector<EncEvent *> ex;
                for (EncEvent &e : ev[k])
                    if (e.kind == 0) ex.push_back(&e);
                std::stable_sort(ex.begin(), ex.end(), [](const EncEvent *a, const EncEvent *b) {
                    return a->out_end < b->out_end;
                });
                for (EncEvent *e : ex) e->hash = ph[pi++];
            }
        }
        {
            std::vector<uint64_t> hs;
            for (const auto &v : ev)
                for (const EncEvent &e : v) hs.push_back(e.hash);
            if ((rc = c->begin_pass(hs, count0))) return rc;
        }
        t_ev += std::chrono::duration<double>(clk::now() - t0).count();
        t0 = clk::now();
        // replay; stop at the first change a later event depends on.  last[h]: the pass's last
        // event (in order) of hash h, so that a change is checked against the later events in the
        // time of its own hashes (a scan of them all after every change was quadratic: COSS)
        if ((rc = c->unmirrorable())) return rc;
        FlatMap<uint64_t> last;
        {
            uint64_t n = 0;
            for (const auto &v : ev) n += v.size();
            last.reserve(n);
            uint64_t gi = 0;
            for (const auto &v : ev)
                for (const EncEvent &e : v) last[e.hash] = gi++;
        }
        uint64_t gbase = 0;  // the global index of item k's first event
        uint64_t entered = 0;
        bool redo = false;
        std::vector<CItem> next;
        std::vector<Change> held;  // changes nothing later in the pass saw: mirrored at its end
        Touch t;                   // (reused: no allocation per event)
        Change ch;
        for (uint64_t k = 0; k < m && !redo; k++) {
            const CItem &it = items[k];
            for (size_t e = 0; e < ev[k].size(); e++) {
                const EncEvent &E = ev[k][e];
                t.clear();
                if (E.kind == 0) {
                    c->st.enter(E.hash, E.seg, &t);
                    c->entered(E.hash, E.seg);
                    entered++;
                } else if (E.kind == 3) {
                    if (c->st.lookup(E.hash, &t))
                        return xc__set_error(XC_EDEVICE, "cache replay: a device miss the store finds");
                } else if (!c->st.lookup(E.hash, &t)) {
                    return xc__set_error(XC_EDEVICE, "cache replay: a device hit the store does not find");
                }
                ch.clear();
                const auto ts = prof ? clk::now() : clk::time_point{};
                if ((rc = settle(c, t, ch))) return rc;
                if (prof) t_set += std::chrono::duration<double>(clk::now() - ts).count();
                if (!ch.any() && !ch.new_lm) continue;
                n_set++;
                // a segment found now that was not, or a miss that now has side effects: any lookup
                // after this event may differ
                bool dep = !ch.added.empty() || ch.new_lm;
                if (!dep) {
                    const uint64_t cur = gbase + e;
                    for (uint64_t h : ch.removed) {
                        const auto it = last.find(h);
                        if (it != last.end() && it->second > cur) {
                            dep = true;
                            break;
                        }
                    }
                }
                if (!dep) {
                    held.push_back(std::move(ch));
                    n_held++;
                    continue;
                }
                // the lookups up to this event (its own, unless a declaration: the lookup at the
                // same position follows it), then roll the device cache back to this event,
                // follow the changes, run the rest again
                if (E.pos != ~0ull)
                    c->st.count_misses(enc_misses(std::max<uint64_t>(SEG - 1, it.start),
                                                  E.kind == 0 ? E.pos : E.pos + 1, ev[k], e + 1));
                else
                    c->st.count_misses(enc_misses(std::max<uint64_t>(SEG - 1, it.start), it.len, ev[k], e + 1));
                if ((rc = xc__cache_truncate(c->cache, count0 + entered))) return rc;
                for (const Change &h : held)
                    if ((rc = mirror(c, h))) return rc;
                held.clear();
                if ((rc = mirror(c, ch))) return rc;
                // (after flush()'s declaration only the escaped tail follows: no lookups)
                const uint64_t keep = E.pos == ~0ull ? olen[k] : E.out_end;
                if (out_len[it.buf] + keep > out_cap[it.buf])
                    return xc__set_error(XC_EINVAL, "output capacity too small");
                std::memcpy(out + out_off[it.buf] + out_len[it.buf], &obuf[ooff[k]], keep);
                out_len[it.buf] += keep;
                if (E.pos != ~0ull) {
                    CItem r = it;
                    r.data = it.data + E.base;
                    r.len = it.len - E.base;
                    r.off = it.off + E.base;
                    if (E.kind == 0) {  // after a declaration: its lookup at the same position is next
                        r.start = 2 * SEG - 1 - SEG;  // window end 2047 of the rest: not looked up yet
                        r.cand = -1;
                    } else if (E.kind == 1) {  // after a REF: a fresh stream
                        r.start = 0;
                        r.cand = -1;
                    } else {  // after a collision / a miss: same source_, candidate carried
                        r.start = E.pos + 1 - E.base;
                        r.cand = E.cand >= 0 ? E.cand - (int64_t)E.base : -1;
                    }
                    next.push_back(r);
                } else {  // flush()'s declaration ended the item: source_ is empty
                    res_base[it.buf] = it.off + it.len;
                    res_cand[it.buf] = -1;
                }
                for (uint64_t k2 = k + 1; k2 < m; k2++) next.push_back(items[k2]);
                redo = true;
                break;
            }
            gbase += ev[k].size();
            if (!redo) {  // item k is final
                c->st.count_misses(enc_misses(std::max<uint64_t>(SEG - 1, it.start), it.len, ev[k], ev[k].size()));
                if (out_len[it.buf] + olen[k] > out_cap[it.buf])
                    return xc__set_error(XC_EINVAL, "output capacity too small");
                std::memcpy(out + out_off[it.buf] + out_len[it.buf], &obuf[ooff[k]], olen[k]);
                out_len[it.buf] += olen[k];
                res_base[it.buf] = it.off + rbase[k];
                res_cand[it.buf] = rcand[k] >= 0 ? (int64_t)it.off + rcand[k] : -1;
            }
        }
        {
            const auto tm = clk::now();
            for (const Change &h : held)
                if ((rc = mirror(c, h))) return rc;
            n_mir += held.size();
            t_mir += std::chrono::duration<double>(clk::now() - tm).count();
        }
        if ((rc = c->end_pass())) return rc;
        t_rep += std::chrono::duration<double>(clk::now() - t0).count();
        items.swap(next);
    }
    return XC_OK;
}

// Decoder batch: stream i is one decode() call, streams in index order (xc_decode_batch_host's
// semantics), the Store advanced as the reference's cache would be.
template <class C>
int decode(C *c, const uint8_t *in, const uint64_t *in_off, const uint64_t *in_len, uint64_t nbuf, uint8_t *out,
           const uint64_t *out_off, const uint64_t *out_cap, uint64_t *out_len, uint64_t *consumed, int32_t *status,
           uint64_t *unknown, int32_t *has_unknown)
{
    struct Item {
        uint64_t buf, from;  // stream, input offset of the item
    };
    std::vector<Item> items;
    for (uint64_t i = 0; i < nbuf; i++) {
        items.push_back({i, 0});
        out_len[i] = 0;
    }
    while (!items.empty()) {
        const uint64_t m = items.size();
        uint64_t count0 = 0;
        int rc = xc__cache_count_raw(c->cache, &count0);
        if (rc) return rc;
        std::vector<uint64_t> ioff(m), ilen(m), ooff(m), ocap(m), olen(m), cons(m), unk(m);
        std::vector<int32_t> st(m), hu(m);
        uint64_t osz = 0;
        for (uint64_t k = 0; k < m; k++) {
            const Item &it = items[k];
            ioff[k] = in_off[it.buf] + it.from;
            ilen[k] = in_len[it.buf] - it.from;
            ooff[k] = osz;
            ocap[k] = out_cap[it.buf] - out_len[it.buf];
            osz += ocap[k];
        }
        static thread_local Scratch s_dout;
        uint8_t *const obuf = s_dout.get(osz);
        rc = xc__decode_batch_host_raw(c->cache, in, ioff.data(), ilen.data(), m, obuf, ooff.data(),
                                       ocap.data(), olen.data(), cons.data(), st.data(), unk.data(), hu.data());
        if (rc) return rc;
        // events: every EXTRACT / REF token the decoder executed (xcodec_decoder.cc:85-173)
        struct DEv {
            int kind;  // 0 EXTRACT (lookup, enter if absent), 1 REF (lookup)
            uint64_t hash, in_end, out_end;
            const uint8_t *seg;
        };
        std::vector<std::vector<DEv>> ev(m);
        std::vector<const uint8_t *> payloads;
        for (uint64_t k = 0; k < m; k++) {
            const uint8_t *p = in + ioff[k];
            const uint64_t n = ilen[k];
            // the tokens before the stop, and an EXTRACT the decoder stopped on as a collision
            const uint64_t lim = cons[k] + (st[k] == 0 && cons[k] >= 2 && cons[k] <= n &&
                                            p[cons[k] - 2] == 0xF1 && p[cons[k] - 1] == 0x01 ? SEG : 0);
            uint64_t x = 0, y = 0;
            while (x < lim && x < n) {
                if (p[x] != 0xF1) { x++; y++; continue; }
                if (x + 1 >= n) break;
                const uint8_t op = p[x + 1];
                if (op == 0x00) { x += 2; y++; continue; }
                if (op == 0x01 && x + 2 + SEG <= n) {
                    ev[k].push_back({0, 0, x + 2 + SEG, y + SEG, p + x + 2});
                    payloads.push_back(p + x + 2);
                    x += 2 + SEG;
                    y += SEG;
                } else if (op == 0x02 && x + 10 <= n) {
                    if (x + 10 > cons[k]) break;  // (the unknown REF the decoder stopped on: a miss)
                    ev[k].push_back({1, (uint64_t)get_be64(p + x + 2), x + 10, y + SEG, nullptr});
                    x += 10;
                    y += SEG;
                } else {
                    break;
                }
            }
        }
        std::vector<uint64_t> ph(payloads.size());
        if (!payloads.empty()) {
            static thread_local Scratch s_dsegs;
            uint8_t *const segs = s_dsegs.get(payloads.size() * (size_t)SEG);
            for (size_t i = 0; i < payloads.size(); i++) std::memcpy(&segs[i * SEG], payloads[i], SEG);
            if ((rc = xc__hash_segments_host_raw(c->ctx, segs, payloads.size(), ph.data()))) return rc;
            size_t pi = 0;
            for (auto &v : ev)
                for (DEv &e : v)
                    if (e.kind == 0) e.hash = ph[pi++];
        }
        {
            std::vector<uint64_t> hs;
            for (const auto &v : ev)
                for (const DEv &e : v) hs.push_back(e.hash);
            if ((rc = c->begin_pass(hs, count0))) return rc;
        }
        if ((rc = c->unmirrorable())) return rc;
        // last[h]: the pass's last token of hash h in order (a stream's unknown REF after its tokens):
        // a change is checked against the later ones in the time of its own hashes
        std::unordered_map<uint64_t, uint64_t> last;
        std::vector<uint64_t> gbase(m + 1, 0);
        {
            uint64_t gi = 0;
            for (uint64_t k = 0; k < m; k++) {
                gbase[k] = gi;
                for (const DEv &e : ev[k]) last[e.hash] = gi++;
                if (hu[k]) last[unk[k]] = gi;
                gi++;
            }
            gbase[m] = gi;
        }
        auto later = [&](const Change &ch, uint64_t cur) {
            for (const auto *v : {&ch.added, &ch.removed})
                for (uint64_t h : *v) {
                    const auto it = last.find(h);
                    if (it != last.end() && it->second > cur) return true;
                }
            return false;
        };
        uint64_t entered = 0;
        bool redo = false;
        std::vector<Item> next;
        std::vector<Change> held;
        for (uint64_t k = 0; k < m && !redo; k++) {
            const Item &it = items[k];
            for (size_t e = 0; e < ev[k].size(); e++) {
                const DEv &E = ev[k][e];
                Touch t;
                const uint8_t *d = c->st.lookup(E.hash, &t);
                if (E.kind == 0 && !d) {
                    c->st.enter(E.hash, E.seg, &t);
                    c->entered(E.hash, E.seg);
                    entered++;
                } else if (E.kind == 1 && !d) {
                    return xc__set_error(XC_EDEVICE, "cache replay: a device hit the store does not find");
                }
                Change ch;
                if ((rc = settle(c, t, ch))) return rc;
                if (!ch.any() && !ch.new_lm) continue;
                // later tokens, and the unknown REF a later stream stopped on, that saw the change
                const bool dep = ch.new_lm || later(ch, gbase[k] + e);
                if (!dep) {
                    held.push_back(std::move(ch));
                    continue;
                }
                if ((rc = xc__cache_truncate(c->cache, count0 + entered))) return rc;
                for (const Change &h : held)
                    if ((rc = mirror(c, h))) return rc;
                held.clear();
                if ((rc = mirror(c, ch))) return rc;
                std::memcpy(out + out_off[it.buf] + out_len[it.buf], &obuf[ooff[k]], E.out_end);
                out_len[it.buf] += E.out_end;
                next.push_back({it.buf, it.from + E.in_end});
                for (uint64_t k2 = k + 1; k2 < m; k2++) next.push_back(items[k2]);
                redo = true;
                break;
            }
            if (!redo) {
                std::memcpy(out + out_off[it.buf] + out_len[it.buf], &obuf[ooff[k]], olen[k]);
                out_len[it.buf] += olen[k];
                consumed[it.buf] = it.from + cons[k];
                status[it.buf] = st[k];
                unknown[it.buf] = unk[k];
                has_unknown[it.buf] = hu[k];
                if (hu[k]) {  // the unknown REF's lookup (:150): a miss, with side effects in one state
                    Touch t;
                    if (c->st.lookup(unk[k], &t))
                        return xc__set_error(XC_EDEVICE, "cache replay: a device miss the store finds");
                    Change ch;
                    if ((rc = settle(c, t, ch))) return rc;
                    if (ch.any() || ch.new_lm) {
                        const bool dep = ch.new_lm || later(ch, gbase[k] + ev[k].size());
                        if (!dep) {
                            held.push_back(std::move(ch));
                        } else {  // stream k is done; the later ones run again
                            if ((rc = xc__cache_truncate(c->cache, count0 + entered))) return rc;
                            for (const Change &h : held)
                                if ((rc = mirror(c, h))) return rc;
                            held.clear();
                            if ((rc = mirror(c, ch))) return rc;
                            for (uint64_t k2 = k + 1; k2 < m; k2++) next.push_back(items[k2]);
                            redo = true;
                        }
                    }
                }
            }
        }
        for (const Change &h : held)
            if ((rc = mirror(c, h))) return rc;
        if ((rc = c->end_pass())) return rc;
        items.swap(next);
    }
    return XC_OK;
}

}  // namespace replay
