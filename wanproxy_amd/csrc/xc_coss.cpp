// xc_coss.cpp — the persistent COSS cache (XCodecCacheCOSS, xcodec/cache/coss/) as a host tier
// over the device cache.
//
// The reference's COSS cache keeps segments in a file <cache_dir>/<uuid>.wpc of stripes (512
// segments and a header each), 16 stripes in memory, an in-memory index hash -> (stripe, slot),
// and on top the 64-entry recent window of XCodecCache (xcodec/xcodec_cache.h:94-158).  A lookup
// hit has side effects (stripe loads, freshness, use flags, the recent window), and when the file
// is full the stripe to reuse is purged of the segments not used since its last purge
// (xcodec_cache_coss.cc:163-377): which segments the codec finds depends on that history.
//
// Here the device cache holds exactly the segments a COSS lookup would find, with the bytes it would
// return (its mirror), so the device encoder and decoder run as over the memory cache; the Store below
// is the reference's COSS state machine, same file format, driven afterwards by the batch's cache
// events in the reference's order (enters and lookup hits: every EXTRACT and REF token of the
// outputs, and the collisions the walk records).  Every Store operation reports what it touched
// (hashes, stripe ranges, slots); those are looked up again without side effects (Store::peek) and
// compared with the mirror.  What a lookup finds changes at a purge, when a slot takes another
// stripe (lookup takes the first slot whose stripe_range matches, :200-207: an unused slot, or the
// first of two copies of a stripe — best_erasable_stripe returns a loaded stripe when every stripe
// is loaded, :304-321 — shadows the one that holds the entry), when the recent window forgets or
// drops a hash a purge left findable only there, and when a stripe slot's bytes under a window entry
// are replaced.  When a change happens inside a batch and a later event depends on it (for a segment
// that became findable: any later lookup), the device cache is rolled back to that event, follows
// the change, and the rest of the batch runs again from there (a REF or a declaration restarts an
// encoder as a fresh stream item, a collision with its carried candidate; a decoder restarts at the
// token boundary) — so outputs, cache contents and the file bytes equal the reference's.
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cstddef>
#include <cstring>
#include <memory>
#include <new>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "../../include/xcodec_hip.h"

#include "xc_replay.h"

extern "C" void xc__cache_untracked(xc_cache *c);
extern "C" int xc__cache_find(xc_cache *c, const uint64_t *h, uint64_t n, uint64_t *val);
extern "C" int xc__cache_read(xc_cache *c, uint64_t h, uint8_t *out, int *found);

namespace coss {

constexpr uint32_t SEG = XC_SEGMENT_LENGTH;
constexpr uint32_t SIGNATURE = 0xF150E964u;  // xcodec_cache_coss.h:83
constexpr uint32_t VERSION = 2;              // :84
constexpr uint32_t STRIPE_SEGS = 512;        // :85
constexpr int LOADED = 16;                   // :86
constexpr uint64_t BASIC_MB = 1024;          // :87
constexpr int WINDOW = 64;                   // xcodec_cache.h:48

struct Meta {  // COSSMetadata (:147-160), on disk as is
    uint32_t signature, version;
    uint64_t serial_number, stripe_range;
    uint32_t segment_index, segment_count;
    uint64_t freshness, uses, credits;
    uint32_t load_uses, state;
};
static_assert(sizeof(Meta) == 64, "COSSMetadata layout");

constexpr size_t HEADER = 8192;  // ROUND_UP(512 * 12 + 64, 4096) (:91-94)
struct Header {                  // COSSStripeHeader (:162-168)
    Meta m;
    char padding[HEADER - STRIPE_SEGS * 12 - sizeof(Meta)];
    uint32_t flags[STRIPE_SEGS];
    uint64_t hash[STRIPE_SEGS];
};
static_assert(sizeof(Header) == HEADER, "COSSStripeHeader layout");

struct Stripe {  // COSSStripe (:170-177)
    Header h;
    uint8_t seg[STRIPE_SEGS][SEG];
};

using replay::Loc;
using replay::Touch;

class Store {
public:
    int open(const std::string &path, uint64_t size_mb)
    {
        path_ = path;
        struct stat st;
        if (::stat(path.c_str(), &st) == 0 && S_ISREG(st.st_mode)) {
            file_size_ = (uint64_t)st.st_size;
        } else {
            const int t = ::open(path.c_str(), O_CREAT | O_WRONLY | O_TRUNC, 0644);
            if (t < 0) return XC_EINVAL;
            ::close(t);
            file_size_ = 0;
        }
        if (!size_mb) size_mb = BASIC_MB;
        limit_ = (size_mb * 1048576ull + sizeof(Stripe) - 1) / sizeof(Stripe);
        slot_.reset(new (std::nothrow) Stripe[LOADED]());  // COSSStripe(): zeroed headers
        if (!slot_) return XC_ENOMEM;
        for (auto &r : resident_) r = true;  // (zeroed memory is the slots' content)
        dir_.assign(limit_, Meta{});
        fstamp_.assign(limit_, 0);
        owner_.assign(limit_ * STRIPE_SEGS, 0);
        file_hash_.assign(limit_ * STRIPE_SEGS, 0);
        fd_ = ::open(path.c_str(), O_RDWR);
        if (fd_ < 0 || !read_file()) {
            if (fd_ >= 0) ::close(fd_);
            fd_ = ::open(path.c_str(), O_RDWR | O_CREAT | O_TRUNC, 0644);
            if (fd_ < 0) return XC_EINVAL;
            file_size_ = 0;
            index_.clear();
            std::fill(owner_.begin(), owner_.end(), 0);
            std::fill(file_hash_.begin(), file_hash_.end(), 0);
            initialize_stripe(range_, active_, nullptr);
        }
        return XC_OK;
    }

    void close()
    {  // ~XCodecCacheCOSS (:82-105)
        if (fd_ < 0) return;
        for (int i = 0; i < LOADED; ++i)
            if (slot_[i].h.m.state == 1) store_stripe(i, i == active_ ? sizeof(Stripe) : sizeof(Header), nullptr);
        ::close(fd_);
        fd_ = -1;
    }

    // XCodecCacheCOSS::enter (:163-186)
    void enter(uint64_t h, const uint8_t *seg, Touch *t)
    {
        while (slot_[active_].h.m.segment_index >= STRIPE_SEGS) new_active(t);
        Stripe &a = slot_[active_];
        const uint32_t i = a.h.m.segment_index;
        a.h.hash[i] = h;
        std::memcpy(a.seg[i], seg, SEG);
        wstamp_[active_][i] = ++stamp_;
        written_[active_] = true;
        const uint64_t range = a.h.m.stripe_range;
        a.h.m.segment_index++;
        while (a.h.m.segment_index < STRIPE_SEGS && a.h.hash[a.h.m.segment_index]) a.h.m.segment_index++;
        a.h.m.segment_count++;
        a.h.m.freshness = ++freshness_;
        index_put(h, Loc{range, i}, t);
    }

    // XCodecCacheCOSS::lookup (:188-228), with XCodecCache::find_recent / remember: the segment's
    // bytes, or null.
    const uint8_t *lookup(uint64_t h, Touch *t)
    {
        lookups_++;
        for (int i = 0; i < (wcnt_[wbucket(h)] ? WINDOW : 0); i++)  // find_recent (xcodec_cache.h:137-147)
            if (win_[i].hash == h) {
                if (win_[i].data) {
                    found_1_++;
                    return win_[i].data;
                }
                break;
            }
        auto it = index_.find(h);
        if (it == index_.end()) return nullptr;
        const Loc e = it->second;
        int s = first_slot(e.range);
        if (s >= LOADED) {
            s = best_unloadable_slot();
            // A slot read from the file and not written since names the file's bytes at every
            // position (peek's file ids), as the file does once it is detached, and a stripe read
            // from the file into it names the same ids it had in the file: when the two stripes'
            // headers agree with the file and no other slot holds either, no owner of them finds
            // other bytes or a miss of another kind, and their ~1000 owners need no settle (the
            // slot's window entries and the window's forgotten hashes still do).
            const uint64_t old = slot_[s].h.m.stripe_range;
            const bool quiet = t && slot_[s].h.m.signature != 0 && slot_[s].h.m.state == 1 && from_file_[s] &&
                               !written_[s] && old < limit_ && e.range < limit_ && only_holder(s, old) &&
                               std::memcmp(slot_[s].h.hash, &file_hash_[old * STRIPE_SEGS], sizeof(Header::hash)) == 0 &&
                               owners_agree(old) && owners_agree(e.range);
            Touch q;
            detach_stripe(s, quiet ? &q : t);
            const bool loaded = load_stripe(e.range, s, quiet ? &q : t, false);  // (its header: the data stays in the file)
            if (quiet) {
                t->hs.insert(t->hs.end(), q.hs.begin(), q.hs.end());
                t->slots.insert(t->slots.end(), q.slots.begin(), q.slots.end());
                if (!loaded || !from_file_[s]) t->ranges.insert(t->ranges.end(), q.ranges.begin(), q.ranges.end());
            }
        }
        Stripe &st = slot_[s];
        if (st.h.hash[e.pos] != h) return nullptr;
        st.h.m.freshness = ++freshness_;
        st.h.m.uses++;
        st.h.m.credits++;
        st.h.m.load_uses++;
        st.h.flags[e.pos] |= 3u;
        const uint8_t *d = st.seg[e.pos];
        if (t) {  // remember (xcodec_cache.h:130-135)
            t->hs.push_back(h);
            t->hs.push_back(win_[cursor_].hash);
        }
        wset(cursor_, h);
        win_[cursor_].data = d;
        cursor_ = (cursor_ + 1) & (WINDOW - 1);
        found_2_++;
        return d;
    }

    // What lookup(h) returns now, without its side effects: FOUND (*p: the bytes), IN_FILE (the
    // stripe is loaded from the file first, *l: where the bytes are), ABSENT, or LOAD_MISS (not
    // found, after loading a stripe: a miss with side effects).
    enum { ABSENT = replay::ABSENT, FOUND = replay::FOUND, IN_FILE = replay::IN_FILE, LOAD_MISS = replay::LOAD_MISS };
    // id (the replay's settle): where the bytes are and their version there -- slot s, position pos
    // and the stamp of the last load of s or write at (s, pos); or stripe r, position pos of the file
    // and the stamp of r's last full store -- equal ids have equal bytes.
    int peek(uint64_t h, const uint8_t **p, Loc *l, uint64_t *id) const
    {
        if (peek_window(h, p, id)) return FOUND;
        auto it = index_.find(h);
        if (it == index_.end()) return ABSENT;
        const Loc e = it->second;
        return peek_at(h, e, first_slot(e.range), p, l, id);
    }

    // The owners of stripe `range` (the hashes whose index entries point into it), each peeked:
    // f(hash, peek's result, p, l, id).  The index entry of an owner is (range, its position) and
    // the first slot is the range's for every owner: no index lookup, no slot search per hash (the
    // replay's settle peeks every owner of every touched range, ~a million per 64 MiB batch).
    template <class F>
    void peek_owners(uint64_t range, F f) const
    {
        if (range >= limit_) return;
        const int s = first_slot(range);
        const uint64_t *own = &owner_[range * STRIPE_SEGS];
        for (uint32_t i = 0; i < STRIPE_SEGS; i++) {
            const uint64_t h = own[i];
            if (!h) continue;
            const uint8_t *p = nullptr;
            Loc l{0, 0};
            uint64_t id[2] = {0, 0};
            const int r = peek_window(h, &p, id) ? FOUND : peek_at(h, Loc{range, i}, s, &p, &l, id);
            f(h, r, p, l, id);
        }
    }

    // peek's first step: the recent window (find_recent, xcodec_cache.h:137-147)
    bool peek_window(uint64_t h, const uint8_t **p, uint64_t *id) const
    {
        for (int i = 0; i < (wcnt_[wbucket(h)] ? WINDOW : 0); i++)
            if (win_[i].hash == h) {
                if (win_[i].data) {
                    *p = win_[i].data;
                    slot_id(win_[i].data, id);
                    return true;
                }
                break;
            }
        return false;
    }

    // peek's rest, for a hash not in the window whose index entry is e, the first slot of its range s
    int peek_at(uint64_t h, Loc e, int s, const uint8_t **p, Loc *l, uint64_t *id) const
    {
        if (s < LOADED) {
            if (slot_[s].h.hash[e.pos] != h) return ABSENT;
            *p = slot_[s].seg[e.pos];
            slot_id(*p, id);
            return FOUND;
        }
        *l = e;
        if (e.range * sizeof(Stripe) >= file_size_) return LOAD_MISS;
        if (file_hash_[e.range * STRIPE_SEGS + e.pos] != h) return LOAD_MISS;
        id[0] = (1ull << 62) | (e.range << 9) | e.pos;
        id[1] = fstamp_[e.range];
        return IN_FILE;
    }

    // The 2048 bytes at p, a pointer into a slot's data (a lookup's result, a window entry): from
    // memory, or, for a slot whose data was not read in (lazy loads), from the file at the slot's
    // stripe (the file's bytes there are the slot's: they change only by a full store of that
    // stripe, which reads every such slot in first).
    bool copy_bytes(const uint8_t *p, uint8_t *out) const
    {
        const uint8_t *b0 = slot_[0].seg[0];
        const size_t off = (size_t)(p - (const uint8_t *)&slot_[0]);
        const int s = (int)(off / sizeof(Stripe));
        if (p < b0 || s >= LOADED || resident_[s]) {
            std::memcpy(out, p, SEG);
            return true;
        }
        const uint32_t pos = (uint32_t)((p - slot_[s].seg[0]) / SEG);
        const off_t at = (off_t)(slot_[s].h.m.stripe_range * sizeof(Stripe) + HEADER + (uint64_t)pos * SEG);
        return ::pread(fd_, out, SEG, at) == (ssize_t)SEG;
    }

    // A position of a slot loaded from the file and not written since holds the file's bytes of the
    // version it was loaded at: the file's id, so that loading a stripe (a lookup's, every 512 of its
    // hashes settled) reads and fingerprints nothing the mirror already took from the file.
    // p (a lookup's result) points at bytes held in memory (not a lazily loaded slot's)
    bool in_memory(const uint8_t *p) const
    {
        const size_t off = (size_t)(p - (const uint8_t *)&slot_[0]);
        const int s = (int)(off / sizeof(Stripe));
        return p < slot_[0].seg[0] || s >= LOADED || resident_[s];
    }

    void slot_id(const uint8_t *p, uint64_t *id) const
    {
        const size_t off = (size_t)(p - (const uint8_t *)&slot_[0]);
        const uint32_t s = (uint32_t)(off / sizeof(Stripe));
        if (p < slot_[0].seg[0] || s >= (uint32_t)LOADED) return;
        const uint32_t pos = (uint32_t)((p - slot_[s].seg[0]) / SEG);
        if (from_file_[s] && wstamp_[s][pos] < load_stamp_[s]) {
            id[0] = (1ull << 62) | (slot_[s].h.m.stripe_range << 9) | pos;
            id[1] = load_fstamp_[s];
            return;
        }
        id[0] = 1u + ((uint64_t)s << 9 | pos);
        id[1] = std::max(load_stamp_[s], wstamp_[s][pos]);
    }

    bool read_segment(const Loc &l, uint8_t *out) const
    {
        const off_t at = (off_t)(l.range * sizeof(Stripe) + HEADER + (uint64_t)l.pos * SEG);
        return ::pread(fd_, out, SEG, at) == (ssize_t)SEG;
    }

    // The hashes whose index entries point into stripe `range`.
    void owners(uint64_t range, std::vector<uint64_t> &out) const
    {
        if (range >= limit_) return;
        for (uint32_t i = 0; i < STRIPE_SEGS; i++)
            if (owner_[range * STRIPE_SEGS + i]) out.push_back(owner_[range * STRIPE_SEGS + i]);
    }

    // The recent-window hashes whose bytes lie in slot s.
    void window_in_slot(int s, std::vector<uint64_t> &out) const
    {
        const uint8_t *b = slot_[s].seg[0], *e = b + sizeof(Stripe::seg);
        for (int i = 0; i < WINDOW; i++)
            if (win_[i].hash && win_[i].data >= b && win_[i].data < e) out.push_back(win_[i].hash);
    }

    void all_hashes(std::vector<uint64_t> &out) const
    {
        index_.for_each([&](const Index::Entry &e) { out.push_back(e.first); });
    }

    size_t size() const { return index_.size(); }

    // (tests) the stripe headers read again from the file, as after another writer changed them:
    // a header that disagrees with the index is the state where a lookup misses after loading the
    // stripe (LOAD_MISS).  t: every indexed hash.
    bool reread_headers(Touch *t)
    {
        const uint64_t n = std::min<uint64_t>(limit_, file_size_ / sizeof(Stripe));
        for (uint64_t r = 0; r < n; r++)
            if (::pread(fd_, &file_hash_[r * STRIPE_SEGS], sizeof(Header::hash),
                        (off_t)(r * sizeof(Stripe) + offsetof(Header, hash))) != (ssize_t)sizeof(Header::hash))
                return false;
        all_hashes(t->hs);
        return true;
    }
    // Lookups the device made that missed (a miss outside the one state LOAD_MISS flags has no side
    // effect but the count): stats_.lookups counts every call (:194).
    void count_misses(uint64_t n) { lookups_ += n; }
    void stats(uint64_t *o) const
    {
        o[0] = lookups_;
        o[1] = found_1_;
        o[2] = found_2_;
        o[3] = index_.size();
        o[4] = limit_;
        o[5] = serial_;
    }

private:
    // no slot but s holds stripe `range`
    bool only_holder(int s, uint64_t range) const
    {
        for (int i = 0; i < LOADED; i++)
            if (i != s && slot_[i].h.m.stripe_range == range) return false;
        return true;
    }

    // every owner of stripe `range` is the hash the file's header has at its position (a lookup
    // through the file finds it, no load miss)
    bool owners_agree(uint64_t range) const
    {
        const uint64_t *o = &owner_[range * STRIPE_SEGS], *f = &file_hash_[range * STRIPE_SEGS];
        for (uint32_t i = 0; i < STRIPE_SEGS; i++)
            if (o[i] && o[i] != f[i]) return false;
        return true;
    }

    // lookup takes the first slot whose stripe_range matches (:200-207): an unused slot (zeroed
    // header, stripe_range 0) or a second copy of a stripe can shadow the one that holds it
    int first_slot(uint64_t range) const
    {
        int s = 0;
        while (s < LOADED && slot_[s].h.m.stripe_range != range) s++;
        return s;
    }

    void index_put(uint64_t h, Loc l, Touch *t)
    {
        auto it = index_.find(h);
        if (it != index_.end()) {
            uint64_t &o = owner_[it->second.range * STRIPE_SEGS + it->second.pos];
            if (o == h) o = 0;
            it->second = l;
        } else {
            index_.emplace(h, l);
        }
        owner_[l.range * STRIPE_SEGS + l.pos] = h;
        if (t) t->hs.push_back(h);
    }

    void index_erase(uint64_t h, Touch *t)
    {
        auto it = index_.find(h);
        if (it == index_.end()) return;
        uint64_t &o = owner_[it->second.range * STRIPE_SEGS + it->second.pos];
        if (o == h) o = 0;
        index_.erase(it);
        if (t) t->hs.push_back(h);
    }

    // slot s takes another stripe (or a fresh header)
    void retarget(int s, uint64_t range, Touch *t)
    {
        if (!t) return;
        t->ranges.push_back(slot_[s].h.m.stripe_range);
        t->ranges.push_back(range);
        t->slots.push_back(s);
    }

    bool read_file()
    {  // :107-161
        Header h;
        uint64_t serial = 0, range = 0, level = 0;
        uint64_t limit = file_size_ / sizeof(Stripe);
        if (limit * sizeof(Stripe) != file_size_) return false;
        if (limit > limit_) limit = limit_;
        for (uint64_t n = 0; n < limit; ++n) {
            if (::pread(fd_, &h, sizeof h, (off_t)(n * sizeof(Stripe))) != (ssize_t)sizeof h) return false;
            if (h.m.signature != SIGNATURE) return false;
            if (h.m.segment_count > STRIPE_SEGS) return false;
            if (h.m.serial_number > serial) serial = h.m.serial_number, range = n;
            if (h.m.freshness > level) level = h.m.freshness;
            dir_[n] = h.m;
            dir_[n].state = 0;
            std::memcpy(&file_hash_[n * STRIPE_SEGS], h.hash, sizeof h.hash);
            for (uint32_t i = 0; i < STRIPE_SEGS; ++i)
                if (h.hash[i]) index_put(h.hash[i], Loc{n, i}, nullptr);
        }
        if (serial > 0) {
            serial_ = serial;
            range_ = range;
            freshness_ = level;
            load_stripe(range_, active_, nullptr);
        } else {
            initialize_stripe(range_, active_, nullptr);
        }
        return true;
    }

    void initialize_stripe(uint64_t range, int s, Touch *t)
    {  // :230-239
        retarget(s, range, t);
        load_stamp_[s] = ++stamp_;
        from_file_[s] = false;
        written_[s] = false;
        std::memset(&slot_[s].h, 0, sizeof(Header));
        Meta &m = slot_[s].h.m;
        m.signature = SIGNATURE;
        m.version = VERSION;
        m.serial_number = ++serial_;
        m.stripe_range = range;
        m.state = 1;
        dir_[range] = m;
    }

    // full = false: the header only (a stripe loaded for a lookup: its data is never written back,
    // and what reads it, copy_bytes, reads the file instead; materialize reads it in when the slot's
    // memory must hold it)
    bool load_stripe(uint64_t range, int s, Touch *t, bool full = true)
    {  // :241-260
        const uint64_t pos = range * sizeof(Stripe);
        if (pos < file_size_) {
            retarget(s, range, t);
            const size_t n = full ? sizeof(Stripe) : sizeof(Header);
            load_stamp_[s] = ++stamp_;  // (the slot's bytes are another stripe's now)
            from_file_[s] = false;
            written_[s] = false;
            if (::pread(fd_, &slot_[s], n, (off_t)pos) == (ssize_t)n) {
                resident_[s] = full;
                from_file_[s] = range < limit_;
                load_fstamp_[s] = range < limit_ ? fstamp_[range] : 0;
                slot_[s].h.m.stripe_range = range;
                slot_[s].h.m.load_uses = 0;
                slot_[s].h.m.state = 1;
                dir_[range].state = 1;
                return true;
            }
            resident_[s] = false;  // (a short read: the memory's data is undefined, as in the reference)
        }
        return false;
    }

    // Slot s's data into its memory (the file's bytes of its stripe, as a full load would have read).
    void materialize(int s)
    {
        if (resident_[s]) return;
        const uint64_t pos = slot_[s].h.m.stripe_range * sizeof(Stripe) + HEADER;
        if (::pread(fd_, slot_[s].seg, sizeof(Stripe::seg), (off_t)pos) != (ssize_t)sizeof(Stripe::seg))
            std::memset(slot_[s].seg, 0, sizeof(Stripe::seg));  // (past the file's end: never loaded)
        resident_[s] = true;
    }

    void store_stripe(int s, size_t size, Touch *t)
    {  // :262-272
        const uint64_t range = slot_[s].h.m.stripe_range, pos = range * sizeof(Stripe);
        if (size > sizeof(Header)) {
            materialize(s);
            for (int i = 0; i < LOADED; i++)  // (their data is the file's: read it before it changes)
                if (i != s && !resident_[i] && slot_[i].h.m.stripe_range == range) materialize(i);
        }
        // the positions' ids before the store (their bytes are the file's after it)
        replay::IdMove mv[STRIPE_SEGS];
        uint16_t mpos[STRIPE_SEGS];
        uint32_t nmv = 0;
        if (t && size > sizeof(Header) && range < limit_)
            for (uint32_t i = 0; i < STRIPE_SEGS; i++)
                if (slot_[s].h.hash[i]) {
                    mv[nmv] = replay::IdMove{slot_[s].h.hash[i], {0, 0}, {0, 0}};
                    slot_id(slot_[s].seg[i], mv[nmv].from);
                    mpos[nmv++] = (uint16_t)i;
                }
        if (size > sizeof(Header) && range < limit_) fstamp_[range] = ++stamp_;
        if (::pwrite(fd_, &slot_[s], size, (off_t)pos) == (ssize_t)size) {
            for (uint32_t k = 0; k < nmv; k++) {  // (peek's IN_FILE id of the position now)
                mv[k].to[0] = (1ull << 62) | (range << 9) | mpos[k];
                mv[k].to[1] = fstamp_[range];
                if (mv[k].from[0]) t->moves.push_back(mv[k]);
            }
            if (pos + sizeof(Stripe) > file_size_) file_size_ = pos + sizeof(Stripe);
            if (range < limit_) std::memcpy(&file_hash_[range * STRIPE_SEGS], slot_[s].h.hash, sizeof slot_[s].h.hash);
            if (t) t->ranges.push_back(range);
        }
    }

    void new_active(Touch *t)
    {  // :274-283
        store_stripe(active_, sizeof(Stripe), t);
        active_ = best_unloadable_slot();
        materialize(active_);  // (the active slot's memory is written back whole: it holds its data)
        detach_stripe(active_, t);
        range_ = best_erasable_stripe();
        if (load_stripe(range_, active_, t)) purge_stripe(active_, t);
        else initialize_stripe(range_, active_, t);
    }

    int best_unloadable_slot() const
    {  // :285-302
        uint64_t n = ~0ull;
        int j = 0;
        for (int i = 0; i < LOADED; ++i) {
            if (i == active_) continue;
            const Meta &m = slot_[i].h.m;
            if (m.signature == 0) return i;
            const uint64_t v = m.freshness + m.load_uses;
            if (v < n) j = i, n = v;
        }
        return j;
    }

    uint64_t best_erasable_stripe() const
    {  // :304-321 (every stripe loaded: stripe 0, though loaded — a second copy of it)
        uint64_t n = ~0ull, j = 0;
        for (uint64_t i = 0; i < limit_; ++i) {
            const Meta &m = dir_[i];
            if (m.state == 1) continue;
            if (m.signature == 0) return i;
            const uint64_t v = m.freshness + m.uses;
            if (v < n) j = i, n = v;
        }
        return j;
    }

    void detach_stripe(int s, Touch *t)
    {  // :323-345
        Stripe &st = slot_[s];
        if (st.h.m.state != 1) return;
        const uint64_t range = st.h.m.stripe_range;
        dir_[range] = st.h.m;
        dir_[range].state = 2;
        for (uint32_t i = 0; i < STRIPE_SEGS; ++i)
            if (st.h.flags[i] & 1u) {
                for (int w = 0; w < WINDOW; w++)  // forget (xcodec_cache.h:150-158)
                    if (win_[w].hash == st.h.hash[i]) {
                        wset(w, 0);
                        if (t) t->hs.push_back(st.h.hash[i]);
                    }
                st.h.flags[i] &= ~1u;
            }
        st.h.m.state = 0;
        store_stripe(s, sizeof(Header), t);
    }

    void purge_stripe(int s, Touch *t)
    {  // :347-377
        Stripe &st = slot_[s];
        written_[s] = true;  // (its header is not the file's any more)
        if (t) t->ranges.push_back(st.h.m.stripe_range);
        for (int i = (int)STRIPE_SEGS - 1; i >= 0; --i) {
            const uint64_t h = st.h.hash[i];
            if (h && !(st.h.flags[i] & 2u)) {
                index_erase(h, t);
                st.h.hash[i] = 0;
                st.h.flags[i] = 0;
                st.h.m.segment_count--;
            }
            st.h.flags[i] &= ~2u;
            if (!st.h.hash[i]) st.h.m.segment_index = (uint32_t)i;
        }
        st.h.m.serial_number = ++serial_;
        st.h.m.uses = st.h.m.credits;
        st.h.m.credits = 0;
    }

    std::string path_;
    int fd_ = -1;
    uint64_t file_size_ = 0, serial_ = 0, range_ = 0, limit_ = 0, freshness_ = 0;
    std::unique_ptr<Stripe[]> slot_;
    bool resident_[LOADED] = {};  // the slot's data is in its memory (else: in the file at its stripe)
    // versions of the bytes (peek's ids): a counter, the slots' last loads, their positions' last
    // enters, the stripes' last full stores to the file
    uint64_t stamp_ = 0, load_stamp_[LOADED] = {}, wstamp_[LOADED][STRIPE_SEGS] = {};
    // a slot loaded from the file (its unwritten positions: the file's bytes at load_fstamp_)
    bool from_file_[LOADED] = {};
    // a slot written (enter) or purged since it took its stripe
    bool written_[LOADED] = {};
    uint64_t load_fstamp_[LOADED] = {};
    std::vector<uint64_t> fstamp_;
    int active_ = 0;
    std::vector<Meta> dir_;
    using Index = replay::FlatMap<Loc>;
    Index index_;
    std::vector<uint64_t> owner_;      // [range * 512 + pos]: the hash whose index entry is there
    std::vector<uint64_t> file_hash_;  // [range * 512 + pos]: the stripe headers as in the file
    struct {
        uint64_t hash;
        const uint8_t *data;
    } win_[WINDOW] = {};
    // window slots per bucket of their hash (peek skips the 64 compares for almost every hash)
    uint8_t wcnt_[4096] = {WINDOW};
    static uint32_t wbucket(uint64_t h) { return (uint32_t)(h ^ (h >> 27)) & 4095u; }
    void wset(int i, uint64_t h)
    {
        wcnt_[wbucket(win_[i].hash)]--;
        win_[i].hash = h;
        wcnt_[wbucket(h)]++;
    }
    unsigned cursor_ = 0;
    uint64_t lookups_ = 0, found_1_ = 0, found_2_ = 0;
};

}  // namespace coss

// The COSS cache: the Store, and the device cache as its mirror (xc_replay.h's context).
struct xc_coss {
    xc_ctx *ctx = nullptr;
    xc_cache *cache = nullptr;  // the device mirror (null for a host-only store)
    coss::Store st;
    // what the device cache holds: hash -> fingerprint of its bytes
    replay::FlatMap<uint64_t> known;
    // hashes a lookup misses only after loading a stripe (a miss with side effects)
    std::unordered_set<uint64_t> load_miss;

    // per replay pass: hashes the device held before the pass's batch, and those entered in it
    replay::FlatMap<char> pre, inpass;  // (sets)
    int err = XC_OK;

    // the device entered a declared segment: its bytes, unless the hash was there already (the
    // device keeps a key's first segment: a declaration of a hash another connection entered since
    // the candidate's lookup, xcodec_memcache.cpp) -- then the mirror holds what it held, or, for two
    // enters in one batch, whichever the device took
    void entered(uint64_t h, const uint8_t *seg)
    {
        if (pre.count(h)) return;
        seen.erase(h);
        if (inpass.emplace(h, 1).second) {
            known[h] = replay::fingerprint(seg);
            // where the store's lookup finds these bytes now (the settle after the enter then reads
            // and fingerprints nothing)
            const uint8_t *p = nullptr;
            replay::Loc l{0, 0};
            uint64_t id[2] = {0, 0};
            if (st.peek(h, &p, &l, id) == replay::FOUND && id[0] && p && st.in_memory(p) &&
                std::memcmp(p, seg, replay::SEG) == 0)
                seen[h] = Seen{{id[0], id[1]}, {0, 0}};
            return;
        }
        uint8_t b[replay::SEG];
        int found = 0;
        if (!err && (err = xc__cache_read(cache, h, b, &found)) == XC_OK && found) known[h] = replay::fingerprint(b);
    }
    int before_mirror(const replay::Change &) { return XC_OK; }
    void mirrored(const replay::Change &) {}
    // where the mirror's bytes of a hash were last seen in the store (peek's id): unchanged there,
    // the mirror still holds them (xc_replay.h settle)
    // (a hash in seen is in known: both are set together, seen is erased first)
    // Two ids per hash: where the bytes were last seen, and (a full store of their stripe since) the
    // file's id of the same bytes -- the slot keeps them after the store, the file after the slot
    // takes another stripe, and both name them.
    struct Seen {
        uint64_t a[2], b[2];
    };
    replay::FlatMap<Seen> seen;
    bool same_bytes(uint64_t h, const uint64_t *id) const
    {
        auto it = seen.find(h);
        if (it == seen.end()) return false;
        const Seen &v = it->second;
        return (v.a[0] == id[0] && v.a[1] == id[1]) || (v.b[0] && v.b[0] == id[0] && v.b[1] == id[1]);
    }
    void note_bytes(uint64_t h, const uint64_t *id)
    {
        if (id && id[0]) seen[h] = Seen{{id[0], id[1]}, {0, 0}};
        else seen.erase(h);
    }
    // the mirror's bytes of m.h, seen under id m.from, are those under m.to too (a full stripe store)
    void move_id(const replay::IdMove &m)
    {
        // (an id never names other bytes later: versions are stamps, never reused)
        if (!same_bytes(m.h, m.from)) return;
        Seen &v = seen.find(m.h)->second;
        v.b[0] = m.to[0];
        v.b[1] = m.to[1];
    }
    int begin_pass(const std::vector<uint64_t> &hs, uint64_t count0)
    {
        pre.clear();
        inpass.clear();
        std::vector<uint64_t> q(hs);
        std::sort(q.begin(), q.end());
        q.erase(std::unique(q.begin(), q.end()), q.end());
        if (q.empty()) return XC_OK;
        std::vector<uint64_t> v(q.size());
        int rc = xc__cache_find(cache, q.data(), q.size(), v.data());
        for (size_t i = 0; i < q.size() && !rc; i++)
            if (v[i] != ~0ull && v[i] < count0) pre.emplace(q[i], 1);
        return rc;
    }
    int end_pass() { return err; }
    // (lookups that miss after loading a stripe are replayed from the host's window hashes:
    // xc_replay.h add_load_miss_lookups)
    int unmirrorable() { return err; }
};

namespace {
using coss::SEG;
using coss::Store;
using replay::follow;
using replay::Touch;
}  // namespace

extern "C" int xc_coss_open(xc_ctx *ctx, const char *dir, const char *uuid, uint64_t size_mb, xc_coss **out)
{
    if (!dir || !uuid || !out || strlen(uuid) < 36) return xc__set_error(XC_EINVAL, "null or short uuid");
    try {
        std::string path(dir);
        if (!path.empty() && path.back() != '/') path += '/';
        path.append(uuid, 36);
        path += ".wpc";
        xc_coss *c = new xc_coss();
        int rc = c->st.open(path, size_mb);
        if (rc) {
            delete c;
            return xc__set_error(rc, "cannot open the COSS cache file");
        }
        c->ctx = ctx;
        if (ctx) {
            Touch t;
            c->st.all_hashes(t.hs);
            if (!(rc = xc_cache_create(ctx, std::max<uint64_t>(4096, t.hs.size() + t.hs.size() / 4), &c->cache)))
                xc__cache_untracked(c->cache);  // (the Store replays every lookup, its window included)
            if (rc || (rc = follow(c, t))) {
                c->st.close();
                if (c->cache) xc_cache_destroy(c->cache);
                delete c;
                return rc;
            }
        }
        *out = c;
        return XC_OK;
    } catch (const std::bad_alloc &) {
        return xc__set_error(XC_ENOMEM, "host allocation failed");
    }
}

extern "C" int xc_coss_close(xc_coss *c)
{
    if (!c) return XC_OK;
    c->st.close();
    if (c->cache) xc_cache_destroy(c->cache);
    delete c;
    return XC_OK;
}

extern "C" xc_cache *xc_coss_cache(xc_coss *c) { return c ? c->cache : nullptr; }

extern "C" int xc_coss_count(xc_coss *c, uint64_t *n)
{
    if (!c || !n) return xc__set_error(XC_EINVAL, "null");
    *n = c->st.size();
    return XC_OK;
}

// (tests) replay::WindowHash: out[i] = the hash of the window d[i .. i + 2047], i < n - 2047.
extern "C" int xc__window_hashes_host(const uint8_t *d, uint64_t n, uint64_t *out)
{
    if (!d || !out) return xc__set_error(XC_EINVAL, "null");
    replay::WindowHash w(d);
    for (uint64_t p = 0; p < n; p++) {
        w.push();
        if (p >= SEG - 1) out[p - (SEG - 1)] = w.mix();
    }
    return XC_OK;
}

// (tests) Store::reread_headers, and the device mirror follows.
extern "C" int xc__coss_reread_headers(xc_coss *c)
{
    if (!c) return xc__set_error(XC_EINVAL, "null");
    try {
        Touch t;
        if (!c->st.reread_headers(&t)) return xc__set_error(XC_EDEVICE, "COSS: cannot read the cache file");
        return follow(c, t);
    } catch (const std::bad_alloc &) {
        return xc__set_error(XC_ENOMEM, "host allocation failed");
    }
}

extern "C" int xc_coss_stats(xc_coss *c, uint64_t *out6)
{
    if (!c || !out6) return xc__set_error(XC_EINVAL, "null");
    c->st.stats(out6);
    return XC_OK;
}

extern "C" int xc_coss_lookup(xc_coss *c, uint64_t h, uint8_t *out, int *found)
{
    if (!c || !out || !found) return xc__set_error(XC_EINVAL, "null");
    try {
        Touch t;
        const uint8_t *d = c->st.lookup(h, &t);
        *found = d ? 1 : 0;
        if (d && !c->st.copy_bytes(d, out)) return xc__set_error(XC_EDEVICE, "COSS: cannot read the cache file");
        return follow(c, t);
    } catch (const std::bad_alloc &) {
        return xc__set_error(XC_ENOMEM, "host allocation failed");
    }
}

extern "C" int xc_coss_enter(xc_coss *c, uint64_t h, const uint8_t *seg)
{
    if (!c || !seg) return xc__set_error(XC_EINVAL, "null");
    try {
        Touch t;
        c->st.enter(h, seg, &t);
        return follow(c, t);
    } catch (const std::bad_alloc &) {
        return xc__set_error(XC_ENOMEM, "host allocation failed");
    }
}

// Encoder batch over the COSS cache: buffer i is one encode()+flush() on a fresh encoder, buffers
// in index order (xc_encode_batch_host's semantics), the COSS state advanced exactly as the
// reference's would be.
extern "C" int xc_coss_encode_batch_host(xc_coss *c, const uint8_t *in, const uint64_t *in_off,
                                         const uint64_t *in_len, uint64_t nbuf, uint8_t *out,
                                         const uint64_t *out_off, const uint64_t *out_cap, uint64_t *out_len)
{
    if (!c || !c->cache || (nbuf && (!in || !in_off || !in_len || !out || !out_off || !out_cap || !out_len)))
        return xc__set_error(XC_EINVAL, "null (or a host-only COSS store)");
    try {
        std::vector<replay::CItem> items;
        for (uint64_t i = 0; i < nbuf; i++) {
            items.push_back({i, in + in_off[i], in_len[i], 0, -1, 0, false});
            out_len[i] = 0;
        }
        std::vector<uint64_t> rb(nbuf);
        std::vector<int64_t> rc(nbuf);
        return replay::encode(c, std::move(items), out, out_off, out_cap, out_len, rb.data(), rc.data());
    } catch (const std::bad_alloc &) {
        return xc__set_error(XC_ENOMEM, "host allocation failed");
    }
}

// Internal (xc_stream.cpp, xc_coss_encode_streams): xc__encode_gather's contract over the COSS
// cache: item i is head[i] (an encoder's source_) then tail[i] (its new input), with stream state
// start / cand / flags (SF_NOFLUSH: encode() only); `take` receives each item's output and input
// after rbase / rcand are set.
template <class C>
static int replay_gather(C *c, uint64_t nbuf, const uint8_t *const *head, const uint64_t *head_len,
                         const uint8_t *const *tail, const uint64_t *tail_len, const uint64_t *start,
                         const int64_t *cand, const uint32_t *flags, uint64_t *rbase, int64_t *rcand,
                         int (*take)(void *ctx, uint64_t i, const uint8_t *out, uint64_t out_len, const uint8_t *in),
                         void *ctx)
{
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
        if (start[i] > data[i].size() || cand[i] < -1 ||
            (cand[i] >= 0 && ((uint64_t)cand[i] + SEG > start[i] || (uint64_t)cand[i] + 2 * SEG - 1 < start[i])))
            return xc__set_error(XC_EINVAL, "invalid stream state");
        items.push_back({i, data[i].data(), data[i].size(), start[i], cand[i], 0, (flags[i] & 1u) != 0});
    }
    static thread_local replay::Scratch s_out;  // (grow-only, not zeroed)
    uint8_t *const obuf = s_out.get(osz);
    int rc = replay::encode(c, std::move(items), obuf, ooff.data(), ocap.data(), olen.data(), rbase, rcand);
    for (uint64_t i = 0; i < nbuf && !rc; i++) rc = take(ctx, i, obuf + ooff[i], olen[i], data[i].data());
    return rc;
}

extern "C" int xc__coss_encode_gather(xc_coss *c, uint64_t nbuf, const uint8_t *const *head, const uint64_t *head_len,
                                      const uint8_t *const *tail, const uint64_t *tail_len, const uint64_t *start,
                                      const int64_t *cand, const uint32_t *flags, uint64_t *rbase, int64_t *rcand,
                                      int (*take)(void *ctx, uint64_t i, const uint8_t *out, uint64_t out_len,
                                                  const uint8_t *in),
                                      void *ctx)
{
    if (!c || !c->cache || (nbuf && (!head || !head_len || !tail || !tail_len || !start || !cand || !flags || !rbase ||
                                     !rcand || !take)))
        return xc__set_error(XC_EINVAL, "null (or a host-only COSS store)");
    try {
        return replay_gather(c, nbuf, head, head_len, tail, tail_len, start, cand, flags, rbase, rcand, take, ctx);
    } catch (const std::bad_alloc &) {
        return xc__set_error(XC_ENOMEM, "host allocation failed");
    }
}

// Decoder batch over the COSS cache: stream i is one decode() call, streams in index order
// (xc_decode_batch_host's semantics), the COSS state advanced as the reference's would be.
extern "C" int xc_coss_decode_batch_host(xc_coss *c, const uint8_t *in, const uint64_t *in_off,
                                         const uint64_t *in_len, uint64_t nbuf, uint8_t *out,
                                         const uint64_t *out_off, const uint64_t *out_cap, uint64_t *out_len,
                                         uint64_t *consumed, int32_t *status, uint64_t *unknown,
                                         int32_t *has_unknown)
{
    if (!c || !c->cache || (nbuf && (!in || !in_off || !in_len || !out || !out_off || !out_cap || !out_len ||
                                     !consumed || !status || !unknown || !has_unknown)))
        return xc__set_error(XC_EINVAL, "null (or a host-only COSS store)");
    try {
        return replay::decode(c, in, in_off, in_len, nbuf, out, out_off, out_cap, out_len, consumed, status, unknown,
                              has_unknown);
    } catch (const std::bad_alloc &) {
        return xc__set_error(XC_ENOMEM, "host allocation failed");
    }
}

// Host-only store operations (tests of the Store on its own, no device).
extern "C" int xc_coss_store_lookup(xc_coss *c, uint64_t h, uint8_t *out, int *found)
{
    if (!c || !out || !found) return xc__set_error(XC_EINVAL, "null");
    const uint8_t *d = c->st.lookup(h, nullptr);
    *found = d ? 1 : 0;
    if (d && !c->st.copy_bytes(d, out)) return xc__set_error(XC_EDEVICE, "COSS: cannot read the cache file");
    return XC_OK;
}
extern "C" int xc_coss_store_enter(xc_coss *c, uint64_t h, const uint8_t *seg)
{
    if (!c || !seg) return xc__set_error(XC_EINVAL, "null");
    c->st.enter(h, seg, nullptr);
    return XC_OK;
}
