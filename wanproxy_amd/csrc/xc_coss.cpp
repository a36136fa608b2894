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
#include <cstring>
#include <memory>
#include <new>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "../../include/xcodec_hip.h"

extern "C" int xc__set_error(int code, const char *msg);
extern "C" int xc__encode_batch_host_coll(xc_cache *c, const uint8_t *in, const uint64_t *in_off,
                                          const uint64_t *in_len, uint64_t nbuf, uint8_t *out,
                                          const uint64_t *out_off, const uint64_t *out_cap, uint64_t *out_len,
                                          const uint64_t *start, const int64_t *cand, const uint32_t *flags,
                                          uint64_t *rbase, int64_t *rcand, uint32_t *coll_cnt, uint32_t *coll);
extern "C" int xc__cache_truncate(xc_cache *c, uint64_t keep);
extern "C" int xc__cache_kill(xc_cache *c, const uint64_t *h, uint64_t n);
extern "C" int xc__cache_enter_bulk(xc_cache *c, const uint64_t *h, const uint8_t *segs, uint64_t n);

namespace coss {

constexpr uint32_t SEG = XC_SEGMENT_LENGTH;
constexpr uint32_t SIGNATURE = 0xF150E964u;  // xcodec_cache_coss.h:83
constexpr uint32_t VERSION = 2;              // :84
constexpr uint32_t STRIPE_SEGS = 512;        // :85
constexpr int LOADED = 16;                   // :86
constexpr uint64_t BASIC_MB = 1024;          // :87
constexpr int WINDOW = 64;                   // xcodec_cache.h:48
constexpr uint32_t COLL_CAP = 16;            // xc_kernels.h

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

struct Loc {
    uint64_t range;
    uint32_t pos;
};

// What a Store operation touched: the hashes and stripe ranges whose lookup result may have
// changed, and the slots whose bytes were replaced (recent-window entries point into them).
struct Touch {
    std::vector<uint64_t> hs, ranges;
    std::vector<int> slots;
};

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
        dir_.assign(limit_, Meta{});
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
        for (int i = 0; i < WINDOW; i++)  // find_recent (xcodec_cache.h:137-147): the first match
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
            detach_stripe(s, t);
            load_stripe(e.range, s, t);
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
        win_[cursor_].hash = h;
        win_[cursor_].data = d;
        cursor_ = (cursor_ + 1) & (WINDOW - 1);
        found_2_++;
        return d;
    }

    // What lookup(h) returns now, without its side effects: FOUND (*p: the bytes), IN_FILE (the
    // stripe is loaded from the file first, *l: where the bytes are), ABSENT, or LOAD_MISS (not
    // found, after loading a stripe: a miss with side effects).
    enum { ABSENT, FOUND, IN_FILE, LOAD_MISS };
    int peek(uint64_t h, const uint8_t **p, Loc *l) const
    {
        for (int i = 0; i < WINDOW; i++)
            if (win_[i].hash == h) {
                if (win_[i].data) {
                    *p = win_[i].data;
                    return FOUND;
                }
                break;
            }
        auto it = index_.find(h);
        if (it == index_.end()) return ABSENT;
        const Loc e = it->second;
        const int s = first_slot(e.range);
        if (s < LOADED) {
            if (slot_[s].h.hash[e.pos] != h) return ABSENT;
            *p = slot_[s].seg[e.pos];
            return FOUND;
        }
        *l = e;
        if (e.range * sizeof(Stripe) >= file_size_) return LOAD_MISS;
        return file_hash_[e.range * STRIPE_SEGS + e.pos] == h ? IN_FILE : LOAD_MISS;
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
        for (const auto &kv : index_) out.push_back(kv.first);
    }

    size_t size() const { return index_.size(); }
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
        std::memset(&slot_[s].h, 0, sizeof(Header));
        Meta &m = slot_[s].h.m;
        m.signature = SIGNATURE;
        m.version = VERSION;
        m.serial_number = ++serial_;
        m.stripe_range = range;
        m.state = 1;
        dir_[range] = m;
    }

    bool load_stripe(uint64_t range, int s, Touch *t)
    {  // :241-260
        const uint64_t pos = range * sizeof(Stripe);
        if (pos < file_size_) {
            retarget(s, range, t);
            if (::pread(fd_, &slot_[s], sizeof(Stripe), (off_t)pos) == (ssize_t)sizeof(Stripe)) {
                slot_[s].h.m.stripe_range = range;
                slot_[s].h.m.load_uses = 0;
                slot_[s].h.m.state = 1;
                dir_[range].state = 1;
                return true;
            }
        }
        return false;
    }

    void store_stripe(int s, size_t size, Touch *t)
    {  // :262-272
        const uint64_t range = slot_[s].h.m.stripe_range, pos = range * sizeof(Stripe);
        if (::pwrite(fd_, &slot_[s], size, (off_t)pos) == (ssize_t)size) {
            if (pos + sizeof(Stripe) > file_size_) file_size_ = pos + sizeof(Stripe);
            if (range < limit_) std::memcpy(&file_hash_[range * STRIPE_SEGS], slot_[s].h.hash, sizeof slot_[s].h.hash);
            if (t) t->ranges.push_back(range);
        }
    }

    void new_active(Touch *t)
    {  // :274-283
        store_stripe(active_, sizeof(Stripe), t);
        active_ = best_unloadable_slot();
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
                        win_[w].hash = 0;
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
    int active_ = 0;
    std::vector<Meta> dir_;
    std::unordered_map<uint64_t, Loc> index_;
    std::vector<uint64_t> owner_;      // [range * 512 + pos]: the hash whose index entry is there
    std::vector<uint64_t> file_hash_;  // [range * 512 + pos]: the stripe headers as in the file
    struct {
        uint64_t hash;
        const uint8_t *data;
    } win_[WINDOW] = {};
    unsigned cursor_ = 0;
    uint64_t lookups_ = 0, found_1_ = 0, found_2_ = 0;
};

// What a Store operation did to the set of segments a lookup finds (the device mirror's contents).
struct Change {
    std::vector<uint64_t> removed;  // no longer found
    std::vector<uint64_t> added;    // found now, or found with other bytes
    std::vector<uint8_t> bytes;     // their bytes, SEG each
    bool any() const { return !removed.empty() || !added.empty(); }
};

}  // namespace coss

struct xc_coss {
    xc_ctx *ctx = nullptr;
    xc_cache *cache = nullptr;  // the device mirror (null for a host-only store)
    coss::Store st;
    // what the device cache holds: hash -> fingerprint of its bytes
    std::unordered_map<uint64_t, uint64_t> known;
    // hashes a lookup misses only after loading a stripe (a miss with side effects)
    std::unordered_set<uint64_t> load_miss;
};

namespace {
using coss::Change;
using coss::Loc;
using coss::SEG;
using coss::Store;
using coss::Touch;

uint64_t fingerprint(const uint8_t *p)
{
    uint64_t h = 0x9E3779B97F4A7C15ull;
    for (uint32_t i = 0; i < SEG; i += 8) {
        uint64_t w;
        std::memcpy(&w, p + i, 8);
        h = (h ^ w) * 0x100000001B3ull;
        h ^= h >> 29;
    }
    return h;
}

// The hashes an operation touched, looked up again without side effects: those the device holds
// and a lookup no longer finds, and those a lookup finds that the device lacks or holds with other
// bytes, go into ch (and `known` follows).
int settle(xc_coss *c, const Touch &t, Change &ch)
{
    std::vector<uint64_t> cand(t.hs);
    for (uint64_t r : t.ranges) c->st.owners(r, cand);
    for (int s : t.slots) c->st.window_in_slot(s, cand);
    std::sort(cand.begin(), cand.end());
    cand.erase(std::unique(cand.begin(), cand.end()), cand.end());
    uint8_t buf[SEG];
    for (uint64_t h : cand) {
        if (!h) continue;
        const uint8_t *p = nullptr;
        Loc l{0, 0};
        const int r = c->st.peek(h, &p, &l);
        if (r == Store::LOAD_MISS) c->load_miss.insert(h);
        else c->load_miss.erase(h);
        if (r == Store::IN_FILE) {
            if (!c->st.read_segment(l, buf)) return xc__set_error(XC_EDEVICE, "COSS: cannot read the cache file");
            p = buf;
        }
        if (r != Store::FOUND && r != Store::IN_FILE) {
            if (c->known.erase(h)) ch.removed.push_back(h);
            continue;
        }
        const uint64_t fp = fingerprint(p);
        auto it = c->known.find(h);
        if (it != c->known.end() && it->second == fp) continue;
        c->known[h] = fp;
        ch.added.push_back(h);
        ch.bytes.insert(ch.bytes.end(), p, p + SEG);
    }
    return XC_OK;
}

// The device mirror follows a change.
int mirror(xc_coss *c, const Change &ch)
{
    int rc = XC_OK;
    if (!ch.removed.empty()) rc = xc__cache_kill(c->cache, ch.removed.data(), ch.removed.size());
    if (!rc && !ch.added.empty() && !(rc = xc__cache_kill(c->cache, ch.added.data(), ch.added.size())))
        rc = xc__cache_enter_bulk(c->cache, ch.added.data(), ch.bytes.data(), ch.added.size());
    return rc;
}

// A store operation on a device-backed COSS cache: the device follows at once.
int follow(xc_coss *c, const Touch &t)
{
    if (!c->cache) return XC_OK;
    Change ch;
    int rc = settle(c, t, ch);
    return rc ? rc : (ch.any() ? mirror(c, ch) : XC_OK);
}

// Later events of a batch that saw a change: any lookup of a hash it added or removed.
struct Watch {
    std::unordered_set<uint64_t> hs;
    explicit Watch(const Change &ch) : hs(ch.removed.begin(), ch.removed.end())
    {
        hs.insert(ch.added.begin(), ch.added.end());
    }
    bool has(uint64_t h) const { return hs.count(h) != 0; }
};

int unmirrorable(xc_coss *c)
{
    if (c->load_miss.empty()) return XC_OK;
    return xc__set_error(XC_EINVAL, "COSS: a stripe header in the file disagrees with the index (a cache of "
                                    "16 stripes or fewer after a stripe's second copy was detached); "
                                    "lookups that miss after loading a stripe are not mirrored on the device");
}

// One cache event of an encoder item, in the reference's order (xcodec_encoder.cc:72-171).
struct EncEvent {
    uint64_t pos;       // window end of the lookup / declaration point (~0: flush's declaration)
    int kind;           // 0 enter (EXTRACT), 1 lookup hit (REF), 2 lookup hit (collision)
    uint64_t hash;
    uint64_t out_end;   // output bytes up to the end of this event's token (0 for a collision)
    uint64_t base;      // source_ start after the event (REF / EXTRACT), or at it (collision)
    int64_t cand;       // collision: the pending candidate (-1 none)
    const uint8_t *seg; // EXTRACT payload
};

int64_t get_be64(const uint8_t *p)
{
    uint64_t v = 0;
    for (int i = 0; i < 8; i++) v = (v << 8) | p[i];
    return (int64_t)v;
}

// The encoder's lookup calls (xcodec_encoder.cc:111) at window ends [lo, hi) of an item, whose REF
// events are ev[0..n): every window end once the window is full, except the 2047 after a REF (the
// hash restarts, :117-127).  Minus its hits (the replay's Store::lookup counted those): its misses.
uint64_t enc_misses(uint64_t lo, uint64_t hi, const std::vector<EncEvent> &ev, size_t n)
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
            if ((rc = xc_cache_create(ctx, std::max<uint64_t>(4096, t.hs.size() + t.hs.size() / 4), &c->cache)) ||
                (rc = follow(c, t))) {
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
        if (d) std::memcpy(out, d, SEG);
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

namespace {
// An encoder batch item over the COSS cache: `data` (len bytes) is an encoder's pending source_
// followed by its new input, window ends below `start` already looked up, candidate `cand` (or -1),
// encode() only when `noflush`.  `off`: where data lies in the caller's item (restarts move it).
struct CItem {
    uint64_t buf;
    const uint8_t *data;
    uint64_t len, start;
    int64_t cand;
    uint64_t off;
    bool noflush;
};

// The batch on the device, its cache events replayed into the Store in the reference's order
// (items in order), restarting the rest after a change a later event depends on.  Outputs append
// at out + out_off[buf]; res_base / res_cand: the new source_ start and candidate of each buffer,
// relative to its first item's data.
int coss_encode(xc_coss *c, std::vector<CItem> items, uint8_t *out, const uint64_t *out_off, const uint64_t *out_cap,
                uint64_t *out_len, uint64_t *res_base, int64_t *res_cand)
{
    {
        {
        while (!items.empty()) {
            const uint64_t m = items.size();
            uint64_t count0 = 0;
            int rc = xc_cache_count(c->cache, &count0);
            if (rc) return rc;
            // the device batch
            std::vector<uint64_t> ioff(m), ilen(m), start(m), ooff(m), ocap(m), olen(m), rbase(m);
            std::vector<int64_t> cand(m), rcand(m);
            std::vector<uint32_t> fl(m, 0u), ccnt(m);
            for (uint64_t k = 0; k < m; k++) fl[k] = items[k].noflush ? 1u : 0u;  // (SF_NOFLUSH)
            std::vector<uint32_t> coll(m * coss::COLL_CAP * 4);
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
            std::vector<uint8_t> arena(std::max<uint64_t>(isz, 1)), obuf(std::max<uint64_t>(osz, 1));
            for (uint64_t k = 0; k < m; k++)
                if (items[k].len) std::memcpy(&arena[ioff[k]], items[k].data, items[k].len);
            rc = xc__encode_batch_host_coll(c->cache, arena.data(), ioff.data(), ilen.data(), m, obuf.data(), ooff.data(),
                                            ocap.data(), olen.data(), start.data(), cand.data(), fl.data(), rbase.data(),
                                            rcand.data(), ccnt.data(), coll.data());
            if (rc) return rc;
            // the batch's cache events, item by item in the reference's order
            std::vector<std::vector<EncEvent>> ev(m);
            std::vector<const uint8_t *> payloads;
            for (uint64_t k = 0; k < m; k++) {
                if (ccnt[k] > coss::COLL_CAP)
                    return xc__set_error(XC_EINVAL, "too many hash collisions in one buffer to replay on COSS");
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
                    const uint32_t *r = &coll[(k * coss::COLL_CAP + i) * 4];
                    const uint64_t q = r[0];
                    // source_ start at q: after the last token before it
                    uint64_t base = 0, oe = 0;
                    for (const EncEvent &e : ev[k])
                        if (e.kind != 2 && e.pos <= q) base = e.base, oe = e.out_end;
                    ev[k].push_back({q, 2, ((uint64_t)r[2] << 32) | r[1], oe, base,
                                     r[3] == 0xFFFFFFFFu ? -1 : (int64_t)r[3], nullptr});
                }
                // (a declaration precedes the lookup at the same position; flush's comes last)
                std::stable_sort(ev[k].begin(), ev[k].end(), [](const EncEvent &a, const EncEvent &b) {
                    return a.pos != b.pos ? a.pos < b.pos : a.kind < b.kind;
                });
            }
            // EXTRACT hashes (XCodecHash::hash of the payloads) on the device, one call
            std::vector<uint64_t> ph(payloads.size());
            if (!payloads.empty()) {
                std::vector<uint8_t> segs(payloads.size() * (size_t)SEG);
                for (size_t i = 0; i < payloads.size(); i++) std::memcpy(&segs[i * SEG], payloads[i], SEG);
                if ((rc = xc_hash_segments_host(c->ctx, segs.data(), payloads.size(), ph.data()))) return rc;
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
            // replay; stop at the first change a later event depends on
            if ((rc = unmirrorable(c))) return rc;
            uint64_t entered = 0;
            bool redo = false;
            std::vector<CItem> next;
            std::vector<Change> held;  // changes nothing later in the pass saw: mirrored at its end
            for (uint64_t k = 0; k < m && !redo; k++) {
                const CItem &it = items[k];
                for (size_t e = 0; e < ev[k].size(); e++) {
                    const EncEvent &E = ev[k][e];
                    Touch t;
                    if (E.kind == 0) {
                        c->st.enter(E.hash, E.seg, &t);
                        c->known[E.hash] = fingerprint(E.seg);  // (the device entered it)
                        entered++;
                    } else if (!c->st.lookup(E.hash, &t)) {
                        return xc__set_error(XC_EDEVICE, "COSS replay: a device hit the store does not find");
                    }
                    Change ch;
                    if ((rc = settle(c, t, ch))) return rc;
                    if (!ch.any()) continue;
                    // a segment found now that was not: any lookup after this event may differ
                    bool dep = !ch.added.empty();
                    if (!dep) {
                        const Watch w(ch);
                        for (uint64_t k2 = k; k2 < m && !dep; k2++)
                            for (size_t e2 = (k2 == k ? e + 1 : 0); e2 < ev[k2].size() && !dep; e2++)
                                dep = w.has(ev[k2][e2].hash);
                    }
                    if (!dep) {
                        held.push_back(std::move(ch));
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
                        } else {  // after a collision: same source_, candidate carried
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
            for (const Change &h : held)
                if ((rc = mirror(c, h))) return rc;
            items.swap(next);
        }
        }
    }
    return XC_OK;
}
}  // namespace

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
        std::vector<CItem> items;
        for (uint64_t i = 0; i < nbuf; i++) {
            items.push_back({i, in + in_off[i], in_len[i], 0, -1, 0, false});
            out_len[i] = 0;
        }
        std::vector<uint64_t> rb(nbuf);
        std::vector<int64_t> rc(nbuf);
        return coss_encode(c, std::move(items), out, out_off, out_cap, out_len, rb.data(), rc.data());
    } catch (const std::bad_alloc &) {
        return xc__set_error(XC_ENOMEM, "host allocation failed");
    }
}

// Internal (xc_stream.cpp, xc_coss_encode_streams): xc__encode_gather's contract over the COSS
// cache: item i is head[i] (an encoder's source_) then tail[i] (its new input), with stream state
// start / cand / flags (SF_NOFLUSH: encode() only); `take` receives each item's output and input
// after rbase / rcand are set.
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
        std::vector<std::vector<uint8_t>> data(nbuf);
        std::vector<uint64_t> ooff(nbuf), ocap(nbuf), olen(nbuf, 0);
        std::vector<CItem> items;
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
        std::vector<uint8_t> obuf(std::max<uint64_t>(osz, 1));
        int rc = coss_encode(c, std::move(items), obuf.data(), ooff.data(), ocap.data(), olen.data(), rbase, rcand);
        for (uint64_t i = 0; i < nbuf && !rc; i++) rc = take(ctx, i, obuf.data() + ooff[i], olen[i], data[i].data());
        return rc;
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
            int rc = xc_cache_count(c->cache, &count0);
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
            std::vector<uint8_t> obuf(std::max<uint64_t>(osz, 1));
            rc = xc_decode_batch_host(c->cache, in, ioff.data(), ilen.data(), m, obuf.data(), ooff.data(), ocap.data(),
                                      olen.data(), cons.data(), st.data(), unk.data(), hu.data());
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
                std::vector<uint8_t> segs(payloads.size() * (size_t)SEG);
                for (size_t i = 0; i < payloads.size(); i++) std::memcpy(&segs[i * SEG], payloads[i], SEG);
                if ((rc = xc_hash_segments_host(c->ctx, segs.data(), payloads.size(), ph.data()))) return rc;
                size_t pi = 0;
                for (auto &v : ev)
                    for (DEv &e : v)
                        if (e.kind == 0) e.hash = ph[pi++];
            }
            if ((rc = unmirrorable(c))) return rc;
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
                        c->known[E.hash] = fingerprint(E.seg);  // (the device entered it)
                        entered++;
                    } else if (E.kind == 1 && !d) {
                        return xc__set_error(XC_EDEVICE, "COSS replay: a device hit the store does not find");
                    }
                    Change ch;
                    if ((rc = settle(c, t, ch))) return rc;
                    if (!ch.any()) continue;
                    // later tokens, and the unknown REF a later stream stopped on, that saw the change
                    const Watch w(ch);
                    bool dep = false;
                    for (uint64_t k2 = k; k2 < m && !dep; k2++) {
                        for (size_t e2 = (k2 == k ? e + 1 : 0); e2 < ev[k2].size() && !dep; e2++)
                            dep = w.has(ev[k2][e2].hash);
                        if (hu[k2] && w.has(unk[k2])) dep = true;
                    }
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
                    if (hu[k]) c->st.count_misses(1);  // (the unknown REF's lookup, :150)
                    std::memcpy(out + out_off[it.buf] + out_len[it.buf], &obuf[ooff[k]], olen[k]);
                    out_len[it.buf] += olen[k];
                    consumed[it.buf] = it.from + cons[k];
                    status[it.buf] = st[k];
                    unknown[it.buf] = unk[k];
                    has_unknown[it.buf] = hu[k];
                }
            }
            for (const Change &h : held)
                if ((rc = mirror(c, h))) return rc;
            items.swap(next);
        }
        return XC_OK;
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
    if (d) std::memcpy(out, d, SEG);
    return XC_OK;
}
extern "C" int xc_coss_store_enter(xc_coss *c, uint64_t h, const uint8_t *seg)
{
    if (!c || !seg) return xc__set_error(XC_EINVAL, "null");
    c->st.enter(h, seg, nullptr);
    return XC_OK;
}
