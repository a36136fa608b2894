// xc_stream.cpp — stateful XCodec stream encoders over the batch encoder (host side).
//
// Reference: XCodecEncoder (xcodec/xcodec_encoder.h:43-63, xcodec/xcodec_encoder.cc:43-201) as
// EncodeFilter drives it (xcodec/xcodec_filter.cc:122-164): one encoder per connection, called
// once per received buffer, flushed unless the caller marks the data TO_BE_CONTINUED.  Between
// calls an encoder holds exactly its pending `source_` bytes and its candidate
// (candidate_start_; candidate_symbol_ is the hash of the candidate's bytes), so that is the
// state kept here.  A call becomes one buffer of a device batch: source_ followed by the new
// input, with the window ends of source_ marked as already looked up (xc_plan_set_streams).
//
// Cross-connection batching: xc_encode_streams runs the calls of many encoders as one batch,
// with the reference's single-threaded order (call k sees the cache after calls < k).  A batch
// round holds each encoder at most once; a later call of the same encoder starts a new round.
#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <new>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/xcodec_hip.h"

extern "C" int xc__set_error(int code, const char *msg);
extern "C" int xc__encode_gather(xc_cache *c, uint64_t nbuf, const uint8_t *const *head, const uint64_t *head_len,
                                 const uint8_t *const *tail, const uint64_t *tail_len, const uint64_t *start,
                                 const int64_t *cand, const uint32_t *flags, uint64_t *rbase, int64_t *rcand,
                                 int (*take)(void *ctx, uint64_t i, const uint8_t *out, uint64_t out_len,
                                             const uint8_t *in),
                                 void *ctx);

extern "C" int xc__coss_encode_gather(xc_coss *c, uint64_t nbuf, const uint8_t *const *head,
                                      const uint64_t *head_len, const uint8_t *const *tail, const uint64_t *tail_len,
                                      const uint64_t *start, const int64_t *cand, const uint32_t *flags,
                                      uint64_t *rbase, int64_t *rcand,
                                      int (*take)(void *ctx, uint64_t i, const uint8_t *out, uint64_t out_len,
                                                  const uint8_t *in),
                                      void *ctx);

namespace {
constexpr uint64_t MAX_BUFFER = 1u << 20;  // longest device batch item (xc_kernels.h MAX_BUF)
constexpr uint32_t SF_NOFLUSH = 1u;        // xc_kernels.h
std::atomic<uint64_t> g_placed{0};  // caches placed round-robin so far (xc_device_place)
}  // namespace

// Where a proxy's caches go (include/xcodec_hip.h): WanProxyCore::add_cache constructs every cache
// with two arguments (proxy/wanproxy.h:106-116) and a cache's calls are sequential by contract
// (one cache = one stream of codec calls in the reference's order), so the unit of placement is the
// cache: a codec's encoder cache and each peer's decoder cache each live on one device.
extern "C" int xc_device_place(const uint8_t *key, uint64_t key_len, int ndev)
{
    if (ndev < 1) return xc__set_error(XC_EINVAL, "no device to place a cache on");
    std::vector<int> devs;
    if (const char *e = std::getenv("XC_DEVICE"); e && *e) {
        for (const char *p = e; *p;) {
            char *end = nullptr;
            const long d = std::strtol(p, &end, 10);
            if (end == p || d < 0 || d >= ndev) return xc__set_error(XC_EINVAL, "XC_DEVICE names no visible device");
            devs.push_back((int)d);
            p = *end == ',' ? end + 1 : end;
            if (*end && *end != ',') return xc__set_error(XC_EINVAL, "XC_DEVICE: a device index or a comma list");
        }
    } else {
        for (int d = 0; d < ndev; d++) devs.push_back(d);
    }
    const char *pol = std::getenv("XC_DEVICE_POLICY");
    if (pol && std::strcmp(pol, "uuid") == 0) {
        if (!key && key_len) return xc__set_error(XC_EINVAL, "null key");
        uint64_t h = 1469598103934665603ull;  // FNV-1a 64
        for (uint64_t i = 0; i < key_len; i++) h = (h ^ key[i]) * 1099511628211ull;
        return devs[(size_t)(h % devs.size())];
    }
    return devs[(size_t)(g_placed.fetch_add(1) % devs.size())];
}

struct xc_encoder {
    xc_cache *cache;
    std::vector<uint8_t> source;  // source_ (bytes not yet emitted)
    int64_t cand = -1;            // candidate_start_, relative to source[0]
};

extern "C" int xc_encoder_create(xc_cache *c, xc_encoder **out)
{
    if (!c || !out) return xc__set_error(XC_EINVAL, "null");
    *out = new xc_encoder{c, {}, -1};
    return XC_OK;
}

extern "C" int xc_encoder_destroy(xc_encoder *e)
{
    delete e;
    return XC_OK;
}

extern "C" int xc_encoder_pending(xc_encoder *e, uint64_t *bytes)
{
    if (!e || !bytes) return xc__set_error(XC_EINVAL, "null");
    *bytes = e->source.size();
    return XC_OK;
}

namespace {
// One round: calls [i, j) of the request, each encoder once; the last call may be a prefix of
// its input (`take` bytes from `done`), which then keeps its flush for a later round.
struct Item {
    uint64_t call, from, take;
    bool flush;
};
}  // namespace

// XCodecHash::hash of one 2048-byte segment (xcodec/xcodec_hash.h:166-174: the window sums of byte + 1
// and of ffs(byte), weights 2048 - j, mixed with the uint32 shifts of :155-164).
static uint64_t segment_hash(const uint8_t *p)
{
    uint32_t s1w = 0, s2w = 0, s1f = 0, s2f = 0;
    for (uint32_t j = 0; j < XC_SEGMENT_LENGTH; j++) {
        const uint32_t w = p[j] + 1u, f = p[j] ? (uint32_t)__builtin_ctz(p[j]) + 1u : 0u;
        s1w += w;
        s2w += (XC_SEGMENT_LENGTH - j) * w;
        s1f += f;
        s2f += (XC_SEGMENT_LENGTH - j) * f;
    }
    const uint32_t bits = (s1f << 16) + s2f, bytes = (s1w << 20) + s2w;
    return ((uint64_t)bits << 36) + bytes;
}

// encode_escape (xcodec_encoder.cc:217-239): bytes with F1 -> F1 00, appended at o.
static uint64_t escape(uint8_t *o, const uint8_t *p, uint64_t n)
{
    uint64_t k = 0;
    for (uint64_t i = 0; i < n; i++) {
        o[k++] = p[i];
        if (p[i] == 0xF1) o[k++] = 0x00;
    }
    return k;
}

// XCodecEncoder::flush (xcodec_encoder.cc:175-201) of an encoder over a memory cache, on the host: it
// looks nothing up, so it needs no device batch -- the pending candidate declared (its bytes escaped
// before it, F1 01 + the 2048 bytes, cache_->enter: xc_cache_enter, with the memory cache's release
// semantics for a hash already entered), the rest of source_ escaped.  A proxy's EncodeFilter calls
// it after every consume's encode (xcodec_filter.cc:146-157): one device call per consume, not two.
static int host_flush(xc_encoder *e, uint8_t *out, uint64_t *out_len)
{
    const uint8_t *s = e->source.data();
    const uint64_t n = e->source.size();
    uint64_t k = 0, at = 0;
    if (e->cand >= 0) {
        const uint64_t c = (uint64_t)e->cand;
        if (c + XC_SEGMENT_LENGTH > n) return xc__set_error(XC_EDEVICE, "inconsistent stream state");
        k += escape(out + k, s, c);
        out[k++] = 0xF1;
        out[k++] = 0x01;
        std::memcpy(out + k, s + c, XC_SEGMENT_LENGTH);
        k += XC_SEGMENT_LENGTH;
        if (int rc = xc_cache_enter(e->cache, segment_hash(s + c), s + c)) return rc;
        at = c + XC_SEGMENT_LENGTH;
    }
    k += escape(out + k, s + at, n - at);
    *out_len += k;
    e->source.clear();
    e->cand = -1;
    return XC_OK;
}

// coss: the encoders' cache is that COSS cache's device mirror, and the batches run through the
// COSS replay (xc__coss_encode_gather); else the memory cache (xc__encode_gather).
static int encode_streams(xc_coss *coss, xc_encoder *const *enc, const uint8_t *const *in, const uint64_t *in_len,
                          const uint32_t *flags, uint64_t n, uint8_t *out, const uint64_t *out_off,
                          const uint64_t *out_cap, uint64_t *out_len)
{
    if (n && (!enc || !in_len || !out || !out_off || !out_cap || !out_len)) return xc__set_error(XC_EINVAL, "null");
    xc_cache *cache = coss ? xc_coss_cache(coss) : n ? enc[0]->cache : nullptr;
    for (uint64_t k = 0; k < n; k++) {
        if (!enc[k]) return xc__set_error(XC_EINVAL, "null encoder");
        if (enc[k]->cache != cache)
            return xc__set_error(XC_EINVAL, coss ? "encoder not created on this COSS cache (xc_coss_cache)"
                                                 : "encoders of one call must share a cache");
        if (in_len[k] && (!in || !in[k])) return xc__set_error(XC_EINVAL, "null input");
        out_len[k] = 0;
    }
    // Every output capacity is checked before anything runs, so that an argument error leaves the
    // encoders and the cache as they were.  A call emits at most 2 bytes per byte it takes from
    // source_ and its input (escaped F1 literals; EXTRACT 2050 per 2048, REF 10), and source_ at
    // the call holds at most the encoder's pending bytes plus its earlier inputs of this request.
    {
        std::vector<std::pair<const xc_encoder *, uint64_t>> pend;
        for (uint64_t k = 0; k < n; k++) {
            auto it = std::find_if(pend.begin(), pend.end(), [&](const auto &x) { return x.first == enc[k]; });
            if (it == pend.end()) it = pend.insert(pend.end(), {enc[k], enc[k]->source.size()});
            it->second += in_len[k];
            if (out_cap[k] < 2 * it->second) return xc__set_error(XC_EINVAL, "output capacity too small");
        }
    }
    std::vector<uint64_t> done(n, 0);  // input bytes of call k consumed so far
    uint64_t k0 = 0;
    while (k0 < n) {
        // a flush with no input at the head of the remaining calls: on the host (memory caches)
        if (!coss && in_len[k0] == 0 && flags && (flags[k0] & XC_STREAM_FLUSH)) {
            if (int rc = host_flush(enc[k0], out + out_off[k0] + out_len[k0], &out_len[k0])) return rc;
            k0++;
            continue;
        }
        // build the round
        std::vector<Item> items;
        std::vector<const xc_encoder *> used;
        for (uint64_t k = k0; k < n; k++) {
            xc_encoder *e = enc[k];
            if (std::find(used.begin(), used.end(), e) != used.end()) break;
            const uint64_t pend = e->source.size();
            if (pend >= MAX_BUFFER) return xc__set_error(XC_ENOSPC, "stream pending bytes exceed 1 MiB");
            const uint64_t rest = in_len[k] - done[k];
            const uint64_t take = std::min<uint64_t>(rest, MAX_BUFFER - pend);
            const bool whole = take == rest;
            items.push_back({k, done[k], take, whole && flags && (flags[k] & XC_STREAM_FLUSH)});
            used.push_back(e);
            if (!whole) break;  // the rest of this input is the next round's
        }
        const uint64_t m = items.size();
        std::vector<const uint8_t *> head(m), tail(m);
        std::vector<uint64_t> hlen(m), tlen(m), start(m), rbase(m);
        std::vector<int64_t> cand(m), rcand(m);
        std::vector<uint32_t> fl(m);
        for (uint64_t i = 0; i < m; i++) {
            const xc_encoder *e = enc[items[i].call];
            head[i] = e->source.data();
            hlen[i] = e->source.size();
            tail[i] = items[i].take ? in[items[i].call] + items[i].from : nullptr;
            tlen[i] = items[i].take;
            start[i] = e->source.size();
            cand[i] = e->cand;
            fl[i] = items[i].flush ? 0u : SF_NOFLUSH;
        }
        // each item's output goes straight to its call's output, its new source_ (the input from
        // rbase on: empty after a flush) straight from the pinned arena
        struct Take {
            const std::vector<Item> *items;
            xc_encoder *const *enc;
            uint8_t *out;
            const uint64_t *out_off, *out_cap;
            uint64_t *out_len, *done;
            const uint64_t *hlen, *tlen, *rbase;
            const int64_t *rcand;
        } tk{&items, enc, out, out_off, out_cap, out_len, done.data(), hlen.data(), tlen.data(), rbase.data(), rcand.data()};
        auto take = [](void *vp, uint64_t i, const uint8_t *o, uint64_t olen, const uint8_t *inp) -> int {
            Take &t = *(Take *)vp;
            const uint64_t k = (*t.items)[i].call, ilen = t.hlen[i] + t.tlen[i];
            if (t.rbase[i] > ilen || (t.rcand[i] >= 0 && ((uint64_t)t.rcand[i] < t.rbase[i] || (uint64_t)t.rcand[i] >= ilen)))
                return xc__set_error(XC_EDEVICE, "inconsistent stream state from the device");
            if (t.out_len[k] + olen > t.out_cap[k]) return xc__set_error(XC_EINVAL, "output capacity too small");
            std::copy(o, o + olen, t.out + t.out_off[k] + t.out_len[k]);
            t.out_len[k] += olen;
            xc_encoder *e = t.enc[k];
            e->source.assign(inp + t.rbase[i], inp + ilen);
            e->cand = t.rcand[i] < 0 ? -1 : t.rcand[i] - (int64_t)t.rbase[i];
            t.done[k] += (*t.items)[i].take;
            return XC_OK;
        };
        int rc = coss ? xc__coss_encode_gather(coss, m, head.data(), hlen.data(), tail.data(), tlen.data(),
                                               start.data(), cand.data(), fl.data(), rbase.data(), rcand.data(), take,
                                               &tk)
                      : xc__encode_gather(cache, m, head.data(), hlen.data(), tail.data(), tlen.data(), start.data(),
                                          cand.data(), fl.data(), rbase.data(), rcand.data(), take, &tk);
        if (rc) return rc;
        // calls fully done advance the start of the next round
        k0 = items.back().call + (done[items.back().call] == in_len[items.back().call] ? 1 : 0);
    }
    return XC_OK;
}

extern "C" int xc_encode_streams(xc_encoder *const *enc, const uint8_t *const *in, const uint64_t *in_len,
                                 const uint32_t *flags, uint64_t n, uint8_t *out, const uint64_t *out_off,
                                 const uint64_t *out_cap, uint64_t *out_len)
{
    try {  // no exception crosses the C ABI
        return encode_streams(nullptr, enc, in, in_len, flags, n, out, out_off, out_cap, out_len);
    } catch (const std::bad_alloc &) {
        return xc__set_error(XC_ENOMEM, "host allocation failed");
    } catch (const std::exception &x) {
        return xc__set_error(XC_EINVAL, x.what());
    }
}

extern "C" int xc_coss_encode_streams(xc_coss *c, xc_encoder *const *enc, const uint8_t *const *in,
                                      const uint64_t *in_len, const uint32_t *flags, uint64_t n, uint8_t *out,
                                      const uint64_t *out_off, const uint64_t *out_cap, uint64_t *out_len)
{
    if (!c || !xc_coss_cache(c)) return xc__set_error(XC_EINVAL, "null (or a host-only COSS store)");
    try {
        return encode_streams(c, enc, in, in_len, flags, n, out, out_off, out_cap, out_len);
    } catch (const std::bad_alloc &) {
        return xc__set_error(XC_ENOMEM, "host allocation failed");
    } catch (const std::exception &x) {
        return xc__set_error(XC_EINVAL, x.what());
    }
}

extern "C" int xc_encode(xc_encoder *e, const uint8_t *in, uint64_t n, uint8_t *out, uint64_t cap,
                         uint64_t *out_len)
{
    const uint32_t fl = 0;
    const uint64_t off = 0;
    return xc_encode_streams(&e, &in, &n, &fl, 1, out, &off, &cap, out_len);
}

extern "C" int xc_flush(xc_encoder *e, uint8_t *out, uint64_t cap, uint64_t *out_len, int *emitted)
{
    if (!e) return xc__set_error(XC_EINVAL, "null");
    const uint32_t fl = XC_STREAM_FLUSH;
    const uint64_t zero = 0, off = 0;
    const uint8_t *none = nullptr;
    int rc = xc_encode_streams(&e, &none, &zero, &fl, 1, out, &off, &cap, out_len);
    if (!rc && emitted) *emitted = *out_len > 0 ? 1 : 0;
    return rc;
}

// Internal (the Python mirror's decode_batch): an output bound per stream, its length plus 2038 bytes
// per F1 byte in it (only a REF, F1 02 + 8 bytes, grows: 10 -> 2048 bytes; an EXTRACT keeps 2048
// of 2050, an escape shrinks), plus 16.
extern "C" int xc__decode_bound(const uint8_t *in, const uint64_t *off, const uint64_t *len, uint64_t n,
                                uint64_t *cap)
{
    if (n && (!in || !off || !len || !cap)) return xc__set_error(XC_EINVAL, "null");
    for (uint64_t j = 0; j < n; j++) {
        const uint8_t *p = in + off[j], *e = p + len[j];
        uint64_t c = 0;
        while ((p = (const uint8_t *)std::memchr(p, 0xF1, (size_t)(e - p))) != nullptr) {
            c++;
            p++;
        }
        cap[j] = len[j] + 2038u * c + 16u;
    }
    return XC_OK;
}
