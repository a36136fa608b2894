/* xcodec_hip.hpp — the C++ host layer over the C ABI (xcodec_hip.h).
 *
 * RAII handles and byte-vector I/O with the reference's call shapes, for C++ hosts such as the
 * proxy's xcodec/ facade (INTEGRATION.md §2 adapts these to the reference's Buffer):
 *   xchip::Cache          XCodecMemoryCache::lookup / enter   (xcodec/xcodec_cache.h:182-210)
 *   xchip::StreamEncoder  XCodecEncoder::encode / flush       (xcodec/xcodec_encoder.h:53-57)
 *   xchip::encode_streams many connections' calls as one device batch (xcodec_filter.cc:122-164)
 *   xchip::Decoder        XCodecDecoder::decode               (xcodec/xcodec_decoder.h:48-51)
 *   xchip::hash_segment   XCodecHash::hash                    (xcodec/xcodec_hash.h:166-174)
 * Errors of the device library throw xchip::Error; the reference's own bool results (flush's
 * "emitted", decode's status) are returned as they are. */
#pragma once

#include <cstdint>
#include <cstring>
#include <memory>
#include <set>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "xcodec_hip.h"

namespace xchip {

using Bytes = std::vector<uint8_t>;

struct Error : std::runtime_error {
    int code;
    Error(int rc, const char *what) : std::runtime_error(what ? what : "xcodec_hip error"), code(rc) { }
};

inline void check(int rc)
{
    if (rc != XC_OK) throw Error(rc, xc_last_error());
}

inline int device_count()
{
    int n = 0;
    check(xc_device_count(&n));
    return n;
}

class Context {
    xc_ctx *h_ = nullptr;

public:
    explicit Context(int dev = 0) { check(xc_ctx_create(dev, &h_)); }
    ~Context() { if (h_) xc_ctx_destroy(h_); }
    Context(const Context &) = delete;
    Context &operator=(const Context &) = delete;
    xc_ctx *get() const { return h_; }
};

/* XCodecMemoryCache held in HBM, capacity in 2048-byte segments. */
class Cache {
    xc_cache *h_ = nullptr;

public:
    Cache(Context &ctx, uint64_t cap_segments) { check(xc_cache_create(ctx.get(), cap_segments, &h_)); }
    ~Cache() { if (h_) xc_cache_destroy(h_); }
    Cache(const Cache &) = delete;
    Cache &operator=(const Cache &) = delete;
    xc_cache *get() const { return h_; }

    uint64_t size() const
    {
        uint64_t n = 0;
        check(xc_cache_count(h_, &n));
        return n;
    }
    /* lookup(hash, buf): appends the segment to out when present */
    bool lookup(uint64_t hash, Bytes &out) const
    {
        uint8_t seg[XC_SEGMENT_LENGTH];
        int found = 0;
        check(xc_cache_lookup(h_, hash, seg, &found));
        if (found) out.insert(out.end(), seg, seg + XC_SEGMENT_LENGTH);
        return found != 0;
    }
    /* enter(hash, buf, off): the 2048 bytes at seg */
    void enter(uint64_t hash, const uint8_t *seg) { check(xc_cache_enter(h_, hash, seg)); }
};

/* One connection's XCodecEncoder: state (pending source_ bytes, candidate) kept between calls. */
class StreamEncoder {
    xc_encoder *h_ = nullptr;

public:
    explicit StreamEncoder(Cache &c) { check(xc_encoder_create(c.get(), &h_)); }
    ~StreamEncoder() { if (h_) xc_encoder_destroy(h_); }
    StreamEncoder(const StreamEncoder &) = delete;
    StreamEncoder &operator=(const StreamEncoder &) = delete;
    xc_encoder *get() const { return h_; }

    uint64_t pending() const
    {
        uint64_t n = 0;
        check(xc_encoder_pending(h_, &n));
        return n;
    }
    /* encode(output, input): appends exactly what the reference appends for this call */
    void encode(Bytes &output, const uint8_t *in, uint64_t n)
    {
        Bytes out(2 * (pending() + n) + 16);
        uint64_t len = 0;
        check(xc_encode(h_, in, n, out.data(), out.size(), &len));
        output.insert(output.end(), out.begin(), out.begin() + (ptrdiff_t)len);
    }
    void encode(Bytes &output, const Bytes &in) { encode(output, in.data(), in.size()); }
    /* flush(output): the reference's bool (whether anything was emitted) */
    bool flush(Bytes &output)
    {
        Bytes out(2 * pending() + 16);
        uint64_t len = 0;
        int emitted = 0;
        check(xc_flush(h_, out.data(), out.size(), &len, &emitted));
        output.insert(output.end(), out.begin(), out.begin() + (ptrdiff_t)len);
        return emitted != 0;
    }
};

/* One call of a connection for encode_streams: encoder->encode(input) [+ flush]. */
struct StreamCall {
    StreamEncoder *encoder;
    const uint8_t *data;
    uint64_t size;
    bool flush;
};

/* The outputs of one encode_streams batch: call k's bytes at data + off[k], len[k] of them. */
struct EncodedBatch {
    std::unique_ptr<uint8_t[]> data;  // (not value-initialised: the library writes what is read)
    std::vector<uint64_t> off, len;
    const uint8_t *at(size_t k) const { return data.get() + off[k]; }
};

/* Many connections' calls as one device batch, in order, into one output buffer. */
inline void encode_streams(const std::vector<StreamCall> &calls, EncodedBatch &res)
{
    const size_t n = calls.size();
    res.off.assign(n, 0);
    res.len.assign(n, 0);
    if (n == 0) return;
    std::vector<xc_encoder *> enc(n);
    std::vector<const uint8_t *> in(n);
    std::vector<uint64_t> len(n), cap(n);
    std::vector<uint32_t> flags(n);
    std::vector<std::pair<xc_encoder *, uint64_t>> pend;  // pending bytes per encoder so far
    uint64_t total = 0;
    for (size_t k = 0; k < n; k++) {
        enc[k] = calls[k].encoder->get();
        in[k] = calls[k].data;
        len[k] = calls[k].size;
        flags[k] = calls[k].flush ? XC_STREAM_FLUSH : 0u;
        uint64_t *p = nullptr;
        for (auto &e : pend)
            if (e.first == enc[k]) p = &e.second;
        if (!p) {
            pend.emplace_back(enc[k], calls[k].encoder->pending());
            p = &pend.back().second;
        }
        *p += len[k];
        cap[k] = 2 * *p + 16;
        res.off[k] = total;
        total += cap[k];
    }
    res.data.reset(new uint8_t[total ? total : 1]);
    check(xc_encode_streams(enc.data(), in.data(), len.data(), flags.data(), n, res.data.get(), res.off.data(),
                            cap.data(), res.len.data()));
}

/* The same, each call's output as its own byte vector. */
inline std::vector<Bytes> encode_streams(const std::vector<StreamCall> &calls)
{
    EncodedBatch b;
    encode_streams(calls, b);
    std::vector<Bytes> res(calls.size());
    for (size_t k = 0; k < calls.size(); k++) res[k].assign(b.at(k), b.at(k) + b.len[k]);
    return res;
}

/* An output bound for decoding n encoded bytes (xc__decode_bound): every byte, plus 2038 for each
 * F1 (only a REF grows: 10 -> 2048 bytes), plus 16. */
inline uint64_t decode_bound(const uint8_t *p, uint64_t n)
{
    uint64_t c = 0;
    const uint8_t *e = p + n;
    while ((p = (const uint8_t *)std::memchr(p, 0xF1, (size_t)(e - p))) != nullptr) {
        c++;
        p++;
    }
    return n + 2038u * c + 16u;
}

/* XCodecDecoder::decode(output, input, unknown_hashes): decodes as far as it can, removes the
 * consumed bytes from the front of input, adds the REF hash it stopped on to unknown. */
class Decoder {
    Cache *cache_;

public:
    explicit Decoder(Cache &c) : cache_(&c) { }
    bool decode(Bytes &output, Bytes &input, std::set<uint64_t> &unknown)
    {
        uint64_t off = 0, len = input.size();
        if (len == 0) return true;
        uint64_t cap = decode_bound(input.data(), len), olen = 0, consumed = 0, unk = 0;
        int32_t status = 0, has_unknown = 0;
        Bytes out(cap);
        check(xc_decode_batch_host(cache_->get(), input.data(), &off, &len, 1, out.data(), &off, &cap, &olen,
                                   &consumed, &status, &unk, &has_unknown));
        output.insert(output.end(), out.begin(), out.begin() + (ptrdiff_t)olen);
        input.erase(input.begin(), input.begin() + (ptrdiff_t)consumed);
        if (has_unknown) unknown.insert(unk);
        return status != 0;
    }
};

inline uint64_t hash_segment(Context &ctx, const uint8_t *seg)
{
    uint64_t h = 0;
    check(xc_hash_segments_host(ctx.get(), seg, 1, &h));
    return h;
}

}  // namespace xchip
