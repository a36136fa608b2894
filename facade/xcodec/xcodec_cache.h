/*
 * facade/xcodec/xcodec_cache.h — drop-in replacement for the reference's xcodec/xcodec_cache.h
 * (bramfeld/wanproxy), routing the cache to the MI355X device library (include/xcodec_hip.h).
 *
 * Same public surface as xcodec/xcodec_cache.h:89-211: the abstract XCodecCache (identifier(),
 * nominal_size(), virtual enter / lookup) and XCodecMemoryCache(uuid, size).  The recent window of
 * the reference (:94-98,128-158) lives in the library (xc_memcache.cpp), which gives every lookup
 * the reference's answer, including after a hash was entered twice (release semantics, :182-188).
 * The facade adds device()/coss(): the codec classes of this facade reach the library through them.
 *
 * Used with the reference's unchanged xcodec/xcodec_filter.{h,cc}, proxy/wanproxy.h and
 * proxy/wanproxy_codec.h (tests/test_facade.py compiles them against this directory).
 */
#ifndef XCODEC_XCODEC_CACHE_H
#define XCODEC_XCODEC_CACHE_H

#include <common/buffer.h>
#include <common/uuid/uuid.h>
#include <xcodec/xcodec.h>

#include "xcodec_hip.hpp" /* include/ of this repository */

class XCodecCache {
    UUID uuid_;
    size_t size_;

protected:
    XCodecCache(const UUID& uuid, size_t size) : uuid_(uuid), size_(size) { }

public:
    virtual ~XCodecCache() { }

    const UUID& identifier() { return uuid_; }
    size_t nominal_size() { return size_; }

    virtual void enter(const uint64_t& hash, const Buffer& buf, unsigned off) = 0;
    virtual bool lookup(const uint64_t& hash, Buffer& buf) = 0;

    /* the library objects behind the cache (one of them is non-null) */
    virtual xc_cache *device() { return 0; }
    virtual xc_coss *coss() { return 0; }
    virtual xc_ctx *context() = 0;
};

/* XCodecMemoryCache (xcodec_cache.h:162-211) held in HBM.  The device cache starts at
 * cap_segments and grows like the reference's map before any call that could fill it. */
class XCodecMemoryCache : public XCodecCache {
    xchip::Context ctx_;
    xchip::Cache cache_;

public:
    XCodecMemoryCache(const UUID& uuid, size_t size, int gpu = 0, uint64_t cap_segments = 1u << 16)
    : XCodecCache(uuid, size), ctx_(gpu), cache_(ctx_, cap_segments) { }

    void enter(const uint64_t& hash, const Buffer& buf, unsigned off)
    {
        uint8_t seg[XCODEC_SEGMENT_LENGTH];
        buf.copyout(seg, off, sizeof seg);
        cache_.enter(hash, seg);
    }

    bool lookup(const uint64_t& hash, Buffer& buf)
    {
        xchip::Bytes seg;
        if (!cache_.lookup(hash, seg))
            return false;
        buf.append(&seg[0], seg.size());
        return true;
    }

    xc_cache *device() { return cache_.get(); }
    xc_ctx *context() { return ctx_.get(); }
};

#endif /* !XCODEC_XCODEC_CACHE_H */
