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

#include "xcodec_hip.h" /* include/ of this repository */

/* The library's status codes in the reference's contract: the reference's encoder and cache cannot
 * fail (xcodec_encoder.h:53-57, xcodec_cache.h:182-210) and xcodec_filter.cc:122-164 has no
 * exception handling, so nothing is thrown through it.
 *  - XC_EBUSY (a run another caller submitted on this cache is in flight): that run is finished
 *    first (xc_cache_quiesce) and the call is made again;
 *  - any other failure of an encoder or cache call cannot be continued from: it is logged and the
 *    process halts, as the reference does when an allocation fails (HALT, common/log.h:195);
 *  - a decoder's failure is a decode that returns false (DecodeFilter::consume then reports
 *    "Decoder failed", xcodec_filter.cc). */
namespace xcodec_facade {
template <class F>
inline int call(xc_cache* dev, F f)
{
    int rc = f();
    if (rc == XC_EBUSY && dev && xc_cache_quiesce(dev) == XC_OK)
        rc = f();
    return rc;
}

inline void halt_on(int rc, const LogHandle& log, const char* what)
{
    if (rc != XC_OK)
        HALT(log) << what << ": " << xc_last_error() << " (" << rc << ")";
}

/* The device of a cache the proxy constructs with the reference's arguments (WanProxyCore::add_cache,
 * proxy/wanproxy.h:106-116, passes no device): xc_device_place over the visible devices, i.e. caches
 * dealt round-robin in creation order, XC_DEVICE=d (or a list) to pin them, XC_DEVICE_POLICY=uuid to
 * place by UUID. */
inline int place(const UUID& uuid, const char* log)
{
    int n = 0;
    halt_on(xc_device_count(&n), log, "device count");
    const int d = xc_device_place((const uint8_t*) &uuid.uuid_, sizeof uuid.uuid_, n);
    if (d < 0)
        halt_on(d, log, "device placement");
    return d;
}
}

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
 * cap_segments and grows like the reference's map before any call that could fill it.  gpu < 0 (what
 * the reference's two-argument construction gets): the device xcodec_facade::place picks. */
class XCodecMemoryCache : public XCodecCache {
    xc_ctx* ctx_;
    xc_cache* cache_;

public:
    XCodecMemoryCache(const UUID& uuid, size_t size, int gpu = -1, uint64_t cap_segments = 1u << 16)
    : XCodecCache(uuid, size), ctx_(0), cache_(0)
    {
        if (gpu < 0)
            gpu = xcodec_facade::place(uuid, "/xcodec/cache/memory");
        xcodec_facade::halt_on(xc_ctx_create(gpu, &ctx_), "/xcodec/cache/memory", "device context");
        xcodec_facade::halt_on(xc_cache_create(ctx_, cap_segments, &cache_), "/xcodec/cache/memory", "device cache");
    }
    ~XCodecMemoryCache()
    {
        xc_cache_destroy(cache_);
        xc_ctx_destroy(ctx_);
    }

    void enter(const uint64_t& hash, const Buffer& buf, unsigned off)
    {
        uint8_t seg[XCODEC_SEGMENT_LENGTH];
        buf.copyout(seg, off, sizeof seg);
        xcodec_facade::halt_on(xcodec_facade::call(cache_, [&] { return xc_cache_enter(cache_, hash, seg); }),
                               "/xcodec/cache/memory", "enter");
    }

    bool lookup(const uint64_t& hash, Buffer& buf)
    {
        uint8_t seg[XCODEC_SEGMENT_LENGTH];
        int found = 0;
        xcodec_facade::halt_on(xcodec_facade::call(cache_, [&] { return xc_cache_lookup(cache_, hash, seg, &found); }),
                               "/xcodec/cache/memory", "lookup");
        if (!found)
            return false;
        buf.append(seg, sizeof seg);
        return true;
    }

    xc_cache *device() { return cache_; }
    xc_ctx *context() { return ctx_; }
};

#endif /* !XCODEC_XCODEC_CACHE_H */
