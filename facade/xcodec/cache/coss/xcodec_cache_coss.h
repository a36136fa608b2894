/*
 * facade/xcodec/cache/coss/xcodec_cache_coss.h — drop-in replacement for
 * xcodec/cache/coss/xcodec_cache_coss.h (XCodecCacheCOSS(uuid, cache_dir, cache_size), :184-220).
 *
 * The reference's stripe file <cache_dir>/<uuid>.wpc, same bytes, with the device cache as its
 * mirror (xc_coss_*, wanproxy_amd/csrc/xc_coss.cpp); lookups and enters keep the reference's side
 * effects (stripe loads, freshness, the recent window), and the destructor stores the loaded
 * stripes back as the reference's does (:82-105).
 */
#ifndef XCODEC_CACHE_COSS_XCODEC_CACHE_COSS_H
#define XCODEC_CACHE_COSS_XCODEC_CACHE_COSS_H

#include <string>

#include <common/buffer.h>
#include <xcodec/xcodec.h>
#include <xcodec/xcodec_cache.h>

class XCodecCacheCOSS : public XCodecCache {
    xc_ctx* ctx_;
    xc_coss* coss_;

public:
    XCodecCacheCOSS(const UUID& uuid, const std::string& cache_dir, size_t cache_size, int gpu = -1)
    : XCodecCache(uuid, cache_size), ctx_(0), coss_(0)
    {
        uint8_t u[UUID_STRING_SIZE + 1];
        uuid.to_string(u);
        if (gpu < 0)  /* (the reference's three-argument construction: xcodec_facade::place) */
            gpu = xcodec_facade::place(uuid, "/xcodec/cache/coss");
        xcodec_facade::halt_on(xc_ctx_create(gpu, &ctx_), "/xcodec/cache/coss", "device context");
        xcodec_facade::halt_on(xc_coss_open(ctx_, cache_dir.c_str(), (const char*) u, cache_size, &coss_),
                               "/xcodec/cache/coss", "open");
    }
    ~XCodecCacheCOSS()
    {
        xc_coss_close(coss_);
        xc_ctx_destroy(ctx_);
    }

    void enter(const uint64_t& hash, const Buffer& buf, unsigned off)
    {
        uint8_t seg[XCODEC_SEGMENT_LENGTH];
        buf.copyout(seg, off, sizeof seg);
        xcodec_facade::halt_on(xcodec_facade::call(xc_coss_cache(coss_), [&] { return xc_coss_enter(coss_, hash, seg); }),
                               "/xcodec/cache/coss", "enter");
    }

    bool lookup(const uint64_t& hash, Buffer& buf)
    {
        uint8_t seg[XCODEC_SEGMENT_LENGTH];
        int found = 0;
        xcodec_facade::halt_on(
            xcodec_facade::call(xc_coss_cache(coss_), [&] { return xc_coss_lookup(coss_, hash, seg, &found); }),
            "/xcodec/cache/coss", "lookup");
        if (found)
            buf.append(seg, sizeof seg);
        return found != 0;
    }

    xc_coss* coss() { return coss_; }
    xc_ctx* context() { return ctx_; }
};

#endif /* !XCODEC_CACHE_COSS_XCODEC_CACHE_COSS_H */
