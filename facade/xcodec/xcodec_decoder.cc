/*
 * facade/xcodec/xcodec_decoder.cc — XCodecDecoder over the device library (replaces
 * xcodec/xcodec_decoder.cc; see xcodec_decoder.h).
 */
#include <vector>

#include "xcodec_hip.hpp" /* xchip::decode_bound */

#include <common/buffer.h>
#include <xcodec/xcodec.h>
#include <xcodec/xcodec_cache.h>
#include <xcodec/xcodec_decoder.h>

XCodecDecoder::XCodecDecoder(XCodecCache* cache) : log_("/xcodec/decoder"), cache_(cache) { }

XCodecDecoder::~XCodecDecoder() { }

/* The reference's decode returns false on a collision or a bad opcode (xcodec_decoder.cc:76-176);
 * a library failure is reported the same way (the filter then fails the connection), after a run in
 * flight on the cache was finished and the call made again (XC_EBUSY). */
bool XCodecDecoder::decode(Buffer& output, Buffer& input, std::set<uint64_t>& unknown_hashes)
{
    if (input.empty())
        return true;
    const uint64_t n = input.length();
    if (in_.size() < n)
        in_.resize(n);
    uint8_t* in = &in_[0];
    input.copyout(in, n);
    /* a REF (10 bytes) expands to 2048: n plus 2038 per F1 byte (xchip::decode_bound) */
    uint64_t off = 0, len = n, cap = xchip::decode_bound(in, n), olen = 0, consumed = 0, unknown = 0;
    int32_t status = 0, has_unknown = 0;
    if (out_.size() < cap)
        out_.resize(cap);
    uint8_t* out = &out_[0];
    xc_cache* dev = cache_->coss() ? xc_coss_cache(cache_->coss()) : cache_->device();
    int rc;
    if (cache_->coss())
        rc = xcodec_facade::call(dev, [&] {
            return xc_coss_decode_batch_host(cache_->coss(), in, &off, &len, 1, out, &off, &cap, &olen,
                                             &consumed, &status, &unknown, &has_unknown);
        });
    else
        rc = xcodec_facade::call(dev, [&] {
            return xc_decode_batch_host(dev, in, &off, &len, 1, out, &off, &cap, &olen, &consumed, &status,
                                        &unknown, &has_unknown);
        });
    if (rc != XC_OK) {
        ERROR(log_) << "device decode failed: " << xc_last_error() << " (" << rc << ")";
        return false;
    }
    if (olen)
        output.append(out, olen);
    input.skip(consumed);  /* the reference consumes exactly this much (xcodec_decoder.cc:85-173) */
    if (has_unknown)
        unknown_hashes.insert(unknown);
    return status != 0;
}
