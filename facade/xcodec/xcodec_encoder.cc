/*
 * facade/xcodec/xcodec_encoder.cc — XCodecEncoder over the device library (replaces
 * xcodec/xcodec_encoder.cc; see xcodec_encoder.h).
 */
#include <common/buffer.h>
#include <xcodec/xcodec.h>
#include <xcodec/xcodec_cache.h>
#include <xcodec/xcodec_encoder.h>

XCodecEncoder::XCodecEncoder(XCodecCache* cache) : log_("/xcodec/encoder"), cache_(cache), enc_(0)
{
    xcodec_facade::halt_on(xc_encoder_create(dev(), &enc_), log_, "encoder");
}

xc_cache* XCodecEncoder::dev() const
{
    return cache_->coss() ? xc_coss_cache(cache_->coss()) : cache_->device();
}

XCodecEncoder::~XCodecEncoder()
{
    xc_encoder_destroy(enc_);
}

/* One call of this connection: encode(in) [+ flush()] (xcodec_encoder.cc:60-201).  The reference's
 * encoder cannot fail (xcodec_encoder.h:53-57): a run in flight on the cache is finished first
 * (XC_EBUSY), anything else halts (xcodec_cache.h's notes). */
void XCodecEncoder::call(Buffer& output, const uint8_t* in, uint64_t n, uint32_t flags, int* emitted)
{
    uint64_t pend = 0;
    xcodec_facade::halt_on(xc_encoder_pending(enc_, &pend), log_, "encoder state");
    if (out_.size() < 2 * (pend + n) + 16)
        out_.resize(2 * (pend + n) + 16);
    uint8_t* out = &out_[0];
    uint64_t off = 0, cap = 2 * (pend + n) + 16, len = 0;
    int rc;
    if (cache_->coss())
        rc = xcodec_facade::call(dev(), [&] {
            return xc_coss_encode_streams(cache_->coss(), &enc_, &in, &n, &flags, 1, out, &off, &cap, &len);
        });
    else
        rc = xcodec_facade::call(dev(), [&] { return xc_encode_streams(&enc_, &in, &n, &flags, 1, out, &off, &cap, &len); });
    xcodec_facade::halt_on(rc, log_, "encode");
    if (len)
        output.append(out, len);
    if (emitted)
        *emitted = len > 0;
}

void XCodecEncoder::encode(Buffer& output, Buffer& input)
{
    if (in_.size() < input.length() + 1)
        in_.resize(input.length() + 1);
    input.copyout(&in_[0], input.length());  /* (read, not consumed: source_.append(input), :65) */
    call(output, &in_[0], input.length(), 0, 0);
}

bool XCodecEncoder::flush(Buffer& output)
{
    int emitted = 0;
    call(output, 0, 0, XC_STREAM_FLUSH, &emitted);
    return emitted != 0;
}
