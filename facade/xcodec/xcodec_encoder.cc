/*
 * facade/xcodec/xcodec_encoder.cc — XCodecEncoder over the device library (replaces
 * xcodec/xcodec_encoder.cc; see xcodec_encoder.h).
 */
#include <common/buffer.h>
#include <xcodec/xcodec.h>
#include <xcodec/xcodec_cache.h>
#include <xcodec/xcodec_encoder.h>

XCodecEncoder::XCodecEncoder(XCodecCache* cache) : cache_(cache), enc_(0)
{
    xc_cache* dev = cache->coss() ? xc_coss_cache(cache->coss()) : cache->device();
    xchip::check(xc_encoder_create(dev, &enc_));
}

XCodecEncoder::~XCodecEncoder()
{
    xc_encoder_destroy(enc_);
}

/* One call of this connection: encode(in) [+ flush()] (xcodec_encoder.cc:60-201). */
void XCodecEncoder::call(Buffer& output, const uint8_t* in, uint64_t n, uint32_t flags, int* emitted)
{
    uint64_t pend = 0;
    xchip::check(xc_encoder_pending(enc_, &pend));
    std::vector<uint8_t> out(2 * (pend + n) + 16);
    uint64_t off = 0, cap = out.size(), len = 0;
    if (cache_->coss())
        xchip::check(xc_coss_encode_streams(cache_->coss(), &enc_, &in, &n, &flags, 1, &out[0], &off, &cap, &len));
    else
        xchip::check(xc_encode_streams(&enc_, &in, &n, &flags, 1, &out[0], &off, &cap, &len));
    if (len)
        output.append(&out[0], len);
    if (emitted)
        *emitted = len > 0;
}

void XCodecEncoder::encode(Buffer& output, Buffer& input)
{
    std::vector<uint8_t> in(input.length() + 1);
    input.copyout(&in[0], input.length());  /* (read, not consumed: source_.append(input), :65) */
    call(output, &in[0], input.length(), 0, 0);
}

bool XCodecEncoder::flush(Buffer& output)
{
    int emitted = 0;
    call(output, 0, 0, XC_STREAM_FLUSH, &emitted);
    return emitted != 0;
}
