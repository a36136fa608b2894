/*
 * facade/xcodec/xcodec_encoder.h — drop-in replacement for xcodec/xcodec_encoder.h (public
 * surface :43-63: XCodecEncoder(XCodecCache*), encode(output, input), flush(output)).
 *
 * The reference encoder's state between calls (pending source_ bytes and the candidate, :45-50) is
 * kept by the library's xc_encoder; each call appends exactly what the reference appends
 * (xcodec_encoder.cc:60-201).  Over a COSS cache the calls run through xc_coss_encode_streams,
 * which advances the stripe file as the reference's calls would.
 */
#ifndef XCODEC_XCODEC_ENCODER_H
#define XCODEC_XCODEC_ENCODER_H

#include <vector>

#include <common/log.h>
#include <xcodec/xcodec_hash.h>

#include "xcodec_hip.h"

class XCodecCache;

class XCodecEncoder {
    LogHandle log_;
    XCodecCache* cache_;
    xc_encoder* enc_;
    std::vector<uint8_t> in_, out_;  /* host staging, kept across calls (grown, never shrunk) */

    xc_cache* dev() const;
    void call(Buffer& output, const uint8_t* in, uint64_t n, uint32_t flags, int* emitted);

public:
    XCodecEncoder(XCodecCache*);
    ~XCodecEncoder();

    void encode(Buffer&, Buffer&);
    bool flush(Buffer&);
};

#endif /* !XCODEC_XCODEC_ENCODER_H */
