/*
 * facade/xcodec/xcodec_decoder.h — drop-in replacement for xcodec/xcodec_decoder.h (public
 * surface :43-52: XCodecDecoder(XCodecCache*), decode(output, input, unknown_hashes)).
 *
 * decode() decodes as far as the reference does (xcodec_decoder.cc:76-176): it removes the
 * consumed bytes from input, appends the decoded bytes to output, adds the REF hash it stopped on
 * to unknown_hashes, and returns false on a collision or a bad opcode.
 */
#ifndef XCODEC_XCODEC_DECODER_H
#define XCODEC_XCODEC_DECODER_H

#include <set>
#include <vector>

#include <common/log.h>

class XCodecCache;

class XCodecDecoder {
    LogHandle log_;
    XCodecCache* cache_;
    std::vector<uint8_t> in_, out_;  /* host staging, kept across calls (grown, never shrunk) */

public:
    XCodecDecoder(XCodecCache*);
    ~XCodecDecoder();

    bool decode(Buffer&, Buffer&, std::set<uint64_t>&);
};

#endif /* !XCODEC_XCODEC_DECODER_H */
