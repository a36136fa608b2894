/* TEST ONLY (tests/test_facade.py): the reference's own, unchanged EncodeFilter
 * (xcodec/xcodec_filter.cc:122-216) over the facade, linked with the reference's event system,
 * Buffer and log, the C ABI being the CPU stand-in (tests/facade/xc_abi_oracle.cc).  A connection's
 * reads go through EncodeFilter::consume into a sink; the sink's <HELLO>, <FRAME>s and <EOS> are
 * parsed and the frames decoded by the facade's XCodecDecoder over the peer's cache.
 *   busy:        every library call meets XC_EBUSY once (another caller's run in flight): the facade
 *                finishes that run (xc_cache_quiesce) and calls again; the round trip is exact
 *   fail-decode: the decoder's library call fails: decode() returns false
 *   fail-encode: the encoder's library call fails: the facade halts (HALT: log, abort)
 * Prints "facade filter ok" on success. */
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <set>
#include <string>
#include <vector>

#include <common/buffer.h>
#include <xcodec/xcodec_filter.h>

extern "C" void xc__test_inject(int busy, int fail_encode, int fail_decode);
extern "C" int xc__test_quiesced(void);

static uint64_t sm(uint64_t &s)
{
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

class Sink : public Filter {
public:
    std::vector<uint8_t> bytes;
    bool consume(Buffer& buf, int) override
    {
        const size_t n = buf.length();
        const size_t at = bytes.size();
        bytes.resize(at + n);
        if (n) buf.copyout(&bytes[at], n);
        buf.clear();
        return true;
    }
};

int main(int argc, char** argv)
{
    const std::string mode = argc > 1 ? argv[1] : "";
    UUID ua, ub;
    ua.generate();
    ub.generate();
    XCodecMemoryCache ca(ua, 64), cb(ub, 64);
    WANProxyCodec codec;
    codec.xcache_ = &ca;
    EncodeFilter enc("/test/encode", &codec);
    Sink sink;
    enc.chain(&sink);
    xc__test_inject(mode == "busy", mode == "fail-encode", 0);

    uint64_t s = 11;
    std::vector<uint8_t> data(180000);
    for (size_t i = 0; i < data.size(); i++) data[i] = (uint8_t)sm(s);
    for (size_t i = 0; i < 10000; i++) data[140000 + i] = data[20000 + i];
    for (size_t i = 0; i < data.size(); i += 131) data[i] = 0xF1;
    size_t at = 0;
    while (at < data.size()) {
        const size_t n = std::min<size_t>(data.size() - at, 1 + sm(s) % 65536);
        Buffer in(&data[at], n);
        if (!enc.consume(in)) { std::printf("consume failed\n"); return 1; }
        at += n;
    }
    enc.flush(0);

    // <HELLO> FF len uuid(36) size(8), <FRAME> 00 BE16 data, <EOS> FC (xcodec_filter.cc:48-118)
    const std::vector<uint8_t>& w = sink.bytes;
    if (w.size() < 46 || w[0] != 0xFF || w[1] != 44) { std::printf("no <HELLO>\n"); return 1; }
    size_t p = 46;
    Buffer frames;
    while (p < w.size() && w[p] == 0x00) {
        const size_t n = ((size_t)w[p + 1] << 8) | w[p + 2];
        frames.append(&w[p + 3], n);
        p += 3 + n;
    }
    if (p + 1 != w.size() || w[p] != 0xFC) { std::printf("no <EOS> at the end\n"); return 1; }

    xc__test_inject(mode == "busy", 0, mode == "fail-decode");
    XCodecDecoder dec(&cb);
    Buffer out;
    std::set<uint64_t> unknown;
    const bool ok = dec.decode(out, frames, unknown);
    if (mode == "fail-decode") {
        if (ok) { std::printf("decode did not report the failure\n"); return 1; }
        std::printf("facade filter ok (decode false)\n");
        return 0;
    }
    if (!ok || !unknown.empty() || !frames.empty()) { std::printf("decode failed\n"); return 1; }
    if (out.length() != data.size() || !out.equal(&data[0], data.size())) { std::printf("bytes differ\n"); return 1; }
    if (mode == "busy" && xc__test_quiesced() == 0) { std::printf("no XC_EBUSY was met\n"); return 1; }
    std::printf("facade filter ok %u bytes, %d quiesced\n", (unsigned)data.size(), xc__test_quiesced());
    return 0;
}
