/* TEST ONLY (tests/test_facade.py): the facade (facade/xcodec/) with the reference's own Buffer
 * (common/buffer.cc), as the reference's xcodec_filter.cc drives it: a connection's encoder called
 * per read, flushed at the end, the peer's decoder over its own cache decoding the frames' bytes
 * in pieces (a token may straddle two calls: decode leaves it in the input).  Prints "facade ok". */
#include <cstdio>
#include <cstdlib>
#include <set>
#include <vector>

#include <common/buffer.h>
#include <xcodec/xcodec.h>
#include <xcodec/xcodec_cache.h>
#include <xcodec/xcodec_decoder.h>
#include <xcodec/xcodec_encoder.h>

static uint64_t sm(uint64_t &s)
{
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

int main()
{
    UUID ua, ub;
    ua.generate();
    ub.generate();
    XCodecMemoryCache ca(ua, 64), cb(ub, 64);
    XCodecEncoder enc(&ca);
    XCodecDecoder dec(&cb);
    // data: fresh bytes, a repeat of an earlier 4 KiB (REFs), F1 bytes (escapes)
    uint64_t s = 7;
    std::vector<uint8_t> data(200000);
    for (size_t i = 0; i < data.size(); i++) data[i] = (uint8_t)sm(s);
    for (size_t i = 0; i < 8192; i++) data[120000 + i] = data[30000 + i];
    for (size_t i = 0; i < data.size(); i += 97) data[i] = 0xF1;
    Buffer wire;
    size_t at = 0;
    while (at < data.size()) {  // reads of up to 64 KiB (event/io_service.h:25)
        const size_t n = std::min<size_t>(data.size() - at, 1 + sm(s) % 65536);
        Buffer in(&data[at], n);
        enc.encode(wire, in);
        at += n;
    }
    if (!enc.flush(wire)) { std::printf("flush emitted nothing\n"); return 1; }
    const unsigned wire_len = wire.length();
    Buffer pending, out;
    std::set<uint64_t> unknown;
    while (!wire.empty()) {
        const size_t n = std::min<size_t>(wire.length(), 1 + sm(s) % 40000);
        Buffer piece;
        wire.moveout(&piece, n);
        pending.append(piece);
        if (!dec.decode(out, pending, unknown)) { std::printf("decode failed\n"); return 1; }
        if (!unknown.empty()) { std::printf("unknown hash\n"); return 1; }
    }
    if (!pending.empty() || out.length() != data.size()) {
        std::printf("lengths: pending %u out %u\n", (unsigned)pending.length(), (unsigned)out.length());
        return 1;
    }
    if (!out.equal(&data[0], data.size())) { std::printf("bytes differ\n"); return 1; }
    std::printf("facade ok %u bytes -> %u wire\n", (unsigned)data.size(), wire_len);
    return 0;
}
