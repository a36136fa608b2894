// C++ host-layer check (include/xcodec_hip.hpp), run by tests/test_gpu_cpp.py on the GPU.
//
// usage: xchip_roundtrip CALLS_FILE OUT_FILE
// CALLS_FILE: u32 ncalls, then per call: u32 connection, u8 flush, u32 length, bytes.
// The calls run on one cache through per-connection xchip::StreamEncoder objects, one call at a
// time (XCodecEncoder::encode [+ flush], as EncodeFilter::consume makes them); OUT_FILE gets
// every call's output as u32 length + bytes.  The same calls then run as one batch
// (xchip::encode_streams) on a fresh cache and must give the same bytes, and the streams are
// decoded in call order by xchip::Decoder on a third cache and must give back every
// connection's input.  Exit status 0 and "roundtrip ok" when all of that holds.
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>

#include "../../include/xcodec_hip.hpp"

using xchip::Bytes;

struct Call {
    uint32_t conn;
    bool flush;
    Bytes data;
};

static bool read_calls(const char *path, std::vector<Call> &calls)
{
    FILE *f = fopen(path, "rb");
    if (!f) return false;
    uint32_t n = 0;
    bool ok = fread(&n, 4, 1, f) == 1;
    for (uint32_t i = 0; ok && i < n; i++) {
        Call c;
        uint8_t fl = 0;
        uint32_t len = 0;
        ok = fread(&c.conn, 4, 1, f) == 1 && fread(&fl, 1, 1, f) == 1 && fread(&len, 4, 1, f) == 1;
        c.flush = fl != 0;
        c.data.resize(len);
        if (ok && len) ok = fread(c.data.data(), 1, len, f) == len;
        calls.push_back(std::move(c));
    }
    fclose(f);
    return ok;
}

int main(int argc, char **argv)
{
    if (argc != 3) {
        fprintf(stderr, "usage: %s CALLS_FILE OUT_FILE\n", argv[0]);
        return 2;
    }
    std::vector<Call> calls;
    if (!read_calls(argv[1], calls)) {
        fprintf(stderr, "cannot read %s\n", argv[1]);
        return 2;
    }
    try {
        xchip::Context ctx(0);
        // 1. one call at a time
        xchip::Cache cache(ctx, 1u << 16);
        std::map<uint32_t, std::unique_ptr<xchip::StreamEncoder>> enc;
        std::vector<Bytes> outs;
        for (const Call &c : calls) {
            auto &e = enc[c.conn];
            if (!e) e.reset(new xchip::StreamEncoder(cache));
            Bytes o;
            e->encode(o, c.data);
            if (c.flush) e->flush(o);
            outs.push_back(std::move(o));
        }
        FILE *f = fopen(argv[2], "wb");
        for (const Bytes &o : outs) {
            uint32_t len = (uint32_t)o.size();
            fwrite(&len, 4, 1, f);
            if (len) fwrite(o.data(), 1, len, f);
        }
        fclose(f);
        // 2. the same calls as one batch on a fresh cache
        xchip::Cache cache2(ctx, 1u << 16);
        std::map<uint32_t, std::unique_ptr<xchip::StreamEncoder>> enc2;
        std::vector<xchip::StreamCall> batch;
        for (const Call &c : calls) {
            auto &e = enc2[c.conn];
            if (!e) e.reset(new xchip::StreamEncoder(cache2));
            batch.push_back({e.get(), c.data.data(), (uint64_t)c.data.size(), c.flush});
        }
        std::vector<Bytes> outs2 = xchip::encode_streams(batch);
        for (size_t k = 0; k < calls.size(); k++)
            if (outs2[k] != outs[k]) {
                fprintf(stderr, "batch call %zu differs\n", k);
                return 1;
            }
        if (cache2.size() != cache.size()) {
            fprintf(stderr, "cache sizes differ\n");
            return 1;
        }
        // 3. decode every connection's stream in call order on a third cache
        xchip::Cache dcache(ctx, 1u << 16);
        xchip::Decoder dec(dcache);
        std::map<uint32_t, Bytes> pend, got, want;
        for (size_t k = 0; k < calls.size(); k++) {
            const uint32_t c = calls[k].conn;
            want[c].insert(want[c].end(), calls[k].data.begin(), calls[k].data.end());
            pend[c].insert(pend[c].end(), outs[k].begin(), outs[k].end());
            std::set<uint64_t> unknown;
            if (!dec.decode(got[c], pend[c], unknown) || !unknown.empty()) {
                fprintf(stderr, "decode of call %zu failed\n", k);
                return 1;
            }
        }
        for (auto &kv : want)
            if (got[kv.first] != kv.second || !pend[kv.first].empty()) {
                fprintf(stderr, "connection %u does not round-trip\n", kv.first);
                return 1;
            }
        if (dcache.size() != cache.size()) {
            fprintf(stderr, "decoder cache size differs\n");
            return 1;
        }
        // 4. a cached segment comes back by its hash
        if (!outs.empty() && cache.size()) {
            uint8_t seg[XC_SEGMENT_LENGTH];
            for (int i = 0; i < XC_SEGMENT_LENGTH; i++) seg[i] = (uint8_t)(i * 7 + 3);
            const uint64_t h = xchip::hash_segment(ctx, seg);
            Bytes back;
            if (cache.lookup(h, back)) {
                fprintf(stderr, "unexpected hit\n");
                return 1;
            }
            cache.enter(h, seg);
            if (!cache.lookup(h, back) || memcmp(back.data(), seg, sizeof seg) != 0) {
                fprintf(stderr, "enter/lookup failed\n");
                return 1;
            }
        }
    } catch (const xchip::Error &e) {
        fprintf(stderr, "xchip error %d: %s\n", e.code, e.what());
        return 1;
    }
    printf("roundtrip ok\n");
    return 0;
}
