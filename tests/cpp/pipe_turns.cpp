// pipe_turns — the C++ pipe filters (include/xcodec_pipe.hpp) between two proxies on the GPU.
//
//   pipe_turns parity SCENARIO OUT   the scenario's connections turn by turn (tests/test_gpu_pipe_cpp.py
//                                    runs the same scenario through the oracle pipes): every
//                                    connection's wire bytes both ways and both sinks to OUT
//   pipe_turns bench SCENARIO        filter-path throughput (tools/pipe_bench_cpp.py): encode turns
//                                    of every connection with the Batcher, then the peer decoding the
//                                    pipes; one JSON line
//
// SCENARIO (little endian): u32 nconn, turns, waiting, batched; u64 nwarm, then nwarm x (u64 len,
// bytes): proxy A's warm-up buffers (and, for the bench, the peer's copy of A's cache); turns x nconn
// u32: the order of the connections' consume calls per turn; nconn x turns x (u64 len, bytes): the
// reads (len 0: no read that turn).
#include <chrono>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/xcodec_pipe.hpp"

using namespace xchip;
using namespace xchip::pipe;

static const char *UUID_A = "0f1e2d3c-4b5a-6978-8796-a5b4c3d2e1f0";
static const char *UUID_B = "12345678-9abc-def0-1234-56789abcdef0";

namespace {
struct Reader {
    std::vector<uint8_t> d;
    size_t at = 0;
    explicit Reader(const char *path)
    {
        std::ifstream f(path, std::ios::binary);
        d.assign(std::istreambuf_iterator<char>(f), std::istreambuf_iterator<char>());
    }
    template <class T>
    T get()
    {
        T v;
        if (at + sizeof v > d.size()) throw std::runtime_error("short scenario");
        std::memcpy(&v, &d[at], sizeof v);
        at += sizeof v;
        return v;
    }
    Bytes bytes()
    {
        const uint64_t n = get<uint64_t>();
        if (at + n > d.size()) throw std::runtime_error("short scenario");
        Bytes b(d.begin() + (ptrdiff_t)at, d.begin() + (ptrdiff_t)(at + n));
        at += n;
        return b;
    }
};

struct Scenario {
    uint32_t nconn, turns, waiting, batched;
    std::vector<Bytes> warm;
    std::vector<std::vector<uint32_t>> order;
    std::vector<std::vector<Bytes>> in;  // [conn][turn]
    explicit Scenario(const char *path)
    {
        Reader r(path);
        nconn = r.get<uint32_t>();
        turns = r.get<uint32_t>();
        waiting = r.get<uint32_t>();
        batched = r.get<uint32_t>();
        const uint64_t nw = r.get<uint64_t>();
        for (uint64_t i = 0; i < nw; i++) warm.push_back(r.bytes());
        order.assign(turns, std::vector<uint32_t>(nconn));
        for (auto &o : order)
            for (auto &x : o) x = r.get<uint32_t>();
        in.assign(nconn, std::vector<Bytes>(turns));
        for (auto &c : in)
            for (auto &b : c) b = r.bytes();
    }
};

// A socket: bytes queue until the harness delivers them (log: everything ever sent).
struct Wire : Filter {
    Bytes q, log;
    bool keep_log = true;
    bool consume(const uint8_t *p, size_t n, int) override
    {
        q.insert(q.end(), p, p + n);
        if (keep_log) log.insert(log.end(), p, p + n);
        return true;
    }
    void flush(int) override { }
};

struct Sink : Filter {
    Bytes data;
    bool consume(const uint8_t *p, size_t n, int) override
    {
        data.insert(data.end(), p, p + n);
        return true;
    }
    void flush(int) override { }
};

// One proxy's codec side: its cache (shared by every connection's EncodeFilter), the registry of
// the peers' caches its DecodeFilters find by <HELLO>, and the Batcher of its event loop.
struct Proxy {
    CacheRegistry reg;
    CodecCache *cache;
    Batcher batcher;
    Codec codec;
    Proxy(Context &ctx, const char *uuid, bool batched) : reg(ctx, 1u << 16)
    {
        cache = reg.add_cache(64, uuid);
        codec.cache = cache;
        codec.registry = &reg;
        codec.batcher = batched ? &batcher : nullptr;
    }
    void end_turn()
    {
        if (codec.batcher && !codec.batcher->run().empty()) throw std::runtime_error("a deferred consume failed");
    }
};

void warm_cache(Cache &c, const std::vector<Bytes> &warm)
{
    // encode()+flush() of every warm-up buffer on fresh encoders, in order (the pool's declarations)
    StreamEncoder e(c);
    for (const Bytes &b : warm) {
        Bytes out;
        e.encode(out, b);
        e.flush(out);
    }
}

struct Conn {
    EncodeFilter a_enc, b_enc;
    DecodeFilter a_dec, b_dec;
    Wire ab, ba;
    Sink a_sink, b_sink;
    Conn(Proxy &a, Proxy &b, bool waiting)
        : a_enc(&a.codec, waiting ? 1 : 0), b_enc(&b.codec, 0), a_dec(&a.codec), b_dec(&b.codec)
    {
        a_enc.chain(&ab);
        b_enc.chain(&ba);
        a_dec.chain(&a_sink);
        b_dec.chain(&b_sink);
        a_dec.set_upstream(&a_enc);
        b_dec.set_upstream(&b_enc);
    }
};

// Deliver queued wire bytes turn by turn until every wire is idle (tests/pipe_harness.py pump_turns).
void pump_turns(Proxy &a, Proxy &b, std::vector<std::unique_ptr<Conn>> &conns)
{
    for (int guard = 0; guard < 1000000; guard++) {
        std::vector<std::pair<DecodeFilter *, Bytes>> work;
        for (auto &c : conns) {
            if (!c->ab.q.empty()) {
                work.push_back({&c->b_dec, Bytes()});
                work.back().second.swap(c->ab.q);
            }
            if (!c->ba.q.empty()) {
                work.push_back({&c->a_dec, Bytes()});
                work.back().second.swap(c->ba.q);
            }
        }
        if (work.empty()) return;
        for (auto &w : work)
            if (!w.first->consume(w.second.data(), w.second.size(), 0)) throw std::runtime_error("decode filter failed");
        a.end_turn();
        b.end_turn();
    }
    throw std::runtime_error("pipes did not settle");
}

void put(std::ofstream &f, const Bytes &b)
{
    const uint64_t n = b.size();
    f.write((const char *)&n, 8);
    f.write((const char *)b.data(), (std::streamsize)n);
}

int parity(const Scenario &s, const char *out)
{
    Context ctx(0);
    Proxy a(ctx, UUID_A, s.batched != 0), b(ctx, UUID_B, s.batched != 0);
    warm_cache(*a.cache->store, s.warm);
    std::vector<std::unique_ptr<Conn>> conns;
    for (uint32_t i = 0; i < s.nconn; i++) conns.emplace_back(new Conn(a, b, s.waiting != 0));
    for (uint32_t t = 0; t < s.turns; t++) {
        for (uint32_t i : s.order[t]) {
            const Bytes &d = s.in[i][t];
            if (!d.empty() && !conns[i]->a_enc.consume(d.data(), d.size(), 0)) throw std::runtime_error("consume failed");
        }
        a.end_turn();
        b.end_turn();
        if (s.waiting)
            for (auto &c : conns) c->a_enc.on_read_timeout();
        pump_turns(a, b, conns);
    }
    for (auto &c : conns) c->a_enc.flush(0);
    pump_turns(a, b, conns);
    for (auto &c : conns) c->b_enc.flush(0);
    pump_turns(a, b, conns);
    std::ofstream f(out, std::ios::binary);
    for (auto &c : conns) {
        put(f, c->ab.log);
        put(f, c->ba.log);
        put(f, c->b_sink.data);
        put(f, c->a_sink.data);
    }
    std::printf("parity ok: %u connections, %u turns, device calls %llu / %llu\n", s.nconn, s.turns,
                (unsigned long long)a.batcher.device_calls, (unsigned long long)b.batcher.device_calls);
    return 0;
}

double now()
{
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// One measured run: N connections of proxy A, each EncodeFilter consuming its read per turn; then
// the peer's DecodeFilters decoding every pipe (the peer's copy of A's cache holds the pool: steady
// state, no <ASK>/<LEARN>).  Returns {encode s, decode s, input bytes, ok}.
struct Run {
    double enc_s, dec_s;
    uint64_t bytes, calls;
    bool ok;
};
Run bench_once(Context &ctx, const Scenario &s)
{
    Proxy a(ctx, UUID_A, s.batched != 0), b(ctx, UUID_B, s.batched != 0);
    warm_cache(*a.cache->store, s.warm);
    CodecCache *peer = b.reg.add_cache(64, UUID_A);
    warm_cache(*peer->store, s.warm);
    std::vector<std::unique_ptr<Conn>> conns;
    for (uint32_t i = 0; i < s.nconn; i++) {
        conns.emplace_back(new Conn(a, b, false));
        conns.back()->ab.keep_log = false;
    }
    // the reads as a proxy holds them (its read buffers, handed to consume: no copy when deferred)
    std::vector<std::vector<Bytes>> reads(s.turns, std::vector<Bytes>(s.nconn));
    for (uint32_t t = 0; t < s.turns; t++)
        for (uint32_t i = 0; i < s.nconn; i++) reads[t][i] = s.in[i][t];
    uint64_t bytes = 0;
    const double t0 = now();
    for (uint32_t t = 0; t < s.turns; t++) {
        for (uint32_t i : s.order[t]) {
            const size_t n = reads[t][i].size();
            bytes += n;
            if (n && !conns[i]->a_enc.consume(std::move(reads[t][i]), 0)) throw std::runtime_error("consume failed");
        }
        a.end_turn();
    }
    const double t1 = now();
    for (auto &c : conns) {
        Bytes q;
        q.swap(c->ab.q);
        if (!c->b_dec.consume(q.data(), q.size(), 0)) throw std::runtime_error("decode failed");
    }
    b.end_turn();
    const double t2 = now();
    bool ok = true;
    for (uint32_t i = 0; i < s.nconn; i++) {
        Bytes want;
        for (uint32_t t = 0; t < s.turns; t++) want.insert(want.end(), s.in[i][t].begin(), s.in[i][t].end());
        ok = ok && conns[i]->b_sink.data == want;
    }
    return {t1 - t0, t2 - t1, bytes, a.batcher.device_calls, ok};
}

int bench(const Scenario &s)
{
    Context ctx(0);
    bench_once(ctx, s);  // (the first run pays the library pool's one-time allocations)
    Run r = bench_once(ctx, s);
    const double gib = (double)r.bytes / (1u << 30);
    std::printf("{\"connections\": %u, \"turns\": %u, \"batched\": %s, \"encode_GiBs\": %.3f, "
                "\"encode_ms_per_turn\": %.3f, \"decode_GiBs\": %.3f, \"device_calls\": %llu, \"round_trip_ok\": %s}\n",
                s.nconn, s.turns, s.batched ? "true" : "false", gib / r.enc_s, r.enc_s / s.turns * 1e3, gib / r.dec_s,
                (unsigned long long)r.calls, r.ok ? "true" : "false");
    return r.ok ? 0 : 1;
}
}  // namespace

int main(int argc, char **argv)
{
    try {
        if (argc == 4 && std::string(argv[1]) == "parity") return parity(Scenario(argv[2]), argv[3]);
        if (argc == 3 && std::string(argv[1]) == "bench") return bench(Scenario(argv[2]));
        std::fprintf(stderr, "usage: pipe_turns parity SCENARIO OUT | bench SCENARIO\n");
        return 2;
    } catch (const std::exception &e) {
        std::fprintf(stderr, "pipe_turns: %s\n", e.what());
        return 1;
    }
}
