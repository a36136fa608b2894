/* xcodec_pipe.hpp — the XCodec pipe filters in C++ over the device codec, with cross-connection
 * batching of one event-loop turn.
 *
 * EncodeFilter / DecodeFilter mirror xcodec/xcodec_filter.h:25-86 and xcodec/xcodec_filter.cc:
 * 122-526 (the same names, argument meaning and bool results): <HELLO> (cache UUID + nominal size),
 * <FRAME> = 00 BE16(len) data with 1 <= len <= 32768, <ASK> / <LEARN> for REFs the peer's cache
 * lacks, <EOS> / <EOS_ACK>, and the server side's waiting mode (the flush deferred to
 * on_read_timeout(), the reference's 150 ms timer, :148-157,205-216; the caller owns the clock).
 * Filters chain as in common/filter.h:18-70 (consume from upstream, produce to the next, flush
 * down the chain).
 *
 * The reference calls the codec once per consume on its one event thread.  With a Batcher attached
 * to the Codec, every EncodeFilter::consume of a turn becomes one call of a single device batch
 * (xc_encode_streams: every connection's encoder state carried, calls in call order over one
 * cache), every frames-only DecodeFilter::consume one stream of one device decode batch per cache
 * (xc_decode_batch_host), and each deferred consume's framing and produce then run in call order:
 * the wire bytes are those of the unbatched filters.  Batcher::run() at the end of the turn
 * returns the filters whose deferred consume failed (they then refuse their next consume, as the
 * reference's failing consume ends the connection).
 *
 * Header-only, C++17, over xcodec_hip.hpp. */
#pragma once

#include <cstdint>
#include <cstring>
#include <functional>
#include <map>
#include <memory>
#include <set>
#include <string>
#include <vector>

#include "xcodec_hip.hpp"

namespace xchip {
namespace pipe {

constexpr uint8_t OP_HELLO = 0xFF;    // xcodec_filter.cc:52
constexpr uint8_t OP_LEARN = 0xFE;    // :64
constexpr uint8_t OP_ASK = 0xFD;      // :79
constexpr uint8_t OP_EOS = 0xFC;      // :92
constexpr uint8_t OP_EOS_ACK = 0xFB;  // :104
constexpr uint8_t OP_FRAME = 0x00;    // :116
constexpr uint32_t MAX_FRAME = 32768;  // :118
constexpr int TO_BE_CONTINUED = 1;    // common/count_filter.h:17
constexpr uint32_t UUID_LEN = 36;     // common/uuid/uuid.h:54
constexpr uint32_t SEG = XC_SEGMENT_LENGTH;

/* common/filter.h:18-31 */
class Filter {
public:
    virtual ~Filter() { }
    void chain(Filter *next) { recipient_ = next; }
    virtual bool consume(const uint8_t *p, size_t n, int flg = 0) { return produce(p, n, flg); }
    virtual void flush(int flg)
    {
        if (recipient_) recipient_->flush(flg);
    }
    bool produce(const uint8_t *p, size_t n, int flg = 0) { return recipient_ && recipient_->consume(p, n, flg); }
    bool produce(const Bytes &b, int flg = 0) { return produce(b.data(), b.size(), flg); }

protected:
    Filter *recipient_ = nullptr;
};

/* An XCodecCache as the pipe sees it (xcodec/xcodec_cache.h:100-126): the device cache, its
 * identifier (UUID string) and nominal size in MB (sent in <HELLO>). */
struct CodecCache {
    std::unique_ptr<Cache> store;
    std::string uuid;
    uint64_t size = 0;
};

/* WanProxyCore::find_cache / add_cache (proxy/wanproxy.h:106-130): a <HELLO> finds its peer's
 * cache here or adds one. */
class CacheRegistry {
public:
    CacheRegistry(Context &ctx, uint64_t capacity = 1u << 16) : ctx_(ctx), capacity_(capacity) { }
    CodecCache *find_cache(const std::string &uuid)
    {
        auto it = caches_.find(uuid);
        return it == caches_.end() ? nullptr : it->second.get();
    }
    CodecCache *add_cache(uint64_t size, const std::string &uuid)
    {
        std::unique_ptr<CodecCache> c(new CodecCache{std::unique_ptr<Cache>(new Cache(ctx_, capacity_)), uuid, size});
        CodecCache *r = c.get();
        caches_[uuid] = std::move(c);
        return r;
    }
    Context &context() { return ctx_; }

private:
    Context &ctx_;
    uint64_t capacity_;
    std::map<std::string, std::unique_ptr<CodecCache>> caches_;
};

class Batcher;

/* WANProxyCodec (proxy/wanproxy_codec.h:43-71): the local cache (xcache_), the registry, and the
 * optional Batcher of the event loop. */
struct Codec {
    CodecCache *cache = nullptr;
    CacheRegistry *registry = nullptr;
    Batcher *batcher = nullptr;
};

class DecodeFilter;

/* The codec calls of one event-loop turn, for every connection, as few device calls.  Jobs are
 * cut into rounds: the longest prefix of the remaining jobs in which no filter repeats and no cache
 * is both encoded and decoded; a round is one xc_encode_streams call plus one decode batch per
 * cache, then the completions in call order. */
class Batcher {
public:
    // a job's completion: its output bytes (a view into the batch), and for a decode the status,
    // consumed bytes and the unknown hash
    using Done = std::function<bool(const uint8_t *, size_t, int, uint64_t, bool, uint64_t)>;
    struct Job {
        bool encode;
        const void *owner;
        const Cache *store;
        StreamEncoder *encoder;
        Bytes data;  // the read the consume deferred (owned until the turn ends)
        bool flush;
        Done done;
        DecodeFilter *dec;
    };

    void submit_encode(const void *owner, StreamEncoder *enc, const Cache *store, Bytes &&data, bool flush, Done done)
    {
        jobs_.push_back(Job{true, owner, store, enc, std::move(data), flush, std::move(done), nullptr});
    }
    void submit_decode(DecodeFilter *owner, const Cache *store, Done done)
    {
        jobs_.push_back(Job{false, owner, store, nullptr, Bytes(), false, std::move(done), owner});
    }
    bool pending(const void *owner) const
    {
        for (const Job &j : jobs_)
            if (j.owner == owner) return true;
        return false;
    }
    /* end of the turn: every deferred call; the filters that failed since the last run() */
    std::vector<const void *> run()
    {
        drain();
        std::vector<const void *> f;
        f.swap(failed_);
        return f;
    }
    inline void drain();
    bool failed(const void *owner) const { return failed_set_.count(owner) != 0; }
    uint64_t device_calls = 0;

private:
    inline void drain_round(std::vector<Job> &rnd);
    inline void fail_owner(const void *owner);
    std::vector<Job> jobs_;
    std::vector<const void *> failed_;
    std::set<const void *> failed_set_;
};

/* EncodeFilter::encode_frame (xcodec_filter.cc:189-203): one frame of at most 32768 bytes taken
 * from the front of src. */
inline void encode_frame(const uint8_t *&src, size_t &n, Bytes &trg)
{
    const size_t k = n < MAX_FRAME ? n : MAX_FRAME;
    trg.push_back(OP_FRAME);
    trg.push_back((uint8_t)(k >> 8));
    trg.push_back((uint8_t)k);
    trg.insert(trg.end(), src, src + k);
    src += k;
    n -= k;
}

/* xcodec_filter.h:25-57 / xcodec_filter.cc:122-216.  flg & 1: waiting mode. */
class EncodeFilter : public Filter {
public:
    EncodeFilter(Codec *codec, int flg = 0)
        : codec_(codec), cache_(codec ? codec->cache : nullptr), waiting_((flg & 1) != 0) { }

    bool consume(const uint8_t *p, size_t n, int flg = 0) override { return consume(Bytes(p, p + n), flg); }

    /* the read handed over (a proxy's read buffer: no copy when the call is deferred) */
    bool consume(Bytes &&buf, int flg = 0)
    {
        if (failed_ || (codec_->batcher && codec_->batcher->failed(this))) return false;
        auto output = std::make_shared<Bytes>();
        if (!encoder_) {
            if (!cache_ || cache_->uuid.size() != UUID_LEN) return false;  // "Could not encode UUID for <HELLO>."
            output->push_back(OP_HELLO);
            output->push_back((uint8_t)(UUID_LEN + 8));
            output->insert(output->end(), cache_->uuid.begin(), cache_->uuid.end());
            const uint64_t mb = cache_->size;  // host order (x86-64)
            output->insert(output->end(), (const uint8_t *)&mb, (const uint8_t *)&mb + 8);
            encoder_.reset(new StreamEncoder(*cache_->store));
        }
        const bool flush_now = !(flg & TO_BE_CONTINUED) && !waiting_;
        if (!(flg & TO_BE_CONTINUED) && waiting_) wait_armed_ = true;  // (re)start the timer
        auto done = [this, output, flg](const uint8_t *q, size_t k, int, uint64_t, bool, uint64_t) -> bool {
            output->reserve(output->size() + k + 3 * (k / MAX_FRAME + 1));
            while (k) encode_frame(q, k, *output);
            return output->empty() ? true : produce(*output, flg);
        };
        if (Batcher *b = codec_->batcher) {  // deferred to the end of the turn
            b->submit_encode(this, encoder_.get(), cache_->store.get(), std::move(buf), flush_now, done);
            return true;
        }
        // one device call: encode(buf) [+ flush()] (xc_encode_streams with one call)
        EncodedBatch eb;
        encode_streams({StreamCall{encoder_.get(), buf.data(), buf.size(), flush_now}}, eb);
        return done(eb.at(0), eb.len[0], 1, 0, false, 0);
    }

    void flush(int flg) override
    {
        drain();
        if (flg == OP_EOS_ACK) {
            eos_ack_ = true;
        } else {
            flushing_ = true;
            flush_flags_ |= flg;
            wait_armed_ = false;
            if (!sent_eos_) {
                Bytes enc, output;
                if (encoder_ && encoder_->flush(enc)) {
                    const uint8_t *q = enc.data();
                    size_t k = enc.size();
                    encode_frame(q, k, output);  // (one frame, as the reference)
                }
                output.push_back(OP_EOS);
                sent_eos_ = produce(output);
            }
        }
        if (flushing_ && eos_ack_) Filter::flush(flush_flags_);
    }

    /* EncodeFilter::on_read_timeout (xcodec_filter.cc:205-216): the waiting-mode flush */
    void on_read_timeout()
    {
        wait_armed_ = false;
        drain();
        Bytes enc;
        if (!flushing_ && encoder_ && encoder_->flush(enc)) {
            Bytes output;
            const uint8_t *q = enc.data();
            size_t k = enc.size();
            encode_frame(q, k, output);
            produce(output);
        }
    }
    bool wait_armed() const { return wait_armed_; }
    void fail() { failed_ = true; }

private:
    void drain()
    {
        if (codec_ && codec_->batcher) codec_->batcher->drain();
    }
    Codec *codec_;
    CodecCache *cache_;
    std::unique_ptr<StreamEncoder> encoder_;
    bool waiting_, wait_armed_ = false, sent_eos_ = false, eos_ack_ = false, flushing_ = false, failed_ = false;
    int flush_flags_ = 0;
};

/* xcodec_filter.h:59-86 / xcodec_filter.cc:220-526.  set_upstream names the filter that carries
 * <ASK>, <LEARN> and <EOS_ACK> back to the peer (the local EncodeFilter of the reverse direction). */
class DecodeFilter : public Filter {
public:
    explicit DecodeFilter(Codec *codec) : codec_(codec), encoder_cache_(codec ? codec->cache : nullptr) { }
    void set_upstream(Filter *f) { upstream_ = f; }

    bool consume(const uint8_t *p, size_t n, int flg = 0) override
    {
        if (!upstream_) return false;  // "Decoder not configured"
        if (failed_) return false;
        Batcher *b = codec_ ? codec_->batcher : nullptr;
        if (b) {
            if (b->failed(this)) return false;
            if (!received_eos_ && unknown_.empty() && !b->pending(this) && frames_only(p, n)) {
                // frames only: parse now, decode at the end of the turn in the device batch (the
                // frames of one consume decode in one call as they do one by one: the decoder keeps
                // a token that straddles frames, and stops at the first unknown REF)
                pending_.insert(pending_.end(), p, p + n);
                if (!parse(flg, true)) return false;
                if (!frame_buffer_.empty() && unknown_.empty())
                    b->submit_decode(this, decoder_cache_->store.get(),
                                     [this, flg](const uint8_t *o, size_t k, int st, uint64_t consumed, bool hu,
                                                 uint64_t unk) { return decoded(st != 0, o, k, consumed, hu, unk, flg); });
                return true;
            }
            b->drain();  // anything else runs now, after every earlier deferred call
            if (b->failed(this)) return false;
        }
        pending_.insert(pending_.end(), p, p + n);
        return parse(flg, false);
    }

    void flush(int flg) override
    {
        if (codec_ && codec_->batcher) codec_->batcher->drain();  // (a failure: the turn's run())
        flushing_ = true;
        flush_flags_ |= flg;
        if (!upflushed_ && upstream_) {
            upflushed_ = true;
            upstream_->flush(OP_EOS_ACK);
        }
        Filter::flush(flush_flags_);
    }

    Bytes &frame_buffer() { return frame_buffer_; }
    CodecCache *decoder_cache() { return decoder_cache_; }

private:
    friend class Batcher;

    // Whether pending + (p, n) holds only <HELLO> (first) and <FRAME> messages, the last one possibly
    // incomplete: such a consume changes nothing but the frame buffer before its decode.
    bool frames_only(const uint8_t *p, size_t n) const
    {
        Bytes d(pending_);
        d.insert(d.end(), p, p + n);
        size_t i = 0;
        while (i < d.size()) {
            if (d[i] == OP_FRAME) {
                if (d.size() - i < 3) return true;
                i += 3 + (((size_t)d[i + 1] << 8) | d[i + 2]);
            } else if (d[i] == OP_HELLO && i == 0 && !decoder_cache_) {
                if (d.size() - i < 2) return true;
                i += 2 + d[i + 1];
            } else {
                return false;
            }
        }
        return true;
    }

    // The part of the frame loop after XCodecDecoder::decode (xcodec_filter.cc:414-455).
    bool decoded(bool ok, const uint8_t *out, size_t n, uint64_t consumed, bool has_unknown, uint64_t unknown, int flg)
    {
        if (!ok) return false;  // "Decoder exiting with error."
        frame_buffer_.erase(frame_buffer_.begin(), frame_buffer_.begin() + (ptrdiff_t)consumed);
        if (has_unknown) unknown_.insert(unknown);
        if (n && !produce(out, n, flg)) return false;
        Bytes ask;
        for (uint64_t h : unknown_) {
            ask.push_back(OP_ASK);
            for (int k = 7; k >= 0; k--) ask.push_back((uint8_t)(h >> (8 * k)));
        }
        if (!ask.empty() && !upstream_->produce(ask)) return false;
        return true;
    }

    // The message loop (xcodec_filter.cc:232-455) over pending_ from its read offset; the bytes
    // taken go at the end (one erase per call, not one per message).
    bool parse(int flg, bool defer)
    {
        size_t at = 0;
        struct Trim {  // (every return path)
            Bytes &p;
            size_t &at;
            ~Trim() { p.erase(p.begin(), p.begin() + (ptrdiff_t)at); }
        } trim{pending_, at};
        while (at < pending_.size()) {
            const uint8_t *m = pending_.data() + at;
            const size_t avail = pending_.size() - at;
            const uint8_t op = m[0];
            if (op == OP_HELLO) {
                if (decoder_cache_) return false;  // "Got <HELLO> twice."
                if (avail < 2) return true;
                const size_t ln = m[1];
                if (avail < 2 + ln) return true;
                if (ln != UUID_LEN + 8) return false;  // "Unsupported <HELLO> length"
                const std::string uuid((const char *)m + 2, UUID_LEN);
                uint64_t mb = 0;
                std::memcpy(&mb, m + 2 + UUID_LEN, 8);
                at += 2 + ln;
                if (!valid_uuid(uuid)) return false;  // "Invalid UUID in <HELLO>."
                CacheRegistry *reg = codec_->registry;
                decoder_cache_ = reg->find_cache(uuid);
                if (!decoder_cache_) decoder_cache_ = reg->add_cache(mb, uuid);
                decoder_ = decoder_cache_ != nullptr;
            } else if (op == OP_ASK) {
                if (!encoder_cache_) return false;
                if (avail < 9) return true;
                uint64_t h = 0;
                for (int k = 1; k <= 8; k++) h = (h << 8) | m[k];
                at += 9;
                Bytes learn{OP_LEARN};
                if (!encoder_cache_->store->lookup(h, learn)) return false;  // "Unknown hash in <ASK>"
                if (!upstream_->produce(learn)) return false;
            } else if (op == OP_LEARN) {
                if (!decoder_cache_) return false;  // "Got <LEARN> before <HELLO>."
                if (avail < 1 + SEG) return true;
                const uint64_t h = hash_segment(codec_->registry->context(), m + 1);
                unknown_.erase(h);  // (else: a gratuitous <LEARN>)
                Bytes old;
                if (decoder_cache_->store->lookup(h, old)) {
                    if (std::memcmp(old.data(), m + 1, SEG) != 0) return false;  // "Collision in <LEARN>."
                } else {
                    decoder_cache_->store->enter(h, m + 1);
                }
                at += 1 + SEG;
            } else if (op == OP_EOS) {
                if (received_eos_) return false;  // "Duplicate <EOS>."
                at += 1;
                received_eos_ = true;
            } else if (op == OP_EOS_ACK) {
                if (received_eos_ack_) return false;  // "Duplicate <EOS_ACK>."
                at += 1;
                received_eos_ack_ = true;
            } else if (op == OP_FRAME) {
                if (!decoder_) return false;  // "Got frame data before decoder initialized."
                if (avail < 3) return true;
                const size_t ln = ((size_t)m[1] << 8) | m[2];
                if (ln == 0 || ln > MAX_FRAME) return false;  // "Invalid framed data length."
                if (avail < 3 + ln) return true;
                frame_buffer_.insert(frame_buffer_.end(), m + 3, m + 3 + ln);
                at += 3 + ln;
            } else {
                return false;  // "Unsupported operation in pipe stream."
            }
            if (frame_buffer_.empty() || !unknown_.empty() || defer) continue;
            Bytes out;
            Decoder dec(*decoder_cache_->store);
            Bytes in(frame_buffer_);
            std::set<uint64_t> unk;
            const bool ok = dec.decode(out, in, unk);
            const uint64_t consumed = frame_buffer_.size() - in.size();
            if (!decoded(ok, out.data(), out.size(), consumed, !unk.empty(), unk.empty() ? 0 : *unk.begin(), flg))
                return false;
        }
        if (received_eos_ && !sent_eos_ack_ && frame_buffer_.empty()) {
            sent_eos_ack_ = true;
            const uint8_t a = OP_EOS_ACK;
            if (!upstream_->produce(&a, 1)) return false;
        }
        if (received_eos_ && !flushing_) {
            if (unknown_.empty()) {
                if (!frame_buffer_.empty()) return false;
                flushing_ = true;
                Filter::flush(0);
            } else if (frame_buffer_.empty()) {
                return false;
            }
        }
        if (sent_eos_ack_ && received_eos_ack_ && !upflushed_) {
            upflushed_ = true;
            upstream_->flush(OP_EOS_ACK);
        }
        return true;
    }

    static bool valid_uuid(const std::string &u)
    {
        if (u.size() != UUID_LEN) return false;
        for (size_t i = 0; i < u.size(); i++) {
            const char c = u[i];
            if (i == 8 || i == 13 || i == 18 || i == 23) {
                if (c != '-') return false;
            } else if (!((c >= '0' && c <= '9') || (c >= 'a' && c <= 'f') || (c >= 'A' && c <= 'F'))) {
                return false;
            }
        }
        return true;
    }

    Codec *codec_;
    CodecCache *encoder_cache_;
    CodecCache *decoder_cache_ = nullptr;
    bool decoder_ = false;
    std::set<uint64_t> unknown_;
    Bytes frame_buffer_, pending_;
    bool received_eos_ = false, sent_eos_ack_ = false, received_eos_ack_ = false, upflushed_ = false,
         flushing_ = false, failed_ = false;
    int flush_flags_ = 0;
    Filter *upstream_ = nullptr;
};

inline void Batcher::drain()
{
    while (!jobs_.empty()) {
        size_t r = 0;
        std::set<const void *> owners;
        std::set<const Cache *> enc_stores, dec_stores;
        for (; r < jobs_.size(); r++) {
            const Job &j = jobs_[r];
            if (owners.count(j.owner)) break;
            if ((j.encode && dec_stores.count(j.store)) || (!j.encode && enc_stores.count(j.store))) break;
            owners.insert(j.owner);
            (j.encode ? enc_stores : dec_stores).insert(j.store);
        }
        std::vector<Job> rnd(std::make_move_iterator(jobs_.begin()), std::make_move_iterator(jobs_.begin() + (ptrdiff_t)r));
        jobs_.erase(jobs_.begin(), jobs_.begin() + (ptrdiff_t)r);
        try {
            drain_round(rnd);
        } catch (...) {
            // a library error: the device state of this round's encoders is unknown, so every filter
            // of the round and of the jobs still deferred fails (its next consume refuses, as the
            // reference's failing consume ends the connection); the caller sees the error
            for (const Job &j : rnd) fail_owner(j.owner);
            for (const Job &j : jobs_) fail_owner(j.owner);
            jobs_.clear();
            throw;
        }
    }
}

inline void Batcher::fail_owner(const void *owner)
{
    if (failed_set_.insert(owner).second) failed_.push_back(owner);
}

inline void Batcher::drain_round(std::vector<Job> &rnd)
{
    const size_t r = rnd.size();
    {
        std::vector<const uint8_t *> op(r, nullptr);
        std::vector<size_t> on(r, 0);
        std::vector<int> st(r, 1);
        std::vector<uint64_t> cons(r, 0), unk(r, 0);
        std::vector<char> hu(r, 0);
        std::vector<StreamCall> calls;
        std::vector<size_t> eidx;
        for (size_t k = 0; k < r; k++)
            if (rnd[k].encode) {
                calls.push_back({rnd[k].encoder, rnd[k].data.data(), rnd[k].data.size(), rnd[k].flush});
                eidx.push_back(k);
            }
        EncodedBatch eb;
        if (!calls.empty()) {
            encode_streams(calls, eb);
            device_calls++;
            for (size_t i = 0; i < eidx.size(); i++) {
                op[eidx[i]] = eb.at(i);
                on[eidx[i]] = eb.len[i];
            }
        }
        // one decode batch per cache: stream k is XCodecDecoder::decode of its frame buffer
        std::map<const Cache *, std::vector<size_t>> by_store;
        std::vector<std::unique_ptr<uint8_t[]>> douts;
        for (size_t k = 0; k < r; k++)
            if (!rnd[k].encode) by_store[rnd[k].store].push_back(k);
        for (auto &kv : by_store) {
            const std::vector<size_t> &ks = kv.second;
            const size_t m = ks.size();
            std::vector<uint64_t> ioff(m), ilen(m), ooff(m), ocap(m), olen(m), c(m), u(m);
            std::vector<int32_t> s(m), h(m);
            uint64_t isz = 0, osz = 0;
            for (size_t i = 0; i < m; i++) {
                const Bytes &fb = rnd[ks[i]].dec->frame_buffer();
                ioff[i] = isz;
                ilen[i] = fb.size();
                isz += fb.size();
                ooff[i] = osz;
                ocap[i] = decode_bound(fb.data(), fb.size());
                osz += ocap[i];
            }
            std::unique_ptr<uint8_t[]> in(new uint8_t[isz ? isz : 1]), out(new uint8_t[osz ? osz : 1]);
            for (size_t i = 0; i < m; i++) {
                const Bytes &fb = rnd[ks[i]].dec->frame_buffer();
                if (!fb.empty()) std::memcpy(in.get() + ioff[i], fb.data(), fb.size());
            }
            check(xc_decode_batch_host(const_cast<Cache *>(kv.first)->get(), in.get(), ioff.data(), ilen.data(), m,
                                       out.get(), ooff.data(), ocap.data(), olen.data(), c.data(), s.data(),
                                       u.data(), h.data()));
            device_calls++;
            for (size_t i = 0; i < m; i++) {
                const size_t k = ks[i];
                op[k] = out.get() + ooff[i];
                on[k] = olen[i];
                st[k] = s[i];
                cons[k] = c[i];
                hu[k] = h[i] != 0;
                unk[k] = u[i];
            }
            douts.push_back(std::move(out));
        }
        for (size_t k = 0; k < r; k++)
            if (!rnd[k].done(op[k], on[k], st[k], cons[k], hu[k] != 0, unk[k])) fail_owner(rnd[k].owner);
    }
}

}  // namespace pipe
}  // namespace xchip
