/*
 * xc_oracle.c — TEST INFRASTRUCTURE ONLY (see xc_oracle.h).
 *
 * Plain-C restatement of the reference XCodec encoder, decoder, hash and memory
 * cache.  Each function cites the reference lines it follows.  It is a checker:
 * the HIP product path (wanproxy_amd/) never links or calls this file.
 */
#define _GNU_SOURCE
#include "xc_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#define SEG XO_SEGMENT_LENGTH

/* ---------------------------------------------------------------- hash ---
 * xcodec/xcodec_hash.h:32-71 (RollingHash) and :93-164 (add/roll/reset/mix). */
typedef struct {
    uint32_t sum1, sum2;
    uint32_t ring[SEG];
} xo_rolling;

typedef struct {
    xo_rolling bytes, bits;
    unsigned start;
} xo_hash;

static unsigned xo_ffs8(uint8_t ch) { return ch ? (unsigned)__builtin_ctz(ch) + 1u : 0u; }

static void rolling_add(xo_rolling *r, uint32_t ch, unsigned start)
{ /* xcodec_hash.h:43-49 */
    r->ring[start] = ch;
    r->sum1 += ch;
    r->sum2 += r->sum1;
}

static void rolling_roll(xo_rolling *r, uint32_t ch, unsigned start)
{ /* xcodec_hash.h:57-70 */
    uint32_t dead = r->ring[start];
    r->sum1 -= dead;
    r->sum2 -= dead * SEG;
    r->ring[start] = ch;
    r->sum1 += ch;
    r->sum2 += r->sum1;
}

static void hash_reset(xo_hash *h)
{ /* xcodec_hash.h:111-120 */
    h->bytes.sum1 = h->bytes.sum2 = 0;
    h->bits.sum1 = h->bits.sum2 = 0;
    h->start = 0;
}

static void hash_add(xo_hash *h, uint8_t ch)
{ /* xcodec_hash.h:93-109: word = byte + 1, bit = ffs(byte) */
    rolling_add(&h->bytes, (uint32_t)ch + 1u, h->start);
    rolling_add(&h->bits, xo_ffs8(ch), h->start);
    h->start = (h->start + 1) % SEG;
}

static void hash_roll(xo_hash *h, uint8_t ch)
{ /* xcodec_hash.h:122-135 */
    rolling_roll(&h->bytes, (uint32_t)ch + 1u, h->start);
    rolling_roll(&h->bits, xo_ffs8(ch), h->start);
    h->start = (h->start + 1) % SEG;
}

static uint64_t hash_mix(const xo_hash *h)
{ /* xcodec_hash.h:155-164: the shifts are done in uint32 before widening. */
    uint64_t bits_hash = (uint32_t)((h->bits.sum1 << 16) + h->bits.sum2);
    uint64_t bytes_hash = (uint32_t)((h->bytes.sum1 << 20) + h->bytes.sum2);
    return (bits_hash << 36) + bytes_hash;
}

uint64_t xo_hash_segment(const uint8_t *seg)
{ /* xcodec_hash.h:166-174 */
    xo_hash *h = (xo_hash *)calloc(1, sizeof *h);
    for (unsigned i = 0; i < SEG; i++) hash_add(h, seg[i]);
    uint64_t r = hash_mix(h);
    free(h);
    return r;
}

void xo_window_hashes(const uint8_t *data, size_t n, uint64_t *out)
{
    xo_hash *h = (xo_hash *)calloc(1, sizeof *h);
    for (size_t p = 0; p < n; p++) {
        if (p < SEG) hash_add(h, data[p]);
        else hash_roll(h, data[p]);
        out[p] = p + 1 >= SEG ? hash_mix(h) : 0;
    }
    free(h);
}

/* --------------------------------------------------------------- cache ---
 * XCodecMemoryCache: hash_map<Hash64, uint8_t*> (xcodec_cache.h:162-211), identity hash
 * (:76-86), no eviction; plus the base class's 64-entry recent window (:94-98,128-158). */
#define XO_WINDOW_COUNT 64 /* xcodec_cache.h:48 */

struct xo_cache {
    uint64_t *keys;  /* open addressing, EMPTY marked by idx == UINT32_MAX */
    uint32_t *idx;
    size_t mask, count; /* count: segments stored (every enter) */
    size_t nkeys;       /* the map's size (a hash entered twice counts once) */
    uint64_t *seg_hash; /* insertion order */
    uint8_t *segs;
    size_t seg_cap;
    struct {
        uint64_t hash;
        const uint8_t *data;
        size_t slot; /* segment index the pointer refers to (stable across realloc) */
    } window[XO_WINDOW_COUNT];
    unsigned cursor;
    xo_coss *coss; /* non-null: XCodecCacheCOSS instead of the memory cache */
};

static size_t slot_of(uint64_t h, size_t mask) { return (size_t)((h * 0x9E3779B97F4A7C15ull) >> 17) & mask; }

static void cache_rehash(xo_cache *c, size_t newsize)
{
    uint64_t *ok = c->keys;
    uint32_t *oi = c->idx;
    size_t omask = c->mask;
    c->keys = (uint64_t *)malloc(newsize * sizeof(uint64_t));
    c->idx = (uint32_t *)malloc(newsize * sizeof(uint32_t));
    memset(c->idx, 0xff, newsize * sizeof(uint32_t));
    c->mask = newsize - 1;
    if (ok) {
        for (size_t i = 0; i <= omask; i++) {
            if (oi[i] == UINT32_MAX) continue;
            size_t s = slot_of(ok[i], c->mask);
            while (c->idx[s] != UINT32_MAX) s = (s + 1) & c->mask;
            c->keys[s] = ok[i];
            c->idx[s] = oi[i];
        }
        free(ok);
        free(oi);
    }
}

xo_cache *xo_cache_new(void)
{
    xo_cache *c = (xo_cache *)calloc(1, sizeof *c);
    cache_rehash(c, 1024);
    return c;
}

xo_cache *xo_cache_clone(const xo_cache *s)
{
    xo_cache *c = (xo_cache *)calloc(1, sizeof *c);
    *c = *s;
    c->keys = (uint64_t *)malloc((s->mask + 1) * sizeof(uint64_t));
    c->idx = (uint32_t *)malloc((s->mask + 1) * sizeof(uint32_t));
    memcpy(c->keys, s->keys, (s->mask + 1) * sizeof(uint64_t));
    memcpy(c->idx, s->idx, (s->mask + 1) * sizeof(uint32_t));
    c->seg_hash = (uint64_t *)malloc((s->seg_cap ? s->seg_cap : 1) * sizeof(uint64_t));
    c->segs = (uint8_t *)malloc((s->seg_cap ? s->seg_cap : 1) * SEG);
    if (s->count) {
        memcpy(c->seg_hash, s->seg_hash, s->count * sizeof(uint64_t));
        memcpy(c->segs, s->segs, s->count * SEG);
    }
    for (int i = 0; i < XO_WINDOW_COUNT; i++)
        c->window[i].data = s->window[i].data ? c->segs + s->window[i].slot * SEG : NULL;
    return c;
}

xo_cache *xo_cache_new_coss(const char *dir, const char *uuid, uint64_t size_mb)
{
    xo_cache *c = xo_cache_new();
    c->coss = xo_coss_open(dir, uuid, size_mb);
    return c;
}

void xo_cache_free(xo_cache *c)
{
    if (!c) return;
    if (c->coss) xo_coss_close(c->coss);
    free(c->keys);
    free(c->idx);
    free(c->seg_hash);
    free(c->segs);
    free(c);
}

/* The map's entries (segment_hash_map_.size(), xcodec_cache.h:164). */
size_t xo_cache_count(const xo_cache *c) { return c->coss ? xo_coss_count(c->coss) : c->nkeys; }
size_t xo_cache_segments(const xo_cache *c) { return c->coss ? xo_coss_count(c->coss) : c->count; }

/* COSSStats of a COSS cache (xcodec_cache_coss.h:179-187); 0 for the memory cache. */
/* (checks only) lookups that loaded a stripe and then missed: the <=16-stripe second-copy state */
uint64_t xo_cache_coss_load_misses(const xo_cache *c) { return c->coss ? xo_coss_load_misses(c->coss) : 0; }

int xo_cache_coss_stats(const xo_cache *c, uint64_t *out6)
{
    if (!c->coss) return 0;
    xo_coss_stats(c->coss, out6);
    return 1;
}

static long cache_find(const xo_cache *c, uint64_t h)
{
    size_t s = slot_of(h, c->mask);
    while (c->idx[s] != UINT32_MAX) {
        if (c->keys[s] == h) return (long)c->idx[s];
        s = (s + 1) & c->mask;
    }
    return -1;
}

int xo_cache_lookup(xo_cache *c, uint64_t h, const uint8_t **data)
{ /* xcodec_cache.h:190-210 */
    if (c->coss) return xo_coss_lookup(c->coss, h, data);
    for (int i = 0; i < XO_WINDOW_COUNT; i++) { /* find_recent, :137-147: the first entry with */
        if (c->window[i].hash == h) {           /* the hash (an unused slot: hash 0, no data) */
            if (!c->window[i].data) break;
            *data = c->window[i].data;
            return 1;
        }
    }
    long k = cache_find(c, h);
    if (k < 0) return 0;
    *data = c->segs + (size_t)k * SEG;
    /* remember, :130-135 */
    c->window[c->cursor].hash = h;
    c->window[c->cursor].data = *data;
    c->window[c->cursor].slot = (size_t)k;
    c->cursor = (c->cursor + 1) & (XO_WINDOW_COUNT - 1);
    return 1;
}

void xo_cache_enter(xo_cache *c, uint64_t h, const uint8_t *seg)
{ /* xcodec_cache.h:182-188.  A duplicate enter is an assert in the reference; release
   * builds overwrite the map value, which is what we do. */
    if (c->coss) {
        xo_coss_enter(c->coss, h, seg);
        return;
    }
    long k = cache_find(c, h);
    if (c->count == c->seg_cap) {
        size_t nc = c->seg_cap ? c->seg_cap * 2 : 1024;
        c->seg_hash = (uint64_t *)realloc(c->seg_hash, nc * sizeof(uint64_t));
        c->segs = (uint8_t *)realloc(c->segs, nc * SEG);
        c->seg_cap = nc;
        for (int i = 0; i < XO_WINDOW_COUNT; i++)
            if (c->window[i].data) c->window[i].data = c->segs + c->window[i].slot * SEG;
    }
    size_t id = c->count++;
    c->seg_hash[id] = h;
    memcpy(c->segs + id * SEG, seg, SEG);
    if (k >= 0) {
        size_t s = slot_of(h, c->mask);
        while (c->keys[s] != h || c->idx[s] == UINT32_MAX) s = (s + 1) & c->mask;
        c->idx[s] = (uint32_t)id;
        return;
    }
    c->nkeys++;
    if ((c->count) * 2 > c->mask + 1) cache_rehash(c, (c->mask + 1) * 2);
    size_t s = slot_of(h, c->mask);
    while (c->idx[s] != UINT32_MAX) s = (s + 1) & c->mask;
    c->keys[s] = h;
    c->idx[s] = (uint32_t)id;
}

int xo_cache_entry(const xo_cache *c, size_t i, uint64_t *h, uint8_t *seg)
{
    if (i >= c->count) return -1;
    *h = c->seg_hash[i];
    if (seg) memcpy(seg, c->segs + i * SEG, SEG);
    return 0;
}

/* --------------------------------------------------------------- bytes --- */
static void bytes_reserve(xo_bytes *b, size_t extra)
{
    if (b->len + extra <= b->cap) return;
    size_t nc = b->cap ? b->cap : 4096;
    while (nc < b->len + extra) nc *= 2;
    b->data = (uint8_t *)realloc(b->data, nc);
    b->cap = nc;
}

static void bytes_put(xo_bytes *b, const uint8_t *p, size_t n)
{
    if (!n) return;
    bytes_reserve(b, n);
    memcpy(b->data + b->len, p, n);
    b->len += n;
}

static void bytes_put1(xo_bytes *b, uint8_t v) { bytes_put(b, &v, 1); }

void xo_bytes_free(xo_bytes *b)
{
    free(b->data);
    b->data = NULL;
    b->len = b->cap = 0;
}

/* ------------------------------------------------------------- encoder ---
 * State: xcodec_encoder.h:45-50 (source_, xcodec_hash_, candidate_start_, candidate_symbol_).
 * source_ is kept as a byte vector plus a read offset (Buffer::skip == advance). */
struct xo_encoder {
    xo_cache *cache;
    xo_bytes src;
    size_t src_head; /* bytes skipped from the front of src */
    xo_hash hash;
    int cand;
    uint64_t cand_sym;
};

xo_encoder *xo_encoder_new(xo_cache *c)
{ /* xcodec_encoder.cc:22-28 */
    xo_encoder *e = (xo_encoder *)calloc(1, sizeof *e);
    e->cache = c;
    e->cand = -1;
    return e;
}

/* Bytes pending in source_ (XCodecEncoder's state between calls, xcodec_encoder.h:45-50). */
size_t xo_encoder_pending(const xo_encoder *e) { return e->src.len - e->src_head; }

void xo_encoder_free(xo_encoder *e)
{
    if (!e) return;
    xo_bytes_free(&e->src);
    free(e);
}

static size_t src_len(const xo_encoder *e) { return e->src.len - e->src_head; }
static const uint8_t *src_ptr(const xo_encoder *e) { return e->src.data + e->src_head; }

static void src_skip(xo_encoder *e, size_t n)
{
    e->src_head += n;
    if (e->src_head == e->src.len) e->src_head = e->src.len = 0;
}

static void encode_escape(xo_encoder *e, xo_bytes *out, size_t length)
{ /* xcodec_encoder.cc:217-239: emit runs, each 0xF1 as F1 00 */
    while (length > 0) {
        const uint8_t *p = src_ptr(e);
        const uint8_t *m = (const uint8_t *)memchr(p, XO_MAGIC, length);
        if (m) {
            size_t pos = (size_t)(m - p);
            bytes_put(out, p, pos);
            bytes_put1(out, XO_MAGIC);
            bytes_put1(out, XO_OP_ESCAPE);
            src_skip(e, pos + 1);
            length -= pos + 1;
        } else {
            bytes_put(out, p, length);
            src_skip(e, length);
            break;
        }
    }
}

static void encode_declaration(xo_encoder *e, xo_bytes *out, unsigned start, uint64_t h)
{ /* xcodec_encoder.cc:203-215 */
    if (start > 0) encode_escape(e, out, start);
    xo_cache_enter(e->cache, h, src_ptr(e));
    bytes_put1(out, XO_MAGIC);
    bytes_put1(out, XO_OP_EXTRACT);
    bytes_put(out, src_ptr(e), SEG);
    src_skip(e, SEG);
}

static int encode_reference(xo_encoder *e, xo_bytes *out, unsigned start, uint64_t h,
                            const uint8_t *old)
{ /* xcodec_encoder.cc:241-260 */
    if (memcmp(old, src_ptr(e) + start, SEG) != 0) return 0;
    if (start > 0) encode_escape(e, out, start);
    bytes_put1(out, XO_MAGIC);
    bytes_put1(out, XO_OP_REF);
    for (int i = 7; i >= 0; i--) bytes_put1(out, (uint8_t)(h >> (8 * i))); /* BigEndian */
    src_skip(e, SEG);
    return 1;
}

void xo_encode(xo_encoder *e, const uint8_t *in, size_t n, xo_bytes *out)
{ /* xcodec_encoder.cc:60-173 */
    int off = (int)src_len(e);
    /* source_.append(input): compact first so src_ptr stays contiguous */
    if (e->src_head) {
        memmove(e->src.data, e->src.data + e->src_head, src_len(e));
        e->src.len -= e->src_head;
        e->src_head = 0;
    }
    bytes_put(&e->src, in, n);
    for (size_t i = 0; i < n; i++) {
        uint8_t ch = in[i];
        if (++off < SEG) {
            hash_add(&e->hash, ch);
            continue;
        }
        if (off == SEG) hash_add(&e->hash, ch);
        else hash_roll(&e->hash, ch);
        uint64_t h = hash_mix(&e->hash);

        if (e->cand >= 0 && e->cand + SEG * 2 <= off) { /* :77-82 */
            encode_declaration(e, out, (unsigned)e->cand, e->cand_sym);
            off -= e->cand + SEG;
            e->cand = -1;
        }
        const uint8_t *old;
        if (xo_cache_lookup(e->cache, h, &old)) { /* :89-118 */
            if (encode_reference(e, out, (unsigned)(off - SEG), h, old)) {
                off = 0;
                hash_reset(&e->hash);
                e->cand = -1;
            } /* else: collision, nothing */
        } else if (e->cand < 0) { /* :119-147 */
            e->cand = off - SEG;
            e->cand_sym = h;
        }
    }
}

int xo_flush(xo_encoder *e, xo_bytes *out)
{ /* xcodec_encoder.cc:175-201 */
    int vld = 0;
    if (e->cand >= 0) {
        encode_declaration(e, out, (unsigned)e->cand, e->cand_sym);
        e->cand = -1;
        vld = 1;
    }
    if (src_len(e) > 0) {
        encode_escape(e, out, src_len(e));
        vld = 1;
    }
    hash_reset(&e->hash);
    return vld;
}

/* ------------------------------------------------------------- decoder --- */
int xo_decode(xo_cache *c, const uint8_t *in, size_t n, size_t *consumed, xo_bytes *out,
              uint64_t *unknown, int *has_unknown)
{ /* xcodec_decoder.cc:76-176 */
    size_t pos = 0;
    int ret = 1;
    *has_unknown = 0;
    while (pos < n) {
        const uint8_t *m = (const uint8_t *)memchr(in + pos, XO_MAGIC, n - pos);
        if (!m) { /* :87-90 moveout */
            bytes_put(out, in + pos, n - pos);
            pos = n;
            break;
        }
        size_t off = (size_t)(m - (in + pos));
        bytes_put(out, in + pos, off); /* :92-96 */
        pos += off;
        if (n - pos == 1) break; /* :102-103 */
        uint8_t op = in[pos + 1];
        if (op == XO_OP_ESCAPE) { /* :109-112 */
            bytes_put1(out, XO_MAGIC);
            pos += 2;
        } else if (op == XO_OP_EXTRACT) { /* :114-140 */
            if (n - pos < 2 + SEG) break;
            pos += 2;
            const uint8_t *data = in + pos;
            uint64_t h = xo_hash_segment(data);
            const uint8_t *old;
            if (xo_cache_lookup(c, h, &old)) {
                if (memcmp(old, data, SEG) != 0) { ret = 0; break; } /* collision */
            } else {
                xo_cache_enter(c, h, data);
            }
            bytes_put(out, data, SEG);
            pos += SEG;
        } else if (op == XO_OP_REF) { /* :142-166 */
            if (n - pos < 10) break;
            uint64_t h = 0;
            for (int i = 0; i < 8; i++) h = (h << 8) | in[pos + 2 + i];
            const uint8_t *old;
            if (xo_cache_lookup(c, h, &old)) {
                bytes_put(out, old, SEG);
                pos += 10;
            } else {
                *unknown = h;
                *has_unknown = 1;
                break;
            }
        } else { /* :168-171 */
            ret = 0;
            break;
        }
    }
    *consumed = pos;
    return ret;
}

/* --------------------------------------------------------------- batch --- */
int xo_encode_batch(xo_cache *c, const uint8_t *in, const uint64_t *in_off, const uint64_t *in_len,
                    size_t nb, uint8_t *out, const uint64_t *out_off, const uint64_t *out_cap,
                    uint64_t *out_len)
{
    int rc = 0;
    xo_bytes o = {0, 0, 0};
    for (size_t i = 0; i < nb; i++) {
        xo_encoder *e = xo_encoder_new(c);
        o.len = 0;
        xo_encode(e, in + in_off[i], in_len[i], &o);
        xo_flush(e, &o);
        xo_encoder_free(e);
        out_len[i] = o.len;
        if (o.len > out_cap[i]) { rc = -1; continue; }
        memcpy(out + out_off[i], o.data, o.len);
    }
    xo_bytes_free(&o);
    return rc;
}

int xo_decode_batch(xo_cache *c, const uint8_t *in, const uint64_t *in_off, const uint64_t *in_len,
                    size_t nb, uint8_t *out, const uint64_t *out_off, const uint64_t *out_cap,
                    uint64_t *out_len, uint64_t *consumed, int32_t *status, uint64_t *unknown,
                    int32_t *has_unknown)
{
    int rc = 0;
    xo_bytes o = {0, 0, 0};
    for (size_t i = 0; i < nb; i++) {
        size_t cons = 0;
        int hu = 0;
        uint64_t u = 0;
        o.len = 0;
        status[i] = xo_decode(c, in + in_off[i], in_len[i], &cons, &o, &u, &hu);
        consumed[i] = cons;
        unknown[i] = u;
        has_unknown[i] = hu;
        out_len[i] = o.len;
        if (o.len > out_cap[i]) { rc = -1; continue; }
        memcpy(out + out_off[i], o.data, o.len);
    }
    xo_bytes_free(&o);
    return rc;
}

typedef struct {
    const xo_cache *base;
    const uint8_t *in;
    const uint64_t *in_off, *in_len;
    size_t nb;
    int tid, nthreads;
    uint64_t out_bytes;
} shard_job;

static void *shard_main(void *arg)
{
    shard_job *j = (shard_job *)arg;
    xo_cache *c = xo_cache_clone(j->base);
    xo_bytes o = {0, 0, 0};
    for (size_t i = (size_t)j->tid; i < j->nb; i += (size_t)j->nthreads) {
        xo_encoder *e = xo_encoder_new(c);
        o.len = 0;
        xo_encode(e, j->in + j->in_off[i], j->in_len[i], &o);
        xo_flush(e, &o);
        xo_encoder_free(e);
        j->out_bytes += o.len;
    }
    xo_bytes_free(&o);
    xo_cache_free(c);
    return NULL;
}

double xo_encode_sharded_timed(const xo_cache *c, const uint8_t *in, const uint64_t *in_off,
                               const uint64_t *in_len, size_t nb, int nthreads,
                               uint64_t *total_out)
{
    if (nthreads < 1) nthreads = 1;
    pthread_t *th = (pthread_t *)calloc((size_t)nthreads, sizeof(pthread_t));
    shard_job *jobs = (shard_job *)calloc((size_t)nthreads, sizeof(shard_job));
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (int t = 0; t < nthreads; t++) {
        jobs[t] = (shard_job){c, in, in_off, in_len, nb, t, nthreads, 0};
        pthread_create(&th[t], NULL, shard_main, &jobs[t]);
    }
    uint64_t tot = 0;
    for (int t = 0; t < nthreads; t++) {
        pthread_join(th[t], NULL);
        tot += jobs[t].out_bytes;
    }
    clock_gettime(CLOCK_MONOTONIC, &t1);
    if (total_out) *total_out = tot;
    free(th);
    free(jobs);
    return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}
