/*
 * xc_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference XCodec hot path (bramfeld/wanproxy,
 * xcodec/).  It is the checker for the HIP path: only tests/, the smoke()
 * entry point and bench.py's cpu_baseline leg may load it.  Nothing in
 * wanproxy_amd/ links or calls it.
 *
 * Pinning: the hash is checked against the reference's own 256 KATs
 * (xcodec/test/xcodec-hash1/xcodec-hash1.cc:34-291) and against the
 * reference XCodecHash class compiled from its header (oracle/Makefile,
 * target _ref/libxcref_hash.so).  The encoder / decoder restatement is pinned
 * by the reference's char-run round-trip intent
 * (xcodec/test/xcodec-encode-decode1/xcodec-encode-decode1.cc:38-105) and the
 * survey-time reference measurements; the reference
 * encoder/decoder TUs themselves are unbuildable here (they need
 * <uuid/uuid.h>, absent from this image) — see DESIGN.md "Oracle".
 */
#ifndef XC_ORACLE_H
#define XC_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define XO_SEGMENT_LENGTH 2048 /* xcodec/xcodec.h:78 */
#define XO_MAGIC 0xF1          /* xcodec/xcodec.h:39 */
#define XO_OP_ESCAPE 0x00      /* xcodec/xcodec.h:49 */
#define XO_OP_EXTRACT 0x01     /* xcodec/xcodec.h:63 */
#define XO_OP_REF 0x02         /* xcodec/xcodec.h:76 */

/* Hash of one full 2048-byte segment (xcodec/xcodec_hash.h:166-174). */
uint64_t xo_hash_segment(const uint8_t *seg);

/* Rolling hash at every window end p >= 2047 of data[0..n): out[p] = H(data[p-2047..p]);
 * out[p] for p < 2047 is set to 0.  Follows add/roll/mix (xcodec/xcodec_hash.h:93-164). */
void xo_window_hashes(const uint8_t *data, size_t n, uint64_t *out);

/* XCodecMemoryCache (xcodec/xcodec_cache.h:162-211) with the 64-entry recent window
 * (xcodec/xcodec_cache.h:94-98,128-158). */
typedef struct xo_cache xo_cache;
xo_cache *xo_cache_new(void);
xo_cache *xo_cache_clone(const xo_cache *c);
void xo_cache_free(xo_cache *c);
size_t xo_cache_count(const xo_cache *c);
/* Returns 1 and sets *data when present. */
int xo_cache_lookup(xo_cache *c, uint64_t h, const uint8_t **data);
void xo_cache_enter(xo_cache *c, uint64_t h, const uint8_t *seg);
/* i-th entered (hash, segment) pair, insertion order. */
int xo_cache_entry(const xo_cache *c, size_t i, uint64_t *h, uint8_t *seg);

/* XCodecCacheCOSS (xcodec/cache/coss/xcodec_cache_coss.{h,cc}): oracle/xc_coss.c.  The file is
 * <dir>/<uuid>.wpc; size_mb 0 = 1024. */
typedef struct xo_coss xo_coss;
xo_coss *xo_coss_open(const char *dir, const char *uuid, uint64_t size_mb);
void xo_coss_close(xo_coss *c);
void xo_coss_enter(xo_coss *c, uint64_t h, const uint8_t *seg);
int xo_coss_lookup(xo_coss *c, uint64_t h, const uint8_t **data);
size_t xo_coss_count(const xo_coss *c);
uint64_t xo_coss_load_misses(const xo_coss *c);
void xo_coss_stats(const xo_coss *c, uint64_t *out);
size_t xo_coss_hashes(const xo_coss *c, uint64_t *out, size_t cap);
/* An xo_cache whose lookup / enter are the COSS cache's (the encoder and decoder take it like
 * the memory cache).  xo_cache_free closes the COSS cache (its destructor's stores). */
xo_cache *xo_cache_new_coss(const char *dir, const char *uuid, uint64_t size_mb);

/* XCodecEncoder (xcodec/xcodec_encoder.{h,cc}). Output is appended to a growable byte vector. */
typedef struct {
    uint8_t *data;
    size_t len, cap;
} xo_bytes;
void xo_bytes_free(xo_bytes *b);

typedef struct xo_encoder xo_encoder;
xo_encoder *xo_encoder_new(xo_cache *c);
void xo_encoder_free(xo_encoder *e);
size_t xo_encoder_pending(const xo_encoder *e);
void xo_encode(xo_encoder *e, const uint8_t *in, size_t n, xo_bytes *out);
int xo_flush(xo_encoder *e, xo_bytes *out);

/* XCodecDecoder::decode (xcodec/xcodec_decoder.cc:76-176).  Consumes from in[0..n);
 * *consumed = bytes the reference would have removed from its input Buffer.
 * Returns 1 (true) or 0 (false).  On an unknown REF, *unknown = hash and *has_unknown = 1. */
int xo_decode(xo_cache *c, const uint8_t *in, size_t n, size_t *consumed, xo_bytes *out,
              uint64_t *unknown, int *has_unknown);

/* Batch helpers for ctypes: every buffer is one encode()+flush() on a fresh encoder against
 * the shared cache, buffers in index order.  out must have room for out_cap[i] bytes at out_off[i].
 * Returns 0, or -1 if an output did not fit. */
int xo_encode_batch(xo_cache *c, const uint8_t *in, const uint64_t *in_off, const uint64_t *in_len,
                    size_t nb, uint8_t *out, const uint64_t *out_off, const uint64_t *out_cap,
                    uint64_t *out_len);
/* Every stream is one decode() call against the shared cache, streams in index order. */
int xo_decode_batch(xo_cache *c, const uint8_t *in, const uint64_t *in_off, const uint64_t *in_len,
                    size_t nb, uint8_t *out, const uint64_t *out_off, const uint64_t *out_cap,
                    uint64_t *out_len, uint64_t *consumed, int32_t *status, uint64_t *unknown,
                    int32_t *has_unknown);

/* Multi-threaded encode baseline: buffer i goes to thread i % nthreads, each thread with a
 * private clone of `c` (mirrors the per-GPU caches of the sharded bench).  Returns seconds. */
double xo_encode_sharded_timed(const xo_cache *c, const uint8_t *in, const uint64_t *in_off,
                               const uint64_t *in_len, size_t nb, int nthreads,
                               uint64_t *total_out);

#ifdef __cplusplus
}
#endif
#endif
