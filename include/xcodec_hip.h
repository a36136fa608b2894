/*
 * xcodec_hip.h — C ABI of the MI355X-native XCodec codec (libxcodec_hip.so).
 *
 * Plain C: opaque handles, plain pointers and sizes, int status (0 = ok,
 * negative errno-style on failure).  No exceptions cross this boundary and
 * no torch / HIP types appear in the signatures (streams are passed as void*,
 * NULL = the context's own stream).
 *
 * Each entry point names the reference interface it replaces
 * (bramfeld/wanproxy, file:line).  INTEGRATION.md shows the reference-side
 * binding (the C++ facade a maintainer drops under xcodec/).
 *
 * Semantics are the reference's, bit for bit: a batch is processed as if its
 * buffers were fed, in index order, each to a fresh XCodecEncoder
 * (encode + flush) / XCodecDecoder (one decode call) sharing one
 * XCodecMemoryCache (xcodec/xcodec_cache.h:162-211).
 */
#ifndef XCODEC_HIP_H
#define XCODEC_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define XC_SEGMENT_LENGTH 2048 /* xcodec/xcodec.h:78 */

#define XC_OK 0
#define XC_EINVAL (-22)
#define XC_ENOMEM (-12)
#define XC_ENOSPC (-28)  /* device cache capacity exhausted */
#define XC_EDEVICE (-5)  /* HIP runtime error */
#define XC_ENOENT (-2)
#define XC_EBUSY (-16)   /* a run of this plan is in flight (xc_encode_submit) */

typedef struct xc_ctx xc_ctx;     /* one per GPU; use from one host thread at a time */
typedef struct xc_cache xc_cache; /* replaces XCodecMemoryCache (xcodec/xcodec_cache.h:162-211) */
typedef struct xc_plan xc_plan;   /* a device-resident batch layout + workspace */

/* Number of visible HIP devices. */
int xc_device_count(int *n);

/* Device placement of a new cache among ndev devices (the drop-in facade's two-argument
 * XCodecMemoryCache(uuid, size) / XCodecCacheCOSS(uuid, dir, size), which the unchanged
 * WanProxyCore::add_cache calls, proxy/wanproxy.h:106-116).  key = the cache's 16 UUID bytes.
 * XC_DEVICE in the environment: "d" pins every cache to device d, "d0,d1,..." deals caches over
 * that list; XC_DEVICE_POLICY=uuid places by a hash of the key (the same UUID lands on the same
 * device in every process); otherwise caches are dealt round-robin over all ndev devices in
 * creation order (process-wide).  Returns the device index, or XC_EINVAL (ndev < 1, or XC_DEVICE
 * names a device >= ndev).  Touches no device. */
int xc_device_place(const uint8_t *key, uint64_t key_len, int ndev);

/* Context on device `dev` with its own HIP stream. */
int xc_ctx_create(int dev, xc_ctx **out);
int xc_ctx_destroy(xc_ctx *ctx);
/* The device the context is on. */
int xc_ctx_device(xc_ctx *ctx, int *dev);
/* The context's hipStream_t, as void*. */
void *xc_ctx_stream(xc_ctx *ctx);
/* Wait for all work queued on the context stream. */
int xc_ctx_sync(xc_ctx *ctx);

/* XCodecMemoryCache(UUID, size) (xcodec/xcodec_cache.h:169-172), device resident.
 * cap_segments is the initial capacity.  Like the reference's map, which is unbounded
 * (xcodec/xcodec_cache.h:164,182-188), the cache grows before any call that could fill it (its
 * tables are rebuilt into larger arrays; snapshots stay valid).  Segment bytes fill 2^25 slots of
 * HBM (64 GiB) and then spill to pinned host memory (read by the device over PCIe when a lookup
 * hits them); the tables stay on the device up to 2^28 segments (512 GiB of segments).  Only past
 * that, or when host memory for the spill tier runs out, does a call fail (XC_ENOSPC / XC_ENOMEM). */
int xc_cache_create(xc_ctx *ctx, uint64_t cap_segments, xc_cache **out);
/* Current capacity in segments (grows on demand). */
int xc_cache_capacity(xc_cache *c, uint64_t *cap);
int xc_cache_destroy(xc_cache *c);
int xc_cache_count(xc_cache *c, uint64_t *n);
/* Remember the current contents; xc_cache_restore() rolls every later enter() back. */
/* Diagnostic: the false-positive rates of the cache's level-1 (LDS) and level-2 (L2) filters for
 * a random window end, estimated from their word occupancy. */
int xc_cache_filter_stats(xc_cache *c, double *l1_fp, double *l2_fp);
int xc_cache_snapshot(xc_cache *c);
int xc_cache_restore(xc_cache *c);
/* XCodecCache::lookup (xcodec/xcodec_cache.h:190-210): *found = 1 and 2048 bytes to out (host). */
int xc_cache_lookup(xc_cache *c, uint64_t hash, uint8_t *out, int *found);
/* XCodecCache::enter (xcodec/xcodec_cache.h:182-188): seg = 2048 host bytes. */
int xc_cache_enter(xc_cache *c, uint64_t hash, const uint8_t *seg);

/* XCodecHash::hash (xcodec/xcodec_hash.h:166-174) of n device-resident, 2048-byte-strided
 * segments -> n hashes (device).  stream may be NULL. */
int xc_hash_segments(xc_ctx *ctx, const uint8_t *d_segs, uint64_t n, uint64_t *d_out, void *stream);
/* The same from host memory (n segments at segs, hashes to out; synchronous): the hash of a
 * <LEARN>ed segment, DecodeFilter::consume (xcodec/xcodec_filter.cc:320-322). */
int xc_hash_segments_host(xc_ctx *ctx, const uint8_t *segs, uint64_t n, uint64_t *out);

/* The encoder's rolling hash (xcodec/xcodec_hash.h:93-164 as driven by
 * xcodec/xcodec_encoder.cc:72-84) at every window end of one device buffer:
 * d_out[p] = H(d_in[p-2047..p]) for p >= 2047, 0 below. */
int xc_window_hashes(xc_ctx *ctx, const uint8_t *d_in, uint64_t n, uint64_t *d_out, void *stream);

/* ---- batch encode: XCodecEncoder::encode + flush (xcodec/xcodec_encoder.cc:60-201) ----
 *
 * A plan fixes the buffer lengths of a batch and owns the device workspace.
 * Input arena layout: buffer i at in_off[i] (256-byte aligned), output arena:
 * buffer i's encoded stream at out_off[i] with capacity 2*len+16
 * (the reference's worst case is 2*len: every byte an escaped 0xF1). */
int xc_encode_plan_create(xc_cache *c, const uint64_t *lengths, uint64_t nbuf, xc_plan **out);
/* The same with a bound on each sub-batch's input bytes (0: the default, half the batch between
 * 512 MiB and 1 GiB; at least 1 MiB).  A plan run from host memory (xc_encode_run_host) copies
 * and packs per sub-batch, so smaller sub-batches overlap more of its PCIe transfers: 256 MiB
 * (cfg5 end to end 38 -> 43 GiB/s); device-resident runs are fastest with the default. */
int xc_encode_plan_create_sub(xc_cache *c, const uint64_t *lengths, uint64_t nbuf, uint64_t sub_bytes,
                              xc_plan **out);
int xc_plan_destroy(xc_plan *p);
/* Arena sizes and per-buffer offsets (host arrays of nbuf, may be NULL). */
int xc_plan_layout(xc_plan *p, uint64_t *in_off, uint64_t *out_off, uint64_t *in_bytes,
                   uint64_t *out_bytes);
/* Device-resident encode: d_in / d_out are device arenas in the plan's layout, d_out_len
 * receives nbuf uint64 lengths (device).  Blocks the host until the batch is decided
 * (the codec's sequential-order fix-ups need a host decision), results are on the device.
 * Ordering: the run starts after everything enqueued on the context stream (xc_ctx_stream)
 * before the call, e.g. an async copy into d_in or xc_cache_restore_async; input written on any
 * other stream must be complete (or ordered before the context stream by the caller). */
int xc_encode_run(xc_plan *p, const uint8_t *d_in, uint8_t *d_out, uint64_t *d_out_len);
/* xc_encode_run for an event loop: xc_encode_submit enqueues the run and returns at once;
 * xc_encode_poll never blocks while the device works (*done = 0) and finishes the run once it
 * has (*done = 1, returning the run's status, as xc_encode_run would); xc_encode_wait blocks
 * (yielding the CPU) until then.  Until the run is finished the plan, its cache and the arenas
 * belong to it (another submit on the plan fails with XC_EBUSY).  A run whose sub-batches need
 * the host (declaration growth, cross-buffer conflicts: rare) completes those inside the poll
 * or wait that finishes it.  xc_encode_run = submit + wait.  On a memory cache where a stateful
 * stream entered a hash twice with other bytes (the release build's XCodecMemoryCache::enter,
 * DESIGN.md §5.6) the device hands the run back and the library replays it on the host through the
 * recent window's engine (as xc_encode_batch_host / xc_encode_streams do), writing the streams,
 * lengths and stream results into the run's arenas: same results, slower (a submit refused before
 * any launch is replayed inside the submit; its poll / wait then returns at once). */
int xc_encode_submit(xc_plan *p, const uint8_t *d_in, uint8_t *d_out, uint64_t *d_out_len);
int xc_encode_poll(xc_plan *p, int *done);
int xc_encode_wait(xc_plan *p);
/* Finish the run in flight on the cache, if any (submitted with xc_encode_submit and not yet
 * finished by its poll / wait): blocks until it is done; the submitter's next xc_encode_poll /
 * xc_encode_wait then returns that run's status (until then a submit on that plan fails with
 * XC_EBUSY, so the status cannot be lost).  For synchronous callers that met XC_EBUSY (the
 * drop-in facade): the reference's encoder has no busy state to report. */
int xc_cache_quiesce(xc_cache *c);
/* The caller guarantees that the input arena a run is submitted with is complete when the submit is
 * called (not written by work still pending on any stream, the context stream included) and stays
 * unchanged until the run is finished.  The run's first sub-batch is then hashed at once on a side
 * stream, beside the device work of the plan's previous run (its last kernels and the host's turn),
 * instead of after everything enqueued before the submit.  Default 0. */
int xc_plan_set_input_ready(xc_plan *p, int ready);
/* When xc_encode_run / xc_encode_wait / xc_encode_poll report a run finished:
 * XC_COMPLETE_RUN (the default): every device write of the run is complete;
 * XC_COMPLETE_STREAM: the run is decided (its control words are final, the host has nothing left
 * to do) and its remaining device work completes in the order of the context stream
 * (xc_ctx_stream): work enqueued there afterwards (the next run, a restore, a copy of the outputs)
 * sees the results; other streams and the host must synchronize with that stream first
 * (xc_ctx_sync).  The host then returns while the last kernel still writes the wire bytes, so the
 * next call's launches overlap it.  Applies to device-resident runs without per-kernel timing (a
 * run whose sub-batch the host redoes returns after the redo). */
#define XC_COMPLETE_RUN 0
#define XC_COMPLETE_STREAM 1
int xc_plan_set_completion(xc_plan *p, int mode);
/* Host-to-host convenience: pinned H2D, xc_encode_run, D2H.  out_len receives nbuf lengths. */
int xc_encode_batch_host(xc_cache *c, const uint8_t *in, const uint64_t *in_off,
                         const uint64_t *in_len, uint64_t nbuf, uint8_t *out,
                         const uint64_t *out_off, const uint64_t *out_cap, uint64_t *out_len);

/* Pinned, device-mapped host memory (hipHostMalloc) for the end-to-end host path. */
int xc_host_alloc(xc_ctx *ctx, uint64_t bytes, void **out);
int xc_host_free(void *ptr);

/* End-to-end from host memory, the proxy's path (socket buffers in, encoded frames out):
 * h_in is a host arena in the plan's input layout (xc_plan_layout in_off), h_out pinned host
 * memory from xc_host_alloc.  Each sub-batch's input is copied to the device on a copy stream
 * while earlier sub-batches encode, and each sub-batch's encoded streams are packed in buffer
 * order straight into h_out by a kernel as soon as they are emitted (buffer i at h_pos[i],
 * h_len[i] bytes; h_pos may be NULL).  Fails with XC_EINVAL if they exceed h_out_cap.
 * Same results as xc_encode_run; device arenas are owned by the plan. */
int xc_encode_run_host(xc_plan *p, const uint8_t *h_in, uint8_t *h_out, uint64_t h_out_cap,
                       uint64_t *h_len, uint64_t *h_pos);

/* Enqueue xc_cache_restore() on the context stream without blocking the host. */
int xc_cache_restore_async(xc_cache *c);

/* Per-kernel device time of the plan's runs, from HIP events recorded on the stream of every
 * launch while timing is enabled (kernel ids: XC_K_*).  XC_K_BLOCKHASH runs on a side stream,
 * concurrently with the scans, so its time overlaps theirs. */
#define XC_K_SCAN 0
#define XC_K_RESOLVE 1
#define XC_K_WALK 2
#define XC_K_DECLHASH 3   /* declaration prediction (k_blockpredict); k_walk hashes the unknown ones */
#define XC_K_EMIT 4
#define XC_K_BLOCKHASH 5
#define XC_K_COUNT 6
typedef struct {
    double ms[XC_K_COUNT];        /* summed device time */
    uint64_t launches[XC_K_COUNT];
    uint64_t scan_bytes;          /* input bytes covered by the scan launches */
} xc_kernel_times;
#define XC_TIMING_ALL 1   /* every kernel (each event pair adds a few us between launches) */
#define XC_TIMING_SCAN 2  /* the scan launches only */
int xc_plan_set_timing(xc_plan *p, int mode);
int xc_plan_kernel_times(xc_plan *p, xc_kernel_times *out, int reset);

/* Counters of the last run (for benchmarks / profiling). */
typedef struct {
    uint64_t n_extract;  /* EXTRACT tokens emitted (segments declared) */
    uint64_t n_ref;      /* REF tokens emitted */
    uint64_t in_bytes, out_bytes;
    uint32_t sub_batches, walk_rounds, outer_rounds, dense_chunks;
    uint32_t redone;     /* sub-batches the asynchronous pass handed back to the host */
    uint32_t shadow_misses; /* ... of which because a predicted REF was not emitted */
    uint32_t anchor_scans;  /* sub-batches whose first scan took its events from the anchor index */
    uint32_t anchor_fallbacks; /* ... handed to the exact scan (a collision at a candidate, an
                               anchorless declaration, an overflowing record list) */
    uint32_t early_hashed;  /* 1: the first sub-batch was hashed at the submit (xc_plan_set_input_ready) */
    uint32_t reserved;
} xc_run_stats;
int xc_plan_stats(xc_plan *p, xc_run_stats *st);

/* The first scan of a sub-batch.  XC_SCAN_AUTO (the default): the anchor index
 * when the run qualifies (a memory cache whose segments all have an anchor, fresh encoders, at
 * least 200000 cached + new segments, XC_ANCHOR_MIN_KEYS in the environment), else the exact scan, which tests every window
 * end against the cache.  XC_SCAN_EXACT: always the exact scan.  XC_SCAN_ANCHOR: the anchor index
 * whenever the run qualifies, whatever its size (tests).  Results are identical in every mode. */
#define XC_SCAN_AUTO 0
#define XC_SCAN_EXACT 1
#define XC_SCAN_ANCHOR 2
int xc_plan_set_scan(xc_plan *p, int mode);

/* ---- stateful streams: XCodecEncoder across calls (xcodec/xcodec_encoder.h:43-63) ----
 *
 * Stream state of a batch item (xc_plan_set_streams): buffer i is an encoder's pending source_
 * (the reference's Buffer source_, xcodec/xcodec_encoder.h:47) followed by new input.
 * start[i] = bytes of source_ (their window ends were looked up by earlier calls), cand[i] =
 * the pending candidate_start_ (-1 = none), flags[i] & 1 = encode() only (no flush: the
 * candidate and the trailing literals stay pending).  All three NULL = fresh encode + flush per
 * buffer (the default).  After a run, xc_plan_stream_results gives the new source_ start
 * base[i] (buffer offset; == length after a flush) and candidate cand[i] (buffer offset, -1). */
int xc_plan_set_streams(xc_plan *p, const uint64_t *start, const int64_t *cand, const uint32_t *flags);
int xc_plan_stream_results(xc_plan *p, uint64_t *base, int64_t *cand);

typedef struct xc_encoder xc_encoder; /* XCodecEncoder: one per connection (xcodec_filter.h:43-48) */
/* new XCodecEncoder(cache) (xcodec/xcodec_encoder.cc:43-49). */
int xc_encoder_create(xc_cache *c, xc_encoder **out);
int xc_encoder_destroy(xc_encoder *e);
/* Bytes of source_ not yet emitted (an output of 2 * (pending + n) + 16 bytes always suffices). */
int xc_encoder_pending(xc_encoder *e, uint64_t *bytes);
/* XCodecEncoder::encode(out, in) (xcodec/xcodec_encoder.cc:60-173): out receives exactly the
 * bytes the reference appends during this call. */
int xc_encode(xc_encoder *e, const uint8_t *in, uint64_t n, uint8_t *out, uint64_t cap, uint64_t *out_len);
/* XCodecEncoder::flush(out) (xcodec/xcodec_encoder.cc:175-201); *emitted = its bool result. */
int xc_flush(xc_encoder *e, uint8_t *out, uint64_t cap, uint64_t *out_len, int *emitted);
/* Cross-connection batch of calls, in the reference's single-thread order: call k is
 * enc[k]->encode(in[k]) and, with flags[k] & XC_STREAM_FLUSH, enc[k]->flush() (EncodeFilter::consume
 * without TO_BE_CONTINUED, xcodec/xcodec_filter.cc:146-160).  An encoder may appear in several
 * calls.  Call k's output goes to out + out_off[k] (capacity out_cap[k], at least twice the
 * encoder's pending bytes plus its inputs up to and including call k, else XC_EINVAL before
 * anything runs).  After a device error (XC_EDEVICE / XC_ENOMEM / XC_ENOSPC) the encoders and the
 * cache may hold part of the batch: destroy them. */
#define XC_STREAM_FLUSH 1
int xc_encode_streams(xc_encoder *const *enc, const uint8_t *const *in, const uint64_t *in_len,
                      const uint32_t *flags, uint64_t n, uint8_t *out, const uint64_t *out_off,
                      const uint64_t *out_cap, uint64_t *out_len);

/* ---- batch decode: XCodecDecoder::decode (xcodec/xcodec_decoder.cc:76-176) ----
 * status[i] = 1 (decode returned true) or 0 (false); consumed[i] = input bytes the
 * reference removes from its Buffer; has_unknown[i]/unknown[i] = the REF hash the
 * reference inserted into unknown_hashes and stopped on. */
int xc_decode_batch_host(xc_cache *c, const uint8_t *in, const uint64_t *in_off,
                         const uint64_t *in_len, uint64_t nbuf, uint8_t *out,
                         const uint64_t *out_off, const uint64_t *out_cap, uint64_t *out_len,
                         uint64_t *consumed, int32_t *status, uint64_t *unknown,
                         int32_t *has_unknown);

/* Device-resident decode: a plan fixes the stream lengths and output capacities of a batch and
 * owns the device workspace.  Input arena: stream j at in_off[j]; output arena: stream j's bytes
 * at out_off[j] (capacity out_cap[j]).  xc_decode_run takes device arenas in that layout and
 * device arrays of nbuf results (same meaning as xc_decode_batch_host's); it returns once the
 * batch is decoded (one host round trip decides the provider rounds). */
typedef struct xc_dplan xc_dplan;
typedef struct {
    uint64_t in_bytes;   /* encoded bytes of the batch */
    uint64_t n_extract;  /* EXTRACT tokens executed */
    uint64_t n_ref;      /* REF tokens executed */
    uint64_t n_entered;  /* segments entered into the cache (xcodec_decoder.cc:133-135) */
    uint32_t rounds;     /* provider resolution rounds */
} xc_decode_stats;
int xc_decode_plan_create(xc_cache *c, const uint64_t *in_len, const uint64_t *out_cap, uint64_t nbuf,
                          xc_dplan **out);
int xc_dplan_destroy(xc_dplan *p);
int xc_dplan_layout(xc_dplan *p, uint64_t *in_off, uint64_t *out_off, uint64_t *in_bytes,
                    uint64_t *out_bytes);
int xc_decode_run(xc_dplan *p, const uint8_t *d_in, uint8_t *d_out, uint64_t *d_out_len,
                  uint64_t *d_consumed, int32_t *d_status, uint64_t *d_unknown, int32_t *d_has_unknown);
int xc_dplan_stats(xc_dplan *p, xc_decode_stats *st);
/* As xc_plan_set_completion: with XC_COMPLETE_STREAM xc_decode_run returns once the batch is
 * decided (its statistics and errors are final: the streams' stops, the cache slots) and the
 * output copies and cache inserts complete in the order of the plan's stream (the context
 * stream); a batch whose outputs may not fit their capacities returns after the whole run. */
int xc_dplan_set_completion(xc_dplan *p, int mode);
/* As xc_plan_set_input_ready for decode runs: the input arena is complete when xc_decode_run is
 * called and unchanged until the run is finished; the run's input is then parsed (tokens, EXTRACT
 * hashes) on a side stream at once, beside the device work of the plan's previous run. */
int xc_dplan_set_input_ready(xc_dplan *p, int ready);

/* ---- persistent COSS cache: XCodecCacheCOSS (xcodec/cache/coss/xcodec_cache_coss.{h,cc}) ----
 *
 * XCodecCacheCOSS(uuid, cache_dir, size) (xcodec_cache_coss.cc:31-80): the stripe file
 * <dir>/<uuid>.wpc (uuid: the 36-character UUID string), size_mb 0 = 1024, read back if valid.
 * The segments a lookup can find are mirrored in a device cache on ctx; encode and decode batches
 * run on the device and advance the COSS state (stripes, freshness, use flags, the recent window,
 * purges, the file) exactly as the reference's codec calls would (wanproxy_amd/csrc/xc_coss.cpp).
 * ctx NULL: the host store alone (lookup / enter only). */
typedef struct xc_coss xc_coss;
int xc_coss_open(xc_ctx *ctx, const char *dir, const char *uuid, uint64_t size_mb, xc_coss **out);
/* ~XCodecCacheCOSS (:82-105): the loaded stripes are stored. */
int xc_coss_close(xc_coss *c);
/* The device mirror (NULL for a host-only store): for device-resident plans on a COSS cache only
 * while nothing is purged (use the batch calls below to keep the COSS state). */
xc_cache *xc_coss_cache(xc_coss *c);
int xc_coss_count(xc_coss *c, uint64_t *n);
/* {lookups (every call, misses included, as the reference counts them: the batch paths add the
 * encoder's and decoder's missed lookups of each replayed item), found in the recent window, found in the
 * stripes, index size, stripe limit, serial number} (COSSStats, xcodec_cache_coss.h:179-187). */
int xc_coss_stats(xc_coss *c, uint64_t *out6);
/* XCodecCacheCOSS::lookup / enter (:188-228, :163-186); the device mirror follows. */
int xc_coss_lookup(xc_coss *c, uint64_t hash, uint8_t *out, int *found);
int xc_coss_enter(xc_coss *c, uint64_t hash, const uint8_t *seg);
/* xc_encode_batch_host / xc_decode_batch_host over the COSS cache. */
int xc_coss_encode_batch_host(xc_coss *c, const uint8_t *in, const uint64_t *in_off, const uint64_t *in_len,
                              uint64_t nbuf, uint8_t *out, const uint64_t *out_off, const uint64_t *out_cap,
                              uint64_t *out_len);
int xc_coss_decode_batch_host(xc_coss *c, const uint8_t *in, const uint64_t *in_off, const uint64_t *in_len,
                              uint64_t nbuf, uint8_t *out, const uint64_t *out_off, const uint64_t *out_cap,
                              uint64_t *out_len, uint64_t *consumed, int32_t *status, uint64_t *unknown,
                              int32_t *has_unknown);
/* xc_encode_streams over the COSS cache: stateful encoders (xcodec_encoder.h:45-50) created with
 * xc_encoder_create(xc_coss_cache(c), ...), their calls run in call order as one batch each round,
 * the COSS state advanced as the reference's sequential calls would (the server side's waiting
 * mode, encode() without flush, included). */
int xc_coss_encode_streams(xc_coss *c, xc_encoder *const *enc, const uint8_t *const *in, const uint64_t *in_len,
                           const uint32_t *flags, uint64_t n, uint8_t *out, const uint64_t *out_off,
                           const uint64_t *out_cap, uint64_t *out_len);
/* The host store's own lookup / enter, without the device mirror (tests of the store). */
int xc_coss_store_lookup(xc_coss *c, uint64_t hash, uint8_t *out, int *found);
int xc_coss_store_enter(xc_coss *c, uint64_t hash, const uint8_t *seg);

/* Library self-test of the wave primitives on device (returns XC_OK or a negative code). */
int xc_selftest(xc_ctx *ctx);

/* Human-readable text of the last error recorded on this thread. */
const char *xc_last_error(void);

#ifdef __cplusplus
}
#endif
#endif
