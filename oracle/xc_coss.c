/*
 * xc_coss.c — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference's persistent COSS cache, XCodecCacheCOSS
 * (xcodec/cache/coss/xcodec_cache_coss.{h,cc}), with the base class's 64-entry recent window
 * (xcodec/xcodec_cache.h:46-48,94-158, USING_XCODEC_CACHE_RECENT_WINDOW is defined).  It is the
 * checker for the product's COSS tier (wanproxy_amd/csrc/xc_coss.cpp): the same operations on
 * both must give the same lookup results, the same evictions and the same <uuid>.wpc file bytes.
 *
 * Parity unpinned by the reference itself: xcodec_cache_coss.cc includes xcodec/xcodec_cache.h,
 * which pulls <uuid/uuid.h> (absent from this image), and the reference's COSS test
 * (xcodec/cache/coss/test/xcodec-coss1) does not compile against the current class; this file is
 * checked by review against the source (line citations below) and by that test's intent
 * (segments entered, the cache reopened, lookups match).
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>

#include "xc_oracle.h"

#define SEG XO_SEGMENT_LENGTH
#define SIGNATURE 0xF150E964u   /* xcodec_cache_coss.h:83 */
#define VERSION 2               /* :84 */
#define STRIPE_SEGS 512         /* :85 */
#define LOADED 16               /* :86 */
#define BASIC_MB 1024           /* :87 */
#define WINDOW 64               /* xcodec_cache.h:48 */

typedef struct { /* COSSMetadata, xcodec_cache_coss.h:147-160 */
    uint32_t signature, version;
    uint64_t serial_number, stripe_range;
    uint32_t segment_index, segment_count;
    uint64_t freshness, uses, credits;
    uint32_t load_uses, state;
} meta_t;

/* COSSStripeHeader (:162-168): metadata, padding to 8192 - 6144, flags[512], hash_array[512] */
#define HEADER_SIZE 8192
#define PADDING (HEADER_SIZE - STRIPE_SEGS * 12 - (int)sizeof(meta_t))
typedef struct {
    meta_t m;
    char padding[PADDING];
    uint32_t flags[STRIPE_SEGS];
    uint64_t hash[STRIPE_SEGS];
} header_t;
typedef struct { /* COSSStripe (:170-177) */
    header_t h;
    uint8_t seg[STRIPE_SEGS][SEG];
} stripe_t;

_Static_assert(sizeof(meta_t) == 64, "COSSMetadata");
_Static_assert(sizeof(header_t) == HEADER_SIZE, "COSSStripeHeader");

typedef struct { /* COSSIndexEntry + the hash (:89-121: hash_map<Hash64, entry>) */
    uint64_t hash;
    uint64_t range;
    uint32_t pos;
    int used;
} ientry;

struct xo_coss {
    char path[4096];
    FILE *f;
    uint64_t file_size, serial, stripe_range, stripe_limit, freshness_level;
    stripe_t *stripe; /* [LOADED] */
    int active;
    meta_t *dir;
    ientry *idx; /* open addressing (erase by backward shift) */
    size_t imask, icount;
    struct { uint64_t hash; const uint8_t *data; } window[WINDOW];
    unsigned cursor;
    uint64_t lookups, found_1, found_2;
    uint64_t load_misses; /* (checks only) lookups that loaded a stripe and then missed */
};

/* ------------------------------------------------------------- index --- */
static size_t islot(uint64_t h, size_t mask) { return (size_t)((h * 0x9E3779B97F4A7C15ull) >> 21) & mask; }

static ientry *ifind(xo_coss *c, uint64_t h)
{
    for (size_t s = islot(h, c->imask);; s = (s + 1) & c->imask) {
        if (!c->idx[s].used) return NULL;
        if (c->idx[s].hash == h) return &c->idx[s];
    }
}

static void iinsert(xo_coss *c, uint64_t h, uint64_t range, uint32_t pos)
{ /* index[hash] = entry (:96-99): insert or overwrite */
    if ((c->icount + 1) * 2 > c->imask + 1) {
        ientry *old = c->idx;
        size_t om = c->imask;
        c->imask = om * 2 + 1;
        c->idx = (ientry *)calloc(c->imask + 1, sizeof(ientry));
        c->icount = 0;
        for (size_t i = 0; i <= om; i++)
            if (old[i].used) iinsert(c, old[i].hash, old[i].range, old[i].pos);
        free(old);
    }
    size_t s = islot(h, c->imask);
    while (c->idx[s].used && c->idx[s].hash != h) s = (s + 1) & c->imask;
    if (!c->idx[s].used) c->icount++;
    c->idx[s] = (ientry){h, range, pos, 1};
}

static void ierase(xo_coss *c, uint64_t h)
{ /* index.erase (:107-110) */
    size_t s = islot(h, c->imask);
    while (c->idx[s].used && c->idx[s].hash != h) s = (s + 1) & c->imask;
    if (!c->idx[s].used) return;
    c->idx[s].used = 0;
    c->icount--;
    for (size_t j = (s + 1) & c->imask; c->idx[j].used; j = (j + 1) & c->imask) {
        const size_t home = islot(c->idx[j].hash, c->imask);
        /* keep j if its home lies cyclically in (s, j] */
        if ((j > s && (home <= s || home > j)) || (j < s && home <= s && home > j)) {
            c->idx[s] = c->idx[j];
            c->idx[j].used = 0;
            s = j;
        }
    }
}

/* ------------------------------------------------------- recent window --- */
static void remember(xo_coss *c, uint64_t h, const uint8_t *d)
{ /* xcodec_cache.h:130-135 */
    c->window[c->cursor].hash = h;
    c->window[c->cursor].data = d;
    c->cursor = (c->cursor + 1) & (WINDOW - 1);
}

static const uint8_t *find_recent(xo_coss *c, uint64_t h)
{ /* :137-147 */
    for (int i = 0; i < WINDOW; i++)
        if (c->window[i].hash == h) return c->window[i].data;
    return NULL;
}

static void forget(xo_coss *c, uint64_t h)
{ /* :150-158 */
    for (int i = 0; i < WINDOW; i++)
        if (c->window[i].hash == h) c->window[i].hash = 0;
}

/* ---------------------------------------------------------------- file --- */
static void store_stripe(xo_coss *c, int slot, size_t size)
{ /* xcodec_cache_coss.cc:262-272 */
    const uint64_t pos = c->stripe[slot].h.m.stripe_range * sizeof(stripe_t);
    fseeko(c->f, (off_t)pos, SEEK_SET);
    if (fwrite(&c->stripe[slot], 1, size, c->f) == size && pos + sizeof(stripe_t) > c->file_size)
        c->file_size = pos + sizeof(stripe_t);
    fflush(c->f);
}

static int load_stripe(xo_coss *c, uint64_t range, int slot)
{ /* :241-260 */
    const uint64_t pos = range * sizeof(stripe_t);
    if (pos < c->file_size) {
        fseeko(c->f, (off_t)pos, SEEK_SET);
        if (fread(&c->stripe[slot], 1, sizeof(stripe_t), c->f) == sizeof(stripe_t)) {
            c->stripe[slot].h.m.stripe_range = range;
            c->stripe[slot].h.m.load_uses = 0;
            c->stripe[slot].h.m.state = 1;
            c->dir[range].state = 1;
            return 1;
        }
    }
    clearerr(c->f);
    return 0;
}

static void initialize_stripe(xo_coss *c, uint64_t range, int slot)
{ /* :230-239 */
    memset(&c->stripe[slot].h, 0, sizeof(header_t));
    c->stripe[slot].h.m.signature = SIGNATURE;
    c->stripe[slot].h.m.version = VERSION;
    c->stripe[slot].h.m.serial_number = ++c->serial;
    c->stripe[slot].h.m.stripe_range = range;
    c->stripe[slot].h.m.state = 1;
    c->dir[range] = c->stripe[slot].h.m;
}

static int best_unloadable_slot(xo_coss *c)
{ /* :285-302 */
    uint64_t n = ~0ull;
    int j = 0;
    for (int i = 0; i < LOADED; i++) {
        if (i == c->active) continue;
        if (c->stripe[i].h.m.signature == 0) return i;
        const uint64_t v = c->stripe[i].h.m.freshness + c->stripe[i].h.m.load_uses;
        if (v < n) j = i, n = v;
    }
    return j;
}

static uint64_t best_erasable_stripe(xo_coss *c)
{ /* :304-321 */
    uint64_t n = ~0ull, j = 0;
    for (uint64_t i = 0; i < c->stripe_limit; i++) {
        const meta_t *m = &c->dir[i];
        if (m->state == 1) continue;
        if (m->signature == 0) return i;
        const uint64_t v = m->freshness + m->uses;
        if (v < n) j = i, n = v;
    }
    return j;
}

static void detach_stripe(xo_coss *c, int slot)
{ /* :323-345 */
    stripe_t *s = &c->stripe[slot];
    if (s->h.m.state != 1) return;
    const uint64_t range = s->h.m.stripe_range;
    c->dir[range] = s->h.m;
    c->dir[range].state = 2;
    for (int i = 0; i < STRIPE_SEGS; i++)
        if (s->h.flags[i] & 1) {
            forget(c, s->h.hash[i]);
            s->h.flags[i] &= ~1u;
        }
    s->h.m.state = 0;
    store_stripe(c, slot, sizeof(header_t));
}

static void purge_stripe(xo_coss *c, int slot)
{ /* :347-377 */
    stripe_t *s = &c->stripe[slot];
    for (int i = STRIPE_SEGS - 1; i >= 0; --i) {
        const uint64_t h = s->h.hash[i];
        if (h && !(s->h.flags[i] & 2)) {
            ierase(c, h);
            s->h.hash[i] = 0;
            s->h.flags[i] = 0;
            s->h.m.segment_count--;
        }
        s->h.flags[i] &= ~2u;
        if (!s->h.hash[i]) s->h.m.segment_index = (uint32_t)i;
    }
    s->h.m.serial_number = ++c->serial;
    s->h.m.uses = s->h.m.credits;
    s->h.m.credits = 0;
}

static void new_active(xo_coss *c)
{ /* :274-283 */
    store_stripe(c, c->active, sizeof(stripe_t));
    c->active = best_unloadable_slot(c);
    detach_stripe(c, c->active);
    c->stripe_range = best_erasable_stripe(c);
    if (load_stripe(c, c->stripe_range, c->active)) purge_stripe(c, c->active);
    else initialize_stripe(c, c->stripe_range, c->active);
}

static int read_file(xo_coss *c)
{ /* :107-161 */
    header_t h;
    uint64_t serial = 0, range = 0, level = 0;
    uint64_t limit = c->file_size / sizeof(stripe_t);
    if (limit * sizeof(stripe_t) != c->file_size) return 0;
    if (limit > c->stripe_limit) limit = c->stripe_limit;
    fseeko(c->f, 0, SEEK_SET);
    for (uint64_t n = 0; n < limit; ++n) {
        if (fread(&h, 1, sizeof h, c->f) != sizeof h) return 0;
        if (h.m.signature != SIGNATURE) return 0;
        if (h.m.segment_count > STRIPE_SEGS) return 0;
        fseeko(c->f, (off_t)(sizeof(stripe_t) - sizeof h), SEEK_CUR);
        if (h.m.serial_number > serial) serial = h.m.serial_number, range = n;
        if (h.m.freshness > level) level = h.m.freshness;
        c->dir[n] = h.m;
        c->dir[n].state = 0;
        for (int i = 0; i < STRIPE_SEGS; ++i)
            if (h.hash[i]) iinsert(c, h.hash[i], n, (uint32_t)i);
    }
    if (serial > 0) {
        c->serial = serial;
        c->stripe_range = range;
        c->freshness_level = level;
        load_stripe(c, c->stripe_range, c->active);
    } else {
        initialize_stripe(c, c->stripe_range, c->active);
    }
    return 1;
}

/* ---------------------------------------------------------------- API --- */
xo_coss *xo_coss_open(const char *dir, const char *uuid, uint64_t size_mb)
{ /* XCodecCacheCOSS::XCodecCacheCOSS (:31-80) */
    xo_coss *c = (xo_coss *)calloc(1, sizeof *c);
    size_t dl = strlen(dir);
    snprintf(c->path, sizeof c->path, "%s%s%.36s.wpc", dir, (dl && dir[dl - 1] != '/') ? "/" : "", uuid);
    struct stat st;
    if (stat(c->path, &st) == 0 && S_ISREG(st.st_mode)) {
        c->file_size = (uint64_t)st.st_size;
    } else {
        FILE *t = fopen(c->path, "wb");
        if (t) fclose(t);
        c->file_size = 0;
    }
    if (!size_mb) size_mb = BASIC_MB;
    const uint64_t bytes = (size_mb * 1048576ull + sizeof(stripe_t) - 1) / sizeof(stripe_t) * sizeof(stripe_t);
    c->stripe_limit = bytes / sizeof(stripe_t);
    c->stripe = (stripe_t *)calloc(LOADED, sizeof(stripe_t)); /* COSSStripe() zeroes the headers */
    c->dir = (meta_t *)calloc(c->stripe_limit, sizeof(meta_t));
    c->imask = 1023;
    c->idx = (ientry *)calloc(c->imask + 1, sizeof(ientry));
    c->f = fopen(c->path, "r+b");
    if (c->f) setvbuf(c->f, NULL, _IONBF, 0);
    if (!c->f || !read_file(c)) {
        if (c->f) fclose(c->f);
        c->f = fopen(c->path, "w+b"); /* trunc */
        setvbuf(c->f, NULL, _IONBF, 0);
        c->file_size = 0;
        initialize_stripe(c, c->stripe_range, c->active);
    }
    return c;
}

void xo_coss_close(xo_coss *c)
{ /* ~XCodecCacheCOSS (:82-105) */
    if (!c) return;
    for (int i = 0; i < LOADED; ++i)
        if (c->stripe[i].h.m.state == 1) store_stripe(c, i, i == c->active ? sizeof(stripe_t) : sizeof(header_t));
    fclose(c->f);
    free(c->stripe);
    free(c->dir);
    free(c->idx);
    free(c);
}

void xo_coss_enter(xo_coss *c, uint64_t h, const uint8_t *seg)
{ /* :163-186 */
    while (c->stripe[c->active].h.m.segment_index >= STRIPE_SEGS) new_active(c);
    stripe_t *a = &c->stripe[c->active];
    const uint32_t i = a->h.m.segment_index;
    a->h.hash[i] = h;
    memcpy(a->seg[i], seg, SEG);
    const uint64_t range = a->h.m.stripe_range;
    a->h.m.segment_index++;
    while (a->h.m.segment_index < STRIPE_SEGS && a->h.hash[a->h.m.segment_index]) a->h.m.segment_index++;
    a->h.m.segment_count++;
    a->h.m.freshness = ++c->freshness_level;
    iinsert(c, h, range, i);
}

int xo_coss_lookup(xo_coss *c, uint64_t h, const uint8_t **data)
{ /* :188-228 */
    c->lookups++;
    const uint8_t *d = find_recent(c, h);
    if (d) {
        *data = d;
        c->found_1++;
        return 1;
    }
    const ientry *e = ifind(c, h);
    if (!e) return 0;
    const uint64_t range = e->range;
    const uint32_t pos = e->pos;
    int slot;
    for (slot = 0; slot < LOADED; ++slot)
        if (c->stripe[slot].h.m.stripe_range == range) break;
    int loaded = 0;
    if (slot >= LOADED) {
        loaded = 1;
        slot = best_unloadable_slot(c);
        detach_stripe(c, slot);
        load_stripe(c, range, slot);
    }
    stripe_t *s = &c->stripe[slot];
    if (s->h.hash[pos] != h) {
        if (loaded) c->load_misses++;
        return 0;
    }
    s->h.m.freshness = ++c->freshness_level;
    s->h.m.uses++;
    s->h.m.credits++;
    s->h.m.load_uses++;
    s->h.flags[pos] |= 3;
    *data = s->seg[pos];
    remember(c, h, *data);
    c->found_2++;
    return 1;
}

size_t xo_coss_count(const xo_coss *c) { return c->icount; }

uint64_t xo_coss_load_misses(const xo_coss *c) { return c->load_misses; }

void xo_coss_stats(const xo_coss *c, uint64_t *out)
{
    out[0] = c->lookups;
    out[1] = c->found_1;
    out[2] = c->found_2;
    out[3] = c->icount;
    out[4] = c->stripe_limit;
    out[5] = c->serial;
}

/* The index's hashes (any order), for checks: returns the count written (at most cap). */
size_t xo_coss_hashes(const xo_coss *c, uint64_t *out, size_t cap)
{
    size_t k = 0;
    for (size_t i = 0; i <= c->imask && k < cap; i++)
        if (c->idx[i].used) out[k++] = c->idx[i].hash;
    return k;
}
