/*
 * ref_hash_harness.cc — TEST INFRASTRUCTURE ONLY.
 *
 * Exposes the reference XCodecHash class (compiled from the reference's own
 * header, xcodec/xcodec_hash.h, where it lies under /root/reference) through a
 * C ABI so tests can pin oracle/xc_oracle.c's hash against the real thing.
 * Built by oracle/Makefile into oracle/_ref/libxcref_hash.so (git-ignored).
 */
#include <stdint.h>
#include <stddef.h>
#include <xcodec/xcodec.h>
#include <xcodec/xcodec_hash.h>

extern "C" {

/* XCodecHash::hash — xcodec/xcodec_hash.h:166-174 */
uint64_t xcref_hash_segment(const uint8_t *seg) { return XCodecHash::hash(seg); }

/* The encoder's add-then-roll use of XCodecHash (xcodec/xcodec_encoder.cc:72-84):
 * out[p] = mix() after byte p for p >= 2047, 0 before. */
void xcref_window_hashes(const uint8_t *data, size_t n, uint64_t *out)
{
    XCodecHash *h = new XCodecHash();
    for (size_t p = 0; p < n; p++) {
        if (p < XCODEC_SEGMENT_LENGTH) h->add(data[p]);
        else h->roll(data[p]);
        out[p] = (p + 1 >= XCODEC_SEGMENT_LENGTH) ? h->mix() : 0;
    }
    delete h;
}

}
