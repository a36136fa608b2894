/*
 * ref_zlib_harness.cc — TEST INFRASTRUCTURE ONLY.
 *
 * The reference's DeflateFilter / InflateFilter (zlib/zlib_filter.{h,cc}, compiled where they lie
 * under /root/reference together with common/{buffer,log}.cc, against the system libz) behind a
 * C ABI, so tests can pin wanproxy_amd/pipe.py's zlib stage against the real filters.  A consume
 * receives one Buffer built by Buffer::append of the whole input (2048-byte segments, as a socket
 * read arrives: event/io_service.cc:160-180); whatever the filter produces is collected.
 * Built by oracle/Makefile into oracle/_ref/libzref.so (git-ignored).
 */
#include <stdint.h>
#include <stddef.h>
#include <string.h>
#include <string>

#include <common/filter.h>
#include <zlib/zlib_filter.h>

namespace {
struct Collect : public Filter {
    std::string out;
    int flushes = 0;
    bool consume(Buffer &buf, int) override
    {
        size_t n = buf.length();
        if (n) {
            std::string tmp(n, '\0');
            buf.copyout((uint8_t *)&tmp[0], n);
            out += tmp;
        }
        return true;
    }
    void flush(int) override { flushes++; }
};

struct Z {
    Filter *f;
    Collect sink;
};

int take(Z *z, uint8_t *out, size_t cap, size_t *len)
{
    *len = z->sink.out.size();
    if (*len > cap) return -1;
    memcpy(out, z->sink.out.data(), *len);
    z->sink.out.clear();
    return 0;
}
}  // namespace

extern "C" {

void *zref_new(int deflate, int level)
{
    Z *z = new Z();
    z->f = deflate ? (Filter *)new DeflateFilter(level) : (Filter *)new InflateFilter();
    z->f->chain(&z->sink);
    return z;
}

void zref_free(void *h)
{
    Z *z = (Z *)h;
    delete z->f;
    delete z;
}

/* consume(): 1 / 0 = the filter's result; the produced bytes to out (-1 if cap is too small). */
int zref_consume(void *h, const uint8_t *data, size_t n, uint8_t *out, size_t cap, size_t *len)
{
    Z *z = (Z *)h;
    Buffer b;
    if (n) b.append(data, n);
    const bool ok = z->f->consume(b, 0);
    if (take(z, out, cap, len)) return -1;
    return ok ? 1 : 0;
}

int zref_flush(void *h, uint8_t *out, size_t cap, size_t *len)
{
    Z *z = (Z *)h;
    z->f->flush(0);
    return take(z, out, cap, len);
}

}
