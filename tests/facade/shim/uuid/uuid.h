/* TEST ONLY (tests/test_facade.py): the three libuuid declarations common/uuid/uuid.h uses.  The
 * image has libuuid.so.1 but not its header.  This makes a compile / link check of the facade
 * (facade/xcodec/) against the reference's unchanged filter sources possible; it is not an oracle
 * and nothing built with it runs on the GPU box. */
#pragma once
typedef unsigned char uuid_t[16];
extern "C" {
void uuid_generate(uuid_t out);
int uuid_parse(const char *in, uuid_t uu);
void uuid_unparse(const uuid_t uu, char *out);
}
