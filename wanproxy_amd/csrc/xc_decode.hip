// xc_decode.hip — XCodec batch decoder (placeholder until the device decoder lands).
#include <hip/hip_runtime.h>
#include "../../include/xcodec_hip.h"

extern "C" int xc_decode_batch_host(xc_cache *, const uint8_t *, const uint64_t *, const uint64_t *, uint64_t,
                                    uint8_t *, const uint64_t *, const uint64_t *, uint64_t *, uint64_t *,
                                    int32_t *, uint64_t *, int32_t *)
{
    return XC_EINVAL;
}
