// xc_env.h — the library's environment switches.
//
// A release build reads only the documented deployment knobs, each with a GPU parity test against the
// reference results ("Environment"): XC_DEVICE / XC_DEVICE_POLICY (placement), XC_SUB_MB,
// XC_CHUNK_BLOCKS, XC_NO_SHADOW, XC_SCAN, XC_ANCHOR_MIN_KEYS (sub-batch and scan sizing),
// XC_REPLAY_THREADS (the recent window's replay), XC_GRAPH (a one-sub-batch run as a HIP graph) and
// XC_FORCE_REPLAY (tests: a device-resident run through the replay engine).
//
// Timing ablations and diagnostics (XC_ABL_*, XC_SCAN_ABLATION, XC_NO_HITS, XC_DEBUG_*,
// XC_REPLAY_PROF and the grid overrides) are read through abl_env only in builds with
// -DXC_ABLATIONS=1 (tools/build_variant.sh): in a release build abl_env is a constant nullptr, so
// no such switch can change what the library computes or how much of it it skips.
#pragma once
#include <stdlib.h>

#ifndef XC_ABLATIONS
#define XC_ABLATIONS 0
#endif

namespace xc {

inline const char *abl_env(const char *name)
{
#if XC_ABLATIONS
    return getenv(name);
#else
    (void)name;
    return nullptr;
#endif
}

// an ablation flag: set and non-zero
inline bool abl_flag(const char *name)
{
    const char *e = abl_env(name);
    return e && atoi(e) != 0;
}

}  // namespace xc
