"""wanproxy_amd — MI355X-native XCodec (WANProxy's deduplicating stream codec).

The hot path (rolling window hash, cache probe, encode state machine, decode
reference expansion) runs as hand-written gfx950 HIP kernels in
``libxcodec_hip.so`` behind the C ABI declared in ``include/xcodec_hip.h``.
"""
from . import pipe, workloads  # noqa: F401
from .xcodec import (Context, CossCache, DecodePlan, EncodePlan, HostBuffer, XCodecCache, XCodecDecoder,  # noqa: F401
                     XCodecEncoder, XCodecError, XCodecStreamEncoder, device_count,
                     encode_streams, load_library)

__all__ = ["Context", "CossCache", "DecodePlan", "EncodePlan", "HostBuffer", "XCodecCache", "XCodecDecoder", "XCodecEncoder",
           "XCodecError", "XCodecStreamEncoder", "device_count", "encode_streams", "load_library",
           "pipe", "workloads"]
