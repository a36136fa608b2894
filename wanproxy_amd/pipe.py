"""XCodec pipe filters over the device codec: ``EncodeFilter`` / ``DecodeFilter``.

A mirror of ``xcodec/xcodec_filter.h:25-86`` and ``xcodec/xcodec_filter.cc:122-526`` (SURVEY.md
§8(f)1) with the same names, argument meaning and ``bool`` error behaviour:

* the pipe framing: ``<HELLO>`` (cache UUID + nominal size) at the start of a stream,
  ``<FRAME>`` = ``00 BE16(len) data`` with 1 <= len <= 32768, ``<EOS>`` / ``<EOS_ACK>``;
* the ``<ASK>`` / ``<LEARN>`` exchange for REFs the peer's cache does not hold: the decoder stops
  on the unknown REF, asks for it through its upstream filter, and resumes after the ``<LEARN>``;
* stateful multi-call encoding: ``consume`` without ``TO_BE_CONTINUED`` flushes the encoder,
  except in "waiting" mode, where the flush is deferred to ``on_read_timeout`` (the reference's
  150 ms timer, ``xcodec_filter.cc:148-157,205-216``; the caller owns the clock here).

Filters chain as in ``common/filter.h:18-70``: ``consume`` takes bytes from upstream,
``produce`` hands bytes to the next filter, ``flush`` propagates down the chain.

The codec is the device library (``wanproxy_amd.xcodec``) through :class:`DeviceBackend`; the
filters hold no codec logic of their own.  There is no CPU fallback: a backend is always given
explicitly (the CPU tests pass their CPU restatement of the codec, to check the framing state
machine).
"""
from __future__ import annotations

import re
import struct
import uuid as _uuid

OP_HELLO = 0xFF    # xcodec_filter.cc:52
OP_LEARN = 0xFE    # :64
OP_ASK = 0xFD      # :79
OP_EOS = 0xFC      # :92
OP_EOS_ACK = 0xFB  # :104
OP_FRAME = 0x00    # :116
MAX_FRAME = 32768  # :118
TO_BE_CONTINUED = 1  # common/count_filter.h:17
UUID_STRING_SIZE = 36  # common/uuid/uuid.h:54
SEGMENT_LENGTH = 2048
_UUID_RE = re.compile(rb"^[0-9a-fA-F]{8}-[0-9a-fA-F]{4}-[0-9a-fA-F]{4}-[0-9a-fA-F]{4}-[0-9a-fA-F]{12}$")


class Filter:
    """``common/filter.h:18-31``."""

    def __init__(self):
        self.recipient: Filter | None = None

    def chain(self, nxt: "Filter") -> None:
        self.recipient = nxt

    def consume(self, buf: bytes, flg: int = 0) -> bool:
        return self.produce(buf, flg)

    def produce(self, buf: bytes, flg: int = 0) -> bool:
        return self.recipient is not None and self.recipient.consume(bytes(buf), flg)

    def flush(self, flg: int) -> None:
        if self.recipient is not None:
            self.recipient.flush(flg)


class Sink(Filter):
    """End of a chain: keeps what reaches it, and the flush flags."""

    def __init__(self):
        super().__init__()
        self.data = bytearray()
        self.flushes: list[int] = []

    def consume(self, buf: bytes, flg: int = 0) -> bool:
        self.data += buf
        return True

    def flush(self, flg: int) -> None:
        self.flushes.append(flg)

    def take(self) -> bytes:
        d = bytes(self.data)
        self.data.clear()
        return d


class DeviceBackend:
    """The device codec: stores are :class:`~wanproxy_amd.xcodec.XCodecCache` (HBM), encoders
    :class:`~wanproxy_amd.xcodec.XCodecStreamEncoder`, decode one device decode call, segment
    hashes ``xc_hash_segments_host``."""

    def __init__(self, ctx, capacity: int = 1 << 16):
        from . import xcodec
        self._x = xcodec
        self.ctx = ctx
        self.capacity = capacity

    def new_store(self):
        return self._x.XCodecCache(self.ctx, self.capacity)

    def new_encoder(self, store):
        return self._x.XCodecStreamEncoder(store)

    def encode(self, encoder, data: bytes, flush: bool) -> bytes:
        # encode(enc, buf) [+ flush(enc)] as one device call
        return self._x.encode_streams([(encoder, data, flush)])[0]

    def flush(self, encoder) -> tuple[bool, bytes]:
        return encoder.flush()

    def decode(self, store, data: bytes) -> tuple[bool, bytes, int, int | None]:
        st, out, consumed, unknown = self._x.XCodecDecoder(store).decode_batch([data])[0]
        return bool(st), out, consumed, unknown

    def hash_segment(self, seg: bytes) -> int:
        return int(self._x.hash_segments_host(self.ctx, seg)[0])


class CodecCache:
    """An XCodecCache as the pipe sees it (``xcodec/xcodec_cache.h:100-126``): the store plus
    its identifier (UUID string) and nominal size in MB (sent in ``<HELLO>``)."""

    def __init__(self, store, uuid: str | None = None, size: int = 0):
        self.store = store
        self.uuid = (uuid or str(_uuid.uuid4())).lower()
        self.size = size

    def identifier(self) -> str:
        return self.uuid

    def nominal_size(self) -> int:
        return self.size

    def lookup(self, h: int) -> bytes | None:
        return self.store.lookup(h)

    def enter(self, h: int, seg: bytes) -> None:
        self.store.enter(h, seg)


class CacheRegistry:
    """``WanProxyCore::find_cache`` / ``add_cache`` (``proxy/wanproxy.h:106-130``): the caches of
    a process by UUID; a decoder's ``<HELLO>`` finds its peer's cache here or adds one."""

    def __init__(self, backend):
        self.backend = backend
        self.caches: dict[str, CodecCache] = {}

    def find_cache(self, uuid: str) -> CodecCache | None:
        return self.caches.get(uuid.lower())

    def add_cache(self, size: int, uuid: str) -> CodecCache:
        assert uuid.lower() not in self.caches
        c = CodecCache(self.backend.new_store(), uuid, size)
        self.caches[c.uuid] = c
        return c

    def register(self, cache: CodecCache) -> CodecCache:
        self.caches[cache.uuid] = cache
        return cache


class Codec:
    """``WANProxyCodec`` (``proxy/wanproxy_codec.h:43-71``): the local cache (``xcache_``), the
    backend that makes caches and codecs, and the registry peer caches are found in."""

    def __init__(self, backend, cache: CodecCache | None, registry: CacheRegistry):
        self.backend = backend
        self.cache = cache
        self.registry = registry


def _frame(src: bytearray, trg: bytearray) -> None:
    """``EncodeFilter::encode_frame`` (``xcodec_filter.cc:189-203``): one frame of at most
    32768 bytes taken from the front of ``src``."""
    n = min(len(src), MAX_FRAME)
    trg.append(OP_FRAME)
    trg += struct.pack(">H", n)
    trg += src[:n]
    del src[:n]


class EncodeFilter(Filter):
    """``xcodec_filter.h:25-57`` / ``xcodec_filter.cc:122-216``.  ``flg & 1`` = waiting mode."""

    def __init__(self, codec: Codec | None, flg: int = 0):
        super().__init__()
        self.codec = codec
        self.cache = codec.cache if codec else None
        self.encoder = None
        self.waiting = bool(flg & 1)
        self.wait_armed = False  # wait_action_: a flush is due at on_read_timeout()
        self.sent_eos = False
        self.eos_ack = False
        self.flushing = False
        self.flush_flags = 0

    def consume(self, buf: bytes, flg: int = 0) -> bool:
        assert not self.flushing
        output = bytearray()
        if self.encoder is None:
            if self.cache is None or not _UUID_RE.match(self.cache.identifier().encode()):
                return False  # "Could not encode UUID for <HELLO>."
            output.append(OP_HELLO)
            output.append(UUID_STRING_SIZE + 8)
            output += self.cache.identifier().encode()
            output += struct.pack("<Q", self.cache.nominal_size())  # host order (x86-64)
            self.encoder = self.codec.backend.new_encoder(self.cache.store)
        flush_now = not (flg & TO_BE_CONTINUED) and not self.waiting
        if not (flg & TO_BE_CONTINUED) and self.waiting:
            self.wait_armed = True  # (re)start the timer; on_read_timeout() flushes
        enc = bytearray(self.codec.backend.encode(self.encoder, bytes(buf), flush_now))
        while enc:
            _frame(enc, output)
        return self.produce(output, flg) if output else True

    def flush(self, flg: int) -> None:
        if flg == OP_EOS_ACK:
            self.eos_ack = True
        else:
            self.flushing = True
            self.flush_flags |= flg
            self.wait_armed = False
            if not self.sent_eos:
                output = bytearray()
                if self.encoder is not None:
                    emitted, enc = self.codec.backend.flush(self.encoder)
                    if emitted:
                        _frame(bytearray(enc), output)  # (one frame, as the reference)
                output.append(OP_EOS)
                self.sent_eos = self.produce(output)
        if self.flushing and self.eos_ack:
            Filter.flush(self, self.flush_flags)

    def on_read_timeout(self) -> None:
        """``EncodeFilter::on_read_timeout`` (``xcodec_filter.cc:205-216``): the waiting-mode
        flush, when the caller's 150 ms timer fires."""
        self.wait_armed = False
        if not self.flushing and self.encoder is not None:
            emitted, enc = self.codec.backend.flush(self.encoder)
            if emitted:
                output = bytearray()
                _frame(bytearray(enc), output)
                self.produce(output)


class DecodeFilter(Filter):
    """``xcodec_filter.h:59-86`` / ``xcodec_filter.cc:220-526``.  ``set_upstream`` names the
    filter that carries ``<ASK>``, ``<LEARN>`` and ``<EOS_ACK>`` back to the peer (the local
    EncodeFilter of the reverse direction)."""

    def __init__(self, codec: Codec):
        super().__init__()
        self.codec = codec
        self.encoder_cache = codec.cache if codec else None
        self.decoder = False
        self.decoder_cache: CodecCache | None = None
        self.unknown_hashes: set[int] = set()
        self.frame_buffer = bytearray()
        self.pending = bytearray()
        self.received_eos = False
        self.sent_eos_ack = False
        self.received_eos_ack = False
        self.upflushed = False
        self.flushing = False
        self.flush_flags = 0
        self.upstream: Filter | None = None

    def set_upstream(self, f: Filter) -> None:
        self.upstream = f

    def consume(self, buf: bytes, flg: int = 0) -> bool:
        if self.upstream is None:
            return False  # "Decoder not configured"
        backend = self.codec.backend
        self.pending += buf
        while self.pending:
            op = self.pending[0]
            if op == OP_HELLO:
                if self.decoder_cache is not None:
                    return False  # "Got <HELLO> twice."
                if len(self.pending) < 2:
                    return True
                ln = self.pending[1]
                if len(self.pending) < 2 + ln:
                    return True
                if ln != UUID_STRING_SIZE + 8:
                    return False  # "Unsupported <HELLO> length"
                del self.pending[:2]
                text = bytes(self.pending[:UUID_STRING_SIZE])
                del self.pending[:UUID_STRING_SIZE]
                if not _UUID_RE.match(text):
                    return False  # "Invalid UUID in <HELLO>."
                mb = struct.unpack("<Q", bytes(self.pending[:8]))[0]
                del self.pending[:8]
                uuid = text.decode().lower()
                reg = self.codec.registry
                self.decoder_cache = reg.find_cache(uuid) or reg.add_cache(mb, uuid)
                self.decoder = self.decoder_cache is not None
            elif op == OP_ASK:
                if self.encoder_cache is None:
                    return False
                if len(self.pending) < 9:
                    return True
                h = struct.unpack(">Q", bytes(self.pending[1:9]))[0]
                del self.pending[:9]
                seg = self.encoder_cache.lookup(h)
                if seg is None:
                    return False  # "Unknown hash in <ASK>"
                if not self.upstream.produce(bytes([OP_LEARN]) + seg):
                    return False
            elif op == OP_LEARN:
                if self.decoder_cache is None:
                    return False  # "Got <LEARN> before <HELLO>."
                if len(self.pending) < 1 + SEGMENT_LENGTH:
                    return True
                data = bytes(self.pending[1:1 + SEGMENT_LENGTH])
                del self.pending[:1]
                h = backend.hash_segment(data)
                self.unknown_hashes.discard(h)  # (else: a gratuitous <LEARN>)
                old = self.decoder_cache.lookup(h)
                if old is not None:
                    if old != data:
                        return False  # "Collision in <LEARN>."
                else:
                    self.decoder_cache.enter(h, data)
                del self.pending[:SEGMENT_LENGTH]
            elif op == OP_EOS:
                if self.received_eos:
                    return False  # "Duplicate <EOS>."
                del self.pending[:1]
                self.received_eos = True
            elif op == OP_EOS_ACK:
                if self.received_eos_ack:
                    return False  # "Duplicate <EOS_ACK>."
                del self.pending[:1]
                self.received_eos_ack = True
            elif op == OP_FRAME:
                if not self.decoder:
                    return False  # "Got frame data before decoder initialized."
                if len(self.pending) < 3:
                    return True
                ln = struct.unpack(">H", bytes(self.pending[1:3]))[0]
                if ln == 0 or ln > MAX_FRAME:
                    return False  # "Invalid framed data length."
                if len(self.pending) < 3 + ln:
                    return True
                self.frame_buffer += self.pending[3:3 + ln]
                del self.pending[:3 + ln]
            else:
                return False  # "Unsupported operation in pipe stream."

            if not self.frame_buffer:
                continue
            if self.unknown_hashes:
                continue  # waiting for <LEARN>s
            ok, output, consumed, unknown = backend.decode(self.decoder_cache.store, bytes(self.frame_buffer))
            if not ok:
                return False  # "Decoder exiting with error."
            del self.frame_buffer[:consumed]
            if unknown is not None:
                self.unknown_hashes.add(unknown)
            if output:
                assert not self.flushing
                if not self.produce(output, flg):
                    return False
            ask = b"".join(bytes([OP_ASK]) + struct.pack(">Q", h) for h in sorted(self.unknown_hashes))
            if ask and not self.upstream.produce(ask):
                return False

        if self.received_eos and not self.sent_eos_ack and not self.frame_buffer:
            self.sent_eos_ack = True
            if not self.upstream.produce(bytes([OP_EOS_ACK])):
                return False
        if self.received_eos and not self.flushing:
            if not self.unknown_hashes:
                if self.frame_buffer:
                    return False
                self.flushing = True
                Filter.flush(self, 0)
            elif not self.frame_buffer:
                return False
        if self.sent_eos_ack and self.received_eos_ack and not self.upflushed:
            self.upflushed = True
            self.upstream.flush(OP_EOS_ACK)
        return True

    def flush(self, flg: int) -> None:
        self.flushing = True
        self.flush_flags |= flg
        if not self.upflushed and self.upstream is not None:
            self.upflushed = True
            self.upstream.flush(OP_EOS_ACK)
        Filter.flush(self, self.flush_flags)
