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

Cross-connection batching: the reference calls the codec once per ``consume``
on its one event thread (``event/event_system.cc:45-56``), one connection at a time.  A
:class:`Batcher` attached to the :class:`Codec` defers the codec calls of one event-loop turn:
every ``EncodeFilter.consume`` becomes one call of a single device batch (``xc_encode_streams``),
every frames-only ``DecodeFilter.consume`` one stream of a device decode batch per cache, and the
framing and ``produce`` of each deferred consume then run in call order.  The device batches keep
the reference's single-thread order exactly (one cache shared by the calls in call order), so the
wire bytes are those of the unbatched filters.
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

    def encode_many(self, calls) -> list[bytes]:
        """One device call for ``(encoder, data, flush)`` calls in order (xc_encode_streams)."""
        return self._x.encode_streams(calls)

    def decode_many(self, store, datas) -> list[tuple[bool, bytes, int, int | None]]:
        """One device call: XCodecDecoder::decode of each input in order, one cache."""
        res = self._x.XCodecDecoder(store).decode_batch(list(datas))
        return [(bool(st), out, consumed, unknown) for st, out, consumed, unknown in res]

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
    backend that makes caches and codecs, and the registry peer caches are found in; ``batcher``
    (optional) defers the filters' codec calls to the end of the event-loop turn."""

    def __init__(self, backend, cache: CodecCache | None, registry: CacheRegistry,
                 batcher: "Batcher | None" = None):
        self.backend = backend
        self.cache = cache
        self.registry = registry
        self.batcher = batcher


class Batcher:
    """The codec calls of one event-loop turn, for every connection, as few device calls.

    Filters submit jobs in call order: an encode job is ``(encoder, data, flush)`` plus a
    completion that frames and produces the output; a decode job is a DecodeFilter whose frame
    buffer is decoded when the job runs.  :meth:`run` (end of the turn; also whenever a filter
    needs every earlier call finished) cuts the job list into rounds, each the longest prefix of the
    remaining jobs in which no filter repeats and no cache is both encoded and decoded, and runs a
    round as one ``backend.encode_many`` call plus one ``backend.decode_many`` call per decoder
    cache, then the completions in call order.  Calls in a round share their caches exactly as the
    reference's sequential calls do (the device batches process their items in order against one
    cache), and every call of a round precedes every call of the next in call order, so the
    results are the unbatched ones.

    :meth:`run` returns the filters whose deferred consume failed since the last :meth:`run`,
    including failures of the runs a filter triggers itself (``flush``, ``on_read_timeout``, a
    decoder consume that needs the earlier calls finished).  A failed filter is also marked
    (``deferred_failed``): its next ``consume`` returns False, as the reference's consume of that
    call would have (``xcodec_filter.cc:146-164,414-418``), and the caller tears the connection
    down."""

    def __init__(self, backend):
        self.backend = backend
        self.jobs: list = []
        self.device_calls = 0
        self._failed: list = []  # not reported by run() yet

    def submit_encode(self, owner, encoder, store, data: bytes, flush: bool, done) -> None:
        self.jobs.append(("e", owner, store, (encoder, data, flush), done))

    def submit_decode(self, owner, store, done) -> None:
        self.jobs.append(("d", owner, store, None, done))

    def pending(self, owner) -> bool:
        return any(j[1] is owner for j in self.jobs)

    def run(self) -> list:
        """End of the event-loop turn: every deferred call; the filters that failed since the last
        ``run``."""
        self.drain()
        failed, self._failed = self._failed, []
        return failed

    def drain(self) -> None:
        """Every deferred call now (a filter needs its earlier calls finished); failures are kept
        for the next :meth:`run` and marked on the filters."""
        while self.jobs:
            rnd, owners, enc_stores, dec_stores = [], set(), set(), set()
            for j in self.jobs:
                kind, owner, store = j[0], j[1], j[2]
                if id(owner) in owners:
                    break
                if (kind == "e" and id(store) in dec_stores) or (kind == "d" and id(store) in enc_stores):
                    break
                owners.add(id(owner))
                (enc_stores if kind == "e" else dec_stores).add(id(store))
                rnd.append(j)
            del self.jobs[:len(rnd)]
            results = [None] * len(rnd)
            enc = [k for k, j in enumerate(rnd) if j[0] == "e"]
            if enc:
                outs = self.backend.encode_many([rnd[k][3] for k in enc])
                self.device_calls += 1
                for k, o in zip(enc, outs):
                    results[k] = o
            by_store: dict = {}
            for k, j in enumerate(rnd):
                if j[0] == "d":
                    by_store.setdefault(id(j[2]), []).append(k)
            for ks in by_store.values():
                store = rnd[ks[0]][2]
                outs = self.backend.decode_many(store, [bytes(rnd[k][1].frame_buffer) for k in ks])
                self.device_calls += 1
                for k, o in zip(ks, outs):
                    results[k] = o
            for j, r in zip(rnd, results):
                if not j[4](r):
                    j[1].deferred_failed = True
                    self._failed.append(j[1])


def _frame(src: bytearray, trg: bytearray) -> None:
    """``EncodeFilter::encode_frame`` (``xcodec_filter.cc:189-203``): one frame of at most
    32768 bytes taken from the front of ``src``."""
    n = min(len(src), MAX_FRAME)
    trg.append(OP_FRAME)
    trg += struct.pack(">H", n)
    trg += src[:n]
    del src[:n]


def _frames(enc: bytes, trg: bytearray) -> None:
    """Every frame of ``enc`` (``encode_frame`` until the encoded bytes are used up)."""
    mv = memoryview(enc)
    for o in range(0, len(enc), MAX_FRAME):
        n = min(len(enc) - o, MAX_FRAME)
        trg.append(OP_FRAME)
        trg += struct.pack(">H", n)
        trg += mv[o:o + n]


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
        self.deferred_failed = False  # a deferred consume of this filter failed (Batcher)

    def consume(self, buf: bytes, flg: int = 0) -> bool:
        if self.deferred_failed:
            return False
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

        def done(enc: bytes) -> bool:
            _frames(enc, output)
            return self.produce(output, flg) if output else True
        b = self.codec.batcher
        if b is not None:  # deferred to the end of the turn: one device call for every connection
            b.submit_encode(self, self.encoder, self.cache.store, bytes(buf), flush_now, done)
            return True
        return done(self.codec.backend.encode(self.encoder, bytes(buf), flush_now))

    def _drain(self) -> None:
        # a direct codec call must follow every deferred one (the reference's order)
        if self.codec is not None and self.codec.batcher is not None:
            self.codec.batcher.drain()

    def flush(self, flg: int) -> None:
        self._drain()
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
        self._drain()
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
        self.deferred_failed = False  # a deferred decode of this filter failed (Batcher)

    def set_upstream(self, f: Filter) -> None:
        self.upstream = f

    def _frames_only(self, data: bytes) -> bool:
        """Whether ``data`` (pending bytes) holds only <HELLO> (first) and <FRAME> messages, the
        last one possibly incomplete: such a consume changes nothing but the frame buffer before
        its decode, which can then be deferred."""
        i, n = 0, len(data)
        while i < n:
            op = data[i]
            if op == OP_FRAME:
                if n - i < 3:
                    return True
                i += 3 + struct.unpack(">H", data[i + 1:i + 3])[0]
            elif op == OP_HELLO and i == 0 and self.decoder_cache is None:
                if n - i < 2:
                    return True
                i += 2 + data[i + 1]
            else:
                return False
        return True

    def _decoded(self, res, flg: int) -> bool:
        """The part of the frame loop after ``XCodecDecoder::decode`` (xcodec_filter.cc:414-455)."""
        ok, output, consumed, unknown = res
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
        return True

    def consume(self, buf: bytes, flg: int = 0) -> bool:
        if self.upstream is None:
            return False  # "Decoder not configured"
        if self.deferred_failed:
            return False
        b = self.codec.batcher if self.codec is not None else None
        if b is not None:
            if (not self.received_eos and not self.unknown_hashes and not b.pending(self)
                    and self._frames_only(bytes(self.pending) + bytes(buf))):
                # frames only: parse now, decode at the end of the turn in the device batch (the
                # frames of one consume decode in one call as they do one by one: the decoder
                # keeps a token that straddles frames, and stops at the first unknown REF)
                self.pending += buf
                if not self._parse(flg, defer=True):
                    return False
                if self.frame_buffer and not self.unknown_hashes:
                    b.submit_decode(self, self.decoder_cache.store, lambda r: self._decoded(r, flg))
                return True
            b.drain()  # anything else runs now, after every earlier deferred call
            if self.deferred_failed:
                return False  # (its own deferred decode failed: this consume is the teardown)
        self.pending += buf
        return self._parse(flg, defer=False)

    def _parse(self, flg: int, defer: bool) -> bool:
        backend = self.codec.backend
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
            if defer:
                continue  # (the batch decodes the frame buffer once every frame is in)
            if not self._decoded(backend.decode(self.decoder_cache.store, bytes(self.frame_buffer)), flg):
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
        if self.codec is not None and self.codec.batcher is not None:
            self.codec.batcher.drain()  # (a failure is reported by the turn's run())
        self.flushing = True
        self.flush_flags |= flg
        if not self.upflushed and self.upstream is not None:
            self.upflushed = True
            self.upstream.flush(OP_EOS_ACK)
        Filter.flush(self, self.flush_flags)
