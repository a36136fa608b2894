"""Test harness for wanproxy_amd.pipe: a duplex pair of XCodec pipes (one EncodeFilter and one
DecodeFilter per side, each side with its own cache registry, as two proxies would have),
connected by queued "wires" so that <ASK>/<LEARN> round trips happen between consume calls as
they do over sockets (xcodec/xcodec_filter.cc, proxy/proxy_connector.cc:154-189).

OracleBackend runs the filters over the oracle restatement (test infrastructure only): the CPU
tests use it to check the framing state machine, the GPU tests as the expected wire bytes."""
import numpy as np

from wanproxy_amd import pipe as P

UUID_A = "0f1e2d3c-4b5a-6978-8796-a5b4c3d2e1f0"
UUID_B = "12345678-9abc-def0-1234-56789abcdef0"


class OracleBackend:
    def __init__(self, oracle_mod):
        self.o = oracle_mod

    def new_store(self):
        return self.o.Cache()

    def new_encoder(self, store):
        return self.o.Encoder(store)

    def encode(self, encoder, data, flush):
        out = encoder.encode(data)
        if flush:
            out += encoder.flush()[1]
        return out

    def flush(self, encoder):
        return encoder.flush()

    def decode(self, store, data):
        st, out, consumed, unknown = store.decode_batch([data])[0]
        return bool(st), out, consumed, unknown

    def hash_segment(self, seg):
        return int(self.o.hash_segment(np.frombuffer(seg, np.uint8)))

    # the Batcher's entry points: sequential, as the reference runs them
    def encode_many(self, calls):
        return [self.encode(e, d, f) for e, d, f in calls]

    def decode_many(self, store, datas):
        return [self.decode(store, d) for d in datas]


class Wire(P.Filter):
    """A socket: bytes queue up until pump() delivers them."""

    def __init__(self):
        super().__init__()
        self.q = bytearray()
        self.log = bytearray()  # everything ever sent
        self.flushes = []

    def consume(self, buf, flg=0):
        self.q += buf
        self.log += buf
        return True

    def flush(self, flg):
        self.flushes.append(flg)


class Side:
    def __init__(self, backend, uuid, warm=None, waiting=False, size=64):
        self.registry = P.CacheRegistry(backend)
        store = backend.new_store()
        if warm is not None:
            warm(store)
        self.cache = self.registry.register(P.CodecCache(store, uuid, size))
        self.codec = P.Codec(backend, self.cache, self.registry)
        self.enc = P.EncodeFilter(self.codec, 1 if waiting else 0)
        self.dec = P.DecodeFilter(self.codec)
        self.sink = P.Sink()
        self.wire = Wire()
        self.enc.chain(self.wire)
        self.dec.chain(self.sink)
        self.dec.set_upstream(self.enc)


def pump(a: Side, b: Side, chunk=None, max_rounds=10**7):
    """Deliver queued wire bytes (a -> b.dec, b -> a.dec) until both wires are idle; every
    consume must succeed.  ``chunk``: deliver at most that many bytes per consume call."""
    for _ in range(max_rounds):
        moved = False
        for src, dst in ((a, b), (b, a)):
            if src.wire.q:
                n = len(src.wire.q) if chunk is None else min(chunk, len(src.wire.q))
                data = bytes(src.wire.q[:n])
                del src.wire.q[:n]
                assert dst.dec.consume(data), "decode filter failed"
                moved = True
        if not moved:
            return
    raise AssertionError("pipes did not settle")


def parse(stream: bytes):
    """Split a pipe stream into (op, payload) messages."""
    out, i = [], 0
    while i < len(stream):
        op = stream[i]
        if op == P.OP_HELLO:
            n = stream[i + 1]
            out.append((op, stream[i + 2:i + 2 + n]))
            i += 2 + n
        elif op == P.OP_FRAME:
            n = int.from_bytes(stream[i + 1:i + 3], "big")
            out.append((op, stream[i + 3:i + 3 + n]))
            i += 3 + n
        elif op == P.OP_ASK:
            out.append((op, stream[i + 1:i + 9]))
            i += 9
        elif op == P.OP_LEARN:
            out.append((op, stream[i + 1:i + 1 + 2048]))
            i += 1 + 2048
        elif op in (P.OP_EOS, P.OP_EOS_ACK):
            out.append((op, b""))
            i += 1
        else:
            raise AssertionError(f"bad op {op:#x} at {i}")
    return out


def esc_buffer(n, seed, frac=0.05):
    rng = np.random.default_rng(seed)
    b = rng.integers(0, 256, n, dtype=np.uint8)
    b[rng.random(n) < frac] = 0xF1
    return b


class Proxy:
    """One WANProxy process's codec side: a local cache (its UUID) shared by every connection's
    EncodeFilter, a registry holding the peers' caches shared by every DecodeFilter, and an
    optional Batcher for the codec calls of each event-loop turn."""

    def __init__(self, backend, uuid, warm=None, batched=False, waiting=False):
        self.registry = P.CacheRegistry(backend)
        store = backend.new_store()
        if warm is not None:
            warm(store)
        self.cache = self.registry.register(P.CodecCache(store, uuid, 64))
        self.batcher = P.Batcher(backend) if batched else None
        self.codec = P.Codec(backend, self.cache, self.registry, self.batcher)
        self.waiting = waiting

    def end_turn(self):
        if self.batcher is not None:
            failed = self.batcher.run()
            assert not failed, "a deferred consume failed"


class Conn:
    """A connection between two proxies: a pipe each way (EncodeFilter -> wire -> DecodeFilter)."""

    def __init__(self, a: Proxy, b: Proxy):
        self.a, self.b = a, b
        self.a_enc = P.EncodeFilter(a.codec, 1 if a.waiting else 0)
        self.a_dec = P.DecodeFilter(a.codec)
        self.b_enc = P.EncodeFilter(b.codec, 1 if b.waiting else 0)
        self.b_dec = P.DecodeFilter(b.codec)
        self.ab, self.ba = Wire(), Wire()
        self.a_sink, self.b_sink = P.Sink(), P.Sink()
        self.a_enc.chain(self.ab)
        self.b_enc.chain(self.ba)
        self.a_dec.chain(self.a_sink)
        self.b_dec.chain(self.b_sink)
        self.a_dec.set_upstream(self.a_enc)
        self.b_dec.set_upstream(self.b_enc)


def pump_turns(a: Proxy, b: Proxy, conns, chunk=None, max_turns=10**6):
    """Deliver queued wire bytes turn by turn: in a turn every connection's queued bytes (as they
    stood when the turn began, at most ``chunk`` per wire) reach the other side's DecodeFilter,
    then both proxies end the turn (the batchers run).  Until every wire is idle."""
    for _ in range(max_turns):
        work = []
        for c in conns:
            for w, dec in ((c.ab, c.b_dec), (c.ba, c.a_dec)):
                if w.q:
                    n = len(w.q) if chunk is None else min(chunk, len(w.q))
                    work.append((dec, bytes(w.q[:n])))
                    del w.q[:n]
        if not work:
            return
        for dec, data in work:
            assert dec.consume(data), "decode filter failed"
        a.end_turn()
        b.end_turn()
    raise AssertionError("pipes did not settle")


def run_connections(backend, warm_a, inputs, batched, chunk=None, order_seed=5, waiting=False):
    """Proxies A (warm cache) and B; connection i sends inputs[i][0], inputs[i][1], ... from A,
    one consume per connection per turn in a seeded shuffled order, pumping between turns; then
    EOS both ways.  Returns (a, b, conns)."""
    a = Proxy(backend, UUID_A, warm=warm_a, batched=batched, waiting=waiting)
    b = Proxy(backend, UUID_B, batched=batched)
    conns = [Conn(a, b) for _ in inputs]
    rng = np.random.default_rng(order_seed)
    turns = max(len(x) for x in inputs)
    for t in range(turns):
        for i in rng.permutation(len(conns)):
            if t < len(inputs[i]):
                assert conns[i].a_enc.consume(inputs[i][t].tobytes())
        a.end_turn()
        b.end_turn()
        if waiting:
            for c in conns:
                c.a_enc.on_read_timeout()
        pump_turns(a, b, conns, chunk)
    for c in conns:
        c.a_enc.flush(0)
    pump_turns(a, b, conns, chunk)
    for c in conns:
        c.b_enc.flush(0)
    pump_turns(a, b, conns, chunk)
    return a, b, conns


# ---- the C++ filters' scenario files (tests/cpp/pipe_turns.cpp) ----------------------------------

def write_scenario(path, warm, order, inputs, waiting=False, batched=True):
    """order[t]: the connections' consume order of turn t; inputs[i][t]: connection i's read of turn
    t (empty: none)."""
    import struct
    nconn, turns = len(inputs), len(order)
    with open(path, "wb") as f:
        f.write(struct.pack("<IIII", nconn, turns, int(waiting), int(batched)))
        f.write(struct.pack("<Q", len(warm)))
        for b in warm:
            f.write(struct.pack("<Q", len(b)) + bytes(b))
        for o in order:
            f.write(struct.pack("<%dI" % nconn, *o))
        for i in range(nconn):
            for t in range(turns):
                b = bytes(inputs[i][t])
                f.write(struct.pack("<Q", len(b)) + b)


def read_outputs(path, nconn):
    """Per connection: (A->B wire bytes, B->A wire bytes, B's sink, A's sink)."""
    import struct
    d = open(path, "rb").read()
    at, res = 0, []
    for _ in range(nconn):
        v = []
        for _ in range(4):
            n = struct.unpack_from("<Q", d, at)[0]
            v.append(d[at + 8:at + 8 + n])
            at += 8 + n
        res.append(tuple(v))
    return res


def run_scenario(backend, warm, order, inputs, waiting=False, batched=True):
    """The scenario of write_scenario through the Python pipes (the expected bytes with the oracle
    backend): the same steps as pipe_turns.cpp's parity mode."""
    a = Proxy(backend, UUID_A, warm=lambda s: s.encode_batch(warm), batched=batched, waiting=waiting)
    b = Proxy(backend, UUID_B, batched=batched)
    conns = [Conn(a, b) for _ in inputs]
    for t, o in enumerate(order):
        for i in o:
            d = bytes(inputs[i][t])
            if d:
                assert conns[i].a_enc.consume(d)
        a.end_turn()
        b.end_turn()
        if waiting:
            for c in conns:
                c.a_enc.on_read_timeout()
        pump_turns(a, b, conns)
    for c in conns:
        c.a_enc.flush(0)
    pump_turns(a, b, conns)
    for c in conns:
        c.b_enc.flush(0)
    pump_turns(a, b, conns)
    return [(bytes(c.ab.log), bytes(c.ba.log), bytes(c.b_sink.data), bytes(c.a_sink.data)) for c in conns]
