"""The drop-in boundary compiles (CPU, this container only: it needs /root/reference's sources).

facade/xcodec/ replaces the reference's xcodec_cache.h, xcodec_encoder.{h,cc}, xcodec_decoder.{h,cc}
and cache/coss/xcodec_cache_coss.h.  This test compiles the reference's own,
unchanged xcodec/xcodec_filter.cc (the EncodeFilter / DecodeFilter that call the codec,
xcodec_filter.cc:122-512) and proxy/wanproxy_codec.h (WANProxyCodec::xcache_, :43-71) against it,
then links the facade with the reference's Buffer (common/buffer.cc) and round-trips a stream.

Two test-only pieces make that possible here (tests/facade/): the three libuuid declarations
common/uuid/uuid.h needs (the image has libuuid.so.1 but not its header), and, for the CPU round
trip, the part of the C ABI the facade calls over the CPU oracle (the product library needs a GPU).
This is a check of our headers against the reference's code, not an oracle claim; nothing built
here goes to the GPU box."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"

pytestmark = pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "xcodec")), reason="needs the reference sources")

FLAGS = ["-std=gnu++17", "-O1", "-DNDEBUG=1", "-Wno-deprecated", "-include", "common/common.h",
         "-I" + os.path.join(ROOT, "facade"), "-I" + os.path.join(ROOT, "include"), "-I" + REF,
         "-I" + os.path.join(ROOT, "tests", "facade", "shim")]


def _cc(args, cwd):
    r = subprocess.run(["g++"] + FLAGS + args, cwd=cwd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-4000:]


def test_reference_filter_compiles_against_the_facade(tmp_path):
    _cc(["-c", os.path.join(REF, "xcodec", "xcodec_filter.cc"), "-o", "filter.o"], tmp_path)
    (tmp_path / "codec_tu.cc").write_text("#include <proxy/wanproxy_codec.h>\n#include <proxy/wanproxy.h>\n")
    _cc(["-c", "codec_tu.cc", "-o", "codec.o"], tmp_path)
    # the filter calls exactly the facade's codec and cache classes
    nm = subprocess.run(["nm", "-C", "-u", str(tmp_path / "filter.o")], capture_output=True, text=True).stdout
    for sym in ("XCodecEncoder::XCodecEncoder(XCodecCache*)", "XCodecEncoder::encode(Buffer&, Buffer&)",
                "XCodecEncoder::flush(Buffer&)", "XCodecDecoder::XCodecDecoder(XCodecCache*)",
                "XCodecDecoder::decode(Buffer&, Buffer&, std::set<unsigned long"):
        assert sym in nm, sym


def test_facade_round_trip_with_the_reference_buffer(tmp_path):
    make = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], capture_output=True, text=True)
    assert make.returncode == 0, make.stderr
    fac = os.path.join(ROOT, "facade", "xcodec")
    t = os.path.join(ROOT, "tests", "facade")
    _cc(["-o", "rt", os.path.join(t, "facade_roundtrip.cc"), os.path.join(fac, "xcodec_encoder.cc"),
         os.path.join(fac, "xcodec_decoder.cc"), os.path.join(t, "xc_abi_oracle.cc"),
         os.path.join(REF, "common", "buffer.cc"), os.path.join(REF, "common", "log.cc"),
         os.path.join(REF, "common", "uuid", "uuid.cc"), "-L" + os.path.join(ROOT, "oracle"), "-loracle",
         "-Wl,-rpath," + os.path.join(ROOT, "oracle"), "-l:libuuid.so.1"], tmp_path)
    r = subprocess.run([str(tmp_path / "rt")], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "facade ok" in r.stdout, r.stdout + r.stderr


def _build_filter_program(tmp_path):
    """The reference's unchanged xcodec_filter.cc with its event system, Buffer and log, over the
    facade and the CPU stand-in of the C ABI (tests/facade/facade_filter.cc)."""
    make = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], capture_output=True, text=True)
    assert make.returncode == 0, make.stderr
    fac = os.path.join(ROOT, "facade", "xcodec")
    t = os.path.join(ROOT, "tests", "facade")
    ref = [os.path.join(REF, f) for f in ("xcodec/xcodec_filter.cc", "event/event_system.cc", "event/io_service.cc",
                                          "event/event_poll_epoll.cc", "common/thread/thread.cc", "common/log.cc",
                                          "common/buffer.cc", "common/uuid/uuid.cc")]
    # (sections: the DecodeFilter half of the TU needs the proxy's globals, which this program does
    # not link; the linker drops it, EncodeFilter is what runs)
    _cc(["-w", "-ffunction-sections", "-fdata-sections", "-Wl,--gc-sections", "-o", "ff",
         os.path.join(t, "facade_filter.cc"), os.path.join(fac, "xcodec_encoder.cc"),
         os.path.join(fac, "xcodec_decoder.cc"), os.path.join(t, "xc_abi_oracle.cc")] + ref +
        ["-L" + os.path.join(ROOT, "oracle"), "-loracle", "-Wl,-rpath," + os.path.join(ROOT, "oracle"),
         "-l:libuuid.so.1", "-lpthread"], tmp_path)
    return str(tmp_path / "ff")


def test_reference_filter_over_the_facade_never_throws(tmp_path):
    """No exception crosses the reference's filter (xcodec_filter.cc:122-164 has no handler, and the
    reference's encoder cannot fail, xcodec_encoder.h:53-57): EncodeFilter::consume meets XC_EBUSY on
    every library call and the facade finishes the run in flight (xc_cache_quiesce) and calls again,
    the stream round-trips exactly; a failing decode is decode() == false; a failing encode halts
    (the reference's HALT: logged, abort), as a failed allocation would."""
    ff = _build_filter_program(tmp_path)
    r = subprocess.run([ff], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "facade filter ok" in r.stdout, r.stdout + r.stderr
    r = subprocess.run([ff, "busy"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "facade filter ok" in r.stdout and " 0 quiesced" not in r.stdout, r.stdout + r.stderr
    r = subprocess.run([ff, "fail-decode"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "decode false" in r.stdout and "device decode failed" in r.stderr, r.stdout + r.stderr
    r = subprocess.run([ff, "fail-encode"], capture_output=True, text=True, timeout=120)
    assert r.returncode == -6 and "Halting: encode" in r.stderr, (r.returncode, r.stdout, r.stderr)


def test_filter_turns_driver_over_the_stand_in(tmp_path):
    """The driver of the GPU drop-in test (tests/facade/filter_turns.cc, tests/test_gpu_facade.py)
    with the CPU stand-in of the C ABI: the reference's EncodeFilter / DecodeFilter pipes between two
    proxies, <ASK>/<LEARN> included, give the oracle pipes' bytes.  (This checks the harness; the GPU
    test runs the same driver over the product library.)"""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    from pipe_harness import OracleBackend, read_outputs, run_scenario, write_scenario
    from test_gpu_pipe_cpp import _scenario
    make = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], capture_output=True, text=True)
    assert make.returncode == 0, make.stderr
    fac = os.path.join(ROOT, "facade", "xcodec")
    t = os.path.join(ROOT, "tests", "facade")
    ref = [os.path.join(REF, f) for f in ("xcodec/xcodec_filter.cc", "event/event_system.cc", "event/io_service.cc",
                                          "event/event_poll_epoll.cc", "common/thread/thread.cc", "common/log.cc",
                                          "common/buffer.cc", "common/uuid/uuid.cc")]
    _cc(["-w", "-ffunction-sections", "-fdata-sections", "-Wl,--gc-sections", "-o", "ft",
         os.path.join(t, "filter_turns.cc"), os.path.join(fac, "xcodec_encoder.cc"),
         os.path.join(fac, "xcodec_decoder.cc"), os.path.join(t, "xc_abi_oracle.cc")] + ref +
        ["-L" + os.path.join(ROOT, "oracle"), "-loracle", "-Wl,-rpath," + os.path.join(ROOT, "oracle"),
         "-l:libuuid.so.1", "-lpthread"], tmp_path)
    warm, order, inputs = _scenario(3, nconn=6, turns=3)
    sc, out = tmp_path / "sc.bin", tmp_path / "out.bin"
    write_scenario(sc, warm, order, inputs, waiting=False, batched=False)
    r = subprocess.run([str(tmp_path / "ft"), "parity", str(sc), str(out)], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0 and "parity ok" in r.stdout, r.stdout + r.stderr
    got = read_outputs(out, len(inputs))
    want = run_scenario(OracleBackend(oracle), warm, order, inputs, waiting=False, batched=False)
    assert got == want
    assert sum(g[1].count(b"\xfd") for g in got) > 0
