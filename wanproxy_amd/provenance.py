"""Which library sources a measurement was taken with: a digest of the kernel and runtime sources
(wanproxy_amd/csrc, include/).  The GPU box gets a snapshot without .git, so a commit id is not
available there; the digest is.  bench.py attaches a committed PMC traffic record only when its
digest matches the sources it runs (tools/pmc_traffic.py writes it)."""
import glob
import hashlib
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def source_stamp() -> str:
    h = hashlib.sha256()
    files = sorted(glob.glob(os.path.join(ROOT, "wanproxy_amd", "csrc", "*.hip")) +
                   glob.glob(os.path.join(ROOT, "wanproxy_amd", "csrc", "*.h")) +
                   glob.glob(os.path.join(ROOT, "wanproxy_amd", "csrc", "*.cpp")) +
                   glob.glob(os.path.join(ROOT, "wanproxy_amd", "csrc", "Makefile")) +
                   glob.glob(os.path.join(ROOT, "include", "*.h")))
    for f in files:
        h.update(os.path.relpath(f, ROOT).encode())
        h.update(open(f, "rb").read())
    return h.hexdigest()[:16]
