"""Source hash of the native libraries: the build embeds it (lib/libalert_engine.so:
ae_source_hash, lib/libalert_host.so: ah_source_hash) and the loaders refuse a library whose
hash differs from the sources in this tree — the prebuilt .so files travel with the tree to the
GPU box, so a library left over from other sources must fail loudly, never run.

    python3 buildinfo.py engine|host      (prints the hash; the Makefile's use)
"""
from __future__ import annotations

import hashlib
import pathlib
import sys

PKG = pathlib.Path(__file__).resolve().parent
ROOT = PKG.parent

# what each library is built from (the Makefile's SRCS / HDRS and HOSTSRCS / HOSTHDRS)
PATTERNS = {
    "engine": [(PKG / "csrc", "*.hip"), (PKG / "csrc", "*.h"), (ROOT / "include", "alert_engine.h")],
    "host": [(PKG / "csrc" / "host", "*.cpp"), (PKG / "csrc" / "host", "*.h"),
             (ROOT / "include", "alert_host.h")],
}


def source_hash(kind: str) -> str:
    h = hashlib.sha1()
    files = sorted({p for d, pat in PATTERNS[kind] for p in d.glob(pat)})
    for p in files:
        h.update(p.name.encode() + b"\0")
        h.update(p.read_bytes())
    return h.hexdigest()[:16]


if __name__ == "__main__":
    print(source_hash(sys.argv[1]))
