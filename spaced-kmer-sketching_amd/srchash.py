"""Source hash of libsks.so: sha256 over the library's source files (every
csrc/*.hip, csrc/*.cpp, csrc/*.hpp, cpp/*.cpp, cpp/*.hpp and include/sks.h),
each as its package-relative path, a NUL, its bytes and a NUL, in sorted path
order; first 16 hex digits.  The Makefile compiles it into the library
(sks_build_info) and tests/conftest.py recomputes it, so a test run proves the
loaded binary was built from the sources it sits next to."""
import glob
import hashlib
import os
import sys

PKG = os.path.dirname(os.path.abspath(__file__))


def files():
    pats = ["csrc/*.hip", "csrc/*.cpp", "csrc/*.hpp", "cpp/*.cpp", "cpp/*.hpp", "../include/sks.h"]
    out = []
    for p in pats:
        out += [os.path.relpath(f, PKG) for f in glob.glob(os.path.join(PKG, p))]
    return sorted(out)


# the sources the fused scan kernel is compiled from (profiles/rNN/traffic.json
# records this hash; bench.py uses a traffic figure only when it still matches)
SCAN_FILES = ["csrc/scan.hip", "csrc/sks_hash.hpp", "csrc/sks_internal.hpp"]


def source_hash(rels=None):
    h = hashlib.sha256()
    for rel in (files() if rels is None else sorted(rels)):
        h.update(rel.encode() + b"\0")
        with open(os.path.join(PKG, rel), "rb") as f:
            h.update(f.read())
        h.update(b"\0")
    return h.hexdigest()[:16]


# the sources of the all-pairs join (k_join and its layout build):
# profiles/rNN/pair_lds.json records this hash
JOIN_FILES = ["csrc/join.hip", "csrc/join_common.hpp", "csrc/layout.hip", "csrc/sks_internal.hpp"]


def scan_hash():
    return source_hash(SCAN_FILES)


def join_hash():
    return source_hash(JOIN_FILES)


if __name__ == "__main__":
    sys.stdout.write(source_hash())
