"""Source hashes of the prebuilt binaries the GPU box runs but cannot rebuild
(it has no /root/reference, so no Eigen / reference headers): the workload
library math_amd/lib/libsmg_bench.so, the C++ drop-in tests tests/cpp/_bin/*
and the reference harness oracle/_ref/*.  Each is compiled with
-DSMG_SOURCE_HASH=<this hash of its sources> (include/smg_source_tag.h keeps
the tag "SMG_SOURCE_HASH=<hex>" in the binary); bench.py, smoke() and the
tests that run them compare the tag with the tree's sources and refuse a
stale binary.

    python3 math_amd/srchash.py GROUP      print GROUP's hash (the Makefiles)
"""
import glob
import hashlib
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_TAG = re.compile(rb"SMG_SOURCE_HASH=([0-9a-f]{16})")


def _headers():
    h = sorted(glob.glob(os.path.join(ROOT, "math_amd", "include", "**", "*.hpp"), recursive=True))
    return h + [os.path.join(ROOT, "include", "smg_hip.h")]


def group_files(group):
    """The sources a binary of `group` is built from: "bench", "ref", or
    "cpp:<stem>" (tests/cpp/<stem>.cpp)."""
    if group == "bench":
        return [os.path.join(ROOT, "math_amd", "bench", "smg_bench.cpp")] + _headers()
    if group == "ref":
        return [os.path.join(ROOT, "oracle", f) for f in ("ref_harness.cpp", "gen.h")] + \
            [os.path.join(ROOT, "tests", "cpp", "boundary_cases.hpp")]
    if group.startswith("cpp:"):
        own = os.path.join(ROOT, "tests", "cpp", group[4:] + ".cpp")
        return [own] + sorted(glob.glob(os.path.join(ROOT, "tests", "cpp", "*.hpp"))) + _headers()
    raise ValueError(f"unknown source group {group!r}")


def source_hash(group):
    h = hashlib.sha256()
    for p in group_files(group):
        h.update(os.path.relpath(p, ROOT).encode() + b"\0")
        with open(p, "rb") as f:
            h.update(f.read())
        h.update(b"\0")
    return h.hexdigest()[:16]


def embedded_hash(path):
    """The SMG_SOURCE_HASH tag compiled into a binary, or None."""
    with open(path, "rb") as f:
        m = _TAG.search(f.read())
    return m.group(1).decode() if m else None


def check(path, group):
    """Raise when the binary at `path` was not built from the tree's sources of `group`."""
    want, got = source_hash(group), embedded_hash(path)
    if got != want:
        raise RuntimeError(f"{os.path.relpath(path, ROOT)} is stale: built from sources {got}, the tree has "
                           f"{want} ({group}); rebuild it in the container (__graft_entry__.build())")


if __name__ == "__main__":
    print(source_hash(sys.argv[1]))
