"""Build-on-demand for libsdp.so.

The shared library is a build artefact (git-ignored), so a fresh checkout has none. ``ensure_built()``
compiles it with the csrc Makefile when it is missing or when the sources changed since it was
built, and raises with the compiler's output if that fails. "Changed" is decided by a content
hash of every csrc file and include/sdp.h, written next to the library as ``libsdp.so.stamp``
(mtimes are not trusted: a tree copied to another machine may carry arbitrary ones -- so a
rebuild is ``make -B``, which recompiles every object whatever its mtime; ``write_stamp()`` marks
a library built by hand with ``make`` in csrc/ as current, for the edit-build loop).

A lock file serialises concurrent callers (e.g. several ranks of one job starting together).
This module imports neither torch nor the library, so it is safe to call before any GPU work.
"""
from __future__ import annotations

import fcntl
import hashlib
import os
import subprocess
import sys

_HERE = os.path.dirname(os.path.abspath(__file__))
PKG_DIR = os.path.dirname(_HERE)
CSRC = os.path.join(PKG_DIR, "csrc")
HEADER = os.path.join(os.path.dirname(PKG_DIR), "include", "sdp.h")
LIB_PATH = os.environ.get("SDP_LIB", os.path.join(_HERE, "_lib", "libsdp.so"))
STAMP = LIB_PATH + ".stamp"


def source_hash() -> str:
    h = hashlib.sha256()
    files = sorted(f for f in os.listdir(CSRC) if f.endswith((".hip", ".h", ".cpp")) or f == "Makefile")
    for f in files:
        h.update(f.encode())
        with open(os.path.join(CSRC, f), "rb") as fh:
            h.update(fh.read())
    with open(HEADER, "rb") as fh:
        h.update(fh.read())
    return h.hexdigest()


CONV_SOURCES = ("common.h", "conv_kernel.h", "conv_launch.h", "conv.hip", "conv_inst.hip")


def conv_source_hash() -> str:
    """Hash of the files the forward conv kernel is built from (tools/conv_bench compiles exactly
    these): the key of the PMC traffic record bench.py reports (profiles/*_traffic.json)."""
    h = hashlib.sha256()
    for f in CONV_SOURCES:
        h.update(f.encode())
        with open(os.path.join(CSRC, f), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()


def _stamp_ok(digest: str) -> bool:
    if not os.path.exists(LIB_PATH) or not os.path.exists(STAMP):
        return False
    with open(STAMP) as fh:
        return fh.read().strip() == digest


def write_stamp() -> None:
    """Mark the current libsdp.so as built from the current sources (after a manual ``make``)."""
    if not os.path.exists(LIB_PATH):
        raise FileNotFoundError(LIB_PATH)
    with open(STAMP, "w") as fh:
        fh.write(source_hash() + "\n")


def ensure_built(force_make: bool = False, verbose: bool = True) -> str:
    """Return the library path, building it first if it is missing or stale."""
    if "SDP_LIB" in os.environ:          # an explicitly provided library is used as is
        return LIB_PATH
    digest = source_hash()
    if not force_make and _stamp_ok(digest):
        return LIB_PATH
    os.makedirs(os.path.dirname(LIB_PATH), exist_ok=True)
    with open(LIB_PATH + ".lock", "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        try:
            if not force_make and _stamp_ok(digest):   # another process built it meanwhile
                return LIB_PATH
            jobs = str(max(1, min(16, os.cpu_count() or 4)))
            if verbose:
                print(f"[sdp] building libsdp.so (make -j{jobs} in {CSRC})", file=sys.stderr, flush=True)
            p = subprocess.Popen(["make", "-B", "-j", jobs, "-C", CSRC], stdout=subprocess.PIPE,
                                 stderr=subprocess.STDOUT, text=True)
            log = []
            for line in p.stdout:
                log.append(line)
                if verbose:
                    print("[sdp] " + line.rstrip()[:200], file=sys.stderr, flush=True)
            if p.wait() != 0 or not os.path.exists(LIB_PATH):
                raise RuntimeError("building libsdp.so failed:\n" + "".join(log[-80:]))
            with open(STAMP, "w") as fh:
                fh.write(digest + "\n")
        finally:
            fcntl.flock(lk, fcntl.LOCK_UN)
    return LIB_PATH
