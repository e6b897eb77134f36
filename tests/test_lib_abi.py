"""CPU-side checks of the C-ABI library: it loads, and exports every symbol include/sdp.h declares."""
import os
import re
import subprocess

from conftest import PKG_DIR, REPO

HEADER = os.path.join(REPO, "include", "sdp.h")
LIB = os.path.join(PKG_DIR, "sdp", "_lib", "libsdp.so")


def declared():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(sdp_\w+)\s*\(", src, re.M)))


def test_header_declares_the_boundary():
    d = declared()
    for s in ("sdp_net_create", "sdp_net_forward", "sdp_langevin_step", "sdp_consistency_merge"):
        assert s in d


def test_library_exports_every_declared_symbol():
    assert os.path.exists(LIB), "build libsdp.so first (python __graft_entry__.py build)"
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r" T (sdp_\w+)", out))
    missing = [s for s in declared() if s not in exported]
    assert not missing, missing


def test_library_loads_and_reports_version():
    from sdp import _lib
    L = _lib.lib()
    assert L.sdp_version() == 100
    assert set(_lib.exported_symbols()) == set(declared())


def test_errors_are_reported_not_crashing():
    from sdp import _lib
    L = _lib.lib()
    d = _lib.NetDesc(64, 2, 64, 1024, 232, 1)   # ngf=64 is not built
    h = _lib.P()
    assert L.sdp_net_create(_lib.C.byref(d), _lib.C.byref(h)) != 0
    assert b"ngf" in L.sdp_last_error()


def test_one_hip_runtime_in_process():
    """libsdp must bind to torch's libamdhip64 instance (shared SONAME), never a second copy."""
    from sdp import _lib
    _lib.lib()
    maps = open("/proc/self/maps").read()
    paths = set(re.findall(r"\S*libamdhip64\S*", maps))
    assert len(paths) == 1, paths
