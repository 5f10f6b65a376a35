"""The C-ABI library loads on a GPU-less host and exports every symbol that
include/cronsun_gpu.h declares (no compute calls here)."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "cronsun_gpu.h")
LIB = os.path.join(ROOT, "cronsun_amd", "libcronsun_gpu.so")


def declared():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(cg_[a-z0-9_]+)\s*\(", txt)))


def test_header_declares_entry_points():
    names = declared()
    for must in ("cg_parse", "cg_next_batch", "cg_expand", "cg_expand_per_node", "cg_init"):
        assert must in names


def test_library_exports_every_declared_symbol():
    assert os.path.exists(LIB), "build the library first (__graft_entry__.build())"
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r"\bT (cg_[a-z0-9_]+)", out))
    missing = [n for n in declared() if n not in exported]
    assert not missing, missing


def test_library_loads_and_binds_all_symbols():
    from cronsun_amd import _lib
    L = _lib.lib()
    assert L.cg_abi_version() == _lib.ABI_VERSION == 3
    assert set(_lib.SYMBOLS) == set(declared())


def test_no_device_here_fails_loudly():
    from cronsun_amd import _lib, engine
    if engine.device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(_lib.CgError) as e:
        engine.Engine(0)
    assert e.value.code == _lib.CG_ENODEV


def test_library_does_not_link_oracle():
    out = subprocess.run(["nm", "-D", LIB], capture_output=True, text=True, check=True).stdout
    assert "or_spec_next" not in out and "or_expand" not in out
    deps = subprocess.run(["readelf", "-d", LIB], capture_output=True, text=True, check=True).stdout
    assert "oracle" not in deps


def test_go_binding_calls_only_declared_symbols():
    """The cgo package (node/cron/gpu/gpu.go, uncompiled here: no Go
    toolchain) calls only entry points the header declares."""
    src = open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                            "node", "cron", "gpu", "gpu.go")).read()
    called = set(re.findall(r"\bC\.(cg_[a-z0-9_]+)\s*\(", src))
    assert called and not (called - set(declared())), sorted(called - set(declared()))
