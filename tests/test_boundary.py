"""The drop-in boundary: the C-ABI library builds, loads and exports every entry point
declared in include/ragen_amd.h (no kernel is launched: runs without a GPU)."""
import os
import re
import subprocess

import pytest

from ragen_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "ragen_amd.h")).read()
    return sorted(set(re.findall(r"\b(rmi_[a-z0-9_]+)\s*\(", src)))


def test_library_loads():
    L = _lib.lib()
    assert L.rmi_version().startswith(b"ragen_amd")


def test_every_declared_symbol_is_exported():
    L = _lib.lib()
    decl = declared_symbols()
    assert len(decl) >= 18
    for name in decl:
        assert hasattr(L, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r" T (rmi_\w+)", out))
    assert set(decl) <= exported, set(decl) - exported
    # nothing beyond the C ABI leaks out of the library
    assert all(s.startswith("rmi_") for s in exported)


def test_bindings_cover_header():
    assert set(declared_symbols()) == set(_lib.exported_symbols())


def test_code_object_is_gfx950():
    blob = open(_lib.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob


def test_ops_refuse_cpu_tensors():
    import torch
    from ragen_amd import ops
    with pytest.raises(ValueError):
        ops.row_sum(torch.zeros(2, 3))
