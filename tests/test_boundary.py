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


STRUCTS = {  # ctypes mirror in ragen_amd/_lib.py -> C type in include/ragen_amd.h
    "Episode": "rmi_episode_t", "Turn": "rmi_turn_t", "Sokoban": "rmi_sokoban_t", "Finalize": "rmi_finalize_t",
    "FrozenLake": "rmi_frozenlake_t", "Bandit": "rmi_bandit_t", "Countdown": "rmi_countdown_t",
    "ParseCfg": "rmi_parse_cfg_t", "Piece": "rmi_piece_t", "Prompt": "rmi_prompt_t", "tokenizer.Bpe": "rmi_bpe_t",
    "Render": "rmi_render_t", "TurnChain": "rmi_turn_chain_t",
    "FormulateChain": "rmi_formulate_chain_t", "TokenRows": "rmi_token_rows_t", "XGather": "rmi_xgather_t",
}


def _struct(py):
    """'Name' -> ragen_amd._lib.Name; 'module.Name' -> ragen_amd.module.Name."""
    if "." in py:
        import importlib
        mod, name = py.rsplit(".", 1)
        return getattr(importlib.import_module("ragen_amd." + mod), name)
    return getattr(_lib, py)


def test_ctypes_structs_match_the_c_layout(tmp_path):
    """Every ctypes Structure the binding passes by pointer has the C struct's size and field
    offsets (compiled from the header with gcc: the ABI the kernels read)."""
    import ctypes
    lines = ["#include <stdio.h>", "#include <stddef.h>", '#include "ragen_amd.h"', "int main(void) {"]
    for py, c in STRUCTS.items():
        cls = _struct(py)
        lines.append(f'  printf("{py} size %zu\\n", sizeof({c}));')
        for name, _ in cls._fields_:
            lines.append(f'  printf("{py} {name} %zu\\n", offsetof({c}, {name}));')
    lines.append("  return 0; }")
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split("\n")
    c_vals = {tuple(l.split()[:2]): int(l.split()[2]) for l in out if l.strip()}
    for py in STRUCTS:
        cls = _struct(py)
        assert c_vals[(py, "size")] == ctypes.sizeof(cls), py
        for name, _ in cls._fields_:
            assert c_vals[(py, name)] == getattr(cls, name).offset, (py, name)
