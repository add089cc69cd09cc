"""The Sokoban turn's bitboard block (ragen_amd/csrc/board_step.hpp) on the host: its slot-vector
form against the straight per-slot restatement, bit for bit, over random rooms, action slots,
budgets and step counts (tests/board_step_check.cpp, built with g++).  The GPU parity tests run
the same header inside the turn kernel against the oracle."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_board_step_matches_per_slot_form(tmp_path):
    exe = str(tmp_path / "board_step_check")
    subprocess.run(["g++", "-O2", "-std=c++17", "-I", os.path.join(ROOT, "include"), "-I",
                    os.path.join(ROOT, "ragen_amd", "csrc"), os.path.join(ROOT, "tests", "board_step_check.cpp"),
                    "-o", exe], check=True)
    r = subprocess.run([exe, "100000"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and r.stdout.startswith("ok"), r.stdout + r.stderr
