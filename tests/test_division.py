"""The open-case SOR divide (device.hpp div_denom: split reciprocal + one FMA
correction; the former two-correction form and the one-correction form for
denominators with |1 - y*d| <= 2^-54 alongside) is bit-identical to the IEEE
divide the reference performs
(channel-01.cpp:663, backwards_step-01.cpp:908): random numerators over
+-100 binades for the config denominators and random / adversarial ones.
CPU only (gcc, hardware FMA); the GPU path is covered bit-for-bit by the
solver parity tests."""
from __future__ import annotations

import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc not available")
def test_fma_division_matches_ieee_divide(tmp_path):
    exe = str(tmp_path / "division_check")
    subprocess.check_call(["gcc", "-O2", "-mfma", "-ffp-contract=off", "-o", exe,
                           os.path.join(HERE, "division_check.c"), "-lm"])
    out = subprocess.run([exe, "40000", "300"], capture_output=True, text=True)
    print(out.stdout)
    assert out.returncode == 0, out.stdout
    assert out.stdout.strip().endswith(f"0 mismatches of {40000 * (11 + 300)}")
