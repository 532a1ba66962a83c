"""Host-side logic on CPU: the C-ABI library loads and exports every declared
symbol, parameter derivations agree (Python vs C++ vs the reference's printed
values), CLI-style overrides, and the product refuses to run without a GPU
(no silent CPU fallback)."""
from __future__ import annotations

import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import ROOT

import cfd_amd as C
from cfd_amd import _lib

HEADER = os.path.join(ROOT, "include", "cfd_amd.h")


def declared_functions() -> list[str]:
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(cfd_[a-z_0-9]+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    names = declared_functions()
    assert len(names) >= 25
    L = ctypes.CDLL(_lib.LIB_PATH)
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing
    # and the Python binding covers all of them
    assert set(names) <= set(_lib.SIGNATURES), set(names) - set(_lib.SIGNATURES)


def test_nm_exports_match_header():
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    exported = {l.split()[-1] for l in out.splitlines() if " T " in l and l.split()[-1].startswith("cfd_")}
    assert set(declared_functions()) == exported


def test_abi_version():
    assert _lib.lib().cfd_abi_version() == 13


def test_params_struct_layout_matches_header(tmp_path):
    """The ctypes mirror of cfd_params has the C struct's size and field
    offsets (ABI 7 appended proof_test / small_solve / overlap)."""
    fields = [f for f, _ in _lib.CfdParams._fields_]
    src = tmp_path / "layout.c"
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "cfd_amd.h"\nint main(void){\n'
                   '  printf("%zu\\n", sizeof(cfd_params));\n'
                   + "".join(f'  printf("%zu\\n", offsetof(cfd_params, {f}));\n' for f in fields)
                   + '  printf("%d %d %d\\n", CFD_AUTO, CFD_ON, CFD_OFF);\n  return 0;\n}\n')
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split("\n")
    assert int(out[0]) == ctypes.sizeof(_lib.CfdParams)
    for k, f in enumerate(fields):
        assert int(out[1 + k]) == getattr(_lib.CfdParams, f).offset, f
    assert out[1 + len(fields)].split() == [str(_lib.SWITCH[n]) for n in ("auto", "on", "off")]


def test_timing_struct_layout_and_kernel_enum(tmp_path):
    """The ctypes mirror of cfd_timing matches the C struct (ABI 8 appended
    sor_kernel), and _lib.SOR_KERNEL names enum cfd_sor_kernel's values."""
    fields = [f for f, _ in _lib.Timing._fields_]
    names = ["CFD_SOR_NONE", "CFD_SOR_MARCH", "CFD_SOR_TILE", "CFD_SOR_SMALL", "CFD_SOR_LEXW", "CFD_SOR_LEX"]
    src = tmp_path / "timing.c"
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "cfd_amd.h"\nint main(void){\n'
                   '  printf("%zu\\n", sizeof(cfd_timing));\n'
                   + "".join(f'  printf("%zu\\n", offsetof(cfd_timing, {f}));\n' for f in fields)
                   + "".join(f'  printf("%d\\n", {n});\n' for n in names) + '  return 0;\n}\n')
    exe = tmp_path / "timing"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()
    assert int(out[0]) == ctypes.sizeof(_lib.Timing)
    for k, f in enumerate(fields):
        assert int(out[1 + k]) == getattr(_lib.Timing, f).offset, f
    vals = [int(x) for x in out[1 + len(fields):]]
    assert [_lib.SOR_KERNEL[v] for v in vals] == ["none", "march", "tile", "small", "lexw", "lex"]


def test_switches_default_to_auto_and_map():
    """cfd_params_init leaves the ABI-7 switches at CFD_AUTO; the Python
    mirror passes "auto" / "on" / "off" through unchanged."""
    lp = C.params_from_library(C.CAVITY)
    assert (lp.proof_test, lp.small_solve, lp.overlap) == (0, 0, 0)
    cp = C.solver.to_cparams(C.make_params("cavity"), proof_test="off", small_solve="on", overlap="off")
    assert (cp.proof_test, cp.small_solve, cp.overlap) == (2, 1, 2)
    assert set(_lib.TUNING.values()) == set(range(13))


@pytest.mark.parametrize("case", ["cavity", "channel", "backwards_step"])
@pytest.mark.parametrize("over", [{}, {"re": 400.0}, {"nx": 128, "ny": 96}, {"dt": 1e-3}, {"nx": 4096, "ny": 4096}])
def test_params_python_equals_cpp(case, over):
    if case == "backwards_step" and over.get("nx") == 128:
        over = {"nx": 512, "ny": 64}
    cp = C.make_params(case, **over)
    lp = C.params_from_library(cp.case_id, over.get("re", 0.0), over.get("nx", 0), over.get("ny", 0),
                               over.get("dt", 0.0))
    for f in ("nx", "ny", "dx", "dy", "nu", "dt", "omega", "total_steps", "step_i", "inlet_jmax", "max_iters",
              "tol_factor", "abs_tol", "print_interval", "save_interval", "height"):
        assert getattr(cp, f) == getattr(lp, f), f


@pytest.mark.parametrize("over", [{}, {"nx": 128, "ny": 32}, {"nx": 8192, "ny": 2048, "ra": 1e6}, {"dt": 1e-3},
                                  {"ra": 2e4, "pr": 7.0, "nx": 64, "ny": 16}])
def test_rayleigh_benard_params_python_equals_cpp(over):
    """BASELINE configs[4] (no reference solver): params.py == cfd_params_init_rb."""
    cp = C.make_params("rayleigh_benard", **over)
    lp = C.params_from_library_rb(over.get("ra", 1e6), over.get("pr", 0.71), over.get("nx", 0), over.get("ny", 0),
                                  over.get("dt", 0.0))
    for f in ("nx", "ny", "dx", "dy", "nu", "kappa", "buoyancy", "t_hot", "t_cold", "t_ref", "t_perturb", "dt",
              "omega", "total_steps", "max_iters", "tol_factor", "abs_tol", "height", "length", "re", "ra", "pr",
              "u_ref"):
        assert getattr(cp, f) == getattr(lp, f), f
    assert lp.case_id == C.RAYLEIGH_BENARD and lp.dx == lp.dy
    # cfd_params_init(case 3, re=Ra) = the same derivation with Pr 0.71
    if "pr" not in over:
        lq = C.params_from_library(C.RAYLEIGH_BENARD, over.get("ra", 1e6), over.get("nx", 0), over.get("ny", 0),
                                   over.get("dt", 0.0))
        assert bytes(lq) == bytes(lp)


def test_rayleigh_benard_oracle_onset():
    """Oracle sanity (parity unpinned): the conduction state is linearly unstable
    above Ra_c ~ 1708 (rigid walls) and stable below it."""
    import oracle as O
    ke = {}
    for ra in (1e3, 2e4):
        o = O.Oracle(C.make_params("rayleigh_benard", nx=32, ny=8, ra=ra, max_iters=400), ordering=O.RB)
        k = []
        for n in range(240):
            o.step()
            if n in (80, 239):
                k.append(o.stats()[1])
        ke[ra] = k
        nu = o.nusselt()
        assert 0.99 < nu < 1.2, nu
    assert ke[1e3][1] < ke[1e3][0]
    assert ke[2e4][1] > 2 * ke[2e4][0]


def test_baseline_configs_derive():
    # BASELINE.json configs: cavity Re=100 128^2 dt=1e-3; cavity Re=1000 1024^2; channel Re=1000 4096x512;
    # backwards step Re=400 8192x512
    a = C.make_params("cavity", re=100, nx=128, ny=128, dt=1e-3)
    assert a.dt == 1e-3 and a.nu == pytest.approx(0.01) and a.total_steps == 20000
    b = C.make_params("cavity", re=1000, nx=1024)
    assert b.ny == 1024 and b.dx == 1.0 / 1024
    c = C.make_params("channel", re=1000, nx=4096, ny=512)
    assert c.dx == 3.0 / 4096 and c.dy == 1.0 / 512
    d = C.make_params("backwards_step", re=400, nx=8192, ny=512)
    assert d.step_i == 2048 and d.inlet_jmax == 256


def test_invalid_params_rejected():
    with pytest.raises(ValueError):
        C.make_params("cavity", nx=1)
    out = _lib.CfdParams()
    assert _lib.lib().cfd_params_init(7, 0, 0, 0, 0, ctypes.byref(out)) != 0
    assert b"unknown case" in _lib.lib().cfd_last_error()


@pytest.mark.parametrize("case,spl,kw,msg", [
    ("channel", 3, {"ordering": "rb"}, b"cavity only"),
    ("channel", 4, {"ordering": "rb", "proof_test": "off"}, b"proof-mode test"),
    ("cavity", 5, {"ordering": "rb"}, b"sweeps_per_launch"), ("cavity", -1, {}, b"sweeps_per_launch"),
    ("cavity", 4, {"ordering": "rb", "proof_test": "off"}, b"proof-mode test"),
    ("cavity", 6, {"ordering": "lex"}, b"sweeps_per_launch"), ("channel", 5, {}, b"sweeps_per_launch"),
    ("channel", 3, {"ordering": "lex"}, b"4 sweeps per launch"),
])
def test_sweeps_per_launch_validated_before_device(case, spl, kw, msg):
    """Parameter errors are reported before any device is touched (the checks
    run first in the solver constructor), so they hold on CPU-only hosts too.
    Four sweeps per launch (the default proof-mode plan, stated) are accepted
    in red-black order with the proof test (every case since the open cases'
    proof launches, open.hip); five for the cavity's reference-order kernel
    only."""
    with pytest.raises(_lib.CfdError) as e:
        C.solver_for(C.make_params(case), sweeps_per_launch=spl, **kw)
    assert msg.decode() in str(e.value)


def test_reference_order_is_the_default():
    """cfd_params_init selects the reference's own sweep order (bit-identical
    output) for the three reference cases; the Python classes take it on one
    device and on ranks (ABI 12). A backwards step whose block is under 2 cells
    wide runs the one-workgroup kernel, one strip only: on ranks it is rejected
    before any device is touched."""
    for case in ("cavity", "channel", "backwards_step"):
        out = _lib.CfdParams()
        assert _lib.lib().cfd_params_init(C.params.CASE_IDS[case], 0, 0, 0, 0, ctypes.byref(out)) == 0
        assert out.ordering == _lib.ORDER["lex"]
    out = _lib.CfdParams()
    assert _lib.lib().cfd_params_init_rb(0, 0, 0, 0, 0, ctypes.byref(out)) == 0
    assert out.ordering == _lib.ORDER["rb"]  # (no reference solver: the rank path's order)
    cp = C.solver.to_cparams(C.make_params("cavity"))
    assert cp.ordering == _lib.ORDER["lex"]
    sp = C.solver.to_cparams(C.make_params("backwards_step"))
    sp.step_i = 1
    h = _lib.lib().cfd_create_rank(ctypes.byref(sp), 0, 1, sp.ny, None)
    assert not h
    assert b"no ranks" in _lib.lib().cfd_last_error()


@pytest.mark.parametrize("case,knob,value", [
    ("cavity", "march_min_th", 16), ("channel", "march_min_th", 16), ("backwards_step", "march_min_th", 16),
    ("cavity/rb", "march_min_th", 24), ("channel/rb", "march_min_th", 16), ("backwards_step/rb", "march_min_th", 24),
    ("cavity", "pair_edge_pct", 80), ("channel", "pair_edge_pct", 45), ("backwards_step", "pair_edge_pct", 45),
    ("cavity", "tile_rounds", 1), ("channel", "tile_rounds", 0), ("rayleigh_benard", "tile_rounds", 1),
    ("cavity", "tent_th", 64), ("channel", "lexw_edge_pct", 75), ("backwards_step", "lexw_ramp_pct", 100), ("cavity", "lexw_ramp_pct", 0),
    ("cavity@4096", "lexw_edge_pct", 100), ("cavity@1024", "lexw_edge_pct", 75),
    ("backwards_step", "lexw_left", 1), ("cavity", "lexw_left", 1), ("cavity", "lexw_updown", 1), ("cavity/rb", "resident", 1), ("channel/rb", "resident", 1),
    ("channel", "resident", 1), ("backwards_step", "resident", 0),
])
def test_tuning_defaults(case, knob, value):
    """The launch-plan defaults a solver starts with (cfd_tuning_default, host
    only): the measured band floors (16 rows for the channel and every
    reference-order march, 24 for the red-black step and cavity -
    profiles/r4_tune), boundary-column band lengths (reference order: 75 %
    up to 2048 rows, 100 % above), LDS tiles for the cavity only."""
    case, _, order = case.partition("/")
    case, _, n = case.partition("@")
    cp = C.solver.to_cparams(C.make_params(case, **({"nx": int(n), "ny": int(n)} if n else {})),
                             ordering=order or "lex")
    v = ctypes.c_int(-1)
    assert _lib.lib().cfd_tuning_default(ctypes.byref(cp), _lib.TUNING[knob], ctypes.byref(v)) == 0
    assert v.value == value
    assert _lib.lib().cfd_tuning_default(ctypes.byref(cp), _lib.TUNING["pair_wps"], ctypes.byref(v)) != 0
    assert b"occupancy" in _lib.lib().cfd_last_error()


def test_thin_step_lex_on_strips_rejected_at_create():
    """A backwards step whose block is under 2 cells wide or high runs the
    reference order on the one-workgroup kernel (one strip): with more strips
    cfd_create rejects it before any device is touched, not the first solve."""
    p = C.make_params("backwards_step", nx=64, ny=32)
    p.h_inlet = 1.9375  # inlet_jmax = 31 = ny - 1: the block is one cell high
    cp = C.solver.to_cparams(p)
    assert cp.inlet_jmax == p.ny - 1
    assert cp.ordering == _lib.ORDER["lex"]
    h = _lib.lib().cfd_create(ctypes.byref(cp), 0, 2)
    assert not h
    assert b"one strip" in _lib.lib().cfd_last_error()
    cp.ordering = _lib.ORDER["rb"]  # red-black takes any block on strips (fails here only for want of a GPU)
    h = _lib.lib().cfd_create(ctypes.byref(cp), 0, 2)
    assert b"one strip" not in _lib.lib().cfd_last_error()


def test_bad_switch_rejected_before_device():
    cp = C.solver.to_cparams(C.make_params("cavity"))
    cp.overlap = 7
    h = _lib.lib().cfd_create(ctypes.byref(cp), 0, 1)
    assert not h
    assert b"cfd_switch" in _lib.lib().cfd_last_error()


def test_no_cpu_fallback_without_gpu():
    """cfd_create must fail loudly when there is no gfx950 device (here: no GPU at all)."""
    probe = subprocess.run(["python", "-c", "import torch;print(torch.cuda.is_available())"], capture_output=True,
                           text=True)
    if probe.stdout.strip() == "True":
        pytest.skip("a GPU is present")
    with pytest.raises(_lib.CfdError):
        C.CavitySolver(C.make_params("cavity", nx=32), ordering="rb")


def test_pvd_writer(tmp_path):
    fn = tmp_path / "c.pvd"
    C.write_pvd(str(fn), ["a_000000.vtk", "a_000100.vtk"], [0.0, 0.7936507936507936])
    assert fn.read_text() == (
        '<?xml version="1.0"?>\n'
        '<VTKFile type="Collection" version="0.1" byte_order="LittleEndian">\n'
        "  <Collection>\n"
        '    <DataSet timestep="0.000000" group="" part="0" file="a_000000.vtk"/>\n'
        '    <DataSet timestep="0.793651" group="" part="0" file="a_000100.vtk"/>\n'
        "  </Collection>\n"
        "</VTKFile>\n")


def test_vtk_writer_rejects_bad_shapes(tmp_path):
    cp = C.make_params("cavity", nx=8)
    z = np.zeros((cp.ny + 2, cp.nx + 2))
    with pytest.raises(ValueError):
        C.write_vtk_arrays(cp, str(tmp_path / "x.vtk"), 0.0, z[:-1], z, z)


def test_host_binaries_built_and_print_usage():
    for name in ("cavity", "channel", "backwards_step", "rayleigh_benard"):
        exe = os.path.join(ROOT, "computational-fluid-dynamics_amd", "bin", name)
        assert os.access(exe, os.X_OK), exe
        r = subprocess.run([exe, "--help"], capture_output=True, text=True)
        assert r.returncode == 0 and "--Re" in r.stderr and "--Nx" in r.stderr and "--dt" in r.stderr


def test_bench_traffic_provenance(tmp_path, monkeypatch):
    """bench.py reports roofline.traffic from the newest committed PMC pass of
    the same workload only when that pass profiled the kernel instance that
    ran (its kernel_match) from the same translation-unit sources (its
    source_hash), with the file, commit and hash as traffic_source; a
    mismatched kernel, grid, sweep count or source hash gives traffic null."""
    import json as _json

    import bench

    assert bench.sor_template("cavity", "march", 4, True) == "poisson_multi_kernel<0, 4, true>"
    assert bench.sor_template("channel", "march", 4, True) == "poisson_open_proof_kernel<1, 4>"
    assert bench.sor_template("cavity", "tile", 4, True) == "poisson_tile_kernel<0, true>"
    assert bench.sor_template("backwards_step", "lexw", 4, False) == "poisson_lexw_kernel<2, 4, false, true>"
    prof = tmp_path / "profiles"
    prof.mkdir()
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    from cfd_amd.provenance import source_hash, tu_sources

    h = source_hash("poisson_multi_kernel<0, 4, true>")
    assert h and len(h) == 64 and any(f.endswith("march.hpp") for f in tu_sources("solver"))
    assert source_hash("poisson_tile_kernel<0, true>") != h  # (another translation unit)
    rec = {"kernel_match": "poisson_multi_kernel<0, 4, true>", "nx": 64, "rows": 66, "sweeps_per_launch": 4,
           "hbm_bytes_per_launch": 123.0, "commit": "abc123", "source_hash": h}
    (prof / "r4_pmc_cavity_rb_64x64.json").write_text(_json.dumps(dict(rec, hbm_bytes_per_launch=99.0)))
    (prof / "r5_pmc_cavity_rb_64x64.json").write_text(_json.dumps(rec))
    t, src = bench.pmc_traffic("cavity", "rb", 64, 64, 66, 4, "poisson_multi_kernel<0, 4, true>")
    assert t == 123.0 and src["file"].endswith("r5_pmc_cavity_rb_64x64.json") and src["commit"] == "abc123"
    t, src = bench.pmc_traffic("cavity", "rb", 64, 64, 66, 4, "poisson_multi_kernel<0, 3, true>")
    assert t is None and "kernel mismatch" in src["reason"]  # (the older r4 file is not a fallback)
    t, src = bench.pmc_traffic("cavity", "rb", 64, 64, 66, 3, "poisson_multi_kernel<0, 4, true>")
    assert t is None and "mismatch" in src["reason"]
    t, src = bench.pmc_traffic("channel", "rb", 64, 64, 66, 4, "poisson_open_proof_kernel<1, 4>")
    assert t is None and "no profiles" in src["reason"]
    # a profile taken on other kernel sources (stale) or without a hash: traffic null
    for stale in ({"source_hash": "0" * 64}, {"source_hash": None}):
        (prof / "r6_pmc_cavity_rb_64x64.json").write_text(_json.dumps(dict(rec, **stale)))
        t, src = bench.pmc_traffic("cavity", "rb", 64, 64, 66, 4, "poisson_multi_kernel<0, 4, true>")
        assert t is None and "stale" in src["reason"]
