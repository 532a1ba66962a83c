"""ctypes binding of libcfd_amd.so (include/cfd_amd.h).

The library is the product: HIP kernels for gfx950 behind a C-ABI. There is
no CPU fallback — if the library is missing or no gfx950 device is present,
loading / solver construction raises.

Import-order note: PyTorch-ROCm bundles its own libamdhip64.so.7. If torch is
imported in the same process it must be imported BEFORE this library is
loaded, so both resolve to one HIP runtime (same soname).
"""
from __future__ import annotations

import ctypes
import os

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# CFD_AMD_LIB: an alternative in-tree build of the same library (A/B timing of
# kernel build variants, scripts/); the product default is libcfd_amd.so
LIB_PATH = os.path.join(PKG_DIR, os.environ.get("CFD_AMD_LIB", "libcfd_amd.so"))

CFD_FIELD = {"p": 0, "src": 1, "us": 3, "vs": 4, "u": 5, "v": 6, "uc": 7, "vc": 8, "t": 9}
COMM_ID_BYTES = 128


class CfdParams(ctypes.Structure):
    _fields_ = [
        ("case_id", ctypes.c_int), ("nx", ctypes.c_int), ("ny", ctypes.c_int),
        ("length", ctypes.c_double), ("height", ctypes.c_double),
        ("re", ctypes.c_double), ("u_ref", ctypes.c_double), ("rho", ctypes.c_double), ("cfl", ctypes.c_double),
        ("final_time", ctypes.c_double),
        ("dx", ctypes.c_double), ("dy", ctypes.c_double), ("nu", ctypes.c_double), ("dt", ctypes.c_double),
        ("omega", ctypes.c_double),
        ("tol_factor", ctypes.c_double), ("abs_tol", ctypes.c_double),
        ("max_iters", ctypes.c_int), ("total_steps", ctypes.c_int),
        ("print_interval", ctypes.c_int), ("save_interval", ctypes.c_int),
        ("h_inlet", ctypes.c_double), ("step_x", ctypes.c_double),
        ("step_i", ctypes.c_int), ("inlet_jmax", ctypes.c_int),
        ("check_every", ctypes.c_int), ("chunk", ctypes.c_int), ("ordering", ctypes.c_int),
        ("sweeps_per_launch", ctypes.c_int),
        ("ra", ctypes.c_double), ("pr", ctypes.c_double), ("kappa", ctypes.c_double), ("buoyancy", ctypes.c_double),
        ("t_hot", ctypes.c_double), ("t_cold", ctypes.c_double), ("t_ref", ctypes.c_double),
        ("t_perturb", ctypes.c_double),
        ("proof_test", ctypes.c_int), ("small_solve", ctypes.c_int), ("overlap", ctypes.c_int),
    ]


ORDER = {"rb": 0, "lex": 1}
SWITCH = {"auto": 0, "on": 1, "off": 2}  # enum cfd_switch
TUNING = {"pair_wps": 0, "wave_wps": 1, "lexw_waves": 2, "lexw_edge_pct": 3, "pair_edge_pct": 4,
          "march_min_th": 5, "tent_th": 6, "lexw_ramp_pct": 7, "tile_rounds": 8, "march_order": 9,
          "lexw_left": 10, "resident": 11, "lexw_updown": 12}  # enum cfd_tuning
SOR_KERNEL = {0: "none", 1: "march", 2: "tile", 3: "small", 4: "lexw", 5: "lex", 6: "smlex", 7: "resident"}  # enum cfd_sor_kernel


class StepInfo(ctypes.Structure):
    _fields_ = [("sor_iterations", ctypes.c_int), ("residual", ctypes.c_double)]


class Stats(ctypes.Structure):
    _fields_ = [("max_divergence", ctypes.c_double), ("avg_kinetic_energy", ctypes.c_double)]


class Timing(ctypes.Structure):
    _fields_ = [("poisson_ms", ctypes.c_double), ("poisson_launches", ctypes.c_longlong),
                ("poisson_cell_updates", ctypes.c_longlong), ("step_ms", ctypes.c_double),
                ("steps", ctypes.c_longlong), ("poisson_sweeps", ctypes.c_longlong),
                ("poisson_overlapped", ctypes.c_longlong), ("poisson_steady_ms", ctypes.c_double),
                ("poisson_steady_launches", ctypes.c_longlong),
                ("proof_fallbacks", ctypes.c_longlong), ("sor_kernel", ctypes.c_int),
                ("resident_timeouts", ctypes.c_longlong), ("seqsum_chunks", ctypes.c_longlong),
                ("seqsum_serial_chunks", ctypes.c_longlong)]


# every symbol include/cfd_amd.h declares: name -> (restype, argtypes)
_vp, _i, _d, _sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_double, ctypes.c_size_t
_dp = ctypes.POINTER(ctypes.c_double)
_ip = ctypes.POINTER(ctypes.c_int)
SIGNATURES = {
    "cfd_abi_version": (_i, []),
    "cfd_last_error": (ctypes.c_char_p, []),
    "cfd_params_init": (_i, [_i, _d, _i, _i, _d, ctypes.POINTER(CfdParams)]),
    "cfd_create": (_vp, [ctypes.POINTER(CfdParams), _i, _i]),
    "cfd_create_rank": (_vp, [ctypes.POINTER(CfdParams), _i, _i, _i, _vp]),
    "cfd_destroy": (_i, [_vp]),
    "cfd_apply_bc": (_i, [_vp]),
    "cfd_apply_tentative_bc": (_i, [_vp]),
    "cfd_compute_tentative": (_i, [_vp]),
    "cfd_advance_temperature": (_i, [_vp]),
    "cfd_params_init_rb": (_i, [_d, _d, _i, _i, _d, ctypes.POINTER(CfdParams)]),
    "cfd_build_source": (_i, [_vp]),
    "cfd_solve_pressure": (_i, [_vp, ctypes.POINTER(StepInfo)]),
    "cfd_apply_correction": (_i, [_vp]),
    "cfd_step": (_i, [_vp, ctypes.POINTER(StepInfo)]),
    "cfd_run_steps": (_i, [_vp, _i, ctypes.POINTER(StepInfo)]),
    "cfd_compute_stats": (_i, [_vp, ctypes.POINTER(Stats)]),
    "cfd_field_shape": (_i, [_vp, _i, _ip, _ip]),
    "cfd_get_field": (_i, [_vp, _i, _dp, _sz]),
    "cfd_set_field": (_i, [_vp, _i, _dp, _sz]),
    "cfd_write_vtk": (_i, [_vp, ctypes.c_char_p, _d]),
    "cfd_write_pvd": (_i, [ctypes.c_char_p, ctypes.POINTER(ctypes.c_char_p), _dp, _i]),
    "cfd_write_vtk_arrays": (_i, [ctypes.POINTER(CfdParams), ctypes.c_char_p, _d, _dp, _dp, _dp]),
    "cfd_owned_rows": (_i, [_vp, _ip, _ip]),
    "cfd_get_timing": (_i, [_vp, ctypes.POINTER(Timing)]),
    "cfd_reset_timing": (_i, [_vp]),
    "cfd_synchronize": (_i, [_vp]),
    "cfd_set_tuning": (_i, [_vp, _i, _i]),
    "cfd_tuning_default": (_i, [ctypes.POINTER(CfdParams), _i, _ip]),
    "cfd_comm_unique_id": (_i, [ctypes.POINTER(ctypes.c_ubyte)]),
    "cfd_comm_init": (_vp, [ctypes.POINTER(ctypes.c_ubyte), _i, _i, _i]),
    "cfd_comm_destroy": (_i, [_vp]),
    "cfd_comm_info": (_i, [_vp, _ip, _ip, _ip]),
    "cfd_comm_exchange_check": (_i, [_vp, _i, ctypes.c_size_t, ctypes.POINTER(ctypes.c_longlong)]),
    "cfd_comm_loopback_hub": (_vp, [_i]),
    "cfd_comm_init_loopback": (_vp, [_vp, _i, _i]),
    "cfd_comm_loopback_hub_destroy": (_i, [_vp]),
}

_lib = None


class CfdError(RuntimeError):
    pass


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise CfdError(f"{LIB_PATH} not built: run `python -c 'import __graft_entry__ as g; g.build()'` "
                           "(make -C computational-fluid-dynamics_amd)")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = lib().cfd_last_error().decode(errors="replace")
        raise CfdError(f"{what} failed ({rc}): {msg}")
