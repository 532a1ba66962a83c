"""cfd_amd — MI355X-native 2D incompressible projection solver.

Drop-in for the reference's cavity / channel / backwards-step solvers
(tjjones6/Computational-Fluid-Dynamics cavity-01.cpp, channel-01.cpp,
backwards_step-01.cpp). The compute path is libcfd_amd.so (hand-written HIP
kernels for gfx950 behind a C-ABI, include/cfd_amd.h); this package is the
host-side mirror of the reference classes.
"""
from .params import (BACKSTEP, CASE_IDS, CASE_NAMES, CAVITY, CHANNEL, RAYLEIGH_BENARD, CaseParams, make_params,
                     reference_defaults)
from .solver import (BackwardsStepSolver, CavitySolver, ChannelSolver, RayleighBenardSolver, params_from_library,
                     params_from_library_rb, solver_for, to_cparams, write_pvd, write_vtk_arrays)

__all__ = [
    "RAYLEIGH_BENARD", "RayleighBenardSolver", "params_from_library_rb", "BACKSTEP", "CASE_IDS", "CASE_NAMES", "CAVITY", "CHANNEL", "CaseParams", "make_params", "reference_defaults",
    "BackwardsStepSolver", "CavitySolver", "ChannelSolver", "params_from_library", "solver_for", "to_cparams",
    "write_pvd", "write_vtk_arrays",
]
