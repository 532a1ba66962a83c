"""Residual-log line formatting, identical to the reference's stdout/stderr.

cavity-01.cpp:769-773 (logStatistics), cavity-01.cpp:682-683 (SOR warning),
channel-01.cpp:762-768 and backwards_step-01.cpp:1054-1060 (logStatistics),
channel-01.cpp:684 / backwards_step-01.cpp:934 (PPE warning).
"""
from __future__ import annotations

from .params import CAVITY, RAYLEIGH_BENARD


def step_line(case_id: int, step: int, total: int, t: float, max_div: float, avg_ke: float, iters: int,
              residual: float, nusselt: float | None = None) -> str:
    if case_id == RAYLEIGH_BENARD:  # bin/rayleigh_benard (host/driver.hpp): the cavity line + Nu
        return (f"Step {step:6d}/{total} | t={t:6.2f} | max(div)={max_div:10.2e} | avg_KE={avg_ke:10.6f}"
                f" | Nu={nusselt:.4f} | SOR_iters={iters:4d}")
    if case_id == CAVITY:
        return (f"Step {step:6d}/{total} | t={t:6.2f} | max(div)={max_div:10.2e} | avg_KE={avg_ke:10.6f}"
                f" | SOR_iters={iters:4d}")
    return (f"Step {step:6d}/{total} | t={t:8.3f} | max(div)={max_div:10.2e} | avg_KE={avg_ke:10.6f}"
            f" | PPE iters={iters:4d} | res={residual:10.2e}")


def _g(x: float) -> str:
    """C++ ostream default float format (%g, precision 6)."""
    return "%g" % x


def warning_line(case_id: int, max_iters: int, residual: float) -> str:
    if case_id in (CAVITY, RAYLEIGH_BENARD):
        return f"Warning: SOR solver did not converge in {max_iters} iterations. Final residual: {_g(residual)}"
    return f"Warning: PPE SOR hit max iterations, max_res={_g(residual)}"
