#!/usr/bin/env python3
"""Benchmark: Poisson MLUPS + steps/sec of the lid-driven cavity projection
solver (BASELINE.json metric), 4096^2 fp64 cells per GPU, weak-scaled row strips.

A "step" is one full projection timestep of the reference algorithm
(cavity-01.cpp:387-390): velocity BCs, predictor, source, SOR pressure solve to
the reference tolerance (1e-9 * max|source|, capped at 10000 sweeps), corrector.
All inputs are device-resident when the timed region starts.

  value = interior cells x SOR iterations summed over all ranks / wall time of
          the K timed steps (max over ranks), in MLUPS.

The headline runs the reference's own sweep order (--ordering lex, the
default at every N: poisson_lexw_kernel, bit-identical to the reference's loop
on one GPU and on ranks). Extra fields: steps_per_sec, roofline (the SOR
kernel's steady launches - every cell active -, four sweeps per launch on one
GPU, three on ranks: HIP events on the solver's stream; `achieved` = the
24 B/cell one launch must move / launch time, `effective_sweep_*` the same per
sweep), cpu_baseline (the oracle's lexicographic SOR loop — the reference's
loop restated in C — on a bounded sample of the same grid, rank 0 only) and,
at N=1, the same workload in the other order: red_black (red-black SOR with
the proof-mode test, bit-identical to the red-black oracle; it is not the
reference's iterate where the solve hits the cap) or, with --ordering rb,
reference_order.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--global-ny NY]
For N > 1 launch with torch.distributed.run (one rank per GPU); halos and the
residual all-reduce travel over RCCL inside libcfd_amd.so.

Scaling modes (config.workload says which):
  weak (default): every rank owns --ny rows (4096), global grid nx x (N*ny);
  strong (--global-ny NY): the N ranks split one nx x NY grid (4096² at N=8:
  512 rows per rank).
The residual test runs every SOR iteration at every N (the reference's stop
rule; check_every 1), so 1-GPU and N-GPU runs stop at the same iteration.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "computational-fluid-dynamics_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
FP64_VALU_PEAK_TF = 78.6  # MI355X fp64 vector spec: half the 157.3 TF fp32 vector rate (MI355X_MICROARCH.md)
# the cavity's SOR update: 3 adds, h^2 f, f subtraction, 2 products, 1 add (the other cases' updates -
# an anisotropic sum and a divide - are not priced: no VALU fraction is reported for them)
FLOPS_PER_UPDATE = {"cavity": 8.0}
BYTES_PER_CELL = 24.0  # SOR launch: read p_in + read f + write p_out, fp64
METRIC = "Poisson MLUPS + steps/sec, cavity 4096² @1/2/4/8 GPU; % HBM roofline"
WORKLOAD = {"cavity": "lid-driven cavity", "channel": "channel flow", "backwards_step": "backwards-facing step",
            "rayleigh_benard": "Rayleigh-Benard convection"}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cpu_baseline(nx: int, ny: int, budget_s: float, case: str = "cavity") -> dict:
    """The reference's SOR loop (sweep + residual per iteration, cavity-01.cpp:635-678)
    restated in C (oracle/), single core, on the same grid for a bounded time."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    from cfd_amd.params import make_params

    cp = make_params(case, nx=nx, ny=ny)
    o = O.Oracle(cp, ordering=O.LEX)
    o.velocity_bc(False)
    o.tentative()
    o.source()
    t0 = time.perf_counter()
    n = 0
    while True:
        o.poisson_fixed(1)
        n += 1
        el = time.perf_counter() - t0
        if el >= budget_s or n >= 1000:
            break
    del o
    mlups = nx * ny * n / el / 1e6
    cpu_model = None
    try:
        with open("/proc/cpuinfo") as fh:
            cpu_model = next((ln.split(":", 1)[1].strip() for ln in fh if ln.startswith("model name")), None)
    except OSError:
        pass
    return {"value": round(mlups, 3), "unit": "MLUPS", "cores": 1, "kind": "port", "cpu_model": cpu_model,
            "sample": f"{n} lexicographic SOR sweeps + residual (reference loop restated in C, gcc -O2) on the "
                      f"{nx}x{ny} {case} after one predictor step, {el:.1f} s single-threaded"}


def reference_binary(timeout_s: float = 60.0) -> dict | None:
    """The reference's own CPU loop, as compiled from the unmodified reference
    sources (oracle/build_ref.sh -> oracle/_ref/cavity, g++ -std=c++17 -O2),
    on this host: its compiled-in case (63x63, Re 1000; the reference takes no
    arguments), timed from launch until it writes frame 100, i.e. after steps
    1-100. Their SOR sweep counts (tests/golden/cavity_ref_iters.json, from
    the oracle pinned to this binary; step 100's checked against the
    binary's own log) give the cell updates. None when the binary is absent."""
    import shutil
    import subprocess
    import tempfile

    exe = os.path.join(ROOT, "oracle", "_ref", "cavity")
    fix = os.path.join(ROOT, "tests", "golden", "cavity_ref_iters.json")
    if not (os.path.exists(exe) and os.path.exists(fix)):
        return None
    d = json.load(open(fix))
    wd = tempfile.mkdtemp(prefix="cfd_ref_")
    try:
        t0 = time.perf_counter()
        proc = subprocess.Popen([exe], cwd=wd, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        frame = os.path.join(wd, "vtk_output", "cavity_flow_000100.vtk")
        while not os.path.exists(frame) and proc.poll() is None and time.perf_counter() - t0 < timeout_s:
            time.sleep(0.02)
        el = time.perf_counter() - t0
        ok = os.path.exists(frame)
        proc.kill()
        proc.wait()
    finally:
        shutil.rmtree(wd, ignore_errors=True)
    if not ok:
        return None
    sweeps = sum(d["steps"])
    return {"value": round(d["cells"] * sweeps / el / 1e6, 3), "unit": "MLUPS", "cores": 1, "kind": "reference",
            "sample": f"the reference binary (cavity-01.cpp, g++ -O2, unmodified) on its compiled-in 63x63 Re=1000 "
                      f"run, steps 1-100 ({sweeps} SOR sweeps + residuals, predictor, corrector, frame output) "
                      f"in {el:.2f} s single-threaded"}


def red_black(C, cp, args, device: int, check_every: int, cells_per_launch: int, tuning: dict) -> dict:
    """The same workload in red-black order (ordering="rb": proof-mode march
    launches, bit-identical to the red-black oracle; where the solve hits the
    cap its iterate is not the reference's), timed the same way on one GPU:
    value, ms per step and the SOR launch's roofline."""
    import torch

    s = C.solver_for(cp, device=device, check_every=check_every, ordering="rb",
                     sweeps_per_launch=args.sweeps_per_launch, proof_test=args.proof_test, tuning=tuning)
    if args.case == "cavity":
        s.applyBoundaryConditions()
    s.step()  # warmup
    s.synchronize()
    s.reset_timing()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    iters = [s.step()[0] for _ in range(args.lex_steps)]
    s.synchronize()
    el = time.perf_counter() - t0
    tm = s.timing()
    s.close()
    sk = _lib_sor_kernel(tm)
    ns = round(tm.poisson_sweeps / max(tm.poisson_launches, 1))
    launch_ms = tm.poisson_ms / max(tm.poisson_launches, 1)
    proof = args.proof_test != "off" and (sk == "tile" or (sk == "march" and ns >= 3))
    rows = cells_per_launch // (cp.nx + 2)
    traffic, src = pmc_traffic(args.case, "rb", cp.nx, rows - 2, rows, ns,
                               sor_template(kcase_of(args.case), sk, ns, proof))
    achieved = BYTES_PER_CELL * cells_per_launch / (launch_ms * 1e-3) / 1e9
    return {"ordering": "rb", "value": round(tm.poisson_cell_updates / el / 1e6, 2), "unit": "MLUPS",
            "ms_per_step": round(el / args.lex_steps * 1e3, 3), "steps": args.lex_steps,
            "sor_iterations_per_step": iters, "sor_kernel": sk,
            "template": sor_template(kcase_of(args.case), sk, ns, proof),
            "sweeps_per_launch": round(tm.poisson_sweeps / max(tm.poisson_launches, 1), 3),
            "launches_per_step": round(tm.poisson_launches / args.lex_steps, 1),
            "avg_launch_us": round(launch_ms * 1e3, 2), "achieved_GBs": round(achieved, 1),
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_source": src}


def reference_order(C, cp, args, device: int, check_every: int, cells_per_launch: int) -> dict:
    """(--ordering rb) The same workload in the reference's lexicographic sweep
    order (ordering="lex": poisson_lexw_kernel, bit-identical to the
    reference's loop at any size), timed the same way on one GPU: value, ms per
    step and the steady launches' roofline (every cell active; the ramps at
    both ends of a solve touch part of the grid)."""
    import torch

    s = C.solver_for(cp, device=device, check_every=check_every, ordering="lex", sweeps_per_launch=args.lex_sweeps)
    if args.case == "cavity":
        s.applyBoundaryConditions()
    s.step()  # warmup
    s.synchronize()
    s.reset_timing()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    iters = [s.step()[0] for _ in range(args.lex_steps)]
    s.synchronize()
    el = time.perf_counter() - t0
    tm = s.timing()
    s.close()
    steady_ms = tm.poisson_steady_ms / max(tm.poisson_steady_launches, 1)
    ns = round(tm.poisson_sweeps / max(tm.poisson_launches, 1))
    rows = cells_per_launch // (cp.nx + 2)
    st_traffic, st_src = pmc_traffic(args.case, "lex", cp.nx, rows - 2, rows, ns,
                                     sor_template(args.case, _lib_sor_kernel(tm), ns, False))
    achieved = BYTES_PER_CELL * cells_per_launch / (steady_ms * 1e-3) / 1e9 if tm.poisson_steady_launches else None
    return {"ordering": "lex", "value": round(tm.poisson_cell_updates / el / 1e6, 2), "unit": "MLUPS",
            "ms_per_step": round(el / args.lex_steps * 1e3, 3), "steps": args.lex_steps,
            "sor_iterations_per_step": iters,
            "kernel": (f"poisson_resident_kernel<{args.case},lex> (whole solve in one launch)"
                       if _lib_sor_kernel(tm) == "resident" else
                       f"poisson_lexw_kernel<{args.case},{round(tm.poisson_sweeps / max(tm.poisson_launches, 1))},"
                       f"sampled>"),
            "sweeps_per_launch": round(tm.poisson_sweeps / max(tm.poisson_launches, 1), 3),
            "launches_per_step": round(tm.poisson_launches / args.lex_steps, 1),
            "steady_launches_per_step": round(tm.poisson_steady_launches / args.lex_steps, 1),
            "steady_launch_us": round(steady_ms * 1e3, 2) if tm.poisson_steady_launches else None,
            "steady_achieved_GBs": round(achieved, 1) if achieved else None,
            "steady_frac": round(achieved / HBM_PEAK_GBS, 4) if achieved else None,
            "steady_traffic": st_traffic, "steady_traffic_source": st_src}


CASE_ID = {"cavity": 0, "channel": 1, "backwards_step": 2}


def sor_template(kcase: str, sor_kernel: str, sweeps: int, proof: bool) -> str | None:
    """The C++ template instance of the SOR kernel a run's launches went to, as
    rocprofv3 names it (the PMC files' kernel_match): csrc/march.hpp
    poisson_multi_kernel<CASE, NS, PROOF>, tile.hip poisson_tile_kernel<CASE,
    PROOF>, open.hip poisson_open_proof_kernel<CASE, NS>, lexw.hpp
    poisson_lexw_kernel<CASE, NS, RAMP, SAMPLE> (steady launches of a capped
    solve: RAMP false, sampled residual rows)."""
    c = CASE_ID[kcase]
    if sor_kernel == "lexw":
        return f"poisson_lexw_kernel<{c}, {sweeps}, false, true>"
    if sor_kernel == "tile":
        return f"poisson_tile_kernel<{c}, {'true' if proof else 'false'}>"
    if sor_kernel == "march":
        if proof and kcase != "cavity":
            return f"poisson_open_proof_kernel<{c}, {sweeps}>"
        if sweeps >= 2:
            return f"poisson_multi_kernel<{c}, {sweeps}, {'true' if proof else 'false'}>"
    return None


def pmc_traffic(case: str, order: str, nx: int, ny: int, rows: int, sweeps: int, template: str | None):
    """HBM bytes per SOR launch from the newest committed PMC pass of the same
    workload (profiles/r<N>_pmc_<case>_<order>_<nx>x<ny>.json, made by
    scripts/profile_case.sh + pmc_traffic.py), returned only when that file's
    kernel_match is the kernel instance that ran here (same grid rows and
    sweeps per launch) and its source hash is that of the kernel's
    translation unit as built here (cfd_amd.provenance); otherwise None.
    Second value: the provenance (file, kernel, commit and source hash the
    profile was taken at) or why there is none."""
    import glob
    import re

    pat = os.path.join(ROOT, "profiles", f"r*_pmc_{case}_{order}_{nx}x{ny}.json")
    found = []
    for f in glob.glob(pat):
        m = re.match(r"r(\d+)_pmc_", os.path.basename(f))
        if m:
            found.append((int(m.group(1)), f))
    if not found:
        return None, {"reason": f"no profiles/r*_pmc_{case}_{order}_{nx}x{ny}.json"}
    rnd, path = max(found)  # the newest round's pass only (an older one may predate a kernel change)
    src = {"file": os.path.relpath(path, ROOT)}
    try:
        d = json.load(open(path))
    except (OSError, ValueError) as e:
        return None, dict(src, reason=f"unreadable: {e}")
    src.update(kernel_match=d.get("kernel_match"), commit=d.get("commit"))
    if template is None or d.get("kernel_match") != template:
        return None, dict(src, reason=f"kernel mismatch: profile {d.get('kernel_match')!r}, ran {template!r}")
    if not (d.get("nx") == nx and d.get("rows") == rows and d.get("sweeps_per_launch", 1) == sweeps):
        return None, dict(src, reason="grid / sweeps per launch mismatch")
    # code-exact: the profile's kernel sources must be the ones built here
    from cfd_amd.provenance import source_hash
    now = source_hash(template)
    src["source_hash"] = d.get("source_hash")
    if d.get("source_hash") is None or d.get("source_hash") != now:
        return None, dict(src, reason=f"stale: the kernel's sources changed since the profile (now {now})")
    return d.get("hbm_bytes_per_launch"), src


def _lib_sor_kernel(tm) -> str:
    from cfd_amd import _lib
    return _lib.SOR_KERNEL.get(tm.sor_kernel, "?")


def kcase_of(case: str) -> str:
    return "cavity" if case == "rayleigh_benard" else case  # Rayleigh-Benard runs the cavity SOR kernels


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--nx", type=int, default=4096)
    ap.add_argument("--ny", type=int, default=4096, help="rows per GPU (weak scaling)")
    ap.add_argument("--global-ny", type=int, default=0,
                    help="strong scaling: the ranks split one grid of this many rows (0: weak scaling)")
    ap.add_argument("--re", type=float, default=1000.0)
    ap.add_argument("--case", default="cavity", choices=["cavity", "channel", "backwards_step", "rayleigh_benard"],
                    help="workload (the metric is quoted on the cavity; the others are extra measurements)")
    ap.add_argument("--ra", type=float, default=1e6, help="Rayleigh number (--case rayleigh_benard)")
    ap.add_argument("--max-iters", type=int, default=10000)
    ap.add_argument("--check-every", type=int, default=1,
                    help="residual test every N SOR iterations (1 = the reference's stop rule, at every GPU count)")
    ap.add_argument("--sweeps-per-launch", type=int, default=0,
                    help="SOR iterations fused per kernel launch (0: auto = 4 in red-black proof-mode launches - "
                         "3 for the backwards step on ranks -, 3 (cavity) / 2 (open cases) with exact residuals; "
                         "4 in the reference's order, 3 on strips)")
    ap.add_argument("--proof-test", default="auto", choices=["auto", "off"],
                    help="red-black launches (every case): proof-mode convergence test (off: exact residual every "
                         "sweep)")
    ap.add_argument("--ordering", default="lex", choices=["rb", "lex"],
                    help="SOR sweep order of the headline: lex (default: the reference's lexicographic order, "
                         "bit-identical to the reference's loop on one GPU and on ranks) or rb (red-black)")
    ap.add_argument("--lex-sweeps", type=int, default=0,
                    help="reference_order: sweeps per lexicographic-order launch (0: auto = 4; 5 for the cavity)")
    ap.add_argument("--lex-steps", type=int, default=2,
                    help="N=1: also time this many steps in the other sweep order (0: skip); reported as "
                         "red_black (headline lex) or reference_order (headline rb)")
    ap.add_argument("--tile-rounds", type=int, default=-1,
                    help="red-black, one GPU: LDS-tile SOR launches when the grid fits this many resident rounds of "
                         "tiles (0: never; -1: the library default, 1)")
    ap.add_argument("--tune", action="append", default=[], metavar="KNOB=VALUE",
                    help="launch-planning knob (cfd_amd._lib.TUNING names; performance only, same bits)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--loopback-ranks", type=int, default=0,
                    help="test mode: run the multi-rank code path with this many ranks as host threads sharing "
                         "GPU 0 over the library's loopback transport (no RCCL; timings are not a measurement)")
    return ap.parse_args(argv)


class TorchGroup:
    """Barrier / max / sum over the ranks of the torch.distributed group (gloo:
    host scalars only; the data path's halos and residuals travel over RCCL
    inside the library)."""

    def __init__(self, dist, world: int):
        self.dist, self.world = dist, world

    def barrier(self) -> None:
        if self.world > 1:
            self.dist.barrier()

    def max(self, v: float) -> float:
        from cfd_amd.dist import max_over_ranks
        return max_over_ranks(self.dist, v) if self.world > 1 else v

    def sum(self, v: float) -> float:
        from cfd_amd.dist import sum_over_ranks
        return sum_over_ranks(self.dist, v) if self.world > 1 else v


class ThreadGroup:
    """The same three operations for ranks that are host threads of one
    process (--loopback-ranks)."""

    def __init__(self, world: int):
        import threading
        self.world = world
        self.bar = threading.Barrier(world)
        self.vals = [0.0] * world
        self.rank_of = {}

    def barrier(self) -> None:
        self.bar.wait(timeout=600)

    def _reduce(self, rank: int, v: float, op) -> float:
        self.barrier()
        self.vals[rank] = float(v)
        self.barrier()
        out = op(self.vals)
        self.barrier()
        return out

    def bind(self, rank: int) -> "ThreadGroup._Bound":
        return ThreadGroup._Bound(self, rank)

    class _Bound:
        def __init__(self, g, rank):
            self.g, self.rank = g, rank

        def barrier(self) -> None:
            self.g.barrier()

        def max(self, v: float) -> float:
            return self.g._reduce(self.rank, v, max)

        def sum(self, v: float) -> float:
            return self.g._reduce(self.rank, v, lambda xs: float(sum(xs)))


def run(args, rank: int, world: int, local_rank: int, comm, group, loopback: bool = False) -> dict | None:
    """One rank's benchmark: build the solver for its rows, W untimed warmup
    steps, then K timed steps bracketed by a barrier and device syncs on both
    sides; the elapsed time is the max over ranks and the cell updates the sum.
    Returns rank 0's JSON line (None on the other ranks)."""
    import torch

    import cfd_amd as C
    from cfd_amd import _lib

    check_every = max(1, args.check_every)
    strong = args.global_ny > 0
    ny_global = args.global_ny if strong else args.ny * world
    if args.case == "rayleigh_benard":  # BASELINE configs[4]: Pr 0.71, the Ra given
        cp = C.make_params(args.case, ra=args.ra, nx=args.nx, ny=ny_global, max_iters=args.max_iters)
    else:
        cp = C.make_params(args.case, re=args.re, nx=args.nx, ny=ny_global, max_iters=args.max_iters)
    tuning = {} if args.tile_rounds < 0 else {"tile_rounds": args.tile_rounds}
    for kv in args.tune:
        k_, v_ = kv.split("=", 1)
        tuning[k_] = int(v_)
    comm_info = None
    if world > 1:
        from cfd_amd.dist import comm_info as _comm_info
        from cfd_amd.dist import strip_rows, weak_rows
        comm_info = _comm_info(comm)
        rows = strip_rows(rank, world, ny_global) if strong else weak_rows(rank, args.ny)
        solver = C.solver_for(cp, device=local_rank, check_every=check_every, rank_rows=rows, comm=comm,
                              sweeps_per_launch=args.sweeps_per_launch, ordering=args.ordering,
                              proof_test=args.proof_test, tuning=tuning)
    else:
        solver = C.solver_for(cp, device=local_rank, check_every=check_every,
                              sweeps_per_launch=args.sweeps_per_launch, ordering=args.ordering,
                              proof_test=args.proof_test, tuning=tuning)

    if args.case == "cavity":  # cavity-01.cpp:380 (the open cases apply their BCs in the constructor)
        solver.applyBoundaryConditions()
    for _ in range(args.warmup):
        solver.step()
    solver.synchronize()
    solver.reset_timing()

    group.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    iters, resids = [], []
    for _ in range(args.steps):
        it, res = solver.step()
        iters.append(it)
        resids.append(res)
    solver.synchronize()
    torch.cuda.synchronize()
    group.barrier()
    elapsed = time.perf_counter() - t0
    tm = solver.timing()

    updates = float(tm.poisson_cell_updates)
    elapsed = group.max(elapsed)
    updates = group.sum(updates)
    n_gpus = world

    line = None
    if rank == 0:
        g0, g1 = solver.owned_rows()
        wrows = (g1 - g0 + 1) + (1 if g0 == 1 else 0) + (1 if g1 == cp.ny else 0)
        cells_per_launch = wrows * (cp.nx + 2)
        sor_kernel = _lib.SOR_KERNEL.get(tm.sor_kernel, "?")
        lexw = sor_kernel == "lexw"
        if lexw and tm.poisson_steady_launches > 0:
            # lexicographic order: the launches with every cell active (the
            # ramps at both ends of a solve skip or mask part of the grid)
            avg_launch_ms = tm.poisson_steady_ms / tm.poisson_steady_launches
        else:
            avg_launch_ms = tm.poisson_ms / max(tm.poisson_launches, 1)
        sweeps_per_launch = tm.poisson_sweeps / max(tm.poisson_launches, 1)
        # HBM bytes one launch must move: p_in + f read once, p_out written once,
        # whatever the number of sweeps fused into it
        achieved = BYTES_PER_CELL * cells_per_launch / (avg_launch_ms * 1e-3) / 1e9
        # the same launch measured as if each sweep streamed its own 24 B/cell
        # (the unfused algorithm's traffic): the temporal-blocking gain
        effective = achieved * sweeps_per_launch
        mlups = updates / elapsed / 1e6
        kcase = kcase_of(args.case)
        # red-black launches: proof-mode convergence test (DESIGN.md §2;
        # --proof-test off evaluates the residual in every sweep)
        proof = (args.ordering == "rb" and args.proof_test != "off"
                 and (sor_kernel == "tile" or (sor_kernel == "march" and round(sweeps_per_launch) >= 3)))
        # HBM bytes per launch from the committed PMC pass of the same workload
        # and kernel instance (profiles/), with its provenance
        traffic, traffic_src = pmc_traffic(args.case, args.ordering, cp.nx, wrows - 2, wrows, round(sweeps_per_launch),
                                           sor_template(kcase, sor_kernel, round(sweeps_per_launch), proof))
        rows_here = g1 - g0 + 1
        per_gpu = (f"{cp.nx}x{rows_here} fp64 cells per GPU (global {cp.nx}x{cp.ny} split over {n_gpus} GPUs)"
                   if strong else f"{cp.nx}x{args.ny} fp64 cells per GPU (global {cp.nx}x{cp.ny})")
        line = {
            "metric": METRIC,
            "value": round(mlups, 2),
            "unit": "MLUPS",
            "n_gpus": n_gpus,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "strong" if strong else "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic",
            "config": {
                "workload": f"{WORKLOAD[args.case]} "
                            + (f"Ra={cp.ra:g} Pr={cp.pr:g}" if args.case == "rayleigh_benard" else f"Re={args.re:g}")
                            + f", {per_gpu}, reference SOR tolerance {cp.tol_factor:g}*max|src|, "
                            f"cap {cp.max_iters} sweeps/step, {'strong' if strong else 'weak'} scaling",
                "nx": cp.nx, "ny_per_gpu": rows_here, "global_ny": cp.ny,
                "parallelism": f"strip{n_gpus}", "check_every": check_every, "ordering": args.ordering,
                "convergence_test": "proof" if proof else "residual",
            },
            "rccl_ranks": comm_info["nranks"] if comm_info else None,
            "transport": (comm_info["transport"] if comm_info else "none (1 GPU)"),
            "steps_per_sec": round(args.steps / elapsed, 4),
            "elapsed_s": round(elapsed, 6),
            "poisson_cell_updates": int(updates),
            "sor_iterations_per_step": iters,
            "sor_cap_hits": sum(1 for i in iters if i >= cp.max_iters),
            "final_residual_per_step": [float(f"{r:.6e}") for r in resids],
            "proof_fallbacks": int(tm.proof_fallbacks),
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "traffic_source": traffic_src,
                "kernel": (f"poisson_lexw_kernel<{kcase},{round(sweeps_per_launch)},sampled> (steady launches)" if lexw
                           else f"poisson_tile_kernel<{kcase},{'proof' if proof else 'exact'}> "
                                f"({round(sweeps_per_launch)} sweeps per launch)"
                           if sor_kernel == "tile"
                           else f"poisson_multi_kernel<{kcase},{round(sweeps_per_launch)},proof>" if proof and kcase == "cavity"
                           else f"poisson_open_proof_kernel<{kcase},{round(sweeps_per_launch)}>" if proof
                           else f"poisson_multi_kernel<{kcase},3>" if sweeps_per_launch > 2.5
                           else f"poisson_multi_kernel<{kcase},2>" if sweeps_per_launch > 1.5
                           else f"poisson_wave_kernel<{kcase}>" if sor_kernel == "march"
                           else f"{sor_kernel} ({kcase}, whole solve in one launch)"),
                "bytes_per_launch": BYTES_PER_CELL * cells_per_launch,
                "avg_launch_us": round(avg_launch_ms * 1e3, 2),
                "sweeps_per_launch": round(sweeps_per_launch, 4),
                "effective_sweep_GBs": round(effective, 1),
                "effective_sweep_frac": round(effective / HBM_PEAK_GBS, 4),
            },
        }
        if sor_kernel == "resident":
            # the register-resident whole-solve launch (resident.hpp): p and f*h^2
            # stay in VGPRs, HBM carries only the tiles' 8-cell edge bands - the
            # bound is the fp64 VALU work and the group hand-offs, not HBM
            fpu = FLOPS_PER_UPDATE.get(kcase)
            tflops = fpu * updates / elapsed / 1e12 if fpu else None
            line["roofline"] = {
                "bound": "valu", "achieved": round(tflops, 3) if tflops else None, "peak": FP64_VALU_PEAK_TF,
                "unit": "TFLOP/s", "frac": round(tflops / FP64_VALU_PEAK_TF, 4) if tflops else None, "traffic": None,
                "traffic_source": "none: register-resident solve (no per-sweep HBM stream)",
                "kernel": f"poisson_resident_kernel<{kcase},{'lex' if args.ordering == 'lex' else 'rb'}> "
                          "(whole solve in one launch)",
                "avg_launch_us": round(avg_launch_ms * 1e3, 2), "sweeps_per_launch": round(sweeps_per_launch, 4),
                "us_per_sweep": round(avg_launch_ms * 1e3 / max(sweeps_per_launch, 1), 4),
                # what bounds it (phase stamps of the cavity at 1024^2,
                # profiles/r5/resident/, profiles/r6/resident_granules/): per
                # group ~8 K cycles of sweeps per 4 sweeps against ~12-14 K of
                # hand-off (the write-through bands' visibility to the neighbour
                # CUs, ~3 us) - the VALU fraction above is not the limit; the
                # reference order's groups run 8 (cavity) / 6 (channel) sweeps
                "note": "hand-off-latency bound: ~8 K cycles of sweeps per 4 sweeps vs ~12-14 K per edge-band hand-off "
                        "(a group: red-black 4 sweeps, reference order 8 cavity / 6 channel; DESIGN.md section 4)",
            }
        if loopback:
            line["config"]["loopback_ranks_on_one_gpu"] = world
        if not args.no_cpu_baseline and world == 1:  # the CPU leg is timed at N=1 only
            log("timing the CPU baseline ...")
            line["cpu_baseline"] = cpu_baseline(cp.nx, cp.ny, args.cpu_seconds, args.case)
            if args.case == "cavity":  # beside it: the reference's own binary on its own case (same host)
                line["cpu_baseline"]["reference_binary"] = reference_binary()
        if world == 1 and args.lex_steps > 0 and args.case != "rayleigh_benard":
            if args.ordering == "rb":
                line["reference_order"] = reference_order(C, cp, args, local_rank, check_every, cells_per_launch)
            else:
                line["red_black"] = red_black(C, cp, args, local_rank, check_every, cells_per_launch, tuning)
    solver.close()
    return line


def run_loopback(args) -> dict:
    """--loopback-ranks N: the rank path of run() with N host-thread ranks on
    GPU 0 (cfd_comm_init_loopback: the same group send / recv / all-reduce
    call sites as RCCL), for tests/test_gpu_bench_ranks.py."""
    import threading

    import torch  # noqa: F401  (first: PyTorch's HIP runtime is the one the library binds to)

    from cfd_amd import _lib

    world = args.loopback_ranks
    L = _lib.lib()
    hub = L.cfd_comm_loopback_hub(world)
    group = ThreadGroup(world)
    out, errors = [None], []

    def body(r):
        try:
            comm = L.cfd_comm_init_loopback(hub, r, 0)
            if not comm:
                raise _lib.CfdError(L.cfd_last_error().decode())
            line = run(args, r, world, 0, comm, group.bind(r), loopback=True)
            if r == 0:
                out[0] = line
            L.cfd_comm_destroy(comm)
        except BaseException as e:  # noqa: BLE001
            errors.append(e)
            group.bar.abort()

    th = [threading.Thread(target=body, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    L.cfd_comm_loopback_hub_destroy(hub)
    if errors:
        raise errors[0]
    return out[0]


def main() -> int:
    args = parse_args()
    if args.loopback_ranks > 0:
        print(json.dumps(run_loopback(args)), flush=True)
        return 0
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"note: WORLD_SIZE={world} but --gpus={args.gpus}; using WORLD_SIZE")

    import torch  # noqa: E402  (first: PyTorch's HIP runtime is the one the library binds to)
    import torch.distributed as dist

    from cfd_amd import _lib

    torch.cuda.set_device(local_rank)
    comm = None
    if world > 1:
        from cfd_amd.dist import init_comm
        dist.init_process_group("gloo", rank=rank, world_size=world)
        comm = init_comm(dist, rank, world, local_rank)
    line = run(args, rank, world, local_rank, comm, TorchGroup(dist, world))
    if rank == 0:
        print(json.dumps(line), flush=True)
    if comm:
        _lib.lib().cfd_comm_destroy(comm)
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
