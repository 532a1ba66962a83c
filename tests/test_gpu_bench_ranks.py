"""bench.py's multi-rank code path end to end (run(): rank rows, solver on a
communicator, warmup, barrier-bracketed timed loop, max-over-ranks elapsed,
summed cell updates, the JSON line) with 2-3 ranks as host threads sharing one
GPU over the library's loopback transport (--loopback-ranks): what the
driver's N-GPU run executes, minus RCCL itself (tests/rccl_two_ranks.py and
test_gpu_rccl.py cover that on a box with two devices)."""
from __future__ import annotations

import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def bench(*args):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                       timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


@pytest.mark.parametrize("world,extra,scaling,case,order", [
    (2, [], "weak", "cavity", "lex"),
    (3, ["--global-ny", "192"], "strong", "cavity", "lex"),
    (2, [], "weak", "channel", "lex"),
    (4, [], "weak", "backwards_step", "lex"),
    (2, [], "weak", "cavity", "rb"),
    (3, ["--global-ny", "192"], "strong", "channel", "rb"),
])
def test_bench_rank_path_json_line(world, extra, scaling, case, order):
    nx, ny = 256, 64
    d = bench("--loopback-ranks", str(world), "--case", case, "--nx", str(nx), "--ny", str(ny), "--steps", "2",
              "--warmup", "1", "--max-iters", "400", "--no-cpu-baseline", "--lex-steps", "0", "--ordering", order,
              *extra)
    assert d["n_gpus"] == world and d["rccl_ranks"] == world
    assert d["transport"] == "loopback"
    assert d["scaling"] == scaling and f"{scaling} scaling" in d["config"]["workload"]
    assert d["config"]["loopback_ranks_on_one_gpu"] == world
    assert d["config"]["ordering"] == order
    gny = 192 if scaling == "strong" else ny * world
    assert d["config"]["global_ny"] == gny
    assert d["config"]["parallelism"] == f"strip{world}"
    # value = cell updates summed over ranks / the max-over-ranks elapsed time
    assert d["poisson_cell_updates"] == nx * gny * sum(d["sor_iterations_per_step"])
    assert d["value"] == pytest.approx(d["poisson_cell_updates"] / d["elapsed_s"] / 1e6, rel=1e-4)
    assert "cpu_baseline" not in d and "reference_order" not in d and "red_black" not in d  # (N = 1 legs only)
    assert d["roofline"]["frac"] > 0 and d["unit"] == "MLUPS"
    if order == "lex":
        assert "poisson_lexw_kernel" in d["roofline"]["kernel"]


def test_bench_default_is_reference_order_with_red_black_leg():
    """N = 1, defaults: the headline in the reference's order, the red-black
    order of the same workload beside it."""
    d = bench("--nx", "256", "--ny", "256", "--steps", "1", "--warmup", "1", "--max-iters", "300",
              "--no-cpu-baseline", "--lex-steps", "1")
    assert d["config"]["ordering"] == "lex"
    k = d["roofline"]["kernel"]  # (256^2 fits the register-resident launch)
    assert "poisson_lexw_kernel" in k or "poisson_resident_kernel<cavity,lex>" in k
    assert d["red_black"]["ordering"] == "rb" and d["red_black"]["value"] > 0
    assert "reference_order" not in d
