"""Diagnostic: where do the reference order's rank path and one device part?
Channel reference defaults, one step, stage by stage (src after the mean
removal, then the solve), 1 strip / 3 strips / 3 loopback ranks vs the oracle."""
import sys, os, threading
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "computational-fluid-dynamics_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import numpy as np
import cfd_amd as C
import oracle as O
from cfd_amd import _lib
from cfd_amd.dist import strip_rows

case = sys.argv[1] if len(sys.argv) > 1 else "channel"
world = int(sys.argv[2]) if len(sys.argv) > 2 else 3
cp = C.reference_defaults(case)
o = O.Oracle(cp, ordering=O.LEX)
o.tentative(); o.velocity_bc(True); o.source()
osrc = o.field("src").copy()
io, ro = o.poisson()
op = o.field("p").copy()
print("oracle", io, ro)

def bits_eq(a, b):
    return int((a.view(np.int64) != b.view(np.int64)).sum())

for strips in (1, world):
    g = C.solver_for(cp, ordering="lex", small_solve="off", n_strips=strips, tuning={"resident": 0})
    g.computeTentativeVelocities(); g.applyTentativeBoundaryConditions(); g.buildSourceTerm()
    d_src = bits_eq(g.field("src"), osrc)
    it = g.solverPressurePoisson()
    print(f"strips={strips}: src diff {d_src}, solve {it}, p diff {bits_eq(g.field('p'), op)}")
    g.close()

L = _lib.lib()
hub = L.cfd_comm_loopback_hub(world)
out = [None] * world
def body(r):
    comm = L.cfd_comm_init_loopback(hub, r, 0)
    s = C.solver_for(cp, ordering="lex", rank_rows=strip_rows(r, world, cp.ny), comm=comm)
    s.computeTentativeVelocities(); s.applyTentativeBoundaryConditions(); s.buildSourceTerm()
    src = s.field("src")
    it = s.solverPressurePoisson()
    out[r] = (s.owned_rows(), src, it, s.field("p"))
    s.close(); L.cfd_comm_destroy(comm)
th = [threading.Thread(target=body, args=(r,)) for r in range(world)]
[t.start() for t in th]; [t.join() for t in th]
L.cfd_comm_loopback_hub_destroy(hub)
src = np.concatenate([x[1] for x in out]); p = np.concatenate([x[3] for x in out])
print(f"ranks={world}: src diff {bits_eq(src, osrc)}, solves {[x[2] for x in out]}, p diff {bits_eq(p, op)}")
if bits_eq(src, osrc):
    d = np.argwhere(src.view(np.int64) != osrc.view(np.int64))
    print("first src diffs", d[:5], src[tuple(d[0])], osrc[tuple(d[0])])
