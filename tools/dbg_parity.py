"""Debug helper (GPU box): locate where the HIP march departs from the oracle."""
import sys
import numpy as np
sys.path.insert(0, "tests")
sys.path.insert(0, ".")
from finite_difference_amd.engine import Engine
from plan_factory import random_solve
from test_gpu_kernels import OracleBackend


def run(n, m, r, it, ko=True, seed=0):
    rng = np.random.default_rng(seed)
    s = random_solve(rng, n, m, r, it=it, ko=ko)
    g = Engine().run([s])[0]
    o = Engine(OracleBackend()).run([s])[0]
    e = np.abs(g - o) / max(1.0, np.max(np.abs(o)))
    bad = np.nonzero(e > 1e-10)[0]
    print(f"n={n} m={m} r={r} it={it} ko={ko}: max err {e.max():.3e} at {int(e.argmax())}; "
          f"bad nodes {len(bad)}: {bad[:12].tolist()} ... {bad[-6:].tolist()}", flush=True)


for (n, m, r, it, ko) in [(1024, 1, 0, False, False), (1024, 1, 2, False, False),
                          (1024, 2, 0, False, False), (1024, 150, 0, False, False),
                          (1024, 150, 2, False, False), (257, 1, 0, True, False),
                          (257, 2, 0, True, False), (257, 100, 2, True, False),
                          (769, 1, 0, False, False), (772, 1, 0, False, False),
                          (66, 1, 0, False, False), (64, 1, 0, False, False)]:
    run(n, m, r, it, ko)
