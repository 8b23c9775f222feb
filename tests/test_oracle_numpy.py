"""The NumPy batched-over-scenarios restatement (oracle/batched_numpy.py, the
second CPU baseline of SURVEY §8(d)) agrees with the C oracle on the same
plans: IT and knock-out marches, both tau modes, Rannacher on and off.
Tolerance 1e-13 relative: the only difference is np.exp vs libm exp in the
boundary values (same operation order otherwise)."""
import numpy as np
import pytest

from finite_difference_amd.engine import pack
from oracle import batched_numpy, oracle
from plan_factory import random_solve


@pytest.mark.parametrize("it", [True, False], ids=["it", "cn"])
@pytest.mark.parametrize("n_nodes,n_time,n_ranna", [(40, 30, 2), (257, 64, 0), (513, 25, 2)])
def test_numpy_batched_matches_c_oracle(it, n_nodes, n_time, n_ranna):
    rng = np.random.default_rng(n_nodes + n_time + int(it))
    solves = [random_solve(rng, n_nodes, n_time, n_ranna, it=it) for _ in range(5)]
    for k, s in enumerate(solves):
        s.tau_accumulate = k % 2 == 0
        s.tau0 = 0.0 if k < 3 else 0.05
    g = pack(solves, list(range(len(solves))))
    if it:
        ref = oracle.it_batch(g.n_nodes, g.n_time, g.n_ranna, g.params, g.iparams, g.v_init,
                              g.payoff)
        got = batched_numpy.march(True, g.n_nodes, g.n_time, g.n_ranna, g.params, g.iparams,
                                  g.v_init, payoff=g.payoff)
    else:
        ref = oracle.cn_batch(g.n_nodes, g.n_time, g.n_ranna, g.params, g.iparams, g.v_init,
                              g.mon_step, g.mon_rebate)
        got = batched_numpy.march(False, g.n_nodes, g.n_time, g.n_ranna, g.params, g.iparams,
                                  g.v_init, mon_step=g.mon_step, mon_rebate=g.mon_rebate)
    for r, x in zip(ref, got):
        assert np.max(np.abs(x - r)) <= 1e-13 * max(1.0, np.max(np.abs(r)))


def test_numpy_batched_prefix_of_steps():
    rng = np.random.default_rng(9)
    solves = [random_solve(rng, 100, 40, 2, it=True) for _ in range(3)]
    g = pack(solves, [0, 1, 2])
    part = batched_numpy.march(True, g.n_nodes, g.n_time, g.n_ranna, g.params, g.iparams,
                               g.v_init, payoff=g.payoff, max_steps=7)
    g7 = pack(solves, [0, 1, 2])
    for s in solves:
        s.n_time = 7
    g7 = pack(solves, [0, 1, 2])
    ref = oracle.it_batch(g7.n_nodes, 7, g7.n_ranna, g7.params, g7.iparams, g7.v_init,
                          g7.payoff)
    assert np.max(np.abs(part - ref)) <= 1e-13 * max(1.0, np.max(np.abs(ref)))
