"""Solver backends for tests.

OracleBackend runs a packed launch group through the CPU oracle
(oracle/fdcn_oracle.c, test infrastructure).  Tests pass it to the product's
pricers (engine=Engine(OracleBackend())) to check the host-side logic on a
machine without a GPU; the product itself only ever uses the HIP backend.
"""
from finite_difference_amd.engine import Engine


class OracleBackend:
    name = "oracle"

    def __init__(self, nthreads: int = 1):
        self.nthreads = nthreads

    def run_group(self, g):
        from oracle import oracle
        if g.it:
            return oracle.it_batch(g.n_nodes, g.n_time, g.n_ranna, g.params, g.iparams,
                                   g.v_init, g.payoff, self.nthreads)
        return oracle.cn_batch(g.n_nodes, g.n_time, g.n_ranna, g.params, g.iparams, g.v_init,
                               g.mon_step, g.mon_rebate, self.nthreads)

    def run_vc_group(self, g):
        from oracle import oracle
        return oracle.vc_batch(g.n_nodes, g.n_time, g.n_ranna, g.diag, g.bnd, g.v_init,
                               g.iparams, g.mon_step, g.mon_rebate, self.nthreads)


    def run_rr(self, contracts):
        """The host closed form (analytic.BarrierEngine, the reference's
        formulas in NumPy/SciPy) in place of the GPU batch."""
        from finite_difference_amd.analytic import BarrierEngine
        return [BarrierEngine(**c).price() for c in contracts]

    def run_double(self, contracts, m):
        from finite_difference_amd.analytic import DoubleBarrier
        out = []
        for c in contracts:
            c = dict(c)
            b, r, T = c.pop("b"), c.pop("r"), c.pop("T")
            out.append(DoubleBarrier(m=m, **c).price(b=b, r=r, T=T))
        return out


def oracle_engine() -> Engine:
    return Engine(OracleBackend())
