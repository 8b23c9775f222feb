"""FDCN_I_TAU_MODE = 1: the kernels evaluate the reference American loop's
accumulated tau (tau = tau + dt per step, fd_american_equity.py:664-724) in
constant-increment runs instead of one dependent add per step.  The run
construction (tau_next_run, shared by host and device) must reproduce the
serial Python adds bit for bit -- including binade crossings, rounding ties
and stagnation (dt below half an ulp) -- while needing far fewer runs than
steps.  fdcn_tau_sequence exposes it on the host."""
import numpy as np
import pytest

from finite_difference_amd import capi


def serial(tau0, dt, n):
    out, t = [], tau0
    for _ in range(n):
        t = t + dt
        out.append(t)
    return out


CASES = [
    (0.0, (31 / 365) / 4096, 4096),          # config 2: first segment from tau = 0
    (0.0, (31 / 365) / 8192, 8192),
    (0.0, 0.01 / 3.0, 3000),
    (0.02054794520547945, 0.0001234567, 900),  # a later dividend segment
    (1e4, 1e-3 / 3.0, 700),                   # large tau0 (GPU tau-mode test)
    (1.0, 2.0 ** -30 + 2.0 ** -53, 600),      # remainder exactly u/2: ties-to-even
    (1.0, 2.0 ** -54, 50),                    # dt < u/2: tau never moves
    (1.0, 2.0 ** -53 * 3, 400),               # dt = 1.5 u
    (0.5, 0.5, 40),                            # dt == tau: doubling
    (3.0, 7.0, 30),                            # dt > tau
    (0.0, 0.0, 5),
]


@pytest.mark.parametrize("tau0,dt,n", CASES)
def test_runs_are_bitwise_serial(tau0, dt, n):
    got = capi.tau_sequence(tau0, dt, n)
    assert got.tolist() == serial(tau0, dt, n)


def test_random_segments_bitwise():
    rng = np.random.default_rng(2025)
    for _ in range(300):
        T = float(rng.uniform(1e-3, 3.0))
        n = int(rng.integers(1, 5000))
        tau0 = 0.0 if rng.integers(3) == 0 else float(rng.uniform(0.0, 2.0))
        dt = T / n
        assert capi.tau_sequence(tau0, dt, n).tolist() == serial(tau0, dt, n), (tau0, dt, n)


def test_runs_are_few():
    """~3 runs per binade: 4096 steps from tau = 0 need well under 100 runs
    (the serial form is 4096 dependent adds per wave)."""
    n = 4096
    runs = capi.tau_runs(0.0, (31 / 365) / n, n)
    assert runs < 80, runs
    assert capi.tau_runs(0.0, (31 / 365) / 8192, 8192) < 90
