"""libfdcn's host C++ under sanitizers, on the CPU.

`make sanitize` (Makefile) compiles the host-only translation units --
fdcn_host.hip (plan checks, log grid, tau sequence, dividend jump, error
reporting) and fdcn_plan.hip (the whole-file plan builders, which fan rows
out over std::threads) -- for the host alone, and
  asan: with AddressSanitizer + UndefinedBehaviorSanitizer (first report
        aborts) into build/asan/libfdcn.so, then runs the bitwise plan tests
        (test_scenario_batch, test_american_batch, test_tau_sequence,
        test_capi_symbols, the host facades) against that library;
        It also runs tools/sanitize/session_book_driver.cpp: the device
        sessions' host-only bookkeeping (csrc/fdcn_session_book.h -- the
        pinned staging arena, slot and producer-event tables, the destroy
        path's reset + trim) under the same two sanitizers, malloc standing in
        for hipHostMalloc;
  tsan: with ThreadSanitizer into tools/sanitize/plan_driver.cpp, which runs
        the plan builders from two threads at once and checks the results
        bitwise against a sequential run.
Device code is not instrumented (host sanitizers only)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _make(target):
    return subprocess.run(["make", "-s", target], cwd=ROOT, capture_output=True, text=True,
                          timeout=900)


def test_make_asan_plan_tests_clean():
    p = _make("asan")
    assert p.returncode == 0, (p.stdout[-3000:], p.stderr[-3000:])
    assert "passed" in p.stdout and "ERROR: AddressSanitizer" not in p.stderr
    assert "runtime error" not in p.stderr  # UBSan
    assert "session_book_driver: ok" in p.stdout


def test_asan_library_is_instrumented():
    p = subprocess.run(["nm", os.path.join(ROOT, "build", "asan", "fdcn_plan.o")],
                       capture_output=True, text=True)
    if p.returncode:
        pytest.skip("asan objects not built")
    assert "__asan_report" in p.stdout and "__ubsan_handle" in p.stdout


def test_session_book_driver_is_instrumented():
    p = subprocess.run(["nm", os.path.join(ROOT, "build", "asan", "session_book_driver")],
                       capture_output=True, text=True)
    if p.returncode:
        pytest.skip("session_book_driver not built")
    assert "__asan_report" in p.stdout and "__ubsan_handle" in p.stdout


def test_make_tsan_plan_driver_clean():
    p = _make("tsan")
    assert p.returncode == 0, (p.stdout[-3000:], p.stderr[-3000:])
    assert "plan_driver: ok" in p.stdout
    assert "WARNING: ThreadSanitizer" not in p.stderr
