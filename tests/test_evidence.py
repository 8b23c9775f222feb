"""The committed measurement evidence agrees with itself (CPU only).

profiles/r06_final/ is the closing run DESIGN.md §9 cites.  These checks pin
what a reader would otherwise verify by hand:

* each throughput config's rocprofv3 line and the kernel-trace summary of the
  same process agree on the march's average launch time (the summary also
  counts the warm-up and the three host-array launches, so within 2 %);
* every throughput line's parity record passed and compared the scenarios
  the line says;
* profiles/pmc_counters.json is keyed to the kernel sources in this tree, so
  bench.py reports its traffic / issue records (a stale key would null them);
* no record of a line claims more than its stated peak.
"""
import csv
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FINAL = os.path.join(ROOT, "profiles", "r06_final")
THROUGHPUT = ("american", "barrier", "double", "spot_vc")


def _line(path):
    with open(path) as f:
        return json.loads(f.read().strip().splitlines()[-1])


def _march_avg_ms(wl):
    """Average launch time of the march kernels in the summary (the spot-space
    launch is the march plus its factor kernel)."""
    total = 0.0
    with open(os.path.join(FINAL, f"kernel_stats_{wl}.csv")) as f:
        for r in csv.DictReader(f):
            name = r["Name"]
            if "fdcn_march<" in name or "fdcn_vc_march<1, 16, true>" in name or \
                    "fdcn_vc_factor" in name:
                total += float(r["AverageNs"]) / 1e6
    return total


@pytest.mark.parametrize("wl", THROUGHPUT)
def test_rocprof_line_matches_its_summary(wl):
    line = _line(os.path.join(FINAL, f"rocprof_bench_{wl}.json"))
    avg = _march_avg_ms(wl)
    assert avg > 0
    assert abs(line["kernel_ms_per_launch"] - avg) / avg < 0.02, (line["kernel_ms_per_launch"], avg)


@pytest.mark.parametrize("wl", THROUGHPUT)
def test_throughput_lines_carry_passing_parity(wl):
    for name in (f"bench_{wl}.json", f"rocprof_bench_{wl}.json"):
        line = _line(os.path.join(FINAL, name))
        p = line["parity"]
        assert p["ok"] and p["all_finite"] and p["max_rel_err"] <= p["tol"], name
        assert p["n_compared"] >= 1000, name
        assert line["cpu_baseline"]["value"] > 0, name


def test_pmc_counters_keyed_to_this_tree():
    sys.path.insert(0, ROOT)
    import bench
    with open(os.path.join(ROOT, "profiles", "pmc_counters.json")) as f:
        rec = json.load(f)
    for key, r in rec.items():
        want = bench.file_sha("fdcn_vc.hip") if key.startswith("spot_vc") else bench.kernel_src_sha()
        assert r["kernel_src_sha"] == want, key


def _peaked(rec):
    if isinstance(rec, dict):
        if "achieved" in rec and "peak" in rec:
            yield rec
        for v in rec.values():
            yield from _peaked(v)
    elif isinstance(rec, list):
        for v in rec:
            yield from _peaked(v)


def test_no_committed_line_exceeds_a_peak():
    for name in sorted(os.listdir(FINAL)):
        if not name.endswith(".json"):
            continue
        for r in _peaked(_line(os.path.join(FINAL, name))):
            assert 0.0 < r["achieved"] <= r["peak"], (name, r)
