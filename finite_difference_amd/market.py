"""Market plumbing used by the pricer constructors: day counts, NACA curves,
the South African business-day calendar, and the rate helpers of utils.py.

These are host-side (pure Python) because the reference's are
(discrete_barrier_fdm_pricer.py:174-268, fd_american_equity.py:270-334,
utils.py:16-104); they run once per trade, not per grid node.
"""
from __future__ import annotations

import datetime as _dt
import math
from functools import lru_cache
from typing import Dict, Optional

import numpy as np

# ---------------------------------------------------------------------------
# utils.py equivalents
# ---------------------------------------------------------------------------


def nacc_to_naca(nacc_rate: float) -> float:
    """NACA = exp(NACC) - 1 (utils.py:16-41)."""
    return float(np.exp(nacc_rate) - 1.0)


def naca_to_nacc(naca_rate: float) -> float:
    """NACC = ln(1 + NACA) (utils.py:44-68)."""
    return float(np.log(1.0 + naca_rate))


def create_rate_df(rate: float, start: _dt.date = _dt.date(2025, 7, 28),
                   end: _dt.date = _dt.date(2028, 9, 28)):
    """Flat daily NACA curve with "YYYY/MM/DD" dates (utils.py:71-104)."""
    import pandas as pd
    dates = pd.date_range(start=start, end=end, freq="D")
    return pd.DataFrame({"Date": dates.strftime("%Y/%m/%d"), "NACA": rate})


def iso_curve(df):
    """Copy of a curve with ISO "YYYY-MM-DD" dates, as the runners pass it
    (run_config_scenarios.py:56-57)."""
    import pandas as pd
    out = df.copy()
    out["Date"] = pd.to_datetime(out["Date"], format="%Y/%m/%d").dt.strftime("%Y-%m-%d")
    return out


# ---------------------------------------------------------------------------
# day counts
# ---------------------------------------------------------------------------


def normalise_day_count(day_count: str) -> str:
    return day_count.upper().replace("F", "")


def year_denominator(day_count: str) -> int:
    if day_count in ("ACT/365", "ACT/365F"):
        return 365
    if day_count == "ACT/360":
        return 360
    if day_count == "ACT/364":
        return 364
    if day_count in ("30/360", "BOND", "US30/360"):
        return 360
    return 365


def year_fraction(day_count: str, start: _dt.date, end: _dt.date) -> float:
    """Simple year fractions (discrete_barrier_fdm_pricer.py:188-203)."""
    if end <= start:
        return 0.0
    if day_count in ("ACT/365", "ACT/365F", "ACT/360", "ACT/364"):
        return (end - start).days / float(year_denominator(day_count))
    if day_count in ("30/360", "BOND", "US30/360"):
        d1 = min(start.day, 30)
        d2 = end.day
        if d1 == 30:
            d2 = min(d2, 30)
        days = (end.year - start.year) * 360 + (end.month - start.month) * 30 + (d2 - d1)
        return days / 360.0
    return (end - start).days / 365.0


# ---------------------------------------------------------------------------
# curves
# ---------------------------------------------------------------------------


_MAP_CACHE: Dict[tuple, Dict[str, float]] = {}


class NacaCurve:
    """Date -> NACA lookup over a DataFrame with columns "Date" (ISO) / "NACA".

    Same semantics as the reference's row filter (exact ISO match, first row
    wins, missing date raises ValueError) with an O(1) dict instead of a scan.
    A batch of trades usually shares one curve: the map is cached by the
    curve's content (every date string and every NACA bit pattern), so each
    pricer pays a fingerprint, not a rebuild.
    """

    def __init__(self, df):
        self.df = df
        self._map: Optional[Dict[str, float]] = None

    def _build(self) -> Dict[str, float]:
        col = self.df["Date"]
        raw = col.to_numpy()
        if raw.dtype == object and len(raw) and type(raw[0]) is str:
            dates = tuple(raw.tolist())  # a column of date strings
        else:
            dates = tuple(col.astype(str).tolist())
        naca = np.ascontiguousarray(self.df["NACA"].to_numpy(dtype=np.float64))
        key = (dates, naca.tobytes())
        m = _MAP_CACHE.get(key)
        if m is None:
            # reversed, so the first row of a repeated date wins
            m = dict(zip(reversed(dates), reversed(naca.tolist())))
            if len(_MAP_CACHE) > 64:
                _MAP_CACHE.clear()
            _MAP_CACHE[key] = m
        return m

    def naca(self, d: _dt.date) -> Optional[float]:
        if self._map is None:
            self._map = self._build()
        return self._map.get(d.isoformat())


# ---------------------------------------------------------------------------
# calendar
# ---------------------------------------------------------------------------


def _easter(year: int) -> _dt.date:
    """Gregorian Easter Sunday (anonymous Gregorian algorithm)."""
    a = year % 19
    b, c = divmod(year, 100)
    d, e = divmod(b, 4)
    f = (b + 8) // 25
    g = (b - f + 1) // 3
    h = (19 * a + b - d - g + 15) % 30
    i, k = divmod(c, 4)
    l_ = (32 + 2 * e + 2 * i - h - k) % 7
    m = (a + 11 * h + 22 * l_) // 451
    month, day = divmod(h + l_ - 7 * m + 114, 31)
    return _dt.date(year, month, day + 1)


@lru_cache(maxsize=256)
def _sa_holidays(year: int) -> frozenset:
    fixed = [(1, 1), (3, 21), (4, 27), (5, 1), (6, 16), (8, 9), (9, 24), (12, 16), (12, 25),
             (12, 26)]
    days = set()
    for mth, dy in fixed:
        d = _dt.date(year, mth, dy)
        days.add(d)
        if d.weekday() == 6:  # Public Holidays Act: a Sunday holiday moves to Monday
            days.add(d + _dt.timedelta(days=1))
    e = _easter(year)
    days.add(e - _dt.timedelta(days=2))  # Good Friday
    days.add(e + _dt.timedelta(days=1))  # Family Day
    return frozenset(days)


class SouthAfrica:
    """Business-day calendar standing in for workalendar.africa.SouthAfrica
    (used at discrete_barrier_fdm_pricer.py:113,145-149 and
    fd_american_equity.py:190,202-214).  Statutory holidays + Sunday->Monday;
    add_working_days(d, 0) returns d, as workalendar does."""

    def is_working_day(self, d: _dt.date) -> bool:
        return d.weekday() < 5 and d not in _sa_holidays(d.year)

    def add_working_days(self, day: _dt.date, delta) -> _dt.date:
        step = 1 if delta >= 0 else -1
        remaining = abs(delta)
        count = 0
        cur = day
        while count < remaining:
            cur = cur + _dt.timedelta(days=step)
            if self.is_working_day(cur):
                count += 1
        return cur


def discount_factor(curve: NacaCurve, day_count: str, valuation: _dt.date,
                    d: _dt.date) -> float:
    """(1 + NACA)^(-tau), tau from valuation (discrete_barrier_fdm_pricer.py:205-214)."""
    naca = curve.naca(d)
    if naca is None:
        raise ValueError(f"Discount factor not found for date: {d.isoformat()}")
    tau = year_fraction(day_count, valuation, d)
    return (1.0 + naca) ** (-tau)


def forward_nacc(curve: NacaCurve, day_count: str, valuation: _dt.date, start: _dt.date,
                 end: _dt.date) -> float:
    """Continuously compounded forward rate (discrete_barrier_fdm_pricer.py:226-230)."""
    df_far = discount_factor(curve, day_count, valuation, end)
    df_near = discount_factor(curve, day_count, valuation, start)
    tau = year_fraction(day_count, start, end)
    return -math.log(df_far / df_near) / max(1e-12, tau)
