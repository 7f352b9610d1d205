"""get_tisr_by_date's calendar index (sml_tisr_date_index; src/mod_calendar.f90:24-175,
src/mpires.f90:1644-1676), CPU only.  Known answers derived by hand from the
reference's statements (quirks included: hour 0 falls on Dec 31 of the year before,
a day boundary rounds the day down, a February met in a leap year keeps 29 days for
the rest of the run because the month table is a SAVEd local), and a line-by-line
Python restatement of the same subroutines over a 30-year span."""
import ctypes

import pytest

from speedy_ml_amd._lib import lib


def _idx(startyear, hours, feb29=0):
    f = ctypes.c_int(feb29)
    i = ctypes.c_int()
    assert lib().sml_tisr_date_index(startyear, hours, ctypes.byref(f), ctypes.byref(i)) == 0
    return i.value, f.value


@pytest.mark.parametrize("start,hours,want", [
    (1981, 0, 8760),        # day_of_year 0 -> month 0 -> Dec 31 1980 (a leap year: 335 + 30 days) -> 8760
    (1981, 24, 1),          # Jan 1 00 -> 0 hours -> 1
    (1981, 30, 6),          # Jan 1 06
    (1981, 24 * 32 + 12, 31 * 24 + 12),   # Feb 1 12
    (1984, 8760 + 24, 8760),  # one year on, minus 1984's leap day: day 0 of 1985 -> Dec 31 1984 -> 8760
])
def test_known_answers(start, hours, want):
    assert _idx(start, hours)[0] == want


def _leap(y):
    return (y % 4 == 0 and y % 100 != 0) or y % 400 == 0


def _ref(startyear, hours, state):
    """mod_calendar.f90 get_current_time_delta_hour + numof_hours_into_year, statement
    by statement; state['ncal'] is the SAVEd month table."""
    years = hours // 8760
    year = years + startyear
    leap_days = sum(1 for i in range(years) if _leap(startyear + i))
    ncal = state["ncal"]
    day_of_year = (hours % 8760) // 24 - leap_days
    if _leap(year):
        ncal[1] = 29
    c = day_of_year
    month = 1
    while c > 0:
        c -= ncal[month - 1]
        month += 1
    month -= 1
    if month <= 0:
        month = 12
        year -= 1
    day = ncal[month - 1] + c
    hour = hours % 24
    tab = [31, 29 if _leap(year) else 28, 31, 30, 31, 30, 31, 31, 30, 31, 30, 31]
    n = sum(24 * tab[i] for i in range(month - 1)) + 24 * max(0, day - 1) + hour
    if n == 0:
        n = 1
    if n > 8760:
        n -= 8760
    return n


@pytest.mark.parametrize("start", [1981, 1990, 2000])
def test_matches_restatement_over_decades(start):
    state = {"ncal": [31, 28, 31, 30, 31, 30, 31, 31, 30, 31, 30, 31]}
    feb = 0
    for h in range(0, 30 * 8760, 6 * 37):
        got, feb = _idx(start, h, feb)
        assert got == _ref(start, h, state), (start, h)
        assert 1 <= got <= 8784
