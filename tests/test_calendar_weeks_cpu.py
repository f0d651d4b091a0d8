"""DateTime.previousInterval for week intervals (src/utils/DateTime.java:551-571), in the oracle.

Intervals of more than 2 weeks take the `set(MONTH, 0); set(DAY_OF_WEEK, SUNDAY)` branch:
GregorianCalendar resolves YEAR + MONTH + WEEK_OF_MONTH + DAY_OF_WEEK, a Sunday in January, and
the 7-day walk from there ends on the Sunday of ts's week -- TestDateTime.previousIntervalWeeks'
"multiples - still from start of the week" (104 weeks)."""
from __future__ import annotations

import ctypes as C

import pytest

from opentsdb_amd import abi
from oracle import oracle as O

NON_DST_TS = 1431699673432   # TestDateTime.java:53
DST_TS = 1450152145123       # :55


def prev(ts, n, unit=abi.CAL_W):
    L = O.lib()
    L.ref_cal_prev_ex.argtypes = [C.c_int64, C.c_int64, C.c_int, C.c_void_p, C.POINTER(C.c_int64)]
    out = C.c_int64()
    rc = L.ref_cal_prev_ex(ts, n, unit, None, C.byref(out))
    assert rc == 0
    return out.value


@pytest.mark.parametrize("ts,n,want", [
    (DST_TS, 1, 1449964800000), (NON_DST_TS, 1, 1431216000000),                    # :786-789
    (DST_TS, 2, 1449964800000), (NON_DST_TS, 2, 1431216000000),                    # :792-795
    (1435795200000, 2, 1435449600000),                                             # :796-797
    (DST_TS, 104, 1449964800000), (NON_DST_TS, 104, 1431216000000),                # :820-823
])
def test_previous_interval_weeks_known_answers(ts, n, want):
    assert prev(ts, n) == want


@pytest.mark.parametrize("n", [3, 4, 5, 13, 52])
def test_wide_week_intervals_start_on_the_sunday_of_the_week(n):
    """Every day of 2015-2016 (incl. the first days of January, whose week starts in the old
    year): the result is the Sunday 00:00 UTC on or before ts."""
    for day in range(16436, 16436 + 731, 3):
        ts = day * 86400000 + 12345678
        sunday = day - ((day - 3) % 7)
        assert prev(ts, n) == sunday * 86400000, (day, n)
