"""Writes tests/golden/calendar.json: the reference's UTC calendar-downsampling known answers
(test/core/TestDownsampler.java), transcribed by hand.  Each case is a Downsampler over a
fixed data point array (SeekableViewsForTest.fromArray), a spec with the 'c' suffix, an
optional seek, and the expected (timestamp, value) sequence.  The reference's test loops
compute some expected timestamps with java.util.Calendar arithmetic; those are written out
here with Python's proleptic Gregorian calendar in UTC (what the UTC Calendar computes).

Timezone variants of these tests (America/Denver, Pacific/Tuvalu, Pacific/Fiji,
Asia/Kabul, EST) are not transcribed: the engine aligns on UTC only."""
from __future__ import annotations

import calendar
import datetime as dt
import json
import os

DST_TS = 1450137600000          # TestDownsampler.java:69
BASE_TIME = 1356998400000       # TestDownsampler.java:40
DAY = 86400000


def ms(y, m, d=1):
    return calendar.timegm(dt.datetime(y, m, d).timetuple()) * 1000


def add_months(t, n):
    d = dt.datetime.utcfromtimestamp(t / 1000)
    k = d.year * 12 + d.month - 1 + n
    return ms(k // 12, k % 12 + 1, 1) + (t - ms(d.year, d.month, 1))


def long_pts(pairs):
    return [[int(t), True, int(v)] for t, v in pairs]


cases = []


def case(name, src, points, spec, expect, seek=None):
    cases.append({"name": name, "source": src, "points": long_pts(points), "spec": spec, "seek": seek,
                  "expect": [[int(t), False, float(v)] for t, v in expect]})


# testDownsampler_calendarDay control :480-507
case("TestDownsampler.calendarDay", "test/core/TestDownsampler.java:480-507",
     [(DST_TS, 1), (DST_TS + 86399000, 2), (DST_TS + 126001000, 3), (DST_TS + 172799000, 4),
      (DST_TS + 172800000, 5), (DST_TS + 242999000, 6)], "1dc-sum",
     [(DST_TS, 3), (DST_TS + DAY, 7), (DST_TS + 2 * DAY, 11)])

# testDownsampler_calendarWeek control :593-623 (weeks start on Sunday)
case("TestDownsampler.calendarWeek", "test/core/TestDownsampler.java:593-623",
     [(DST_TS, 1), (DST_TS + 7 * DAY, 2), (1451129400000, 3), (DST_TS + 21 * DAY, 4), (1452367799000, 5)],
     "1wc-sum", [(1449964800000, 1), (1450569600000, 5), (1451779200000, 9)])

# testDownsampler_calendarMonth control :712-738
case("TestDownsampler.calendarMonth", "test/core/TestDownsampler.java:712-738",
     [(1448928000000, 1), (1451559600000, 2), (1451606400000, 3), (1454284800000, 4), (1456704000000, 5),
      (1456772400000, 6)], "1nc-sum", [(1448928000000, 3), (1451606400000, 3), (1454284800000, 15)])

# testDownsampler_noDataCalendar :839-845
case("TestDownsampler.noDataCalendar", "test/core/TestDownsampler.java:839-845", [], "1mc-sum", [])

# testDownsampler_1week :897-917
case("TestDownsampler.1week", "test/core/TestDownsampler.java:897-917",
     [(1356825600000, 1), (1357128000000, 2), (1357430400000, 4), (1357732800000, 8)], "1wc-sum",
     [(1356825600000, 3), (1357430400000, 12)])

# testDownsampler_1month_alt :1022-1062 (1dc over month-start points at 04:00 / 05:00 UTC)
alt = [1380600000000, 1383278400000, 1385874000000, 1388552400000, 1391230800000, 1393650000000, 1396324800000,
       1398916800000, 1401595200000, 1404187200000, 1406865600000, 1409544000000]
t0 = ms(2013, 10)
case("TestDownsampler.1month_alt", "test/core/TestDownsampler.java:1022-1062", [(t, 1) for t in alt], "1dc-sum",
     [(add_months(t0, i), 1) for i in range(len(alt))])

# testDownsampler_2months :1064-1098: 24 points, two per month (month start, mid-month)
pts, t = [], ms(2013, 1)
for i in range(0, 24, 2):
    nxt = add_months(t, 1)
    pts += [(t, 1 << i), (t + (nxt - t) // 2, 1 << (i + 1))]
    t = nxt
case("TestDownsampler.2months", "test/core/TestDownsampler.java:1064-1098", pts, "2nc-sum",
     [(add_months(ms(2013, 1), 2 * j), sum(1 << (4 * j + k) for k in range(4))) for j in range(6)])

# testSeek_useCalendar :1345-1381 (second half: 1yc, seek 1 ms past a year start)
case("TestDownsampler.seek_useCalendar", "test/core/TestDownsampler.java:1370-1381",
     [(1356998400000, 1), (1388534400000, 2), (1420070400000, 4), (1451606400000, 8)], "1yc-sum",
     [(1451606400000, 8)], seek=1420070400001)
case("TestDownsampler.seek_useCalendar_yearstart", "test/core/TestDownsampler.java:1345-1368",
     [(1356998400000, 1), (1388534400000, 2), (1420070400000, 4), (1451606400000, 8)], "1yc-sum",
     [(1420070400000, 4), (1451606400000, 8)], seek=1420070400000)

if __name__ == "__main__":
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "calendar.json")
    with open(out, "w") as f:
        json.dump({"source": "reference test/core/TestDownsampler.java (UTC cases)", "cases": cases}, f, indent=1)
    print(out, len(cases))
