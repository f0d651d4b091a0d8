"""Writes tests/golden/calendar.json: the reference's UTC calendar-downsampling known answers
(test/core/TestDownsampler.java), transcribed by hand.  Each case is a Downsampler over a
fixed data point array (SeekableViewsForTest.fromArray), a spec with the 'c' suffix, an
optional seek, and the expected (timestamp, value) sequence.  The reference's test loops
compute some expected timestamps with java.util.Calendar arithmetic; those are written out
here with Python's proleptic Gregorian calendar in UTC (what the UTC Calendar computes).

The timezone variants (America/Denver, Pacific/Funafuti, Pacific/Fiji, Asia/Kabul, EST) follow,
each with its zone id ("tz"); FillingDownsampler cases (test/core/TestFillingDownsampler.java)
carry the ctor's start / end ("fill": [start, end]).  Where the reference's loop runs on until
the source or the fill range ends, the expected sequence below is the one that loop accepts,
counted by hand from the points and the zone's offsets (noted per case)."""
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


def case(name, src, points, spec, expect, seek=None, tz=None, fill=None):
    cases.append({"name": name, "source": src, "points": long_pts(points), "spec": spec, "seek": seek,
                  "tz": tz, "fill": fill,
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

# ---- time zones (TestDownsampler.java:389-711, 870-1172; TestFillingDownsampler.java:271-590) ----
NAN = float("nan")
HOUR = 3600000
TV, AF, FJ, EST = "Pacific/Funafuti", "Asia/Kabul", "Pacific/Fiji", "EST"
hour_pts = [(BASE_TIME, 1), (BASE_TIME + 1800000, 2), (BASE_TIME + 3599000, 3), (BASE_TIME + 3600000, 4),
            (BASE_TIME + 5400000, 5), (BASE_TIME + 7199000, 6)]
day_pts = [(DST_TS, 1), (DST_TS + 86399000, 2), (DST_TS + 126001000, 3), (DST_TS + 172799000, 4),
           (DST_TS + 172800000, 5), (DST_TS + 242999000, 6)]
week_pts = [(DST_TS, 1), (DST_TS + 7 * DAY, 2), (1451129400000, 3), (DST_TS + 21 * DAY, 4), (1452367799000, 5)]
month_pts = [(1448928000000, 1), (1451559600000, 2), (1451606400000, 3), (1454284800000, 4), (1456704000000, 5),
             (1456772400000, 6)]
TD = "test/core/TestDownsampler.java"
TF = "test/core/TestFillingDownsampler.java"

# testDownsampler_calendar :389-415 (America/Denver)
case("TestDownsampler.calendar_Denver", TD + ":389-415",
     [(BASE_TIME + 5000 + 10000 * i, 1 << i) for i in range(6)], "1dc-sum", [(1356937200000, 63)],
     tz="America/Denver")
# testDownsampler_calendarHour :417-477
case("TestDownsampler.calendarHour_TV", TD + ":417-441", hour_pts, "1hc-sum",
     [(BASE_TIME, 6), (BASE_TIME + HOUR, 15)], tz=TV)
case("TestDownsampler.calendarHour_AF", TD + ":443-461", hour_pts, "1hc-sum",
     [(1356996600000, 1), (1356996600000 + HOUR, 9), (1356996600000 + 2 * HOUR, 11)], tz=AF)
case("TestDownsampler.calendarHour_AF_4h", TD + ":463-476", hour_pts, "4hc-sum", [(1356996600000, 21)], tz=AF)
# testDownsampler_calendarDay :479-590
case("TestDownsampler.calendarDay_TV", TD + ":508-528", day_pts, "1dc-sum",
     [(1450094400000 + i * DAY, v) for i, v in enumerate([1, 5, 9, 6])], tz=TV)
case("TestDownsampler.calendarDay_FJ", TD + ":530-550", day_pts, "1dc-sum",
     [(1450090800000 + i * DAY, v) for i, v in enumerate([1, 2, 12, 6])], tz=FJ)
case("TestDownsampler.calendarDay_AF", TD + ":552-570", day_pts, "1dc-sum",
     [(1450121400000 + i * DAY, v) for i, v in enumerate([1, 5, 15])], tz=AF)
case("TestDownsampler.calendarDay_AF_3d", TD + ":572-589", day_pts, "3dc-sum", [(1450121400000, 21)], tz=AF)
# testDownsampler_calendarWeek :592-709
case("TestDownsampler.calendarWeek_TV", TD + ":624-647", week_pts, "1wc-sum",
     [(1449921600000, 1), (1450526400000, 5), (1451736000000, 4), (1452340800000, 5)], tz=TV)
case("TestDownsampler.calendarWeek_FJ", TD + ":649-664", week_pts, "1wc-sum",
     [(1449918000000 + i * 7 * DAY, i + 1) for i in range(5)], tz=FJ)
case("TestDownsampler.calendarWeek_AF", TD + ":666-689", week_pts, "1wc-sum",
     [(1449948600000, 1), (1450553400000, 5), (1451763000000, 9)], tz=AF)
case("TestDownsampler.calendarWeek_AF_2w", TD + ":691-708", week_pts, "2wc-sum",
     [(1449948600000, 6), (1451158200000, 9)], tz=AF)
# testDownsampler_calendarMonth :711-827 (the FJ loop pins timestamps only; its values, 1 5 9 6,
# are the ones the loop computes)
case("TestDownsampler.calendarMonth_TV", TD + ":740-764", month_pts, "1nc-sum",
     [(1448884800000, 3), (1451563200000, 3), (1454241600000, 9), (1456747200000, 6)], tz=TV)
case("TestDownsampler.calendarMonth_FJ", TD + ":766-789", month_pts, "1nc-sum",
     [(1448881200000, 1), (1451559600000, 5), (1454241600000, 9), (1456747200000, 6)], tz=FJ)
case("TestDownsampler.calendarMonth_AF", TD + ":791-810", month_pts, "1nc-sum",
     [(1448911800000, 3), (1451590200000, 3), (1454268600000, 15)], tz=AF)
case("TestDownsampler.calendarMonth_TV_3n", TD + ":812-826", month_pts, "3nc-sum",
     [(1443614400000, 3), (1451563200000, 18)], tz=TV)
# testDownsampler_1day_timezone :870-894, 1week_timezone :920-943 (EST = -05:00)
case("TestDownsampler.1day_timezone", TD + ":870-894",
     [(1357016400000, 1), (1357059600000, 2), (1357102800000, 4), (1357146000000, 8)], "1dc-sum",
     [(1357016400000, 3), (1357102800000, 12)], tz=EST)
case("TestDownsampler.1week_timezone", TD + ":920-943",
     [(1356843600000, 1), (1357146000000, 2), (1357448400000, 4), (1357750800000, 8)], "1wc-sum",
     [(1356843600000, 3), (1357448400000, 12)], tz=EST)


def est_month(y, m):   # the first instant of a month in EST (-05:00)
    return ms(y, m) + 5 * HOUR


# testDownsampler_1month_timezone :1071-1105: two points a month (month start, mid-month) in EST
pts, bk = [], []
for i in range(12):
    a, b = est_month(2013 + i // 12, i % 12 + 1), est_month(2013 + (i + 1) // 12, (i + 1) % 12 + 1)
    pts += [(a, 1 << (2 * i)), (a + (b - a) // 2, 1 << (2 * i + 1))]
    bk.append((a, (1 << (2 * i)) + (1 << (2 * i + 1))))
case("TestDownsampler.1month_timezone", TD + ":1071-1105", pts, "1nc-sum", bk, tz=EST)
# testDownsampler_1year_timezone :1142-1177
y0, y1, y2 = est_month(2013, 1), est_month(2014, 1), est_month(2015, 1)
case("TestDownsampler.1year_timezone", TD + ":1142-1177",
     [(y0, 1), (y0 + (y1 - y0) // 2, 2), (y1, 4), (y1 + (y2 - y1) // 2, 8)], "1yc-sum", [(y0, 3), (y1, 12)], tz=EST)

# FillingDownsampler (fill nan): bucket counts from the ctor's previousInterval(start) ..
# previousInterval(end) in the zone
case("TestFillingDownsampler.calendarHour_TV", TF + ":291-315", hour_pts, "1hc-sum-nan",
     [(BASE_TIME, 6), (BASE_TIME + HOUR, 15), (BASE_TIME + 2 * HOUR, NAN)], tz=TV,
     fill=[BASE_TIME, BASE_TIME + 3 * HOUR])
case("TestFillingDownsampler.calendarHour_AF", TF + ":317-339", hour_pts, "1hc-sum-nan",
     [(1356996600000 + i * HOUR, v) for i, v in enumerate([1, 9, 11, NAN])], tz=AF,
     fill=[1356996600000, 1356996600000 + 4 * HOUR])
case("TestFillingDownsampler.calendarHour_AF_4h", TF + ":341-357", hour_pts, "4hc-sum-nan",
     [(1356996600000, 21), (1357011000000, NAN)], tz=AF, fill=[1356996600000, 1356996600000 + 8 * HOUR])
case("TestFillingDownsampler.calendarDay_TV", TF + ":392-418", day_pts, "1dc-sum-nan",
     [(1450094400000 - DAY + i * DAY, v) for i, v in enumerate([NAN, 1, 5, 9, 6, NAN])], tz=TV,
     fill=[1450094400000 - DAY, DST_TS + 5 * DAY])
case("TestFillingDownsampler.calendarDay_FJ", TF + ":420-444", day_pts, "1dc-sum-nan",
     [(1450090800000 + i * DAY, v) for i, v in enumerate([1, 2, 12, 6, NAN])], tz=FJ,
     fill=[1450094400000, DST_TS + 5 * DAY])
case("TestFillingDownsampler.calendarDay_AF", TF + ":446-468", day_pts, "1dc-sum-nan",
     [(1450121400000 + i * DAY, v) for i, v in enumerate([1, 5, 15, NAN])], tz=AF,
     fill=[1450121400000, DST_TS + 4 * DAY])
case("TestFillingDownsampler.calendarDay_AF_3d", TF + ":470-486", day_pts, "3dc-sum-nan",
     [(1450121400000, 21), (1450121400000 + 3 * DAY, NAN)], tz=AF, fill=[1450121400000, DST_TS + 6 * DAY])
case("TestFillingDownsampler.calendarWeek", TF + ":489-517", week_pts, "1wc-sum-nan",
     [(1449964800000 + i * 7 * DAY, v) for i, v in enumerate([1, 5, NAN, 9, NAN])],
     fill=[1449964800000, DST_TS + 35 * DAY])
case("TestFillingDownsampler.calendarWeek_TV", TF + ":519-543", week_pts, "1wc-sum-nan",
     [(1449921600000 + i * 7 * DAY, v) for i, v in enumerate([1, 5, NAN, 4, 5])], tz=TV,
     fill=[1449964800000, DST_TS + 35 * DAY])
case("TestFillingDownsampler.calendarWeek_FJ", TF + ":545-561", week_pts, "1wc-sum-nan",
     [(1449918000000 + i * 7 * DAY, i + 1) for i in range(5)], tz=FJ, fill=[1449964800000, DST_TS + 35 * DAY])
case("TestFillingDownsampler.calendarWeek_AF", TF + ":563-587", week_pts, "1wc-sum-nan",
     [(1449948600000 + i * 7 * DAY, v) for i, v in enumerate([1, 5, NAN, 9, NAN])], tz=AF,
     fill=[1449964800000, DST_TS + 35 * DAY])
case("TestFillingDownsampler.calendarWeek_AF_2w", TF + ":589-609", week_pts, "2wc-sum-nan",
     [(1449948600000, 6), (1449948600000 + 14 * DAY, 9), (1449948600000 + 28 * DAY, NAN)], tz=AF,
     fill=[1449964800000, DST_TS + 35 * DAY])

if __name__ == "__main__":
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "calendar.json")
    with open(out, "w") as f:
        json.dump({"source": "reference test/core/TestDownsampler.java, TestFillingDownsampler.java (calendar cases)",
                   "cases": cases}, f, indent=1)
    print(out, len(cases))
