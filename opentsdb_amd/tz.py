"""Time-zone transition tables for calendar downsampling (tsdbhip_tz, include/tsdbhip.h).

The reference aligns 'c' intervals with java.util.GregorianCalendar in the zone the query
names (DownsamplingSpecification.setTimezone, src/core/DownsamplingSpecification.java:199-207;
DateTime.previousInterval, src/utils/DateTime.java:445-606).  The engine takes the zone as a
table of UTC offset transitions built by the host from its own time-zone database -- a JVM host
from ZoneRules, this Python host from the IANA data bundled with pytz -- and reproduces the
Calendar arithmetic over it (engine.cpp jcal_*).  pytz tables end in 2037 for zones with
daylight saving time (the last offset then holds)."""
from __future__ import annotations

import ctypes as C
import datetime as dt
import functools

import numpy as np

from . import abi

_EPOCH = dt.datetime(1970, 1, 1)


class TzTable:
    """A tsdbhip_tz and the arrays behind it."""

    def __init__(self, name: str, utc_ms, offset_ms):
        self.name = name
        self.utc_ms = np.ascontiguousarray(utc_ms, np.int64)
        self.offset_ms = np.ascontiguousarray(offset_ms, np.int32)
        assert len(self.offset_ms) == len(self.utc_ms) + 1
        st = abi.TZ()
        st.n = len(self.utc_ms)
        st.utc_ms = self.utc_ms.ctypes.data_as(C.POINTER(C.c_int64))
        st.offset_ms = self.offset_ms.ctypes.data_as(C.POINTER(C.c_int32))
        st._keep = (self.utc_ms, self.offset_ms)   # the arrays live as long as the struct
        self.struct = st

    def offset_at(self, t_ms: int) -> int:
        """Total offset (ms) in effect at UTC instant t_ms."""
        i = int(np.searchsorted(self.utc_ms, t_ms, side="right"))
        return int(self.offset_ms[i])


def _ms(td: dt.timedelta) -> int:
    return int(round(td.total_seconds() * 1000))


@functools.lru_cache(maxsize=64)
def table(name: str) -> TzTable:
    """The transition table of an IANA zone id (pytz); "UTC" / "GMT" -> no transitions."""
    import pytz
    z = pytz.timezone(name)
    times = getattr(z, "_utc_transition_times", None)
    if not times:
        off = z.utcoffset(dt.datetime(2000, 1, 1))
        return TzTable(name, [], [_ms(off)])
    info = z._transition_info
    utc, offs = [], [_ms(info[0][0])]
    for t, (off, _dst, _name) in list(zip(times, info))[1:]:
        utc.append(int((t - _EPOCH).total_seconds() * 1000))
        offs.append(_ms(off))
    return TzTable(name, utc, offs)


def fixed(name: str, offset_ms: int) -> TzTable:
    """A zone with one constant offset (e.g. Java's "EST" = -05:00)."""
    return TzTable(name, [], [offset_ms])
