"""CPU-side checks of the product: libtsdbhip loads and exports every symbol of
include/tsdbhip.h, and its host-logic helpers (no HIP calls) agree with the oracle and
the reference known answers."""
from __future__ import annotations

import ctypes as C
import os
import re

import numpy as np
import pytest

from opentsdb_amd import abi, engine, synth
from oracle import oracle as O
from tests import golden_util as G

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    src = open(os.path.join(ROOT, "include", "tsdbhip.h")).read()
    return sorted(set(re.findall(r"\b(tsdbhip_[a-z_]+)\s*\(", src)))


def test_library_exports_every_header_symbol():
    L = engine.lib()
    syms = header_symbols()
    assert syms == sorted(engine.EXPORTS)
    for s in syms:
        assert hasattr(L, s), s


def test_abi_version():
    assert engine.lib().tsdbhip_abi_version() == 12


def test_multi_device_context_argument_checks():
    """tsdbhip_init_devices validates its arguments before touching a device; without a GPU the
    context is refused with an error, never a crash."""
    import ctypes as C
    L = engine.lib()
    out = C.c_void_p()
    devs = (C.c_int * 2)(0, 0)
    assert L.tsdbhip_init_devices(None, 2, -1, C.byref(out)) == abi.TSDB_E_ILLEGAL_ARGUMENT
    assert L.tsdbhip_init_devices(devs, 0, -1, C.byref(out)) == abi.TSDB_E_ILLEGAL_ARGUMENT
    assert L.tsdbhip_init_devices(devs, 2, 7, C.byref(out)) == abi.TSDB_E_ILLEGAL_ARGUMENT
    assert L.tsdbhip_md_shard_mode(None, 0) == abi.TSDB_E_ILLEGAL_ARGUMENT
    if not os.path.exists("/dev/kfd"):
        with pytest.raises(engine.EngineError):
            engine.Engine(devices=[0, 0])
    assert abi.Timing.exchange_ms.offset == abi.Timing.fused_queries.offset + 8


@pytest.mark.parametrize("name", abi.AGGREGATOR_NAMES)
def test_aggregator_registry(name):
    L = engine.lib()
    assert L.tsdbhip_aggregator_get(name.encode()) == abi.AGG[name]
    assert L.tsdbhip_aggregator_interpolation(abi.AGG[name]) == abi.interpolation_of(abi.AGG[name])


def test_aggregator_unknown():
    assert engine.lib().tsdbhip_aggregator_get(b"nope") == abi.TSDB_E_NO_SUCH_ELEMENT


@pytest.mark.parametrize("spec", ["1m-avg", "1000s-avg", "10s-sum", "100ms-sum-nan", "1m-sum-zero", "0all-sum",
                                  "1h-p99", "1dc-sum", "30000ms-min-null", "1w-count", "2n-max", "1y-dev"])
def test_parse_downsample_matches_oracle(spec):
    a = engine.parse_downsample(spec)
    b = O.parse_downsample(spec)
    for f in ("ds_function", "ds_fill", "ds_all", "ds_calendar", "ds_interval_ms"):
        assert getattr(a, f) == getattr(b, f), f


@pytest.mark.parametrize("spec", ["1m", "1m-foo", "1m-none", "0m-sum", "1m-sum-bogus", "1x-sum", "1m-sum-nan-x"])
def test_parse_downsample_errors(spec):
    with pytest.raises(engine.EngineError) as ei:
        engine.parse_downsample(spec)
    assert ei.value.java == "IllegalArgumentException"


@pytest.mark.parametrize("case", G.load("scan_bounds.json")["cases"], ids=lambda c: c["ref"])
def test_scan_bounds_known_answers(case):
    q = abi.new_query(case["start"], case["end"], "sum", ds_function=abi.AGG["sum"], ds_interval_ms=case["interval"])
    assert engine.scan_bounds(q) == (case["scan_start"], case["scan_end"])


def test_scan_bounds_no_downsample():
    q = abi.new_query(1356998400, 1357041600, "sum")
    assert engine.scan_bounds(q) == O.scan_bounds(q) == (1356998400, 1357045200)


def test_host_synth_is_mockbase_encoding():
    """The synthetic generator produces exactly what MockStore (addPoint + compaction) produces."""
    from opentsdb_amd.store import MockStore
    b = synth.generate(4, 1356998400, 400, 10000, value_kind=2, n_groups=2, int_mod=30000)
    order, grp = synth.series_order(4, 2)
    st = MockStore()
    ks = np.arange(400)
    for i in order:
        is_int, v = synth.values(0x5EED, int(i), ks, 2, 30000)
        for k in range(400):
            ts = 1356998400 + 10 * k
            if is_int:
                st.add_long("m", ts, int(v[k]), {"id": f"s{i:03d}"})
            else:
                st.add_float("m", ts, float(v[k]), {"id": f"s{i:03d}"})
    spans = st.scan("m", 0, 1 << 31)
    by_id = {dict(sk[1])[1]: rows for sk, rows in spans}  # tagk uid 1 -> tagv uid
    # tag value uids follow insertion order of series in `order`
    for pos, i in enumerate(order):
        rows = spans[pos][1] if False else list(by_id.values())[pos]
        for r, (base, q, v) in enumerate(rows):
            row = b.series_row_ptr[pos] + r
            assert base == b.row_base_time[row]
            assert q == bytes(b.qual[b.row_qual_off[row]:b.row_qual_off[row + 1]])
            assert v == bytes(b.val[b.row_val_off[row]:b.row_val_off[row + 1]])


def test_calendar_spec_units_match_oracle():
    """tsdbhip_parse_downsample records the calendar unit of a 'c' interval like the oracle
    (DownsamplingSpecification :140-147 + DateTime.unitsToCalendarType :616-640)."""
    from opentsdb_amd import engine
    from oracle import oracle as O
    for spec in ["1wc-sum", "1dc-avg-nan", "2nc-max", "1yc-sum", "500msc-sum", "30sc-avg", "15mc-min", "6hc-count",
                 "1m-sum", "0all-sum"]:
        a, b = engine.parse_downsample(spec), O.parse_downsample(spec)
        assert (a.ds_calendar, a.ds_interval_ms, a.ds_fill, a.ds_all) == (b.ds_calendar, b.ds_interval_ms, b.ds_fill,
                                                                          b.ds_all), spec


def test_pinned_copy_keeps_its_block_alive(monkeypatch):
    """pinned_copy's arrays (and any view numpy collapses to their base) own the page-locked
    block: it is freed only after the last array over it is gone (a use-after-free here crashed
    an upload from pinned memory)."""
    import ctypes as C
    import gc
    freed, keep = [], {}

    class FakeLib:
        def tsdbhip_host_alloc(self, n, pp):
            buf = C.create_string_buffer(n)
            keep[C.addressof(buf)] = buf
            C.cast(pp, C.POINTER(C.c_void_p))[0] = C.addressof(buf)
            return 0

        def tsdbhip_host_free(self, p):
            freed.append(p)

    fake = FakeLib()
    monkeypatch.setattr(engine, "_lib", fake)
    monkeypatch.setattr(engine, "lib", lambda: fake)
    y = engine.pinned_copy(np.arange(10, dtype=np.int64))
    v = np.ascontiguousarray(y, dtype=np.int64)[2:]
    del y
    gc.collect()
    assert freed == [] and int(v.sum()) == 44
    del v
    gc.collect()
    assert len(freed) == 1
