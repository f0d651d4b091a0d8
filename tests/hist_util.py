"""Helpers of the histogram-path tests: fixture stores, random stores,
and the comparison of two query results (lists of HistogramDataPoints per group)."""
from __future__ import annotations

import json
import math
import os
import struct

import numpy as np

from opentsdb_amd import abi
from opentsdb_amd import histogram as H

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "histogram.json")


def golden():
    with open(GOLDEN) as f:
        return json.load(f)


def store_batch(st) -> H.HostHistBatch:
    series = [[(base, [(bytes.fromhex(q), bytes.fromhex(v)) for q, v in cols]) for base, cols in rows]
              for rows in st["series"]]
    return H.HostHistBatch.from_rows(series, st["groups"], {int(k): v for k, v in st["codecs"].items()})


def golden_query(gq) -> abi.Query:
    ds = gq["downsample"]
    q = abi.new_query(gq["start"], gq["end"], gq["aggregator"])
    if ds:
        from opentsdb_amd import engine as E
        d = E.parse_downsample(ds)
        q.ds_function, q.ds_interval_ms, q.ds_all, q.ds_calendar, q.ds_fill = (d.ds_function, d.ds_interval_ms,
                                                                               d.ds_all, d.ds_calendar, d.ds_fill)
    return q


def check_golden(got, gq):
    """got: list (per group) of HistogramDataPoints lists; gq: a fixture query."""
    exp = gq["expect"]
    assert len(got) == len(exp), (gq["name"], len(got), len(exp))
    tol = gq.get("tol", 0.0)
    for g_got, g_exp in zip(got, exp):
        assert g_got and g_got[0].group_id == g_exp["group"] or not g_got, gq["name"]
        if gq.get("partial_buckets"):
            by_key = {tuple(s.bucket): s for s in g_got if s.bucket is not None}
            for se in g_exp["series"]:
                s = by_key[tuple(se["bucket"])]
                assert list(s.ts) == se["ts"] and list(s.values) == se["values"], (gq["name"], se, s.values)
            continue
        assert len(g_got) == len(g_exp["series"]), gq["name"]
        for s, se in zip(g_got, g_exp["series"]):
            assert list(s.ts) == se["ts"], (gq["name"], list(s.ts)[:5], se["ts"][:5])
            if "percentile" in se:
                assert abs(s.percentile - se["percentile"]) < 1e-6
                np.testing.assert_allclose(s.values, np.array(se["values"], np.float64), rtol=0, atol=tol,
                                           err_msg=gq["name"])
            else:
                assert tuple(s.bucket) == tuple(se["bucket"]) and list(s.values) == se["values"], gq["name"]


def same(a, b, what=""):
    """Bit-exact equality of two query results (NaN == NaN)."""
    assert len(a) == len(b), (what, len(a), len(b))
    for ga, gb in zip(a, b):
        assert len(ga) == len(gb), (what, "series", len(ga), len(gb))
        for sa, sb in zip(ga, gb):
            assert sa.group_id == sb.group_id, (what, sa.group_id, sb.group_id)
            assert (sa.percentile is None) == (sb.percentile is None)
            if sa.percentile is not None:
                assert sa.percentile == sb.percentile
            assert sa.bucket == sb.bucket or (sa.bucket and sb.bucket and tuple(sa.bucket) == tuple(sb.bucket)), \
                (what, sa.bucket, sb.bucket)
            assert np.array_equal(sa.ts, sb.ts), (what, sa.group_id, sa.ts[:8], sb.ts[:8])
            va, vb = np.asarray(sa.values), np.asarray(sb.values)
            if va.dtype.kind == "f":
                ok = (va.view(np.uint64) == vb.view(np.uint64)) | (np.isnan(va) & np.isnan(vb))
                assert ok.all(), (what, sa.group_id, sa.percentile, va[~ok][:4], vb[~ok][:4])
            else:
                assert np.array_equal(va, vb), (what, sa.group_id, sa.bucket, va[:8], vb[:8])


# ---- random stores ------------------------------------------------------------------------
def random_layout(rng, nb, wild=False):
    """nb (lower, upper) float32 pairs; wild: negative, zero, -0.0, inf, NaN bounds."""
    if not wild:
        edges = np.cumsum(rng.uniform(0.5, 20.0, nb + 1)).astype(np.float32)
        return [(float(edges[i]), float(edges[i + 1])) for i in range(nb)]
    pool = [0.0, -0.0, 1.0, -1.0, 2.5, -7.25, 100.0, float("inf"), float("-inf"), float("nan"), 1e-30, 3.0e9]
    out = []
    for _ in range(nb):
        out.append((float(rng.choice(pool)) if rng.random() < 0.5 else float(np.float32(rng.normal(0, 50))),
                    float(rng.choice(pool)) if rng.random() < 0.5 else float(np.float32(rng.normal(0, 50)))))
    return out


def encode_simple(cid, buckets, under, over) -> bytes:
    b = bytes([cid]) + struct.pack(">h", len(buckets))
    for (lo, up), c in buckets:
        b += struct.pack(">ff", lo, up) + H.kryo_varlong(int(c))
    return b + H.kryo_varlong(int(under)) + H.kryo_varlong(int(over))


def random_store(rng, n_series=6, n_rows=3, period_ms=10000, t0=1356998400, groups=2, layouts=3, nb=(3, 12),
                 wild=False, long_frac=0.0, bad_frac=0.0, ms_frac=0.3, sparse=0.2, big_counts=False, codec_id=3):
    """Series of SimpleHistogram (codec_id) / long (codec_id + 1) columns; returns (HostHistBatch, info)."""
    lays = [random_layout(rng, int(rng.integers(nb[0], nb[1] + 1)), wild) for _ in range(layouts)]
    codecs = {codec_id: H.HCODEC_SIMPLE, codec_id + 1: H.HCODEC_LONG}
    series = []
    for s in range(n_series):
        rows = []
        lay = lays[s % layouts]
        use_long = rng.random() < long_frac
        for r in range(n_rows):
            base = t0 + 3600 * r
            cols = []
            ms = rng.random() < ms_frac
            step = period_ms if not ms else max(1, period_ms // 7)
            for off in range(0, 3600 * 1000, step):
                if rng.random() < sparse:
                    continue
                if ms:
                    q = bytes([6]) + struct.pack(">I", off)
                else:
                    if off % 1000:
                        continue
                    q = bytes([6]) + struct.pack(">H", off // 1000)
                if use_long:
                    v = bytes([codec_id + 1]) + struct.pack(">q", int(rng.integers(-1000, 100000)))
                else:
                    hi = (1 << 40) if big_counts else 1000
                    cnt = rng.integers(0, hi, len(lay))
                    if big_counts:
                        cnt[rng.random(len(lay)) < 0.1] = -int(rng.integers(1, 1 << 50))
                    bl = list(zip(lay, cnt))
                    if rng.random() < 0.2 and len(bl) > 1:   # a column with a subset of the layout
                        bl = [bl[i] for i in sorted(rng.choice(len(bl), len(bl) // 2 + 1, replace=False))]
                    v = encode_simple(codec_id, bl, rng.integers(0, 50), rng.integers(0, 50))
                if rng.random() < bad_frac:
                    kind = rng.integers(0, 4)
                    if kind == 0:
                        v = v[: max(0, len(v) - int(rng.integers(1, 6)))]   # truncated: dropped
                    elif kind == 1:
                        v = bytes([200]) + v[1:]                            # no codec with that id
                    elif kind == 2:
                        q = q[:2]                                           # invalid qualifier length
                    else:
                        v = b""
                cols.append((q, v))
            rows.append((base, cols))
        series.append(rows)
    gids = [s % groups for s in range(n_series)]
    return H.HostHistBatch.from_rows(series, gids, codecs)


def query(t0, t1, agg="sum", ds=None, tz=None):
    q = abi.new_query(t0, t1, agg)
    if ds:
        from opentsdb_amd import engine as E
        d = E.parse_downsample(ds)
        q.ds_function, q.ds_interval_ms, q.ds_all, q.ds_calendar, q.ds_fill = (d.ds_function, d.ds_interval_ms,
                                                                               d.ds_all, d.ds_calendar, d.ds_fill)
    return q


def isclose_or_nan(a, b):
    return (math.isnan(a) and math.isnan(b)) or a == b
