"""Query-time compaction on the CPU: the oracle's restatement of
CompactionQueue.Compaction / ColumnDatapointIterator / AppendDataPoints pinned by every
TestCompactionQueue known answer of the query path (tests/golden/compaction.json,
transcribed by tests/golden/make_compaction_golden.py)."""
import importlib.util
import os
import struct

import pytest

from oracle import oracle as O
from tests import golden_util as gu

DOC = gu.load("compaction.json")
_spec = importlib.util.spec_from_file_location(
    "make_compaction_golden", os.path.join(gu.GOLDEN, "make_compaction_golden.py"))
MK = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(MK)
CASES = {c["name"]: c for c in DOC["cases"]}


@pytest.mark.parametrize("name", sorted(CASES))
def test_oracle_compaction_known_answers(name):
    case = CASES[name]
    cols, expect = MK.expand_columns(case)
    kw = dict(timestamps=case.get("timestamps"), use_otsdb_timestamp=case.get("use_otsdb_timestamp", False))
    if expect == "IllegalDataException":
        with pytest.raises(O.OracleError) as e:
            O.compact_row(cols, case["fix_duplicates"], **kw)
        assert e.value.code == -2
        return
    for use_max in (True, False) if kw["use_otsdb_timestamp"] else (True,):
        got = O.compact_row(cols, case["fix_duplicates"], use_max_value=use_max, **kw)
        if expect is None:
            assert got is None
            continue
        assert got is not None
        assert got[0].hex() == expect[0].hex()
        assert got[1].hex() == expect[1].hex()


def test_every_test_method_transcribed():
    src = "/root/reference/test/core/TestCompactionQueue.java"
    if not os.path.exists(src):
        pytest.skip("reference absent")
    import re
    names = set(re.findall(r"public void (\w+)\(\) throws", open(src).read())) - {"before"}
    missing = names - set(CASES)
    assert not missing, missing


def test_newest_column_wins_regardless_of_position():
    q, v1, v2 = bytes([0, 0x07]), (1).to_bytes(8, "big"), (2).to_bytes(8, "big")
    assert O.compact_row([(q, v1), (q + bytes([0, 0x17]), v2 + v2 + b"\0")], True, [5, 3]) == \
        (q + bytes([0, 0x17]), v1 + v2 + b"\0")
    assert O.compact_row([(q, v1), (q + bytes([0, 0x17]), v2 + v2 + b"\0")], True, [3, 5]) == \
        (q + bytes([0, 0x17]), v2 + v2 + b"\0")


# ---- dtcsMergeDataPoints (tsd.storage.use_otsdb_timestamp, CompactionQueue.java:508-547) ----
# Hand-worked answers of the reference's loop (no reference test covers a repeated offset under
# this merge; useMaxTsWhileCompacting repeats none).

def _sq(sec, fl):
    return (sec << 4 | fl).to_bytes(2, "big")


def _mq(ms, fl):
    return (0xF0000000 | ms << 6 | fl).to_bytes(4, "big")


def test_dtcs_keeps_max_or_min_without_duplicate_exception():
    cols = [(_sq(1, 0), b"\x03"), (_sq(1, 0), b"\x07"), (_sq(2, 0), b"\x01")]
    ts = [5, 3, 1]
    q = _sq(1, 0) + _sq(2, 0)
    # default merge: the newest column's 3 is kept, the different 7 raises without fix_duplicates
    assert O.compact_row(cols, True, ts) == (q, b"\x03\x01\x00")
    with pytest.raises(O.OracleError):
        O.compact_row(cols, False, ts)
    assert O.compact_row(cols, False, ts, use_otsdb_timestamp=True) == (q, b"\x07\x01\x00")
    assert O.compact_row(cols, False, ts, use_otsdb_timestamp=True, use_max_value=False) == (q, b"\x03\x01\x00")


def test_dtcs_tie_keeps_heap_head_and_compares_as_double():
    # 1-byte int 5 (older column) vs float 5.0 (newer): equal as doubles, the newer column's kept
    f5 = struct.pack(">f", 5.0)
    cols = [(_sq(1, 0), b"\x05"), (_sq(1, 0xB), f5)]
    assert O.compact_row(cols, True, [1, 2], use_otsdb_timestamp=True) == (_sq(1, 0xB), f5)
    assert O.compact_row(cols, True, [2, 1], use_otsdb_timestamp=True) == (_sq(1, 0), b"\x05")


def test_dtcs_nan_head_is_never_replaced():
    nan = struct.pack(">f", float("nan"))
    big = struct.pack(">f", 1e30)
    cols = [(_sq(1, 0xB), nan), (_sq(1, 0xB), big), (_sq(2, 0), b"\x01")]
    assert O.compact_row(cols, True, [9, 1, 0], use_otsdb_timestamp=True) == (_sq(1, 0xB) + _sq(2, 0), nan + b"\x01\x00")
    # a NaN further down the heap never wins either
    assert O.compact_row(cols, True, [1, 9, 0], use_otsdb_timestamp=True) == (_sq(1, 0xB) + _sq(2, 0), big + b"\x01\x00")


def test_dtcs_meta_byte_reads_the_advanced_column():
    # A = [s@0, ms@500] (newest), B = s@0.  Under the min rule A's 5 is kept at offset 0 and A has
    # advanced to its ms datapoint when isMilliseconds() is read: the row is never seen "in
    # seconds", so no MS_MIXED_COMPACT bit, where the default merge sets it.
    A = (_sq(0, 0) + _mq(500, 0), b"\x05\x06\x01")
    B = (_sq(0, 0), b"\x09")
    q = _sq(0, 0) + _mq(500, 0)
    assert O.compact_row([A, B], True, [10, 1]) == (q, b"\x05\x06\x01")
    assert O.compact_row([A, B], True, [10, 1], use_otsdb_timestamp=True, use_max_value=False) == (q, b"\x05\x06\x00")
    # max rule: B's 9 wins; B (single datapoint) stays "in seconds", A's ms point sets ms: mixed
    assert O.compact_row([A, B], True, [10, 1], use_otsdb_timestamp=True) == (q, b"\x09\x06\x01")


def test_dtcs_unreadable_value_is_a_runtime_exception():
    cols = [(_sq(1, 2), b"\x00\x01\x02"), (_sq(2, 0), b"\x01")]   # a 3-byte integer in a merged row
    with pytest.raises(O.OracleError) as e:
        O.compact_row(cols, True, [1, 2], use_otsdb_timestamp=True)
    assert e.value.code == -6
    # the default merge copies it (the decode raises later); a single column is kept as stored
    assert O.compact_row(cols, True, [1, 2]) is not None
    assert O.compact_row(cols[:1], True, [1], use_otsdb_timestamp=True) == cols[0]
