"""Query-time compaction on the CPU: the oracle's restatement of
CompactionQueue.Compaction / ColumnDatapointIterator / AppendDataPoints pinned by every
TestCompactionQueue known answer of the query path (tests/golden/compaction.json,
transcribed by tests/golden/make_compaction_golden.py)."""
import importlib.util
import os

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
    if expect == "IllegalDataException":
        with pytest.raises(O.OracleError) as e:
            O.compact_row(cols, case["fix_duplicates"])
        assert e.value.code == -2
        return
    got = O.compact_row(cols, case["fix_duplicates"])
    if expect is None:
        assert got is None
        return
    assert got is not None
    assert got[0].hex() == expect[0].hex()
    assert got[1].hex() == expect[1].hex()


def test_every_test_method_transcribed():
    src = "/root/reference/test/core/TestCompactionQueue.java"
    if not os.path.exists(src):
        pytest.skip("reference absent")
    import re
    names = set(re.findall(r"public void (\w+)\(\) throws", open(src).read())) - {"before"}
    missing = names - set(CASES) - {"useMaxTsWhileCompacting"}   # the otsdb-timestamp merge, not the query path
    assert not missing, missing


def test_newest_column_wins_regardless_of_position():
    q, v1, v2 = bytes([0, 0x07]), (1).to_bytes(8, "big"), (2).to_bytes(8, "big")
    assert O.compact_row([(q, v1), (q + bytes([0, 0x17]), v2 + v2 + b"\0")], True, [5, 3]) == \
        (q + bytes([0, 0x17]), v1 + v2 + b"\0")
    assert O.compact_row([(q, v1), (q + bytes([0, 0x17]), v2 + v2 + b"\0")], True, [3, 5]) == \
        (q + bytes([0, 0x17]), v2 + v2 + b"\0")
