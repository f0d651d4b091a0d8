"""Transcribes the known answers of test/core/TestCompactionQueue.java (query-time
compaction) into tests/golden/compaction.json.

Each case is one row: its columns in the order the test adds them (qualifier and value bytes;
the column timestamp is the test's makekv sequence number, i.e. the position), the
fix_duplicates setting (the test class sets true; the "expected = IllegalDataException"
tests set false) and the compacted cell compactionq.compact() returns (qualifier, value),
null, or the exception class.  useMaxTsWhileCompacting (:108-131) sets
tsd.storage.use_otsdb_timestamp, whose merge (dtcsMergeDataPoints, CompactionQueue.java:508-547)
is on the query path too (SaltScanner.processRow -> TSDB.compact); its columns carry random
write timestamps (Math.abs(rnd.nextLong())), transcribed as three fixed ones -- the expected
cell does not depend on them, since no offset repeats.

    python tests/golden/make_compaction_golden.py
"""
from __future__ import annotations

import json
import os
import struct

SRC = "test/core/TestCompactionQueue.java"


def L(x):
    return struct.pack(">q", x)


def I(x):
    return struct.pack(">i", x)


def H(x):
    return struct.pack(">H", x)


ZERO, MIXED = b"\x00", b"\x01"
NOTE_Q = bytes([1, 0, 0])
NOTE = b'{"tsuid":"ABCD","description":"Description","notes":"Notes","custom":null,"endTime":1328140801,"startTime":1328140800}'
APPEND = bytes([0x05, 0x00, 0x00])


def F32(x):
    return struct.unpack(">I", struct.pack(">f", x))[0]


def cases():
    out = []

    def add(name, lines, cols, expect, fix=True, **extra):
        out.append({"name": name, "source": f"{SRC}:{lines}", "fix_duplicates": fix,
                    "columns": [[q.hex(), v.hex()] for q, v in cols],
                    "expect": expect if isinstance(expect, (str, type(None))) else
                    {"qualifier": expect[0].hex(), "value": expect[1].hex()}, **extra})

    q07, q17, q27, q37, q47, q57, q67 = (bytes([0, x]) for x in (0x07, 0x17, 0x27, 0x37, 0x47, 0x57, 0x67))
    m0, m1, m2 = (bytes([0xF0, 0, x, 0x07]) for x in (0x00, 0x01, 0x02))
    add("useMaxTsWhileCompacting", "108-131", [(m0, L(4)), (m1, L(5)), (m2, L(2))],
        (m0 + m1 + m2, L(4) + L(5) + L(2) + ZERO), use_otsdb_timestamp=True,
        timestamps=[6917529027641081857, 1234567890123456789, 4611686018427387905])
    add("emptyRow", "133-145", [], None)
    add("oneCellRow", "147-163", [(q07, L(42))], (q07, L(42)))
    add("oneCellAppend", "165-182", [(APPEND, q07 + L(42))], (q07, L(42)))
    add("oneCellRowWAnnotation", "184-202", [(NOTE_Q, NOTE), (q07, L(42))], (q07, L(42)))
    add("oneCellAppendWAnnotiation", "204-223", [(NOTE_Q, NOTE), (APPEND, q07 + L(42))], (q07, L(42)))
    add("oneCellRowWAnnotationMS", "225-243", [(bytes([1, 0, 0, 0, 0]), NOTE), (q07, L(42))], (q07, L(42)))
    add("oneCellRowBadLength", "245-261", [(bytes([0, 3]), L(42))], (q07, L(42)))
    add("oneCellRowMS", "263-279", [(m0, L(42))], (m0, L(42)))
    add("twoCellRow", "281-301", [(q07, L(4)), (q17, L(5))], (q07 + q17, L(4) + L(5) + ZERO))
    add("twoCellAppend", "303-322", [(APPEND, q07 + L(42) + q17 + L(5))], (q07 + q17, L(42) + L(5) + ZERO))
    add("twoCellRowWAnnotation", "324-346", [(NOTE_Q, NOTE), (q07, L(4)), (q17, L(5))],
        (q07 + q17, L(4) + L(5) + ZERO))
    add("twoCellAppendWAnnotations", "348-369", [(NOTE_Q, NOTE), (APPEND, q07 + L(42) + q17 + L(5))],
        (q07 + q17, L(42) + L(5) + ZERO))
    # the two loop-built rows are stored as their loops (expand_columns below)
    out.append({"name": "fullRowSeconds", "source": f"{SRC}:371-396", "fix_duplicates": True,
                "columns_loop": {"kind": "seconds", "start": 0, "stop": 3600, "step": 1}, "expect": "loop"})
    out.append({"name": "bigRowMs", "source": f"{SRC}:398-422", "fix_duplicates": True,
                "columns_loop": {"kind": "ms", "start": 0, "stop": 3599999, "step": 101}, "expect": "loop"})
    add("twoCellRowMS", "424-444", [(m0, L(4)), (m1, L(5))], (m0 + m1, L(4) + L(5) + ZERO))
    add("sortMsAndS", "446-472", [(q07, L(4)), (m2, L(5)), (m1, L(5))], (q07 + m1 + m2, L(4) + L(5) + L(5) + MIXED))
    add("secondsOutOfOrder", "474-500", [(bytes([2, 7]), L(4)), (q07, L(5)), (bytes([1, 7]), L(6))],
        (q07 + bytes([1, 7]) + bytes([2, 7]), L(5) + L(6) + L(4) + ZERO))
    add("msOutOfOrder", "502-529", [(m2, L(4)), (m0, L(5)), (m1, L(6))], (m0 + m1 + m2, L(5) + L(6) + L(4) + ZERO))
    add("secondAndMs", "531-552", [(q07, L(4)), (m1, L(5))], (q07 + m1, L(4) + L(5) + MIXED))
    add("secondAndMsWAnnotation", "554-577", [(NOTE_Q, NOTE), (q07, L(4)), (m1, L(5))],
        (q07 + m1, L(4) + L(5) + MIXED))
    add("msSameAsSecond", "579-592", [(q07, L(4)), (m0, L(5))], "IllegalDataException", fix=False)
    add("msSameAsSecondFix", "594-613", [(q07, L(4)), (m0, L(5))], (m0, L(5)))
    add("fixQualifierFlags", "615-638", [(bytes([0, 3]), L(4)), (q17, L(5))], (q07 + q17, L(4) + L(5) + ZERO))
    add("fixFloatingPoint", "640-665", [(q07, L(4)), (bytes([0, 0x1B]), L(F32(4.2)))],
        (q07 + bytes([0, 0x1B]), L(4) + I(F32(4.2)) + ZERO))
    add("overlappingDataPoints", "667-681", [(q07, L(4)), (bytes([0, 3]), I(4))], "IllegalDataException", fix=False)
    add("overlappingDataPointsFix", "683-703", [(q07, L(4)), (bytes([0, 3]), I(4))], (bytes([0, 3]), I(4)))
    add("failedCompactNoop", "705-730", [(q07, L(4)), (q17, L(5)), (q07 + q17, L(4) + L(5) + ZERO)],
        (q07 + q17, L(4) + L(5) + ZERO))
    add("annotationOnly", "732-746", [(NOTE_Q, NOTE)], None)
    add("annotationsOnly", "748-765", [(NOTE_Q, NOTE), (bytes([1, 0, 1]), NOTE)], None)
    add("secondCompact", "767-797", [(q07 + q27, L(4) + L(5) + ZERO), (q17, L(6))],
        (q07 + q17 + q27, L(4) + L(6) + L(5) + ZERO))
    add("secondCompactWAnnotation", "799-831", [(NOTE_Q, NOTE), (q07 + q27, L(4) + L(5) + ZERO), (q17, L(6))],
        (q07 + q17 + q27, L(4) + L(6) + L(5) + ZERO))
    add("secondCompactMS", "833-863", [(m0 + m2, L(4) + L(5) + ZERO), (m1, L(6))],
        (m0 + m1 + m2, L(4) + L(6) + L(5) + ZERO))
    mx = bytes([0xF0, 0x0A, 0x41, 0x07])
    add("secondCompactMixedSecond", "865-897", [(q07 + mx, L(4) + L(5) + MIXED), (q57, L(6))],
        (q07 + q57 + mx, L(4) + L(6) + L(5) + MIXED))
    add("secondCompactMixedMS", "899-931", [(q07 + mx, L(4) + L(5) + MIXED), (m1, L(6))],
        (q07 + m1 + mx, L(4) + L(6) + L(5) + MIXED))
    qf7 = bytes([0, 0xF7])
    add("secondCompactMixedMSAndS", "933-966", [(mx + qf7, L(4) + L(5) + MIXED), (q07, L(6))],
        (q07 + mx + qf7, L(6) + L(4) + L(5) + MIXED))
    add("secondCompactOverwrite", "968-989", [(q07 + q27, L(4) + L(5) + ZERO), (q07, L(6))], "IllegalDataException",
        fix=False)
    add("secondCompactOverwriteFix", "991-1022", [(q07 + q27, L(4) + L(5) + ZERO), (q07, L(6))],
        (q07 + q27, L(6) + L(5) + ZERO))
    add("doubleFailedCompactNoop", "1024-1062",
        [(q07, L(4)), (q07 + q17 + q27, L(4) + L(6) + L(5) + ZERO), (q07 + q27, L(4) + L(5) + ZERO), (q17, L(6)),
         (q27, L(5))], (q07 + q17 + q27, L(4) + L(6) + L(5) + ZERO))
    add("weirdOverlappingCompactedCells", "1064-1100",
        [(q07, L(4)), (q07 + q27, L(4) + L(5) + ZERO), (q07 + q17, L(4) + L(6) + ZERO), (q17, L(6)), (q27, L(5))],
        (q07 + q17 + q27, L(4) + L(6) + L(5) + ZERO))
    q3, q4, q5, q6 = bytes([0, 0x37]), bytes([0, 0x47]), bytes([0, 0x57]), bytes([0, 0x67])
    vals6 = L(4) + L(5) + L(6) + L(7) + L(8) + L(9)
    add("tripleCompacted", "1102-1143",
        [(q07 + q27, L(4) + L(5) + ZERO), (q3 + q4, L(6) + L(7) + ZERO), (q5 + q6, L(8) + L(9) + ZERO)],
        (q07 + q27 + q3 + q4 + q5 + q6, vals6 + ZERO))
    add("tripleCompactedOutOfOrder", "1145-1186",
        [(q07 + q27, L(4) + L(5) + ZERO), (q5 + q6, L(8) + L(9) + ZERO), (q3 + q4, L(6) + L(7) + ZERO)],
        (q07 + q27 + q3 + q4 + q5 + q6, vals6 + ZERO))
    a4, a5 = bytes([0xF0, 0x04, 0x65, 0x07]), bytes([0xF0, 0x05, 0x5F, 0x07])
    add("tripleCompactedSecondsAndMs", "1188-1231",
        [(m0 + q27, L(4) + L(5) + ZERO), (q3 + a4, L(6) + L(7) + ZERO), (a5 + q6, L(8) + L(9) + ZERO)],
        (m0 + q27 + q3 + a4 + a5 + q6, vals6 + MIXED))
    v1, v2, v3, v4, v5, v6 = L(42), L(5), L(3), L(2), L(1), L(0)
    four_q, four_v = q07 + q17 + q27 + q37, v1 + v2 + v3 + v4 + ZERO
    six_q, six_v = q07 + q17 + q27 + q37 + q47 + q57, v1 + v2 + v3 + v4 + v5 + v6 + ZERO
    add("appendsAndLaterPuts", "1233-1261", [(APPEND, q07 + v1 + q17 + v2), (q27, v3), (q37, v4)], (four_q, four_v))
    add("appendsAndEarlierPuts", "1262-1290", [(q07, v1), (q17, v2), (APPEND, q27 + v3 + q37 + v4)], (four_q, four_v))
    add("appendsAndInterspersedPuts", "1291-1319", [(q07, v1), (q27, v3), (APPEND, q17 + v2 + q37 + v4)],
        (four_q, four_v))
    add("doubleAppends", "1320-1348", [(APPEND, q07 + v1 + q17 + v2), (APPEND, q27 + v3 + q37 + v4)],
        (four_q, four_v))
    add("tripleAppends", "1349-1383",
        [(APPEND, q07 + v1 + q17 + v2), (APPEND, q27 + v3 + q37 + v4), (APPEND, q47 + v5 + q57 + v6)], (six_q, six_v))
    add("doubleAppendsAndPuts", "1384-1418",
        [(APPEND, q07 + v1 + q17 + v2), (q27, v3), (q37, v4), (APPEND, q47 + v5 + q57 + v6)], (six_q, six_v))
    add("appendsAndCompacted", "1419-1447", [(APPEND, q07 + v1 + q17 + v2), (q27 + q37, v3 + v4 + ZERO)],
        (four_q, four_v))
    add("appendsAndCompactedAndPuts", "1448-1482",
        [(APPEND, q07 + v1 + q17 + v2), (q27 + q37, v3 + v4 + ZERO), (q47, v5), (q57, v6)], (six_q, six_v))
    add("appendsDuplicatePuts", "1483-1505", [(APPEND, q07 + v1 + q17 + v2), (q07, v1), (q17, v2)],
        (q07 + q17, v1 + v2 + ZERO))
    add("appendsDuplicateCompacted", "1506-1528", [(APPEND, q07 + v1 + q17 + v2), (q07 + q17, v1 + v2 + ZERO)],
        (q07 + q17, v1 + v2 + ZERO))
    return out


def expand_columns(case):
    """(columns, expected (qualifier, value)) of a case; a loop-built row's expected cell is its
    columns concatenated in order plus the 0 meta byte, as the test asserts."""
    if "columns_loop" not in case:
        return ([(bytes.fromhex(q), bytes.fromhex(v)) for q, v in case["columns"]],
                case["expect"] if not isinstance(case["expect"], dict) else
                (bytes.fromhex(case["expect"]["qualifier"]), bytes.fromhex(case["expect"]["value"])))
    lp = case["columns_loop"]
    cols = []
    for i in range(lp["start"], lp["stop"], lp["step"]):
        q = H((i << 4) | 0x07) if lp["kind"] == "seconds" else struct.pack(">I", ((i << 6) | 0x07) | 0xF0000000)
        cols.append((q, L(i)))
    return cols, (b"".join(q for q, _ in cols), b"".join(v for _, v in cols) + ZERO)


def main():
    doc = {"about": __doc__.strip().splitlines()[0], "cases": cases()}
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "compaction.json")
    with open(path, "w") as f:
        json.dump(doc, f, separators=(",", ":"))
    print(path, len(doc["cases"]), "cases")


if __name__ == "__main__":
    main()
