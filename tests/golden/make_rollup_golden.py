"""Extracts the rollup codec known answers into tests/golden/rollup.json.

Source: the reference's own unit tests (read as text, nothing executed):
  test/rollup/TestRollupInterval.java  -- RollupInterval ctor / validateAndCompile
  test/rollup/TestRollupUtils.java     -- getRollupBasetime, buildRollupQualifier
Each case records its test method and line, the interval (interval string, row span),
the call's arguments and the expected value, or "error" for tests that expect an
exception.  Cases whose arguments this extractor cannot read are skipped and counted.

Run (in a container that holds the reference):
  python tests/golden/make_rollup_golden.py [/root/reference]
"""
from __future__ import annotations

import json
import os
import re
import sys

HERE = os.path.dirname(os.path.abspath(__file__))


def methods(text):
    """(name, first line, annotation, body) per @Test method."""
    out = []
    lines = text.split("\n")
    i = 0
    while i < len(lines):
        m = re.match(r"\s*@Test\s*(\(.*\))?", lines[i])
        if not m:
            i += 1
            continue
        ann = m.group(1) or ""
        j = i + 1
        while j < len(lines) and "public void" not in lines[j]:
            j += 1
        name = re.search(r"public void (\w+)", lines[j]).group(1)
        depth, body, k = 0, [], j
        started = False
        while k < len(lines):
            depth += lines[k].count("{") - lines[k].count("}")
            body.append(lines[k])
            if "{" in lines[k]:
                started = True
            if started and depth == 0:
                break
            k += 1
        out.append((name, j + 1, ann, "\n".join(body)))
        i = k + 1
    return out


def field_intervals(text):
    """Intervals built in @Before: field name -> (interval, row span)."""
    res = {}
    for m in re.finditer(r"(\w+) = RollupInterval\.builder\(\)(.*?)\.build\(\)", text, re.S):
        iv = re.search(r'setInterval\("([^"]+)"\)', m.group(2))
        rs = re.search(r'setRowSpan\("([^"]+)"\)', m.group(2))
        if iv and rs:
            res[m.group(1)] = (iv.group(1), rs.group(1))
    return res


def body_interval(body, fields):
    iv = re.search(r'setInterval\("([^"]+)"\)', body)
    rs = re.search(r'setRowSpan\("([^"]+)"\)', body)
    if iv and rs:
        return iv.group(1), rs.group(1)
    for name, v in fields.items():
        if re.search(r"[,(]\s*" + name + r"\s*\)", body):
            return v
    return None


def flags_expr(tok):
    """`7`, `0x7` or `( 3 | Const.FLAG_FLOAT)` (Const.FLAG_FLOAT = 0x8, src/core/Const.java:65)."""
    tok = tok.strip()
    if tok.startswith("("):
        return int(re.search(r"\d+", tok).group(0)) | 0x8
    return int(tok, 0)


def jbyte(tok):
    tok = tok.strip().replace("(byte)", "").strip()
    v = int(tok, 16) if tok.lower().startswith("0x") else int(tok)
    return v & 0xFF


def main():
    ref = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
    rel_i = "test/rollup/TestRollupInterval.java"
    rel_u = "test/rollup/TestRollupUtils.java"
    ti = open(os.path.join(ref, rel_i)).read()
    tu = open(os.path.join(ref, rel_u)).read()
    out = {"source": [rel_i, rel_u], "intervals": [], "basetime": [], "qualifier": []}
    skipped = 0

    for name, line, ann, body in methods(ti):
        iv = body_interval(body, {})
        if not iv or "Table" in name:   # table names are not part of the engine's interval API
            skipped += 1
            continue
        case = {"name": name, "ref": f"{rel_i}:{line}", "interval": iv[0], "row_span": iv[1]}
        if "expected" in ann:
            case["error"] = re.search(r"expected\s*=\s*(\w+)", ann).group(1)
        else:
            def get(what):
                m = re.search(r"assertEquals\(([^,]+),\s*interval\.get" + what + r"\(\)\)", body)
                return m.group(1).strip() if m else None
            u, n, s = get("Units"), get("Intervals"), get("IntervalSeconds")
            if u is None or n is None or s is None:
                skipped += 1
                continue
            case.update(units=u.strip("'"), intervals=int(n), interval_seconds=int(s))
        out["intervals"].append(case)

    fields = field_intervals(tu)
    for name, line, ann, body in methods(tu):
        flat = re.sub(r"\s+", " ", body)
        iv = body_interval(body, fields)
        err = re.search(r"expected\s*=\s*(\w+)", ann)
        if "getRollupBasetime" in flat:
            m = re.search(r"getRollupBasetime\((-?\d+)L?, (\w+)\)", flat)
            if not m or m.group(2) == "null" or iv is None:
                skipped += 1
                continue
            case = {"name": name, "ref": f"{rel_u}:{line}", "interval": iv[0], "row_span": iv[1],
                    "timestamp": int(m.group(1))}
            if err:
                case["error"] = err.group(1)
            else:
                e = re.search(r"assertEquals\((-?\d+), RollupUtils\.getRollupBasetime", flat)
                if not e:
                    skipped += 1
                    continue
                case["expected"] = int(e.group(1))
            out["basetime"].append(case)
        elif "buildRollupQualifier" in flat:
            m = re.search(r"buildRollupQualifier\((-?\d+)L?, (-?\d+), ?\(byte\) ?(\( ?\d+ \| Const\.FLAG_FLOAT\)|\w+), "
                          r"(\d+), \w+\)", flat)
            if not m or iv is None:
                skipped += 1
                continue
            case = {"name": name, "ref": f"{rel_u}:{line}", "interval": iv[0], "row_span": iv[1],
                    "timestamp": int(m.group(1)), "basetime": int(m.group(2)),
                    "flags": flags_expr(m.group(3)), "agg_id": int(m.group(4))}
            if err:
                case["error"] = err.group(1)
            else:
                off = re.search(r"offset = \{([^}]*)\}", flat)
                agg = re.search(r"expected_qual\[0\] = (\d+);", flat)
                if not off or not agg:
                    skipped += 1
                    continue
                b = [jbyte(t) for t in off.group(1).split(",")]
                case["expected"] = bytes([int(agg.group(1))] + b).hex()
            out["qualifier"].append(case)
    out["skipped"] = skipped
    with open(os.path.join(HERE, "rollup.json"), "w") as f:
        json.dump(out, f, indent=1)
    print({k: len(v) for k, v in out.items() if isinstance(v, list)}, "skipped", skipped)


if __name__ == "__main__":
    main()
