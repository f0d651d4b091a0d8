"""TEST INFRASTRUCTURE ONLY -- oracle of the /api/query/exp join iterators.

A literal Python restatement, object for object, of
  TimeSyncedIterator ....... src/query/expression/TimeSyncedIterator.java:61-247
  UnionIterator ............ src/query/expression/UnionIterator.java:90-453 (computeUnion :171-244,
                             flattenTags :259-309, next :409-419, next(int) :442-453)
  IntersectionIterator ..... src/query/expression/IntersectionIterator.java:100-519
                             (computeIntersection :270-359, flattenTags :397-444)
  ExpressionIterator ....... src/query/expression/ExpressionIterator.java:135-485 (compile :237-302,
                             next(long) :323-358, next(int) :452-485)
  ExpressionDataPoint ...... src/query/expression/ExpressionDataPoint.java:66-257
  NumericFillPolicy ........ src/query/expression/NumericFillPolicy.java:140-175
  SpanGroup.computeTags .... src/core/SpanGroup.java:350-389 (the tags of a query result)
and of the JEXL 2.1.1 script evaluation ExpressionIterator runs (commons-jexl 2.1.1, pinned by
the reference build, third_party/jexl/include.mk; not vendored, restated from its published
source: JexlArithmetic add / subtract / multiply / divide / mod / negate / comparisons on
Double, Float, Integer and Boolean operands, and the lenient Interpreter's `0.0` for a division or
modulo by zero -- TestExpressionIterator.aDivideByZeroWithTwoSeries pins that one).

Java's HashMap iteration order decides which sub-query an intersection starts from and which
variable's tags an expression's series carry; it is simulated (String.hashCode, table sizes of
HashMap(int) and resizes), since the reference code iterates those maps.

Values are Python ints (Java long / Integer) or floats (double).  Tags are dicts of 3-byte UIDs.
"""
from __future__ import annotations

import math
import re
import struct

LONG_MAX = (1 << 63) - 1


class JavaError(Exception):
    def __init__(self, java, msg=""):
        self.java = java
        super().__init__(f"{java}: {msg}")


# ---- java.util.HashMap iteration order ------------------------------------------------------
def _jhash(s: str) -> int:
    h = 0
    for ch in s:
        h = (31 * h + ord(ch)) & 0xFFFFFFFF
    return h


def _table_size_for(cap: int) -> int:
    n = 1
    while n < cap:
        n <<= 1
    return max(n, 1)


def hashmap_order(keys, initial_capacity=None):
    """Iteration order of a java.util.HashMap<String, ?> filled with `keys` in that order
    (new HashMap() or new HashMap(initial_capacity)); re-puts of a key keep its position."""
    uniq = []
    for k in keys:
        if k not in uniq:
            uniq.append(k)
    n = 16 if initial_capacity is None else _table_size_for(max(1, initial_capacity))
    if initial_capacity == 0:
        n = 1
    size = 0
    buckets: dict[int, list] = {}
    for k in uniq:
        h = _jhash(k)
        h ^= h >> 16
        size += 1
        buckets.setdefault(h, []).append(k)
        while size > n * 0.75:
            n <<= 1
    order = []
    # keys in bucket index order; equal buckets keep insertion order (resize splits preserve it)
    by_bucket = sorted(uniq, key=lambda k: ((_jhash(k) ^ (_jhash(k) >> 16)) & (n - 1), uniq.index(k)))
    order.extend(by_bucket)
    return order


# ---- query results (DataPoints) ---------------------------------------------------------------
class DataPoints:
    """A query result: points [(ts_ms, value)], tag UIDs {tagk: tagv}, aggregated tagks."""

    def __init__(self, points, tags=None, agg_tags=(), metric=b"", name=""):
        self.points = list(points)
        self.tags = dict(tags or {})
        self.agg_tags = sorted(set(agg_tags))
        self.metric = metric
        self.name = name


def compute_tags(span_tags):
    """SpanGroup.computeTags (:350-389): pairs equal in every span that has the key stay tags;
    keys whose values differ become aggregated tags (a key missing from some spans stays)."""
    tag_set, discards = {}, set()
    for uids in span_tags:
        for k in sorted(uids):
            if k in discards:
                continue
            v = tag_set.get(k)
            if v is None:
                tag_set[k] = uids[k]
            elif v != uids[k]:
                discards.add(k)
                del tag_set[k]
    return tag_set, sorted(discards)


class EDP:
    """ExpressionDataPoint (:33-257): metadata plus one MutableDataPoint."""

    def __init__(self, src=None):
        self.tags = {}
        self.agg = set()
        self.metrics = set()
        self.index = 0
        self.ts = LONG_MAX
        self.val = math.nan
        if isinstance(src, DataPoints):       # ExpressionDataPoint(DataPoints) :79-96
            self.metrics = {src.metric}
            self.tags = dict(src.tags)
            self.agg = set(src.agg_tags)
        elif isinstance(src, EDP):            # ExpressionDataPoint(ExpressionDataPoint) :103-114
            self.metrics = set(src.metrics)
            self.tags = dict(src.tags)
            self.agg = set(src.agg)
        elif src is None:                     # default ctor: MutableDataPoint() = (Long.MAX_VALUE, 0L)
            self.val = 0

    def add(self, other: "EDP"):              # add(ExpressionDataPoint) :144-157 (no tag intersection)
        self.metrics |= other.metrics
        self.agg |= other.agg

    def reset_value(self, ts, value):
        self.ts, self.val = ts, value

    def to_double(self):
        return float(self.val)


def flatten_tags(union, use_query_tags, include_agg_tags, tags, agg, sub_query_tagks=None, sub=True):
    """The static flattenTags of UnionIterator (:259-309; `tags` None -> empty key) and of
    IntersectionIterator (:397-444; `tags` None -> NullPointerException).  sub=False: no sub
    iterator (null) -- NullPointerException when the query tagks are needed."""
    if tags is None:
        if union:
            return b""
        raise JavaError("NullPointerException", "tags")
    if not tags:
        return b""
    if use_query_tags and not sub:
        raise JavaError("NullPointerException", "sub iterator")
    return _flat_key(use_query_tags, include_agg_tags, tags, agg, sub_query_tagks)


def _flat_key(use_query_tags, include_agg_tags, tags, agg, query_tagks):
    """UnionIterator.flattenTags (:259-309) / IntersectionIterator.flattenTags (:397-444):
    the tag pairs (only the sub-query's filter tagks with use_query_tags -- none when it has
    none), then the aggregated tagks; an empty tag map gives an empty key."""
    if not tags:
        return b""
    qt = set(query_tagks or ())
    out = bytearray()
    for k in sorted(tags):
        if use_query_tags and k not in qt:
            continue
        out += k + tags[k]
    if include_agg_tags:
        if agg is None:
            raise JavaError("NullPointerException", "aggregated tags")
        for k in sorted(agg):
            out += k
    return bytes(out)


# ---- TimeSyncedIterator ---------------------------------------------------------------------
class TimeSyncedIterator:
    def __init__(self, id_, query_tagks, dps, fill=0.0):
        if not id_:
            raise JavaError("IllegalArgumentException", "Missing ID string")
        self.id = id_
        self.query_tagks = query_tagks
        self.dps = list(dps)
        self.fill = fill                     # NumericFillPolicy(ZERO) by default
        self.index = 0
        self.pos = [0] * len(self.dps)
        self.cur = [None] * len(self.dps)    # current_values
        self.emit = [None] * len(self.dps)   # emitter_values
        for i, d in enumerate(self.dps):     # setupEmitters :234-247
            if d.points:
                self.cur[i] = d.points[0]
                self.pos[i] = 1
                e = EDP(d)
                e.index = i
                self.emit[i] = e

    def copy(self):
        it = TimeSyncedIterator(self.id, self.query_tagks, self.dps, self.fill)
        return it

    def size(self):
        return len(self.dps)

    def has_next(self):
        return any(c is not None for c in self.cur)

    def _advance(self, i):
        d = self.dps[i]
        if self.pos[i] < len(d.points):
            self.cur[i] = d.points[self.pos[i]]
            self.pos[i] += 1
        else:
            self.cur[i] = None

    def next_ts(self, timestamp):            # next(long) :125-144
        for i in range(len(self.cur)):
            if self.emit[i] is None:
                raise JavaError("NullPointerException", "series without data points")
            if self.cur[i] is None:
                self.emit[i].reset_value(timestamp, self.fill)
                continue
            if self.cur[i][0] > timestamp:
                self.emit[i].reset_value(timestamp, self.fill)
            else:
                self.emit[i].reset_value(*self.cur[i])
                self._advance(i)
        return self.emit

    def next_timestamp(self):
        ts = LONG_MAX
        for c in self.cur:
            if c is not None and c[0] < ts:
                ts = c[0]
        return ts

    def next_index(self, i):                 # next(int) :161-171
        if self.cur[i] is None:
            raise JavaError("RuntimeException", "No more elements")
        self.emit[i].reset_value(*self.cur[i])
        self._advance(i)

    def has_next_index(self, i):
        return self.cur[i] is not None

    def null_iterator(self, i):
        if i < 0 or i > len(self.cur):
            raise JavaError("IllegalArgumentException", f"Index out of range: {i}")
        self.cur[i] = None

    def values(self):
        return self.emit

    def flat_tags_of(self, i):
        e = self.emit[i]
        if e is None:
            raise JavaError("NullPointerException", "series without data points")
        return e.tags, e.agg


# ---- UnionIterator / IntersectionIterator -----------------------------------------------------
class _Join:
    def __init__(self, id_, results: dict, use_query_tags, include_agg_tags, results_order=None):
        if results is None:
            raise JavaError("NullPointerException", "results")
        self.id = id_
        self.use_qt = use_query_tags
        self.inc_agg = include_agg_tags
        order = results_order if results_order is not None else hashmap_order(list(results))
        # queries = new HashMap(results.size()), filled in results' iteration order
        self.names = hashmap_order(order, len(results))
        self.queries = {k: results[k] for k in self.names}
        self.index_to_names = list(order)
        for i, k in enumerate(order):
            results[k].index = i
        self.current = {}
        self.series_size = 0
        self.timestamp = LONG_MAX

    def _key(self, sub, i):
        vals = sub.values()
        e = vals[i]
        if e is None:
            raise JavaError("NullPointerException", "series without data points")
        # ExpressionIterator.getQueryTagKs() returns null
        qt = sub.query_tagks if isinstance(sub, TimeSyncedIterator) else None
        return _flat_key(self.use_qt, self.inc_agg, e.tags, e.agg, qt)

    def has_next(self):
        return any(s.has_next() for s in self.queries.values())

    def next_timestamp(self):
        ts = LONG_MAX
        for s in self.queries.values():
            t = s.next_timestamp()
            if t < ts:
                ts = t
        return ts

    def results(self):
        return self.current


class UnionIterator(_Join):
    def __init__(self, id_, results, use_query_tags, include_agg_tags, results_order=None, fill=0.0):
        super().__init__(id_, results, use_query_tags, include_agg_tags, results_order)
        self.fill = fill
        self.fill_dp = EDP()
        self.matrix = {}
        self._compute_union()
        self.timestamp = self.next_timestamp()

    def _compute_union(self):                 # :171-244
        union = {}
        for name in self.names:
            sub = self.queries[name]
            for i in range(sub.size()):
                key = self._key(sub, i)
                udps = union.get(key)
                if udps is None:
                    udps = [None] * len(self.queries)
                    union[key] = udps
                udps[sub.index] = sub.values()[i]
        if not union:
            return
        keys = sorted(union)                  # ByteMap: unsigned lexicographic
        for name in self.names:
            self.current[name] = [None] * len(keys)
            self.matrix[name] = [-1] * len(keys)
        for j, key in enumerate(keys):
            idps = union[key]
            for x, e in enumerate(idps):
                nm = self.index_to_names[x]
                self.current[nm][j] = e
                if e is not None:
                    self.matrix[nm][j] = e.index
        for nm in self.current:
            arr = self.current[nm]
            for j in range(len(arr)):
                if arr[j] is None:
                    arr[j] = self.fill_dp
        self.series_size = len(keys)
        self.keys = keys

    def next(self):                           # :409-419
        if not self.has_next():
            raise JavaError("IllegalDataException", "No more data")
        for s in self.queries.values():
            s.next_ts(self.timestamp)
        self.fill_dp.reset_value(self.timestamp, self.fill)
        self.timestamp = self.next_timestamp()

    def has_next_index(self, j):              # :432-440
        for nm, m in self.matrix.items():
            idx = m[j]
            if idx >= 0 and self.queries[nm].has_next_index(idx):
                return True
        return False

    def next_index(self, j):                  # :443-453
        if not self.has_next():
            raise JavaError("IllegalDataException", "No more data")
        for nm, m in self.matrix.items():
            idx = m[j]
            if idx >= 0:
                self.queries[nm].next_index(idx)


class IntersectionIterator(_Join):
    def __init__(self, id_, results, use_query_tags, include_agg_tags, results_order=None):
        super().__init__(id_, results, use_query_tags, include_agg_tags, results_order)
        max_series = max([s.size() for s in self.queries.values()] or [0])
        if max_series < 1:
            return
        self._compute_intersection()
        self.timestamp = self.next_timestamp()

    def _compute_intersection(self):          # :270-359
        names = self.names
        first = self.queries[names[0]]
        flattened = {}
        tags = {}
        flattened[first.id] = tags
        inter = {}
        for i in range(first.size()):
            key = self._key(first, i)
            tags[key] = i
            idps = [None] * len(self.queries)
            idps[first.index] = first.values()[i]
            inter[key] = idps
        for name in names[1:]:
            sub = self.queries[name]
            tags = {}
            flattened[sub.id] = tags
            for i in range(sub.size()):
                key = self._key(sub, i)
                tags[key] = i
                idps = inter.get(key)
                if idps is None:
                    sub.null_iterator(i)
                    continue
                idps[sub.index] = sub.values()[i]
            for key in sorted(inter):
                if key not in tags:
                    for sid, ftags in flattened.items():
                        if sid == sub.id:
                            continue
                        idx = ftags.get(key)
                        if idx is not None:
                            self._query_by_id(sid).null_iterator(idx)
                    del inter[key]
        if len(names) > 1 and not inter:
            raise JavaError("IllegalDataException", "No intersections found")
        keys = sorted(inter)
        for name in names:
            self.current[name] = [None] * len(keys)
        for j, key in enumerate(keys):
            for x, e in enumerate(inter[key]):
                self.current[self.index_to_names[x]][j] = e
        self.series_size = len(keys)
        self.keys = keys

    def _query_by_id(self, sid):
        for s in self.queries.values():
            if s.id == sid:
                return s
        raise KeyError(sid)

    def next(self):                           # :215-223
        if not self.has_next():
            raise JavaError("IllegalDataException", "No more data")
        for s in self.queries.values():
            s.next_ts(self.timestamp)
        self.timestamp = self.next_timestamp()

    def has_next_index(self, j):              # :502-509 (the index goes to every sub unmapped)
        return any(s.has_next_index(j) for s in self.queries.values())

    def next_index(self, j):                  # :512-519
        if not self.has_next():
            raise JavaError("IllegalDataException", "No more data")
        for s in self.queries.values():
            s.next_index(j)


# ---- JEXL 2.1.1 subset ----------------------------------------------------------------------
class JInt(int):
    """A JEXL integer literal / result (java.lang.Integer / Long): integer arithmetic."""


class JFloat(float):
    """A JEXL decimal literal without suffix: java.lang.Float."""


_TOKEN = re.compile(r"\s*(?:(\d+\.\d*(?:[eE][-+]?\d+)?[fFdD]?|\.\d+(?:[eE][-+]?\d+)?[fFdD]?|\d+[lL]?)"
                    r"|([A-Za-z_$][A-Za-z0-9_$]*)|(<=|>=|==|!=|[-+*/%()<>]))")


def _tokenize(text):
    pos, out = 0, []
    text = text.rstrip()
    while pos < len(text):
        m = _TOKEN.match(text, pos)
        if not m or m.end() == pos:
            raise JavaError("JexlException", f"parse error in {text!r}")
        pos = m.end()
        num, name, op = m.groups()
        if num is not None:
            out.append(("num", num))
        elif name is not None:
            out.append(("var", name))
        else:
            out.append(("op", op))
    return out


def parse(text):
    """Expression AST (tuples) and its variable names (JexlEngine.getVariables)."""
    if text is None or text == "":
        raise JavaError("IllegalArgumentException", "The expression cannot be  null")
    toks = _tokenize(text)
    pos = 0
    names = []

    def peek():
        return toks[pos] if pos < len(toks) else (None, None)

    def take():
        nonlocal pos
        pos += 1
        return toks[pos - 1]

    def primary():
        kind, v = peek()
        if kind == "num":
            take()
            if re.fullmatch(r"\d+[lL]?", v):
                return ("lit", JInt(int(v.rstrip("lL"))))
            if v[-1] in "dD":
                return ("lit", float(v[:-1]))
            s = v[:-1] if v[-1] in "fF" else v
            return ("lit", JFloat(struct.unpack("<f", struct.pack("<f", float(s)))[0]))
        if kind == "var":
            take()
            if v not in names:
                names.append(v)
            return ("var", v)
        if (kind, v) == ("op", "("):
            take()
            e = comparison()
            if peek() != ("op", ")"):
                raise JavaError("JexlException", f"parse error in {text!r}")
            take()
            return e
        if (kind, v) == ("op", "-"):
            take()
            return ("neg", primary())
        raise JavaError("JexlException", f"parse error in {text!r}")

    def multiplicative():
        e = primary()
        while peek()[0] == "op" and peek()[1] in ("*", "/", "%"):
            o = take()[1]
            e = (o, e, primary())
        return e

    def additive():
        e = multiplicative()
        while peek()[0] == "op" and peek()[1] in ("+", "-"):
            o = take()[1]
            e = (o, e, multiplicative())
        return e

    def comparison():
        e = additive()
        while peek()[0] == "op" and peek()[1] in ("<", ">", "<=", ">=", "==", "!="):
            o = take()[1]
            e = (o, e, additive())
        return e

    ast = comparison()
    if pos != len(toks):
        raise JavaError("JexlException", f"parse error in {text!r}")
    return ast, names


def _is_fp(x):
    return isinstance(x, float)


def _to_double(x):
    if isinstance(x, bool):
        return 1.0 if x else 0.0
    return float(x)


def _to_int(x):
    if isinstance(x, bool):
        return 1 if x else 0
    return int(x)


def _jmod_int(l, r):   # BigInteger.mod: non-negative
    return l % r if r > 0 else (_ for _ in ()).throw(ArithmeticError("%"))


def _arith(op, l, r):
    if _is_fp(l) or _is_fp(r):
        a, b = _to_double(l), _to_double(r)
        if op == "+":
            return a + b
        if op == "-":
            return a - b
        if op == "*":
            return a * b
        if b == 0.0:
            raise ArithmeticError(op)
        if op == "/":
            return a / b
        return math.fmod(a, b)
    a, b = _to_int(l), _to_int(r)
    if op == "+":
        return JInt(a + b)
    if op == "-":
        return JInt(a - b)
    if op == "*":
        return JInt(a * b)
    if b == 0:
        raise ArithmeticError(op)
    if op == "/":
        q = abs(a) // abs(b)
        return JInt(q if (a >= 0) == (b >= 0) else -q)
    return JInt(_jmod_int(a, b))


def _compare(op, l, r):
    if _is_fp(l) or _is_fp(r):
        a, b = _to_double(l), _to_double(r)
    else:
        a, b = _to_int(l), _to_int(r)
    return {"<": a < b, ">": a > b, "<=": a <= b, ">=": a >= b, "==": a == b, "!=": a != b}[op]


def evaluate(ast, env):
    kind = ast[0]
    if kind == "lit":
        return ast[1]
    if kind == "var":
        if ast[1] not in env:
            raise JavaError("JexlException", f"undefined variable {ast[1]}")
        return env[ast[1]]
    if kind == "neg":
        v = evaluate(ast[1], env)
        if isinstance(v, bool):
            raise JavaError("JexlException", "negate a boolean")
        return -v if _is_fp(v) else JInt(-int(v))
    l, r = evaluate(ast[1], env), evaluate(ast[2], env)
    if kind in ("<", ">", "<=", ">=", "==", "!="):
        return _compare(kind, l, r)
    try:
        return _arith(kind, l, r)
    except ArithmeticError:
        return 0.0   # lenient Interpreter: a divide / modulo error yields Double 0.0


def _result_double(out, it):
    if isinstance(out, bool):
        return 1.0 if out else 0.0
    if isinstance(out, float) and not isinstance(out, JFloat):
        return float(out)
    raise JavaError("IllegalStateException", f"Expression returned a result of type: "
                    f"{'java.lang.Float' if isinstance(out, JFloat) else 'java.lang.Integer'} for {it}")


class ExpressionIterator:
    def __init__(self, id_, expression, set_operator, use_query_tags, include_agg_tags):
        if expression is None or expression == "":
            raise JavaError("IllegalArgumentException", "The expression cannot be  null")
        if set_operator is None:
            raise JavaError("IllegalArgumentException", "The set operator cannot be null")
        self.id = id_
        self.text = expression
        self.ast, names = parse(expression)
        if not names:
            raise JavaError("IllegalArgumentException", "The expression didn't appear to have any variables")
        self.names = hashmap_order(names)     # HashSet<String> iteration order
        self.set_operator = set_operator
        self.use_qt = use_query_tags
        self.inc_agg = include_agg_tags
        self.results = {}                      # HashMap<String, ITimeSyncedIterator>
        self.results_keys = []
        self.fill = math.nan                   # NumericFillPolicy(NOT_A_NUMBER)
        self.index = 0
        self.query_tagks = None
        self.iterator = None
        self.dps = None

    def add_results(self, id_, iterator):
        if id_ is None:
            raise JavaError("IllegalArgumentException", "Missing ID")
        if iterator is None:
            raise JavaError("IllegalArgumentException", "Iterator cannot be null")
        self.results[id_] = iterator
        self.results_keys.append(id_)

    def copy(self):
        e = ExpressionIterator(self.id, self.text, self.set_operator, self.use_qt, self.inc_agg)
        for k in self.results_keys:
            e.add_results(k, self.results[k].copy())
        return e

    def compile(self):                          # :237-302
        if len(self.results) < 1:
            raise JavaError("IllegalArgumentException", "No results for any variables in the expression")
        if len(self.results) < len(self.names):
            raise JavaError("IllegalArgumentException", "Not enough query results for the expression variables")
        for v in self.names:
            it = self.results.get(v.lower())
            if it is None:
                raise JavaError("IllegalArgumentException", "Missing results for variable " + v)
            if isinstance(it, ExpressionIterator):
                it.compile()
        order = hashmap_order(self.results_keys)
        if self.set_operator == "INTERSECTION":
            self.iterator = IntersectionIterator(self.id, self.results, self.use_qt, self.inc_agg, order)
        else:
            self.iterator = UnionIterator(self.id, self.results, self.use_qt, self.inc_agg, order)
        res = self.iterator.results()
        n = self.iterator.series_size
        self.dps = []
        for i in range(n):
            entries = list(res.items())          # current_values: HashMap in the join's name order
            e0 = entries[0][1] if entries else None
            d = EDP() if (e0 is None or e0[i] is None) else EDP(e0[i])
            for _, arr in entries[1:]:
                if arr is not None and arr[i] is not None:
                    d.add(arr[i])
            self.dps.append(d)

    # ITimeSyncedIterator
    def has_next(self):
        return self.iterator.has_next()

    def next_timestamp(self):
        return self.iterator.next_timestamp()

    def size(self):
        return len(self.dps)

    def values(self):
        return self.dps

    def null_iterator(self, i):
        if i < 0 or i >= len(self.dps):
            raise JavaError("IllegalArgumentException", "Index out of bounds")

    def _bind(self, i, env, ts_out=None):
        res = self.iterator.results()
        for v in self.names:
            arr = res.get(v)
            if arr is None:
                raise JavaError("NullPointerException", f"no results named {v}")
            e = arr[i]
            fill = self.results[v].fill
            if e is None:
                env[v] = fill
            else:
                if ts_out is not None and e.ts < ts_out[0]:
                    ts_out[0] = e.ts
                val = e.to_double()
                env[v] = fill if val != val else val

    def next_ts(self, timestamp):               # next(long) :323-358
        self.iterator.next()
        for i in range(self.iterator.series_size):
            env = {}
            self._bind(i, env)
            self.dps[i].reset_value(timestamp, _result_double(evaluate(self.ast, env), self.id))
        return self.dps

    def has_next_index(self, i):
        return self.iterator.has_next_index(i)

    def next_index(self, i):                    # next(int) :452-485
        self.iterator.next_index(i)
        env = {}
        ts = [LONG_MAX]
        self._bind(i, env, ts)
        self.dps[i].reset_value(ts[0], _result_double(evaluate(self.ast, env), self.id))


def serialize(it: ExpressionIterator, qs, qe):
    """QueryExecutor.SerializeExpressionIterator (src/tsd/QueryExecutor.java:668-708): the rows
    [ts, value of set 0, set 1, ...] of every step with qs <= ts <= qe."""
    rows = []
    ts = it.next_timestamp()
    while it.has_next():
        it.next_ts(ts)
        t = it.dps[0].ts if it.dps else ts
        if qs <= t <= qe:
            rows.append((t, [d.to_double() for d in it.dps]))
        ts = it.next_timestamp()
    return rows
