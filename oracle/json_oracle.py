"""CPU restatement of the demo's record deserializer — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this; the product
path (libcep.so, cep_decode_stock_json) never does.

What it restates: `StockEventSerDe.JsonSerDeserializer.deserialize`
(/root/reference/src/test/java/com/github/fhuz/kafka/streams/cep/demo/StockEventSerDe.java:58-72)
and the `StockEvent` it builds (demo/StockEvent.java:4-14).  The parsing itself is the third-party
dependency json-simple 1.1.1 (`com.googlecode.json-simple:json-simple:1.1.1`, pom.xml:99-104),
absent from /root/reference; it is restated from its published algorithm:
  * `Yylex` (JFlex scanner, longest match): WS [ \\t\\n\\r\\f]; INT -?[0-9]+ -> Long.valueOf
    (NumberFormatException past long); DOUBLE INT(\\.[0-9]+)?([eE][-+]?[0-9]+)? -> Double;
    true/false/null; { } [ ] , : ; strings with \\" \\\\ \\/ \\b \\f \\n \\r \\t \\uXXXX escapes (an
    unmatched escape is the scanner's java.lang.Error); any other char -> ParseException; end of
    input inside a string is end of input (the scanner returns null at EOF).
  * `JSONParser.parse(String)`: the status/value stack machine (S_INIT, S_IN_FINISHED_VALUE,
    S_IN_OBJECT, S_PASSED_PAIR_KEY, S_IN_ARRAY) in which commas/colons are skipped tokens.
Pinned by the README's 8 demo records (README.md:73-80, the values smoke() and the NFA golden
use) and the serializer's format (StockEventSerDe.java:75-82); the error outcomes have no
reference fixture ("parity unpinned" for them — restated from json-simple's published source).

Result per record: (status, price, volume, name_span) with status one of the CEP_JSON_* codes of
include/cep.h, name_span = (offset of the name text in the record, raw length | bit31 escapes)
or None for a null/absent name.
"""
from __future__ import annotations

import re

OK, PARSE, CLASS_CAST, NULL, NUMBER, LEX, NARROW, DEPTH = range(8)
_LONG_MIN, _LONG_MAX = -(1 << 63), (1 << 63) - 1

_INT = re.compile(rb"-?[0-9]+")
_DOUBLE = re.compile(rb"-?[0-9]+(\.[0-9]+)?([eE][-+]?[0-9]+)?")
_ESC = {ord('"'): '"', ord("\\"): "\\", ord("/"): "/", ord("b"): "\b", ord("f"): "\f",
        ord("n"): "\n", ord("r"): "\r", ord("t"): "\t"}
_HEX = set(b"0123456789abcdefABCDEF")


class _Fail(Exception):
    def __init__(self, code):
        self.code = code


class JStr(str):
    """A decoded string token and the raw byte span of its text."""
    span = (0, 0, False)


_EOF = object()


def _tokens(data: bytes):
    """Yylex: yields ('v', value) or the punctuation byte as a 1-char str, then _EOF."""
    i, n = 0, len(data)
    while i < n:
        c = data[i]
        if c in b" \t\n\r\f":
            i += 1
            continue
        if c in b"{}[],:":
            yield chr(c)
            i += 1
            continue
        if c == ord('"'):
            j, out, esc = i + 1, [], False
            while True:
                if j >= n:  # end of input inside a string: the scanner returns EOF
                    yield _EOF
                    return
                d = data[j]
                if d == ord('"'):
                    break
                if d == ord("\\"):
                    esc = True
                    if j + 1 < n and data[j + 1] in _ESC:
                        out.append(_ESC[data[j + 1]])
                        j += 2
                        continue
                    if j + 5 < n and data[j + 1] == ord("u") and all(h in _HEX for h in data[j + 2:j + 6]):
                        out.append(chr(int(data[j + 2:j + 6], 16)))
                        j += 6
                        continue
                    raise _Fail(LEX)
                k = j
                while k < n and data[k] not in b'"\\':
                    k += 1
                out.append(data[j:k].decode("utf-8", "replace"))
                j = k
            s = JStr("".join(out))
            s.span = (i + 1, j - (i + 1), esc)
            yield ("v", s)
            i = j + 1
            continue
        if c == ord("-") or 48 <= c <= 57:
            m = _INT.match(data, i)
            if m is None:
                raise _Fail(PARSE)  # a lone '-' matches only the catch-all rule
            md = _DOUBLE.match(data, i)
            if md.end() > m.end():
                yield ("v", float(md.group(0)))
                i = md.end()
            else:
                v = int(m.group(0))
                if not _LONG_MIN <= v <= _LONG_MAX:
                    raise _Fail(NUMBER)
                yield ("v", v)
                i = m.end()
            continue
        for lit, val in ((b"true", True), (b"false", False), (b"null", None)):
            if data.startswith(lit, i):
                yield ("v", val)
                i += len(lit)
                break
        else:
            raise _Fail(PARSE)  # ERROR_UNEXPECTED_CHAR
    yield _EOF


def _parse(data: bytes):
    """JSONParser.parse: returns the value (dict/list/str/int/float/bool/None)."""
    S_INIT, S_FIN, S_OBJ, S_KEY, S_ARR = range(5)
    status, sstack, vstack = S_INIT, [], []
    for tok in _tokens(data):
        if status == S_INIT:
            if isinstance(tok, tuple):
                status = S_FIN
                sstack.append(status)
                vstack.append(tok[1])
            elif tok == "{":
                status = S_OBJ
                sstack.append(status)
                vstack.append({})
            elif tok == "[":
                status = S_ARR
                sstack.append(status)
                vstack.append([])
            else:
                raise _Fail(PARSE)
        elif status == S_FIN:
            if tok is _EOF:
                return vstack.pop()
            raise _Fail(PARSE)
        elif status == S_OBJ:
            if tok == ",":
                pass
            elif isinstance(tok, tuple) and isinstance(tok[1], str):
                vstack.append(tok[1])
                status = S_KEY
                sstack.append(status)
            elif tok == "}":
                if len(vstack) > 1:
                    sstack.pop()
                    vstack.pop()
                    status = sstack[-1]
                else:
                    status = S_FIN
            else:
                raise _Fail(PARSE)
        elif status == S_KEY:
            if tok == ":":
                pass
            elif isinstance(tok, tuple) or tok in ("{", "["):
                sstack.pop()
                key = vstack.pop()
                parent = vstack[-1]
                if isinstance(tok, tuple):
                    parent[key] = tok[1]
                    status = sstack[-1]
                else:
                    new = {} if tok == "{" else []
                    parent[key] = new
                    status = S_OBJ if tok == "{" else S_ARR
                    sstack.append(status)
                    vstack.append(new)
            else:
                raise _Fail(PARSE)
        elif status == S_ARR:
            if tok == ",":
                pass
            elif isinstance(tok, tuple):
                vstack[-1].append(tok[1])
            elif tok == "]":
                if len(vstack) > 1:
                    sstack.pop()
                    vstack.pop()
                    status = sstack[-1]
                else:
                    status = S_FIN
            elif tok in ("{", "["):
                new = {} if tok == "{" else []
                vstack[-1].append(new)
                status = S_OBJ if tok == "{" else S_ARR
                sstack.append(status)
                vstack.append(new)
            else:
                raise _Fail(PARSE)
    raise _Fail(PARSE)


def _is_long(v):
    return isinstance(v, int) and not isinstance(v, bool)


def deserialize(data: bytes, col_width: int = 8):
    """StockEventSerDe.java:58-72 on one record value -> (status, price, volume, name_span)."""
    try:
        obj = _parse(data)
    except _Fail as f:
        return f.code, 0, 0, None
    if obj is None:
        return NULL, 0, 0, None  # ((JSONObject) null).get(...)
    if not isinstance(obj, dict):
        return CLASS_CAST, 0, 0, None
    name = obj.get("name")
    if name is not None and not isinstance(name, str):
        return CLASS_CAST, 0, 0, None
    vals = []
    for f in ("price", "volume"):  # (Long) cast, then unboxing, in argument order
        v = obj.get(f)
        if v is None:
            return NULL, 0, 0, None
        if not _is_long(v):
            return CLASS_CAST, 0, 0, None
        vals.append(v)
    if col_width == 4 and not all(-(1 << 31) <= v < (1 << 31) for v in vals):
        return NARROW, 0, 0, None
    span = None
    if isinstance(name, JStr):
        span = name.span
    return OK, vals[0], vals[1], span


def serialize(name: str, price: int, volume: int) -> bytes:
    """StockEventSerDe.java:75-82: json-simple's JSONObject is a java.util.HashMap (default
    capacity 16), so toJSONString writes its entries in bucket order, (h ^ h >>> 16) & 15 of
    String.hashCode: volume 0, price 6, name 8.  (Derived from json-simple 1.1.1's published
    source and HashMap's iteration order: parity unpinned; names here need no escaping.)"""
    return b'{"volume":%d,"price":%d,"name":"%s"}' % (volume, price, name.encode())


def readme_record(name: str, price: int, volume: int) -> bytes:
    """The README's demo input records (README.md:73-80), typed into the console producer in
    the order name, price, volume."""
    return b'{"name":"%s","price":%d,"volume":%d}' % (name.encode(), price, volume)


def decode_batch(data: bytes, rec_off, col_width: int = 8):
    return [deserialize(data[int(rec_off[r]):int(rec_off[r + 1])], col_width) for r in range(len(rec_off) - 1)]
