"""StockEvent record values for the JSON ingest tests: the README demo records (the one
reference fixture, README.md:73-80) plus hand-written cases of json-simple 1.1.1 behaviour
(expected outcome per case, restated from its published lexer/parser; "parity unpinned" beyond
the README records) and a seeded fuzzer that mutates well-formed records."""
import random

OK, PARSE, CLASS_CAST, NULL, NUMBER, LEX, NARROW, DEPTH = range(8)

# README.md:73-80 (the demo's 8 StockEvents) -> (price, volume)
README = [
    (b'{"name":"e1","price":100,"volume":1010}', 100, 1010),
    (b'{"name":"e2","price":120,"volume":990}', 120, 990),
    (b'{"name":"e3","price":120,"volume":1005}', 120, 1005),
    (b'{"name":"e4","price":121,"volume":999}', 121, 999),
    (b'{"name":"e5","price":120,"volume":999}', 120, 999),
    (b'{"name":"e6","price":125,"volume":750}', 125, 750),
    (b'{"name":"e7","price":120,"volume":950}', 120, 950),
    (b'{"name":"e8","price":120,"volume":700}', 120, 700),
]

# (record, expected status) — hand-derived from json-simple's grammar
CASES = [
    (b'{"name":"e1","price":100,"volume":1010}', OK),
    (b' {\t"volume" : 7 ,\n"price":-3, "name" : "x"}\r\n', OK),
    (b'{"price":1,"volume":2}', OK),                       # name absent -> null String
    (b'{"name":null,"price":1,"volume":2}', OK),
    (b'{"name":"a","price":1,"volume":2,"extra":[1,{"k":[true,false,null]},"s"]}', OK),
    (b'{"name":"a" "price" 1 "volume" 2}', OK),            # commas/colons are skipped tokens
    (b'{,,"name":"a",,"price"::1,"volume":2,}', OK),
    (b'{"price":1,"price":5,"volume":2}', OK),             # HashMap.put: last wins
    (b'{"pr\\u0069ce":4,"volume":2}', OK),                 # keys compare after unescaping
    (b'{"name":"a\\"b\\\\c\\/d\\n","price":1,"volume":2}', OK),
    (b'{"name":"\xc3\xa9t\xc3\xa9","price":1,"volume":2}', OK),
    (b'{"price":007,"volume":-0}', OK),                    # Long.valueOf accepts leading zeros
    (b'{"price":9223372036854775807,"volume":-9223372036854775808}', OK),
    (b'{"price":1,"volume":2} "unterminated', OK),          # EOF inside a string is EOF
    (b'', PARSE),
    (b'   ', PARSE),
    (b'{"price":1,"volume":2', PARSE),
    (b'{"price":1,"volume":2}}', PARSE),
    (b'{"price":1,"volume":2} {}', PARSE),
    (b'{"price":1.,"volume":2}', PARSE),
    (b'{"price":1e,"volume":2}', PARSE),
    (b'{"price":-,"volume":2}', PARSE),
    (b'{"price":tru,"volume":2}', PARSE),
    (b'{"price":1,"volume":2,x}', PARSE),
    (b'{1:2}', PARSE),                                     # keys must be strings
    (b'{"a"}', PARSE),
    (b'[1,2}', PARSE),
    (b"{'price':1}", PARSE),
    (b'\xef\xbb\xbf{"price":1,"volume":2}', PARSE),        # a BOM is an unexpected char
    (b'[1,2]', CLASS_CAST),
    (b'"str"', CLASS_CAST),
    (b'42', CLASS_CAST),
    (b'true', CLASS_CAST),
    (b'{"name":5,"price":1,"volume":2}', CLASS_CAST),
    (b'{"name":{"x":1},"price":1,"volume":2}', CLASS_CAST),
    (b'{"price":1.5,"volume":2}', CLASS_CAST),
    (b'{"price":1e3,"volume":2}', CLASS_CAST),
    (b'{"price":"1","volume":2}', CLASS_CAST),
    (b'{"price":1,"volume":[2]}', CLASS_CAST),
    (b'{"price":true,"volume":2}', CLASS_CAST),
    (b'{"name":1,"volume":2}', CLASS_CAST),                # name's cast comes before price's unboxing
    (b'{"price":null,"volume":2.5}', NULL),                # price unboxed before volume is cast
    (b'null', NULL),
    (b'{"volume":2}', NULL),
    (b'{"price":1}', NULL),
    (b'{"price":1,"volume":null}', NULL),
    (b'{"price":9223372036854775808,"volume":2}', NUMBER),
    (b'{"price":-9223372036854775809,"volume":2}', NUMBER),
    (b'{"x":99999999999999999999,"price":1,"volume":2}', NUMBER),
    (b'{"x":99999999999999999999.5,"price":1,"volume":2}', OK),   # a Double, no Long.valueOf
    (b'{"x":99999999999999999999.,"price":1,"volume":2}', NUMBER),  # INT first, then '.'
    (b'{"x" 1 2 3 "price":1,"volume":2}', PARSE),
    (b'{"name":"a\\x","price":1,"volume":2}', LEX),
    (b'{"name":"\\u12G4","price":1,"volume":2}', LEX),
    (b'{"price":1,"volume":2,"name":"\\u00', LEX),
    (b'{"price":3000000000,"volume":2}', OK),              # a long; NARROW only for int32 columns
]


def deep(depth):
    return b'{"price":1,"volume":2,"d":' + b"[" * depth + b"]" * depth + b"}"


def fuzz(seed, n):
    """Seeded mutations of well-formed records (byte flips, deletions, duplications, insertions
    of JSON punctuation) — every outcome class shows up."""
    rng = random.Random(seed)
    alphabet = b'{}[],:"\\-.eE0123456789 tfnulra\x00\xff'
    out = []
    for i in range(n):
        price, vol = rng.randint(-10**6, 10**6), rng.randint(0, 10**6)
        r = bytearray(b'{"name":"e%d","price":%d,"volume":%d}' % (i + 1, price, vol))
        for _ in range(rng.choice([0, 0, 1, 1, 2, 3])):
            op, p = rng.randrange(4), rng.randrange(len(r) + 1)
            if op == 0 and p < len(r):
                r[p] = rng.choice(alphabet)
            elif op == 1 and p < len(r):
                del r[p]
            elif op == 2:
                r[p:p] = bytes([rng.choice(alphabet)])
            else:
                q = rng.randrange(len(r) + 1)
                a, b = min(p, q), max(p, q)
                r[p:p] = r[a:b][:12]
        out.append(bytes(r))
    return out
