"""Event schemas: the columnar stand-in for the reference's value type `V`.

The reference's events are Java objects (`StockEvent{price, volume}` in
test:nfa/NFATest.java:247-265, `StockEvent{name, price, volume}` with `long` fields in
test:demo/StockEvent.java:4-24, or plain `String` values in NFATest.java:35-39).
The engine reads key-partitioned columns, so a schema names the columns and their Java
primitive types.  A `String` value (NFATest's "A".."D") becomes an `int` column of
dictionary codes; `value.equals("A")` compares codes.
"""
from __future__ import annotations

from . import expr as X


class EventSchema:
    def __init__(self, fields=None, *, string_value: bool = False):
        self.names: list[str] = []
        self.types: list[int] = []
        self._dict: dict[str, int] = {}
        self.string_value = string_value
        if string_value:
            self.names, self.types = ["value"], [X.I32]
        for n, t in (fields or {}).items():
            self.names.append(n)
            self.types.append(X.as_type(t))
        if not self.names:
            raise ValueError("a schema needs at least one column")

    @classmethod
    def strings(cls) -> "EventSchema":
        """Schema for string-valued events (the reference NFATest's `Event<String, String>`)."""
        return cls(string_value=True)

    # -- tracing --
    def field_index(self, name: str) -> int:
        try:
            return self.names.index(name)
        except ValueError:
            raise AttributeError(f"event has no field '{name}' (schema: {self.names})") from None

    def field_expr(self, name: str) -> X.Expr:
        i = self.field_index(name)
        return X.Field(i, self.types[i], name)

    def value_expr(self) -> X.Expr:
        if not self.string_value:
            raise TypeError("value.equals(...) needs a string-valued schema")
        return X.Field(0, X.I32, "value")

    def encode_literal(self, s) -> int:
        if not isinstance(s, str):
            raise TypeError("string-valued events compare with str literals")
        if s not in self._dict:
            self._dict[s] = len(self._dict) + 1
        return self._dict[s]

    def encode_values(self, values) -> list[int]:
        """Dictionary-encode string values (shares the dictionary with predicate literals)."""
        return [self.encode_literal(v) for v in values]

    def __repr__(self):
        return "EventSchema(" + ", ".join(f"{n}:{X.TYPE_NAMES[t]}" for n, t in zip(self.names, self.types)) + ")"


STOCK_INT = lambda: EventSchema({"price": "int", "volume": "int"})    # NFATest.java:247-265
STOCK_LONG = lambda: EventSchema({"price": "long", "volume": "long"})  # demo/StockEvent.java:4-24
