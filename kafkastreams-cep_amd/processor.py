"""CEPProcessor: the reference's Kafka Streams processor over libcep.

Mirrors `CEPProcessor<K, V>` (CEPProcessor.java:54-193), `Sequence<K, V>` (Sequence.java:9-75)
and `Event<K, V>` (Event.java:27-93).  Records enter one at a time through
`process(key, value)` exactly as in the reference; the matching itself runs on the GPU
in arrival-order micro-batches (`cep_push_batch` on a streaming session, include/cep.h):

* `process(key, value)` skips a null value (CEPProcessor.java:157) and buffers the record
  with its context metadata (topic, partition, offset, timestamp - Event.java:31-41);
* the buffer is flushed when it holds `batch_size` records, on `punctuate()` and on
  `close()` (the reference's `punctuate`/`close` are empty, :167-175: it matches record by
  record, this processor matches a batch of records per launch);
* each flush rebuilds every match as a `Sequence` (stage name -> events, in the walk order of
  `NFA.matchPattern` / `peek`: final stage first, newest event first) and forwards them with
  `context.forward(None, sequence)` (:161) in the reference's order: by the arrival of the
  record that completed them, and in emission order within one record;
* a key whose NFA threw (the per-key errors of `cep_key_errors`) raises that exception after
  every match of an earlier record has been forwarded, like the reference's `process()`
  throwing out of the stream thread; the processor is failed from then on.

One difference is by design: the reference keeps ONE NFA per topic
partition (CEPProcessor.java:117-134), so records of different keys share runs; this
processor keeps one NFA per key (a Kafka partition is usually one key's stream in the
reference's demo, where both give the same matches).

State.  The device session holds every key's NFA (run queue, shared buffer, folds).  The host
keeps, per key, only the records a later match can still contain: after each flush the
session reports, per key, the oldest event a live buffer node holds (`cep_live_floor`) and
older records are dropped - the same events the reference's buffer store still holds
(KVSharedVersionedBuffer.java:143-171 deletes a node once its last reference is walked).  A
query whose runs never die (the README query: WITHIN never prunes in the reference, SURVEY
§0.3) pins its runs' events there as it does in the reference's store.  `max_keys` bounds the
dense key space of the device session.

Persistence (`in_memory=False`, the reference's default, CEPProcessor.java:71-84,144-149).  The
reference writes the NFA's run queue to the `_cep_nfa` store after every record (:159-160) and
reloads it in `init` (:117-134).  Here the processor's whole state - the device session's
snapshot (`cep_session_snapshot`: run queues, buffers, folds, Dewey versions, sequence
numbers of every key) and the retained records - is written to the `_cep_nfa` store, keyed by
(topic, partition) as the reference keys it, at every commit (`punctuate`, `close`), and
reloaded in `init`.  Records processed after the last commit are replayed by the host after a
restart (Kafka's at-least-once delivery), so a processor recreated from the store forwards
exactly what one uninterrupted processor would.  This commit granularity is a deliberate
difference from the reference's per-record store write (it would serialise every key's NFA per
record); the results forwarded are the same.  The store is whatever
`context.get_state_store("_cep_nfa")` returns (any mutable mapping; a real host passes its
persistent store), or the `store` argument.  The blob is a versioned plain encoding (no
pickle): the device snapshot's own binary format, then a JSON document of the retained records
whose keys and values go through `key_serde` / `value_serde` (Kafka-style serdes:
`serialize(obj) -> bytes`, `deserialize(bytes) -> obj`; the default, `JsonSerde`, is JSON that
keeps tuples, non-string dict keys, bytes and numpy scalars exact; process() checks the first
record of every key against the serdes, so an unsupported type fails at once).

There is no CPU matching path: without libcep.so and a GPU, `init()` raises.
"""
from __future__ import annotations

import base64
import json
import operator

import numpy as np

from . import expr as X
from . import native as N

_DTYPES = {X.I32: np.int32, X.I64: np.int64, X.F64: np.float64}


# ---- Java exceptions a key's NFA can throw (cep_key_errors codes) -------------------------
class JavaException(RuntimeError):
    """An exception the reference's `process()` would have thrown (the key and record that
    raised it are in `key` / `event`)."""

    def __init__(self, msg, key=None, event=None):
        super().__init__(msg)
        self.key, self.event = key, event


class NullPointerException(JavaException):
    pass


class IllegalStateException(JavaException):
    pass


class ArithmeticException(JavaException):
    pass


class CapacityError(JavaException):
    """A hard limit of the GPU engine (Dewey run-length pairs, stage depth); the reference
    has no such limit, so this is never a parity result."""


_EXC = {1: NullPointerException, 2: IllegalStateException, 3: ArithmeticException, 16: CapacityError}

NFA_STATES_STORE = "_cep_nfa"  # CEPProcessor.java:56
_CKPT_MAGIC = b"CEPPROC2"  # 2: plain encoding (JSON host half); 1 (pickle) is not read
# host-half versions: 3 = JsonSerde's tagged encoding (tuples, bytes, numpy scalars, non-string
# dict keys); 2 = the plain JSON encoding before it (read back with plain json.loads)
_CKPT_VERSION = 3
_CKPT_READABLE = (2, 3)


class JsonSerde:
    """The default key/value serde of the processor's checkpoint: JSON with the Python types a
    key or a record value usually is kept exact - dicts (any hashable keys), lists, tuples,
    strings, numbers (non-finite floats too), booleans, None, bytes and numpy scalars; a tuple key
    comes back a tuple, a dict value with int keys comes back with int keys.  Anything else (an
    object read by attribute, say) needs a serde of its own: process() checks the first record of
    every key against the serdes, so such a value fails there, not at the first commit (the
    reference's Kryo serde likewise accepts only registered classes, serde/KryoSerDe.java)."""

    TAG = "__cep__"  # a dict holding this key is an encoded non-JSON value

    @classmethod
    def _enc(cls, o):
        if isinstance(o, (np.integer, np.floating, np.bool_)):  # (before float: np.float64 is one)
            return {cls.TAG: "np", "dt": o.dtype.str, "v": cls._enc(o.item())}
        if o is None or isinstance(o, (bool, str)):
            return o
        if isinstance(o, int):
            return int(o)
        if isinstance(o, float):
            return o if o == o and o not in (float("inf"), float("-inf")) else {cls.TAG: "float", "v": repr(o)}
        if isinstance(o, list):
            return [cls._enc(x) for x in o]
        if isinstance(o, tuple):
            return {cls.TAG: "tuple", "v": [cls._enc(x) for x in o]}
        if isinstance(o, dict):
            if cls.TAG not in o and all(isinstance(k, str) for k in o):
                return {k: cls._enc(v) for k, v in o.items()}
            return {cls.TAG: "dict", "v": [[cls._enc(k), cls._enc(v)] for k, v in o.items()]}
        if isinstance(o, (bytes, bytearray)):
            return {cls.TAG: "bytes", "v": base64.b64encode(bytes(o)).decode()}
        raise TypeError(f"cannot checkpoint {type(o).__name__} values as JSON: pass key_serde/value_serde "
                        f"to CEPProcessor")

    @classmethod
    def _dec(cls, o):
        if isinstance(o, list):
            return [cls._dec(x) for x in o]
        if not isinstance(o, dict):
            return o
        tag = o.get(cls.TAG)
        if tag is None:
            return {k: cls._dec(v) for k, v in o.items()}
        if tag == "tuple":
            return tuple(cls._dec(x) for x in o["v"])
        if tag == "dict":
            return {cls._dec(k): cls._dec(v) for k, v in o["v"]}
        if tag == "float":
            return float(o["v"])
        if tag == "bytes":
            return base64.b64decode(o["v"])
        if tag == "np":
            return np.dtype(o["dt"]).type(cls._dec(o["v"]))
        raise ValueError(f"unknown checkpoint value tag {tag!r}")

    @classmethod
    def serialize(cls, obj) -> bytes:
        return json.dumps(cls._enc(obj), separators=(",", ":"), allow_nan=False).encode()

    @classmethod
    def deserialize(cls, data: bytes):
        return cls._dec(json.loads(data.decode()))

    @classmethod
    def deserialize_v2(cls, data: bytes):
        """A value a version-2 checkpoint holds: plain JSON (a dict with a "__cep__" key is data)."""
        return json.loads(data.decode())


# ---- Event / Sequence ---------------------------------------------------------------------
class Event:
    """Event.java:27-93: a record and where it came from.  Equality and hash are on
    (topic, partition, offset) only (:48-61); ordering compares offsets within one
    topic partition, timestamps across partitions (:78-92)."""

    __slots__ = ("key", "value", "timestamp", "topic", "partition", "offset")

    def __init__(self, key, value, timestamp: int, topic: str, partition: int, offset: int):
        self.key, self.value, self.timestamp = key, value, int(timestamp)
        self.topic, self.partition, self.offset = topic, int(partition), int(offset)

    def __eq__(self, o):
        return isinstance(o, Event) and (self.topic, self.partition, self.offset) == \
            (o.topic, o.partition, o.offset)

    def __hash__(self):
        return hash((self.topic, self.partition, self.offset))

    def compare_to(self, o: "Event") -> int:
        if self.topic != o.topic or self.partition != o.partition:
            return (self.timestamp > o.timestamp) - (self.timestamp < o.timestamp)
        return (self.offset > o.offset) - (self.offset < o.offset)

    def __lt__(self, o):
        return self.compare_to(o) < 0

    def __repr__(self):
        return (f"Event{{key={self.key}, value={self.value}, timestamp={self.timestamp}, "
                f"topic='{self.topic}', partition={self.partition}, offset={self.offset}}}")


class Sequence:
    """Sequence.java:9-75: events keyed by stage name, in insertion order (a LinkedHashMap)."""

    def __init__(self, mapping=None):
        self._seq: dict[str, list[Event]] = dict(mapping or {})

    def add(self, stage: str, event: Event) -> "Sequence":
        self._seq.setdefault(stage, []).append(event)
        return self

    def get(self, stage: str):
        return self._seq.get(stage)

    def as_map(self) -> dict:
        return self._seq

    asMap = as_map

    def size(self) -> int:
        return sum(len(v) for v in self._seq.values())

    def __eq__(self, o):
        # :59-73 - every stage of this one is in `o` with the same number of events and all
        # of them contained (order-insensitive; one-directional, as in the reference)
        if self is o:
            return True
        if not isinstance(o, Sequence):
            return False
        for stage, events in self._seq.items():
            other = o.get(stage)
            if other is None or len(events) != len(other) or not all(e in other for e in events):
                return False
        return True

    __hash__ = None

    def __repr__(self):
        return "Sequence(" + ", ".join(f"{k}: {[e.offset for e in v]}" for k, v in self._seq.items()) + ")"


# ---- a minimal ProcessorContext -----------------------------------------------------------
class RecordContext:
    """The part of Kafka's `ProcessorContext` the processor uses: the current record's
    topic / partition / offset / timestamp, and `forward(key, value)`.  `send(key, value,
    timestamp)` plays a record into a processor the way a stream task does (offsets count up
    per topic partition).  A real host passes its own context with the same members."""

    def __init__(self, topic: str = "topic", partition: int = 0, stores: dict | None = None):
        """stores: name -> mutable mapping, the context's state stores (Kafka's
        ProcessorContext.getStateStore); pass the same dict to a new context to play a restart
        from persistent stores."""
        self._topic, self._partition = topic, partition
        self.stores = {} if stores is None else stores
        self._offset, self._timestamp = -1, 0
        self.forwarded: list = []
        self.processor = None

    def topic(self):
        return self._topic

    def partition(self):
        return self._partition

    def offset(self):
        return self._offset

    def timestamp(self):
        return self._timestamp

    def forward(self, key, value):
        self.forwarded.append((key, value))

    def get_state_store(self, name: str):
        """ProcessorContext.getStateStore: the store of that name (created empty on first use)"""
        return self.stores.setdefault(name, {})

    getStateStore = get_state_store

    def send(self, key, value, timestamp: int, offset: int | None = None):
        self._offset = self._offset + 1 if offset is None else int(offset)
        self._timestamp = int(timestamp)
        self.processor.process(key, value)


# ---- the processor ------------------------------------------------------------------------
class CEPProcessor:
    """CEPProcessor.java:54-193 over a streaming libcep session (one NFA per key)."""

    def __init__(self, pattern, in_memory: bool = False, *, batch_size: int = 4096,
                 max_keys: int = 1 << 16, device: int = 0, session_factory=None, semantic_within: bool = False,
                 store=None, key_serde=None, value_serde=None):
        """semantic_within: enforce the query's WITHIN on the record timestamps (this build's
        semantic mode, Pattern.to_ir(semantic_within=True)); the default is the reference's
        behaviour, where WITHIN never prunes.  in_memory=False (the reference's default): the
        state is checkpointed to the `_cep_nfa` store at every commit and reloaded by init();
        `store` overrides the context's store; key_serde / value_serde encode the retained
        records' keys and values in the checkpoint (default JsonSerde)."""
        self.pattern = pattern
        self.key_serde = key_serde or JsonSerde
        self.value_serde = value_serde or JsonSerde
        self.in_memory = in_memory  # the reference's store choice (CEPProcessor.java:144-149)
        self._store = store
        self.batch_size = max(1, int(batch_size))
        self.max_keys = int(max_keys)
        self.device = device
        self.schema = pattern.schema
        # the columns of a record value, one C-level getter (process() runs once per record)
        names = tuple(self.schema.names)
        self._get_item = operator.itemgetter(*names) if names else (lambda v: ())
        self._get_attr = operator.attrgetter(*names) if names else (lambda v: ())
        self._one_col = len(names) == 1
        if self.schema is None:
            raise ValueError("the pattern needs an EventSchema (QueryBuilder(schema))")
        self.ir = pattern.to_ir(semantic_within=semantic_within)  # interns string literals first
        self._session_factory = session_factory
        self.context = None
        self.session = None
        self.query = None
        self._key_ids: dict = {}
        self._keys: list = []
        # per key id: the records a later match can still contain, in arrival order; record i of
        # the list has sequence number _ev_base[k] + i; _ev_total[k] records were given so far
        self._events: list[list[Event]] = []
        self._ev_base: list[int] = []
        self._ev_total: list[int] = []
        self._buf_key: list[int] = []
        self._buf_vals: list[tuple] = []
        self._buf_ts: list[int] = []
        self._failed: JavaException | None = None

    # -- Processor API --
    def init(self, context) -> None:
        """CEPProcessor.java:84-106: binds the context and creates the device session
        (the reference creates its stores here and the NFA lazily on the first record)."""
        self.context = context
        if isinstance(context, RecordContext):
            context.processor = self
        if self._session_factory is not None:
            self.session = self._session_factory(self.ir)
        else:
            self.query = N.Query(self.ir)
            self.session = N.Session(self.query, device=self.device, streaming=True)
        self.stage_names = list(getattr(self.session, "stage_names", None) or self.query.stage_names)
        store = self._state_store()
        if store is not None:  # initializeIfNotAndGet :121-131: the NFA as the store holds it
            blob = store.get(self._store_key())
            if blob is not None:
                self.restore(blob)

    # -- persistence (in_memory=False) --
    def _state_store(self):
        if self.in_memory:
            return None
        if self._store is not None:
            return self._store
        get = getattr(self.context, "get_state_store", None) or getattr(self.context, "getStateStore", None)
        return get(NFA_STATES_STORE) if get is not None else None

    def _store_key(self):
        """TopicAndPartition(context.topic(), context.partition()) (CEPProcessor.java:121-122)"""
        return (self.context.topic(), self.context.partition())

    def checkpoint(self) -> bytes:
        """The processor's whole state as one blob: the device session's snapshot (every key's
        NFA) and the retained records with their per-key sequence numbers.  Layout: magic
        "CEPPROC2", u64 length + the session snapshot, then UTF-8 JSON {version, max_keys, ir
        (hex), keys, base, total, events} where keys and values are base64 of their serde's
        bytes and an event is [timestamp, topic, partition, offset, value]."""
        dev = self.session.snapshot()
        b64 = lambda b: base64.b64encode(b).decode()  # noqa: E731
        ks, vs = self.key_serde, self.value_serde
        host = {"version": _CKPT_VERSION, "max_keys": self.max_keys, "ir": self.ir.hex(),
                "keys": [b64(ks.serialize(k)) for k in self._keys],
                "base": [int(x) for x in self._ev_base], "total": [int(x) for x in self._ev_total],
                "events": [[[e.timestamp, e.topic, e.partition, e.offset, b64(vs.serialize(e.value))] for e in evs]
                           for evs in self._events]}
        hb = json.dumps(host, separators=(",", ":")).encode()
        return _CKPT_MAGIC + len(dev).to_bytes(8, "little") + dev + hb

    def restore(self, blob: bytes) -> None:
        """Loads a checkpoint() blob written by a processor over the same pattern.  Nothing in
        the blob is executed: the host half is JSON data, decoded by the serdes."""
        if blob[:8] != _CKPT_MAGIC:
            raise ValueError("not a CEPProcessor checkpoint (or an older, unsupported version)")
        n = int.from_bytes(blob[8:16], "little")
        host = json.loads(blob[16 + n:].decode())
        if not isinstance(host, dict) or host.get("version") not in _CKPT_READABLE:
            raise ValueError("unsupported CEPProcessor checkpoint version")
        if host["ir"] != self.ir.hex() or host["max_keys"] != self.max_keys:
            raise ValueError("checkpoint of another pattern or key space")

        def dec(serde):  # (version 2: the default serde wrote plain JSON)
            if host["version"] == 2 and ((isinstance(serde, type) and issubclass(serde, JsonSerde)) or isinstance(serde, JsonSerde)):
                return serde.deserialize_v2
            return serde.deserialize
        kdec, vdec = dec(self.key_serde), dec(self.value_serde)
        keys = [kdec(base64.b64decode(k)) for k in host["keys"]]
        events = [[Event(k, vdec(base64.b64decode(v)), ts, topic, part, off)
                   for ts, topic, part, off, v in evs] for k, evs in zip(keys, host["events"])]
        if not (len(events) == len(keys) == len(host["base"]) == len(host["total"])):
            raise ValueError("malformed CEPProcessor checkpoint")
        self.session.restore(blob[16:16 + n])
        self._keys = keys
        self._key_ids = {k: i for i, k in enumerate(self._keys)}
        self._events, self._ev_base, self._ev_total = events, [int(x) for x in host["base"]], \
            [int(x) for x in host["total"]]

    def commit(self) -> None:
        """Writes the checkpoint into the `_cep_nfa` store (a no-op in memory)."""
        store = self._state_store()
        if store is not None and self._failed is None:
            store[self._store_key()] = self.checkpoint()

    def process(self, key, value) -> None:
        """CEPProcessor.java:155-163."""
        if self._failed is not None:
            raise self._failed
        if value is None:  # :157
            return
        kid = self._key_ids.get(key)
        if kid is None:
            if len(self._keys) >= self.max_keys:
                raise ValueError(f"more than max_keys={self.max_keys} distinct keys")
            if not self.in_memory:  # the checkpoint must hold this key and its records
                self._check_serde(self.key_serde, key, "key")
                self._check_serde(self.value_serde, value, "value")
            kid = self._key_ids[key] = len(self._keys)
            self._keys.append(key)
            self._events.append([])
            self._ev_base.append(0)
            self._ev_total.append(0)
        ctx = self.context
        ev = Event(key, value, ctx.timestamp(), ctx.topic(), ctx.partition(), ctx.offset())
        self._events[kid].append(ev)
        self._ev_total[kid] += 1
        self._buf_key.append(kid)
        self._buf_vals.append(self._columns_of(value))
        self._buf_ts.append(ev.timestamp)
        if len(self._buf_key) >= self.batch_size:
            self.flush()

    @staticmethod
    def _check_serde(serde, obj, what) -> None:
        """A key (and the first record value of each key) must survive the checkpoint's serde:
        an unsupported type fails at its first record, not at the next commit.  A key must also
        come back equal and hashable (restore() indexes the keys)."""
        try:
            back = serde.deserialize(serde.serialize(obj))
        except Exception as e:
            raise TypeError(f"CEPProcessor checkpoint: the record {what} {obj!r} does not go through "
                            f"{getattr(serde, '__name__', type(serde).__name__)} ({e}); pass "
                            f"{what}_serde=... or in_memory=True") from e
        if what == "key":
            try:
                ok = back == obj and hash(back) == hash(obj)
            except TypeError:
                ok = False
            if not ok:
                raise TypeError(f"CEPProcessor checkpoint: the key {obj!r} comes back from "
                                f"{getattr(serde, '__name__', type(serde).__name__)} as {back!r}")

    def punctuate(self, timestamp: int) -> None:
        """CEPProcessor.java:167-169 (empty there): forwards what is buffered, then commits
        the state to the `_cep_nfa` store (in_memory=False)."""
        self.flush()
        self.commit()

    def close(self) -> None:
        """CEPProcessor.java:172-175: forwards what is buffered, commits, frees the session."""
        try:
            if self.session is not None and self._failed is None:
                self.flush()
                self.commit()
        finally:
            if self.session is not None and hasattr(self.session, "close"):
                self.session.close()
            self.session = None

    # -- batching --
    def _columns_of(self, value) -> tuple:
        S = self.schema
        if S.string_value:
            return (S.encode_literal(value),)
        v = self._get_item(value) if isinstance(value, dict) else self._get_attr(value)
        return (v,) if self._one_col else v

    def flush(self) -> None:
        """Matches the buffered records on the device and forwards the new Sequences."""
        if self._failed is not None:
            raise self._failed
        n = len(self._buf_key)
        if n == 0:
            return
        keys = np.asarray(self._buf_key, np.uint32)
        vals = self._buf_vals
        cols = [np.asarray([v[f] for v in vals], dtype=_DTYPES[t]) for f, t in enumerate(self.schema.types)]
        ts = np.asarray(self._buf_ts, np.int64)
        self._buf_key, self._buf_vals, self._buf_ts = [], [], []
        # per key: the sequence number of its first record in this batch, and the arrival
        # index of each of its records (a stable partition of the batch by key)
        counts = np.bincount(keys, minlength=len(self._keys)).astype(np.int64)
        total = np.asarray(self._ev_total, np.int64)
        before = total - counts
        base = np.asarray(self._ev_base, np.int64)
        by_key = np.argsort(keys, kind="stable")
        start = np.zeros(len(self._keys) + 1, np.int64)
        np.cumsum(counts, out=start[1:])

        try:
            self.session.push_arrival(keys, cols, self.max_keys, ts)
            m = self.session.matches(0)
            code, err_seq = self.session.key_errors(0, self.max_keys)
        except N.CepError as e:
            # the records are consumed (appended above) but the device state is unknown: the
            # processor cannot continue consistently
            self._failed = JavaException(f"libcep failed on a batch of {n} records: {e}")
            raise self._failed from e

        def arrival(k, seq):
            return by_key[start[k] + (np.asarray(seq, np.int64) - before[k])]

        # the first record (in arrival order) whose key threw in this batch
        fail_at, fail_key = n, -1
        for k in np.flatnonzero(code[:len(self._keys)]):
            s = int(err_seq[k])
            if s >= before[k] and s < total[k]:
                a = int(arrival(k, s))
                if a < fail_at:
                    fail_at, fail_key = a, int(k)
            elif s < before[k]:  # (sticky errors are raised when they first appear)
                raise RuntimeError("key error from an earlier batch was not raised")

        nm = int(m["n_matches"])
        if nm:
            mk = m["key"].astype(np.int64)
            emit = by_key[start[mk] + (m["emit_seq"].astype(np.int64) - before[mk])]
            order = np.argsort(emit, kind="stable")
            off = m["pair_off"].astype(np.int64)
            pseq = m["pair_seq"].astype(np.int64)
            pst = m["pair_stage"]
            names = self.stage_names
            fwd = self.context.forward
            for i in order.tolist():
                if emit[i] >= fail_at:
                    break
                evs, b0 = self._events[mk[i]], base[mk[i]]
                seq = Sequence()
                for p in range(off[i], off[i + 1]):
                    seq.add(names[pst[p]], evs[pseq[p] - b0])
                fwd(None, seq)
        if fail_key >= 0:
            c = int(code[fail_key])
            ev = self._events[fail_key][int(err_seq[fail_key]) - int(base[fail_key])]
            exc = _EXC.get(c, JavaException)
            self._failed = exc(f"{exc.__name__} in the NFA of key {self._keys[fail_key]!r} at "
                               f"offset {ev.offset} (cep_key_errors code {c})",
                               key=self._keys[fail_key], event=ev)
            raise self._failed
        self._drop_unreachable(np.flatnonzero(counts))

    def _drop_unreachable(self, touched) -> None:
        """Drops the records of the batch's keys that no live buffer node holds any more
        (cep_live_floor): no later match can contain them."""
        if len(touched) == 0 or not hasattr(self.session, "live_floor"):
            return
        floor = self.session.live_floor(0, len(self._keys))
        for k in touched.tolist():
            keep = min(int(floor[k]), self._ev_total[k])
            cut = keep - self._ev_base[k]
            if cut > 0:
                del self._events[k][:cut]
                self._ev_base[k] = keep

    def retained_records(self) -> int:
        """records held on the host (the ones a later match can still contain)"""
        return sum(len(e) for e in self._events)
