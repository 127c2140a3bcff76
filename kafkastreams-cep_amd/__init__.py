"""kafkastreams-cep_amd — MI355X-native drop-in for the reference's CEP matching path.

Query API (mirrors pattern/QueryBuilder.java & co.): QueryBuilder, Pattern, Matcher, J,
EventSchema, TimeUnit.  Processor: CEPProcessor / Sequence / Event (processor.py, after
CEPProcessor.java, Sequence.java, Event.java).  Engine: the C-ABI session in `native`
(libcep.so, include/cep.h) running hand-written HIP kernels on gfx950.
"""
from .expr import J, Matcher  # noqa: F401
from .pattern import (Cardinality, Pattern, PredicateBuilder, QueryBuilder,  # noqa: F401
                      SelectBuilder, SelectStrategy, TimeUnit)
from .processor import CEPProcessor, Event, RecordContext, Sequence  # noqa: F401
from .schema import EventSchema  # noqa: F401

__all__ = ["J", "Matcher", "Cardinality", "Pattern", "PredicateBuilder", "QueryBuilder",
           "SelectBuilder", "SelectStrategy", "TimeUnit", "EventSchema", "CEPProcessor", "Event",
           "RecordContext", "Sequence"]
