"""Writes tests/golden/reference_kats.json — the reference's own known-answer vectors.

Every value below is transcribed (as data) from the reference's tests and README; nothing is
computed here, so the fixture is independent of the oracle it pins.
  test:  = /root/reference/src/test/java/com/github/fhuz/kafka/streams/cep/
Run: python tests/golden/make_golden.py
"""
import json
import os

ABC = ["A", "B", "C", "C", "D"]  # test:nfa/NFATest.java:35-39 (offsets 0..4)
STOCK = [  # test:nfa/NFATest.java:206-213 == README.md:73-80 (e1..e8, offsets 0..7)
    [100, 1010], [120, 990], [120, 1005], [121, 999], [120, 999], [125, 750], [120, 950], [120, 700],
]

KATS = {
    "nfa_strict_one_run": {
        "source": "test:nfa/NFATest.java:41-67",
        "events": ABC[:3],
        # expected Sequence: first=[ev1], second=[ev2], latest=[ev3]
        "expected": [{"first": [0], "second": [1], "latest": [2]}],
    },
    "nfa_strict_kleene": {
        "source": "test:nfa/NFATest.java:69-101",
        "events": ABC,
        "expected": [{"firstStage": [0], "secondStage": [1], "thirdStage": [2, 3], "latestState": [4]}],
    },
    "nfa_skip_till_next": {
        "source": "test:nfa/NFATest.java:104-132",
        "events": ABC,
        "expected": [{"first": [0], "second": [2], "latest": [4]}],
    },
    "nfa_skip_till_any": {
        "source": "test:nfa/NFATest.java:134-172",
        "events": ABC,
        # s.get(0) then s.get(1): order is asserted
        "expected": [{"first": [0], "second": [1], "three": [2], "latest": [4]},
                     {"first": [0], "second": [1], "three": [3], "latest": [4]}],
    },
    "stock_test_zero_or_more": {
        "source": "test:nfa/NFATest.java:203-245 (int fields, zeroOrMore, getOrElse)",
        "events": STOCK,
        "expected_count": 4,
    },
    "stock_readme": {
        "source": "README.md:33-49 (query, oneOrMore, int casts), README.md:71-96 (input/output)",
        "events": STOCK,
        # README.md:93-96, in forward order; e1..e8 -> offsets 0..7
        "expected": [{"0": [0], "1": [1, 2, 3, 4], "2": [5]},
                     {"0": [2], "1": [3], "2": [5]},
                     {"0": [0], "1": [1, 2, 3, 4, 5, 6], "2": [7]},
                     {"0": [2], "1": [3, 5], "2": [7]}],
        "ordered": True,
    },
    "stock_demo_long": {
        "source": "test:demo/CEPStockKStreamsDemo.java:37-53 (long fields, zeroOrMore) on README input",
        "events": STOCK,
        "expected": [{"0": [0], "1": [1, 2, 3, 4], "2": [5]},
                     {"0": [2], "1": [3], "2": [5]},
                     {"0": [0], "1": [1, 2, 3, 4, 5, 6], "2": [7]},
                     {"0": [2], "1": [3, 5], "2": [7]}],
        "ordered": True,
    },
    "dewey": {
        "source": "test:nfa/DeweyVersionTest.java:8-44",
        "apply": [["1", "", "1"], ["1.0.1", "", "1.0.1"], ["1", "r", "2"], ["1", "sr", "1.1"], ["1", "s", "1.0"]],
        "compatible": [["1.0", "2.0", False], ["1.0.0", "1.0", True], ["1.1", "1.0", True], ["1.0", "1.1", False]],
    },
    "buffer_one_run": {
        "source": "test:nfa/buffer/SharedVersionedBufferTest.java:28-41",
        # stages: first=(0,BEGIN), second=(1,NORMAL), latest=(2,FINAL)
        "puts": [["first", 0, None, None, "1"], ["second", 1, "first", 0, "1.0"], ["latest", 2, "second", 1, "1.0.0"]],
        "gets": [[["latest", 2, "1.0.0"], {"size": 3, "latest": 1, "second": 1, "first": 1}]],
    },
    "buffer_branching_run": {
        "source": "test:nfa/buffer/SharedVersionedBufferTest.java:43-68",
        "puts": [["first", 0, None, None, "1"], ["second", 1, "first", 0, "1.0"], ["latest", 2, "second", 1, "1.0.0"],
                 ["second", 2, "second", 1, "1.1"], ["second", 3, "second", 2, "1.1"], ["latest", 4, "second", 3, "1.1.0"]],
        "gets": [[["latest", 2, "1.0.0"], {"size": 3, "latest": 1, "second": 1, "first": 1}],
                 [["latest", 4, "1.1.0"], {"size": 5, "latest": 1, "second": 3, "first": 1}]],
    },
}

if __name__ == "__main__":
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "reference_kats.json")
    with open(path, "w") as f:
        json.dump(KATS, f, indent=1)
    print("wrote", path)
