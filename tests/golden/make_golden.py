#!/usr/bin/env python3
"""Generate tests/golden/kat_scenarios.json from the reference's own tests.

Each scenario below is the op sequence of one reference test, written as data:

  KAT-1 TestAWSetXXX                       awset_test.go:10-29
  KAT-2 TestAWSet                          awset_test.go:31-83
  KAT-3 TestAWSetConcurrentAddWinsOverDelete awset_test.go:85-122
  KAT-4 TestAWSetCommutativity             awset_test.go:124-154
  KAT-5 TestAWSetDelta                     awset-delta_test.go:168-189
  KAT-6 TestVersionVector                  crdt-misc_test.go:5-28

Replaying uses the map-based restatement ``oracle/awset_ref.py``.  Two kinds of
check pin it:
  * ``assert_entries`` steps are the reference tests' own assertions (sorted
    element sets) -- these are what the reference pins;
  * ``expect`` blocks are the dot/version-vector hand traces of SURVEY.md
    section 4.1 (the reference's tests never assert dots or clocks).
Every merge step's (dst, src) -> dst' states are written out as golden vectors
for the batched kernels.  Run from the repo root: ``python tests/golden/make_golden.py``.
"""

from __future__ import annotations

import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle.awset_ref import AWSet, AWSetDelta, Dot, VersionVector, snapshot  # noqa: E402

A, B = 0, 1


def D(actor, counter):
    return [actor, counter]


# Each step: ("add", r, keys) | ("del", r, keys) | ("merge", dst, src) |
# ("clone", new, old) | ("assert_entries", r, values) |
# ("expect", r, {key: (actor, counter)}, vv)
SCENARIOS = [
    {
        "name": "KAT-1 TestAWSetXXX",
        "ref": "awset_test.go:10-29",
        "kind": "awset",
        "steps": [
            ("add", "A", ["A", "B", "C"]),
            ("add", "B", ["A", "B", "C"]),
            ("merge", "A", "B"),
            ("expect", "A", {"A": D(B, 1), "B": D(B, 2), "C": D(B, 3)}, [3, 3]),
            ("merge", "B", "A"),
            ("expect", "B", {"A": D(B, 1), "B": D(B, 2), "C": D(B, 3)}, [3, 3]),
            ("assert_entries", "A", ["A", "B", "C"]),
            ("assert_entries", "B", ["A", "B", "C"]),
            ("del", "A", ["B"]),
            ("add", "B", ["B"]),
            ("merge", "B", "A"),
            ("merge", "A", "B"),
            ("assert_entries", "A", ["A", "B", "C"]),
            ("assert_entries", "B", ["A", "B", "C"]),
            ("expect", "A", {"A": D(B, 1), "B": D(B, 4), "C": D(B, 3)}, [3, 4]),
            ("expect", "B", {"A": D(B, 1), "B": D(B, 4), "C": D(B, 3)}, [3, 4]),
        ],
    },
    {
        "name": "KAT-2 TestAWSet",
        "ref": "awset_test.go:31-83",
        "kind": "awset",
        "steps": [
            ("assert_entries", "A", []),
            ("assert_entries", "B", []),
            ("add", "A", ["Shelly"]),
            ("assert_entries", "A", ["Shelly"]),
            ("assert_entries", "B", []),
            ("merge", "B", "A"),
            ("expect", "B", {"Shelly": D(A, 1)}, [1, 0]),
            ("assert_entries", "A", ["Shelly"]),
            ("assert_entries", "B", ["Shelly"]),
            ("add", "B", ["Bob", "Phil", "Pete"]),
            ("assert_entries", "A", ["Shelly"]),
            ("assert_entries", "B", ["Shelly", "Bob", "Phil", "Pete"]),
            ("merge", "A", "B"),
            ("expect", "A", {"Shelly": D(A, 1), "Bob": D(B, 1), "Phil": D(B, 2), "Pete": D(B, 3)}, [1, 3]),
            ("assert_entries", "A", ["Shelly", "Bob", "Phil", "Pete"]),
            ("assert_entries", "B", ["Shelly", "Bob", "Phil", "Pete"]),
            ("del", "A", ["Phil"]),
            ("add", "A", ["Bob"]),
            ("add", "A", ["Anna"]),
            ("expect", "A", {"Shelly": D(A, 1), "Bob": D(A, 2), "Pete": D(B, 3), "Anna": D(A, 3)}, [3, 3]),
            ("assert_entries", "A", ["Shelly", "Bob", "Pete", "Anna"]),
            ("assert_entries", "B", ["Shelly", "Bob", "Phil", "Pete"]),
            ("merge", "B", "A"),
            ("expect", "B", {"Shelly": D(A, 1), "Bob": D(A, 2), "Pete": D(B, 3), "Anna": D(A, 3)}, [3, 3]),
            ("assert_entries", "A", ["Shelly", "Bob", "Pete", "Anna"]),
            ("assert_entries", "B", ["Shelly", "Bob", "Pete", "Anna"]),
            ("del", "A", ["Bob", "Pete"]),
            ("del", "B", ["Bob", "Shelly"]),
            ("merge", "A", "B"),
            ("expect", "A", {"Anna": D(A, 3)}, [3, 3]),
            ("merge", "B", "A"),
            ("expect", "B", {"Anna": D(A, 3)}, [3, 3]),
            ("assert_entries", "A", ["Anna"]),
            ("assert_entries", "B", ["Anna"]),
            ("add", "A", ["A", "B", "C"]),
            ("del", "A", ["A"]),
            ("add", "A", ["A"]),
            ("merge", "B", "A"),
            ("expect", "B", {"Anna": D(A, 3), "A": D(A, 7), "B": D(A, 5), "C": D(A, 6)}, [7, 3]),
            ("assert_entries", "A", ["Anna", "A", "B", "C"]),
            ("assert_entries", "B", ["Anna", "A", "B", "C"]),
        ],
    },
    {
        "name": "KAT-3 TestAWSetConcurrentAddWinsOverDelete",
        "ref": "awset_test.go:85-122",
        "kind": "awset",
        "steps": [
            ("add", "A", ["Anne", "Bob"]),
            ("add", "B", ["Anne"]),
            # fork (awset_test.go:104): shadowed clones
            ("clone", "A'", "A"),
            ("clone", "B'", "B"),
            ("add", "B'", ["Bob"]),
            ("del", "A'", ["Bob"]),
            ("merge", "B'", "A'"),
            ("expect", "B'", {"Anne": D(A, 1), "Bob": D(B, 2)}, [2, 2]),
            ("merge", "A'", "B'"),
            ("expect", "A'", {"Anne": D(A, 1), "Bob": D(B, 2)}, [2, 2]),
            ("assert_entries", "B'", ["Anne", "Bob"]),
            ("assert_entries", "A'", ["Anne", "Bob"]),
            # main line (awset_test.go:114-121)
            ("add", "B", ["Bob"]),
            ("merge", "B", "A"),
            ("expect", "B", {"Anne": D(A, 1), "Bob": D(A, 2)}, [2, 2]),
            ("del", "A", ["Bob"]),
            ("merge", "B", "A"),
            ("expect", "B", {"Anne": D(A, 1)}, [2, 2]),
            ("merge", "A", "B"),
            ("expect", "A", {"Anne": D(A, 1)}, [2, 2]),
            ("assert_entries", "B", ["Anne"]),
            ("assert_entries", "A", ["Anne"]),
        ],
    },
    {
        "name": "KAT-4 TestAWSetCommutativity",
        "ref": "awset_test.go:124-154",
        "kind": "awset",
        "steps": [
            ("add", "A", ["Shelly", "Bob", "Pete", "Anna"]),
            ("add", "B", ["Shelly", "Bob", "Pete", "Anna"]),
            ("del", "A", ["Anna"]),
            ("add", "B", ["Anna"]),
            ("assert_entries", "A", ["Shelly", "Bob", "Pete"]),
            ("assert_entries", "B", ["Shelly", "Bob", "Pete", "Anna"]),
            ("clone", "A'", "A"),
            ("clone", "B'", "B"),
            ("merge", "B'", "A'"),
            ("merge", "A'", "B'"),
            ("assert_entries", "A'", ["Shelly", "Bob", "Pete", "Anna"]),
            ("assert_entries", "B'", ["Shelly", "Bob", "Pete", "Anna"]),
            ("expect", "A'", {"Shelly": D(A, 1), "Bob": D(A, 2), "Pete": D(A, 3), "Anna": D(B, 5)}, [4, 5]),
            ("expect", "B'", {"Shelly": D(A, 1), "Bob": D(A, 2), "Pete": D(A, 3), "Anna": D(B, 5)}, [4, 5]),
            ("merge", "A", "B"),
            ("merge", "B", "A"),
            ("assert_entries", "A", ["Shelly", "Bob", "Pete", "Anna"]),
            ("assert_entries", "B", ["Shelly", "Bob", "Pete", "Anna"]),
            ("expect", "A", {"Shelly": D(B, 1), "Bob": D(B, 2), "Pete": D(B, 3), "Anna": D(B, 5)}, [4, 5]),
            ("expect", "B", {"Shelly": D(B, 1), "Bob": D(B, 2), "Pete": D(B, 3), "Anna": D(B, 5)}, [4, 5]),
        ],
    },
    {
        "name": "KAT-5 TestAWSetDelta",
        "ref": "awset-delta_test.go:168-189",
        "kind": "awset_delta",
        "steps": [
            ("add", "A", ["A", "B"]),
            ("add", "B", ["A", "C"]),
            ("merge", "A", "B"),  # first contact: full merge
            ("expect", "A", {"A": D(B, 1), "B": D(A, 2), "C": D(B, 2)}, [2, 2]),
            ("merge", "B", "A"),
            ("expect", "B", {"A": D(B, 1), "B": D(A, 2), "C": D(B, 2)}, [2, 2]),
            ("assert_entries", "A", ["A", "B", "C"]),
            ("assert_entries", "B", ["A", "B", "C"]),
            ("del", "A", ["B"]),
            ("add", "A", ["D", "E"]),
            ("add", "B", ["E"]),
            ("merge", "B", "A"),  # delta path
            ("expect", "B", {"A": D(B, 1), "C": D(B, 2), "D": D(A, 4), "E": D(A, 5)}, [5, 3]),
            ("assert_entries", "B", ["A", "C", "D", "E"]),
            ("merge", "A", "B"),  # delta path, changed={} deleted={} -> no-op, VV untouched
            ("expect", "A", {"A": D(B, 1), "C": D(B, 2), "D": D(A, 4), "E": D(A, 5)}, [5, 2]),
            ("assert_entries", "A", ["A", "C", "D", "E"]),
        ],
    },
]


def replay(sc):
    cls = AWSetDelta if sc["kind"] == "awset_delta" else AWSet
    reps = {
        "A": cls(0, VersionVector([0, 0])),
        "B": cls(1, VersionVector([0, 0])),
    }
    merges = []
    checks = 0
    for st in sc["steps"]:
        op = st[0]
        if op == "add":
            reps[st[1]].Add(*st[2])
        elif op == "del":
            reps[st[1]].Del(*st[2])
        elif op == "clone":
            reps[st[1]] = reps[st[2]].Clone()
        elif op == "merge":
            dst, src = reps[st[1]], reps[st[2]]
            pre_dst, pre_src = snapshot(dst), snapshot(src)
            dst.Merge(src)
            merges.append({"dst_name": st[1], "src_name": st[2], "dst": pre_dst, "src": pre_src, "out": snapshot(dst)})
        elif op == "assert_entries":
            got = reps[st[1]].SortedValues()
            want = sorted(st[2])
            assert got == want, (sc["name"], st, got)
            checks += 1
        elif op == "expect":
            r = reps[st[1]]
            got = {k: [d.actor, d.counter] for k, d in r.Entries.items()}
            assert got == st[2], (sc["name"], st, got)
            assert list(r.VersionVector) == st[3], (sc["name"], st, list(r.VersionVector))
            checks += 1
        else:
            raise ValueError(op)
    return merges, checks, reps


def kat6():
    # crdt-misc_test.go:23-27
    a, b = VersionVector([1, 1, 0, 4]), VersionVector([2, 0, 3, 0])
    a.Merge(b)
    assert list(a) == [2, 1, 3, 4]
    b.Merge(a)
    assert list(b) == [2, 1, 3, 4]
    return {"a": [1, 1, 0, 4], "b": [2, 0, 3, 0], "a_merge_b": [2, 1, 3, 4], "b_merge_a": [2, 1, 3, 4]}


def main():
    out = {"generator": "tests/golden/make_golden.py", "oracle": "oracle/awset_ref.py", "scenarios": []}
    total = 0
    for sc in SCENARIOS:
        merges, checks, reps = replay(sc)
        total += checks
        out["scenarios"].append({
            "name": sc["name"],
            "ref": sc["ref"],
            "kind": sc["kind"],
            "steps": [list(s) for s in sc["steps"]],
            "merges": merges,
            "final": {k: snapshot(v) for k, v in sorted(reps.items())},
        })
    out["version_vector"] = kat6()
    path = os.path.join(HERE, "kat_scenarios.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
        f.write("\n")
    print("wrote %s: %d scenarios, %d merges, %d checks" % (
        path, len(out["scenarios"]), sum(len(s["merges"]) for s in out["scenarios"]), total))


if __name__ == "__main__":
    main()
