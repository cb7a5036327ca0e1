"""CPU: fixture dumps and debug text through the C ABI.

crdt_awset_format is Go's (AWSet).String() (awset.go:163-171 with
crdt-misc.go:17-19, 57-68) of a packed document; it is checked against the
map-based restatement (oracle/awset_ref.py AWSet.String, %q as
strconv.Quote) on random documents, on keys that need escaping, and on the
golden scenario states.  crdt_batch_dump / crdt_batch_undump round-trip any
batch (slack slots, empty docs) to its compact form and reject a corrupted
image.  The reference never asserts String() output (its tests print it), so
the text format is pinned by the restatement, not by a reference fixture."""

import json
import random

import numpy as np
import pytest

import crdtgpu
from crdtgpu.batch import AWSetBatch
from helpers import GOLDEN, batch_of
from oracle import awset_ref as ref

NAMES = ["a", "b", 'quo"te', "back\\slash", "new\nline", "tab\t", "\x01ctl", "é", "nb sp", "emoji😀", "",
         "z" * 40]


def ref_string(names, ents, vv):
    s = ref.AWSet(0, ref.VersionVector(vv), {names[k]: ref.Dot(a, c) for k, a, c in ents})
    return s.String()


def test_format_matches_reference_string():
    names = sorted(NAMES)  # ids are order-preserving: id order = SortedValues order
    rng = random.Random(1)
    docs = []
    for _ in range(200):
        R = rng.randint(1, 6)
        keys = sorted(rng.sample(range(len(names)), rng.randint(0, len(names))))
        docs.append((R, [(k, rng.randrange(R + 30), rng.randint(0, 10 ** 12)) for k in keys],
                     [rng.randint(0, 2 ** 64 - 1) for _ in range(R)]))
    for R, ents, vv in docs:
        b = batch_of(R, [(ents, vv)])
        assert crdtgpu.format_doc(b, 0, names) == ref_string(names, ents, vv)


def test_format_without_names_and_on_golden_states():
    b = batch_of(2, [([(3, 0, 1), (10, 1, 7)], [2, 9])])
    assert crdtgpu.format_doc(b, 0) == '[(A 2), (B 9)]\n  (A 1)  "#3"\n  (B 7)  "#10"'
    g = json.load(open(GOLDEN))
    for sc in g["scenarios"]:
        for m in sc["merges"]:
            for side in ("dst", "src", "out"):
                st = m[side]
                names = sorted({e[0] for e in st["entries"]})
                ids = {k: i for i, k in enumerate(names)}
                ents = sorted((ids[k], a, c) for k, a, c in st["entries"])
                b = batch_of(len(st["vv"]), [(ents, st["vv"])])
                want = ref.AWSet(0, ref.VersionVector(st["vv"]),
                                 {k: ref.Dot(a, c) for k, a, c in st["entries"]}).String()
                assert crdtgpu.format_doc(b, 0, names) == want


def test_format_truncates_and_reports_length():
    import ctypes

    b = batch_of(2, [([(0, 0, 1)], [1, 0])]).numpy()
    cb = b.c()
    n = ctypes.c_size_t(0)
    buf = ctypes.create_string_buffer(8)
    assert crdtgpu.lib().crdt_awset_format(ctypes.byref(cb), 0, None, buf, 8, ctypes.byref(n)) == 0
    full = '[(A 1), (B 0)]\n  (A 1)  "#0"'
    assert n.value == len(full) and buf.value == full[:7].encode()
    assert crdtgpu.lib().crdt_awset_format(ctypes.byref(cb), 5, None, buf, 8, ctypes.byref(n)) == \
        crdtgpu.CRDT_E_INVALID


def test_dump_round_trip():
    rng = random.Random(2)
    for slack in (0, 3):
        docs = []
        for _ in range(300):
            keys = sorted(rng.sample(range(10 ** 6), rng.choice([0, 1, 5, 64, 200])))
            docs.append(([(k, rng.randrange(4), rng.randint(1, 99)) for k in keys],
                         [rng.randint(0, 2 ** 64 - 1) for _ in range(4)]))
        b = batch_of(4, docs, slack=slack)
        img = crdtgpu.dump_batch(b)
        c = crdtgpu.load_batch(img)
        assert c.n_docs == b.n_docs and c.R == 4
        for d in range(b.n_docs):
            assert c.doc(d) == b.doc(d)
        assert crdtgpu.dump_batch(c) == img  # compact form is a fixed point


def test_dump_rejects_corruption():
    b = batch_of(2, [([(1, 0, 1), (2, 1, 1)], [1, 1])])
    img = bytearray(crdtgpu.dump_batch(b))
    for pos in (0, 9, 30, len(img) - 1):
        bad = bytearray(img)
        bad[pos] ^= 0x40
        with pytest.raises(crdtgpu.CrdtError):
            crdtgpu.load_batch(bytes(bad))
    with pytest.raises(crdtgpu.CrdtError):
        crdtgpu.load_batch(bytes(img[:-1]))
    empty = AWSetBatch(2, np.zeros(1, np.uint32), np.zeros(1, np.uint64), np.zeros(1, np.uint32),
                       np.zeros(1, np.uint64), np.zeros(1, np.uint64))
    assert crdtgpu.load_batch(crdtgpu.dump_batch(empty)).n_docs == 0


def test_image_parser_fuzz_under_sanitizers():
    """crdt_batch_info / crdt_batch_undump parse images a caller may not
    control: tests/cpp/fuzz_serial.cpp mutates dumped images (header fields,
    offsets, lengths, bytes) and re-signs the checksum so the parser's own
    checks are what stands between a bad image and the output arrays; images
    sit at misaligned addresses too.  Built with ASan + UBSan (host code only,
    host/Makefile build/fuzz_serial): any report aborts with a non-zero exit."""
    import os
    import subprocess

    exe = os.path.join(os.path.dirname(crdtgpu.__file__), "..", "host", "build", "fuzz_serial")
    if not os.path.exists(exe):
        subprocess.check_call(["make", "-s", "-C", os.path.dirname(os.path.dirname(exe)), "build/fuzz_serial"])
    for seed in (1, 2, 3):
        r = subprocess.run([exe, "30000", str(seed)], capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
        assert r.stdout.startswith("ok:"), r.stdout
