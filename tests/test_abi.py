"""CPU: the C-ABI library loads, exports every symbol include/crdtgpu.h
declares, and its host-only entry points (validation, strerror) behave.  No
compute call is made here (no GPU in this container)."""

import ctypes
import os

import numpy as np
import pytest

import crdtgpu
from crdtgpu import abi
from crdtgpu.batch import AWSetBatch, SrcBatch
from helpers import batch_of, src_batch_of


def test_exports_every_header_symbol():
    names = crdtgpu.header_functions()
    assert len(names) >= 15
    lib = ctypes.CDLL(crdtgpu.LIB_PATH)
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing


def test_abi_version_and_strerror():
    assert crdtgpu.lib().crdt_abi_version() == 1
    for code in (0, -1, -2, -3, -4, -5, -6, -7, -8, -9):
        assert crdtgpu.strerror(code) != "unknown error"
    assert "panic" in crdtgpu.strerror(crdtgpu.CRDT_E_ACTOR_RANGE)


def test_struct_layouts():
    # pointer-sized fields after two u32: offsets at 8 (no padding surprises)
    assert ctypes.sizeof(abi.CAWSetBatch) == 8 + 6 * 8
    assert ctypes.sizeof(abi.CAWSetOut) == 6 * 8
    assert ctypes.sizeof(abi.CSrcBatch) == 8 + 11 * 8
    assert abi.CAWSetBatch.offsets.offset == 8


def test_validate_batch():
    good = batch_of(2, [([(1, 0, 1), (4, 1, 2)], [1, 2]), ([], [0, 0])])
    assert crdtgpu.validate(good) == 0
    unsorted = batch_of(2, [([(4, 0, 1), (1, 1, 2)], [1, 2])])
    assert crdtgpu.validate(unsorted) == crdtgpu.CRDT_E_UNSORTED
    dup = batch_of(2, [([(4, 0, 1), (4, 1, 2)], [1, 2])])
    assert crdtgpu.validate(dup) == crdtgpu.CRDT_E_UNSORTED
    over = batch_of(2, [([(1, 0, 1)], [1, 0])], slack=1)
    over.counts[0] = 5
    assert crdtgpu.validate(over) == crdtgpu.CRDT_E_CAPACITY
    wide = AWSetBatch(65, good.offsets, good.keys, good.actors, good.counters, np.zeros(130, np.uint64))
    assert crdtgpu.validate(wide) == crdtgpu.CRDT_E_INVALID


def test_validate_src_batch():
    ok = src_batch_of(2, [[(0, [1, 0], [(1, 0, 1)], [(2, 0, 1)])], []])
    assert crdtgpu.validate_src(ok) == 0
    bad = src_batch_of(2, [[(0, [1, 0], [(3, 0, 1), (1, 0, 1)], [])]])
    assert crdtgpu.validate_src(bad) == crdtgpu.CRDT_E_UNSORTED
    badt = src_batch_of(2, [[(0, [1, 0], [], [(3, 0, 1), (3, 0, 2)])]])
    assert crdtgpu.validate_src(badt) == crdtgpu.CRDT_E_UNSORTED


def test_validate_tomb_batch():
    from crdtgpu.batch import TombBatch
    from crdtgpu.engine import validate_tombs

    u32, u64 = np.uint32, np.uint64

    def tb(offs, keys, counts=None):
        n = len(keys)
        return TombBatch(np.array(offs, u32), np.array(keys, u64), np.zeros(n, u32), np.ones(n, u64),
                         None if counts is None else np.array(counts, u32))

    assert validate_tombs(tb([0, 2, 3], [1, 5, 2]), 2) == 0
    assert validate_tombs(tb([0, 2, 3], [5, 1, 2]), 2) == crdtgpu.CRDT_E_UNSORTED
    assert validate_tombs(tb([0, 2, 3], [1, 1, 2]), 2) == crdtgpu.CRDT_E_UNSORTED
    assert validate_tombs(tb([0, 2, 3], [1, 5, 2], counts=[3, 1]), 2) == crdtgpu.CRDT_E_CAPACITY
    assert validate_tombs(tb([0, 3, 2], [1, 2, 5]), 2) == crdtgpu.CRDT_E_INVALID
    # counts below capacity: the unsorted tail past the live count is not read
    assert validate_tombs(tb([0, 3, 3], [1, 5, 0], counts=[2, 0]), 2) == 0


def test_product_has_no_cpu_fallback():
    """The product package must not import the oracle or ship a CPU merge."""
    import os
    import re

    pkg = os.path.dirname(crdtgpu.__file__)
    for fn in os.listdir(pkg):
        if fn.endswith(".py"):
            src = open(os.path.join(pkg, fn)).read()
            assert not re.search(r"\boracle\b", src.replace("oracle/", "")), fn


def test_batch_roundtrip_numpy():
    b = batch_of(3, [([(1, 0, 1), (9, 2, 7)], [1, 0, 7]), ([(2, 1, 1)], [0, 1, 0])])
    assert b.n_docs == 2 and b.live(0) == 2 and b.live(1) == 1
    assert b.doc(0) == ([(1, 0, 1), (9, 2, 7)], [1, 0, 7])
    s = SrcBatch.from_lists(3, [[(1, [0, 1, 0], [(2, 1, 1)], None)], []])
    assert s.n_docs == 2 and s.n_srcs == 1 and s.out_slots(b) == 4


def test_engine_needs_a_gpu_or_works():
    try:
        import torch

        has_gpu = torch.cuda.is_available()
    except Exception:  # pragma: no cover
        has_gpu = False
    if has_gpu:
        pytest.skip("GPU present: covered by -m gpu")
    with pytest.raises(crdtgpu.CrdtError):
        crdtgpu.Engine(0)


def test_single_hip_runtime_in_process():
    """torch and libcrdtgpu.so must share one HIP runtime (torch streams are passed in)."""
    assert len(abi.hip_runtimes_mapped()) <= 1, abi.hip_runtimes_mapped()


def test_go_binding_calls_declared_entry_points():
    """go/crdtgpu/crdtgpu.go (not compiled here: no Go toolchain) calls only C
    names that include/crdtgpu.h declares, and binds the batch entry points."""
    import re

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    go = open(os.path.join(root, "go", "crdtgpu", "crdtgpu.go")).read()
    hdr = open(os.path.join(root, "include", "crdtgpu.h")).read()
    used = set(re.findall(r"\bC\.(crdt_\w+|CRDT_\w+)", go))
    assert used
    for name in used:
        assert re.search(r"\b%s\b" % name, hdr), name
    for must in ("crdt_awset_join_batch", "crdt_awset_exchange_batch", "crdt_awset_fold_batch", "crdt_host_alloc"):
        assert must in used
    code = re.sub(r'//[^\n]*|"(?:[^"\\]|\\.)*"', "", go)  # comments and string literals out
    assert code.count("{") == code.count("}") and code.count("(") == code.count(")")


def _header_api():
    """include/crdtgpu.h -> ({function: n_params}, {struct typedef: [field names]})."""
    import re

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    hdr = open(os.path.join(root, "include", "crdtgpu.h")).read()
    hdr = re.sub(r"/\*.*?\*/", "", hdr, flags=re.S)
    hdr = re.sub(r"//[^\n]*", "", hdr)
    funcs = {}
    for m in re.finditer(r"\b(crdt_\w+)\s*\(([^;{]*?)\)\s*;", hdr, flags=re.S):
        params = m.group(2).strip()
        funcs[m.group(1)] = 0 if params in ("", "void") else params.count(",") + 1
    structs = {}
    for m in re.finditer(r"typedef\s+struct\s*\{(.*?)\}\s*(crdt_\w+)\s*;", hdr, flags=re.S):
        structs[m.group(2)] = re.findall(r"(\w+)\s*(?:\[[^\]]*\])?\s*;", m.group(1))
    return funcs, structs


def _go_calls(code):
    """(name, n_args) of every C.crdt_*(...) call in Go source (comments/strings removed)."""
    import re

    out = []
    for m in re.finditer(r"\bC\.(crdt_\w+)\(", code):
        i, depth, args, cur = m.end(), 1, 0, ""
        while depth:
            ch = code[i]
            if ch in "([{":
                depth += 1
            elif ch in ")]}":
                depth -= 1
            elif ch == "," and depth == 1:
                args += 1
            if depth:
                cur += ch
            i += 1
        out.append((m.group(1), 0 if not cur.strip() else args + 1))
    return out


def test_go_binding_matches_header_and_python_abi():
    """go/crdtgpu/crdtgpu.go is never compiled here (no Go toolchain), so its
    drift against the C ABI is checked by parsing: every C.crdt_* call passes
    as many arguments as include/crdtgpu.h declares (and as crdtgpu/abi.py
    binds, where both bind it); every field it names on a C.crdt_* struct --
    in composite literals and on variables of those types -- is a field of
    that struct in the header."""
    import re

    funcs, structs = _header_api()
    assert {"crdt_awset_join_batch", "crdt_awset_exchange_batch", "crdt_awset_fold_batch"} <= set(funcs)
    assert set(structs) >= {"crdt_awset_batch", "crdt_awset_out", "crdt_src_batch"}
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    go = open(os.path.join(root, "go", "crdtgpu", "crdtgpu.go")).read()
    code = re.sub(r'//[^\n]*|"(?:[^"\\]|\\.)*"', "", go)
    sigs = abi.signatures()
    calls = _go_calls(code)
    assert len(calls) >= 8
    for name, n in calls:
        assert name in funcs, name
        assert n == funcs[name], "%s: Go passes %d arguments, the header declares %d" % (name, n, funcs[name])
        if name in sigs:
            assert len(sigs[name][1]) == n, "%s: abi.py binds %d arguments" % (name, len(sigs[name][1]))
    # every Python binding agrees with the header too
    for name, (_, args) in sigs.items():
        assert funcs.get(name) == len(args), name
    # struct fields in composite literals: C.crdt_x{field: ..., field: ...}
    seen = 0
    for m in re.finditer(r"\bC\.(crdt_\w+)\{", code):
        i, depth, body = m.end(), 1, ""
        while depth:
            ch = code[i]
            depth += ch == "{"
            depth -= ch == "}"
            if depth:
                body += ch
            i += 1
        for f in re.findall(r"(?:^|[,{\s])(\w+)\s*:", body):
            assert f in structs[m.group(1)], "%s has no field %s" % (m.group(1), f)
            seen += 1
    # fields on variables / struct members declared with a C.crdt_* struct type
    bound = []  # (access pattern, struct): locals by name, struct members through their owner
    for m in re.finditer(r"(\.?)\b(\w+)\s*(?::=|=)\s*C\.(crdt_\w+)\{", code):
        owner = r"\w\." if m.group(1) else r"(?<![\w.])"
        bound.append((r"%s%s\.([a-z_]\w*)" % (owner, m.group(2)), m.group(3)))
    for m in re.finditer(r"^\s*(\w+)\s+C\.(crdt_\w+)\s*$", code, flags=re.M):
        bound.append((r"\w\.%s\.([a-z_]\w*)" % m.group(1), m.group(2)))
    for pat, st in bound:
        if st not in structs:
            continue
        for f in re.findall(pat, code):
            assert f in structs[st], "%s (%s) has no field %s" % (pat, st, f)
            seen += 1
    assert seen >= 20
