"""CPU: bench.py reports a PMC traffic figure only for exactly what it times
(a stale entry of the same kernel family must never stand in)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from crdtgpu.srcid import source_id  # noqa: E402


class _W:
    exchange = True
    shared_keys = True
    kernel = "join_wave_kernel"
    kernel_instance = "join_wave_kernel<4, 8, 2, true, true>"
    tus = ("join.hip",)


def _entry(**kw):
    e = {"docs": 1 << 20, "config": 2, "kernel": _W.kernel_instance, "exchange": True, "shared_keys": True,
         "src_id": source_id(_W.tus), "hbm_bytes_per_launch": 123.0, "profile": "profiles/x.txt"}
    e.update(kw)
    return e


def _lookup(tmp_path, entries):
    p = tmp_path / "traffic.json"
    p.write_text(json.dumps(entries))
    return bench._traffic(str(p), 2, 1 << 20, _W())


def test_exact_entry_is_reported(tmp_path):
    b, note, e = _lookup(tmp_path, [_entry()])
    assert b == 123.0 and e is not None and "profiles/x.txt" in note


def test_stale_source_id_is_not_reported(tmp_path):
    b, note, _ = _lookup(tmp_path, [_entry(src_id="0000000000000000")])
    assert b is None and "source id" in note


def test_same_family_other_instance_is_not_reported(tmp_path):
    b, _, _ = _lookup(tmp_path, [_entry(kernel="join_wave_kernel<4, 8, 2, true>")])
    assert b is None
    b, _, _ = _lookup(tmp_path, [_entry(shared_keys=False)])
    assert b is None
    b, _, _ = _lookup(tmp_path, [_entry(docs=1000)])
    assert b is None


def test_source_id_follows_the_translation_unit_and_its_headers():
    j, f, t = source_id(("join.hip",)), source_id(("fold.hip",)), source_id(("join.hip", "tile.hip"))
    assert len({j, f, t}) == 3 and all(len(x) == 16 for x in (j, f, t))
    assert source_id(("join.hip",)) == j  # deterministic


def test_committed_traffic_table_parses():
    table = json.load(open(os.path.join(ROOT, "profiles", "traffic.json")))
    assert isinstance(table, list) and all("kernel" in e and "docs" in e for e in table)


def test_committed_table_covers_every_timed_kernel_at_this_tree():
    """Every bench leg's dominant kernel, at the source id of this tree, has its
    PMC entry in profiles/traffic.json -- so the line's roofline.traffic comes
    from a profile of exactly these sources (a kernel edit needs
    `tools/gpu_run.sh pmcall` before this passes again)."""
    path = os.path.join(ROOT, "profiles", "traffic.json")
    for c, cls in ((2, bench.Config2), (3, bench.Config3), (4, bench.Config4), (5, bench.Config5)):
        W = object.__new__(cls)  # class defaults: the forms the bench times
        b, note, e = bench._traffic(path, c, bench.DEFAULT_DOCS[c], W)
        assert b is not None, "config %d: %s" % (c, note)
        assert os.path.exists(os.path.join(ROOT, e["profile"])), e["profile"]
