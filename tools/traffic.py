#!/usr/bin/env python3
"""Summarise the rocprofv3 PMC passes of tools/pmc.sh.

Per kernel: mean counter value per dispatch.  HBM traffic of the join kernel is
FETCH_SIZE + WRITE_SIZE (KiB units), corrected by the known-byte calibration run
(tools/calib.py: vv_max_kernel, 8 B per lane): correction = known bytes /
counted bytes, applied per direction (the guide's gfx950 note: FETCH_SIZE counts
half of a wide coalesced stream; other widths must be calibrated).
Writes <dir>/traffic.json and, with --emit, adds the entry to profiles/traffic.json.
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict


def load(d):
    vals = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> [per dispatch]
    for fn in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        per = defaultdict(float)
        names = {}
        with open(fn) as f:
            for row in csv.DictReader(f):
                key = (row.get("Dispatch_Id") or row.get("Correlation_Id"), row["Counter_Name"])
                per[key] += float(row["Counter_Value"])
                names[key[0]] = row["Kernel_Name"]
        for (disp, cname), v in per.items():
            vals[names[disp]][cname].append(v)
    return vals


def short(k):
    return k.split("(")[0].replace("void ", "").replace("crdt::", "")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--docs", type=int, default=1 << 20)
    ap.add_argument("--emit", action="store_true")
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--kernel", default="join_wave_kernel")
    ap.add_argument("--shared-keys", type=int, default=0, help="exchange runs: the two outputs shared one key column")
    ap.add_argument("--tus", default="join.hip", help="comma-separated translation units of the kernel (crdtgpu.srcid)")
    ap.add_argument("--profile", default="", help="the profiles/ summary this entry is committed as")
    ap.add_argument("--fetch-pattern", default="stream8", choices=["stream8", "mix"],
                    help="FETCH_SIZE correction: 8-byte streaming (calib.py) or the tile element mix (fetch_calib)")
    a = ap.parse_args()
    out, calib = {}, {}
    for sub in sorted(os.listdir(a.dir)):
        p = os.path.join(a.dir, sub)
        if not os.path.isdir(p):
            continue
        dst = calib if sub.startswith("calib") else out
        for k, cs in load(p).items():
            for c, v in cs.items():
                dst.setdefault(short(k), {})[c] = sum(v) / len(v)
    for k in sorted(out):
        print(k)
        for c, v in sorted(out[k].items()):
            print("   %-24s %.6g" % (c, v))
    cal = calib.get("vv_max_kernel", {})
    print("calibration (vv_max_kernel, 1 GiB read / 512 MiB written per launch):", cal)
    N = 64 << 20
    fcorr = (16 * N) / (cal["FETCH_SIZE"] * 1024) if cal.get("FETCH_SIZE") else None
    wcorr = (8 * N) / (cal["WRITE_SIZE"] * 1024) if cal.get("WRITE_SIZE") else None
    # --fetch-pattern mix: the tile kernel's element (u64 key, u32 actor, u64 counter
    # per lane), calibrated on its own (tools/fetch_calib.hip readmix: 20 B x 64 Mi per launch)
    mix = calib.get("readmix", {})
    if a.fetch_pattern == "mix":
        print("calibration (fetch_calib readmix, 1.25 GiB read per launch):", mix,
              "read1<u64>:", calib.get("read1<unsigned long long>", {}), "read1<u32>:", calib.get("read1<unsigned int>", {}))
        fcorr = (20 * N) / (mix["FETCH_SIZE"] * 1024) if mix.get("FETCH_SIZE") else None
    # the exact instance when --kernel names one (has '<'), else the first of the family
    jk = a.kernel if "<" in a.kernel else next((k for k in out if k.startswith(a.kernel)), "")
    j = out.get(jk, {})
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "go-crdt-playground_amd"))
    from crdtgpu.srcid import source_id

    exch = jk.startswith("join") and (jk.split(",")[3:4] == [" true"] if "tile" not in jk else
                                       jk.split(",")[2:3] == [" true"])
    res = {"docs": a.docs, "config": a.config, "kernel": jk, "exchange": exch,
           "src_id": source_id(tuple(x for x in a.tus.split(",") if x)), "profile": a.profile,
           "fetch_correction": fcorr, "fetch_pattern": a.fetch_pattern, "write_correction": wcorr}
    if res["exchange"]:
        res["shared_keys"] = bool(a.shared_keys)
    if j.get("FETCH_SIZE") is not None and j.get("WRITE_SIZE") is not None:
        rd = j["FETCH_SIZE"] * 1024 * (fcorr or 1.0)
        wr = j["WRITE_SIZE"] * 1024 * (wcorr or 1.0)
        res.update({"fetch_bytes_raw": j["FETCH_SIZE"] * 1024, "write_bytes_raw": j["WRITE_SIZE"] * 1024,
                    "read_bytes": rd, "write_bytes": wr, "hbm_bytes_per_launch": rd + wr})
    print(json.dumps(res, indent=1))
    json.dump(res, open(os.path.join(a.dir, "traffic.json"), "w"), indent=1)
    if a.emit:
        # profiles/traffic.json: one entry per (config, docs, kernel); bench.py picks its own
        path = "profiles/traffic.json"
        table = json.load(open(path)) if os.path.exists(path) else []
        ident = lambda e: (e["config"], e["docs"], e["kernel"], e.get("shared_keys", False))  # noqa: E731
        table = [e for e in table if ident(e) != ident(res)]
        table.append(res)
        json.dump(table, open(path, "w"), indent=1)


if __name__ == "__main__":
    main()
