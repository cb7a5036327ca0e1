"""Source identity of a kernel build: which sources a PMC traffic figure was
measured on.  bench.py reports a profiles/traffic.json entry only when the
entry's kernel instance and source id equal the ones it is timing, so a
figure taken on an older build of the same kernel family never stands in for
the current one (tools/traffic.py records the id; tools/pmc.sh)."""

import hashlib
import os
import re

CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "csrc")
_INC = re.compile(r'^\s*#\s*include\s+"([^"]+)"', re.M)


def _closure(path, seen):
    path = os.path.normpath(path)
    if path in seen or not os.path.exists(path):
        return
    seen.add(path)
    with open(path, encoding="utf-8", errors="replace") as f:
        text = f.read()
    for inc in _INC.findall(text):
        _closure(os.path.join(os.path.dirname(path), inc), seen)


def source_id(tus, csrc=CSRC):
    """sha256 (16 hex) over the build flags (Makefile), the C ABI's launch
    defaults (api.cpp) and each translation unit in `tus` with the local
    headers it includes, transitively."""
    files = set()
    for tu in ("Makefile", "api.cpp") + tuple(tus):
        _closure(os.path.join(csrc, tu), files)
    h = hashlib.sha256()
    for p in sorted(files):
        h.update(os.path.relpath(p, csrc).encode() + b"\0")
        with open(p, "rb") as f:
            h.update(f.read())
        h.update(b"\0")
    return h.hexdigest()[:16]
