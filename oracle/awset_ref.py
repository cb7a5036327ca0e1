"""TEST INFRASTRUCTURE ONLY -- map-based restatement of the reference Go merge.

This module is an ORACLE.  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import it, and only as the checker.  The
product path (``go-crdt-playground_amd/``) never imports it.

It restates, in Python dictionaries, the semantics of the reference package
``crdt`` (rsms/go-crdt-playground, no go.mod, stdlib only) so that small
scenarios can be replayed exactly as the reference tests replay them:

* ``VersionVector`` -- crdt-misc.go:23-74 (HasDot :28-34, Counter :36-41,
  Merge :43-55, String :57-68, Clone :70-74).  Variable length, like the Go
  slice; the out-of-range index the Go code hits when ``actor == len(vv)``
  (crdt-misc.go:29,37 compare with ``<`` not ``<=``) raises ``GoPanic``.
* ``AWSet`` -- awset.go:55-171 (Add :89-94, Del :96-101, Merge/merge :103-161).
* ``AWSetDelta`` -- awset-delta_test.go:9-166 (Del :14-33, Merge :51-65,
  gcDeleted :67-77 (no-op), MakeDeltaMergeData :79-105, deltaMerge :107-166).

The per-key decision log the Go code prints (awset.go:109-121) has no effect on
state and is not restated.  Go map iteration order is random; every decision in
``merge``/``deltaMerge`` reads only pre-merge version vectors and the key's own
presence, so the result is iteration-order independent (SURVEY.md section 8a,
row a7), and plain dict order is used here.

Parity status: the reference cannot be executed in this container (no Go
toolchain).  This restatement is pinned by the element-set
assertions and the one version-vector assertion the reference's own tests make
(awset_test.go, awset-delta_test.go, crdt-misc_test.go), replayed in
``tests/golden/make_golden.py``; dots and version vectors after merges are pinned
only by the hand traces of SURVEY.md section 4.1, which the same script asserts.
"""

from __future__ import annotations

from dataclasses import dataclass


class GoPanic(RuntimeError):
    """The Go code would panic (index out of range) at this point."""


@dataclass(frozen=True)
class Dot:
    """crdt-misc.go:12-15 -- an (Actor, Counter) event id."""

    actor: int
    counter: int

    def __str__(self) -> str:  # crdt-misc.go:17-19
        return "(%s %d)" % (chr(ord("A") + self.actor), self.counter)


class VersionVector(list):
    """crdt-misc.go:23 -- ``[]uint`` indexed by actor."""

    def HasDot(self, d: Dot) -> bool:
        # crdt-misc.go:28-34.  Note the ``<``: actor == len indexes past the end.
        if len(self) < d.actor:
            return False
        if d.actor >= len(self):
            raise GoPanic("index out of range [%d] with length %d" % (d.actor, len(self)))
        return self[d.actor] >= d.counter

    def Counter(self, a: int) -> int:
        # crdt-misc.go:36-41, same off-by-one as HasDot.
        if len(self) < a:
            return 0
        if a >= len(self):
            raise GoPanic("index out of range [%d] with length %d" % (a, len(self)))
        return self[a]

    def Merge(self, src: "VersionVector") -> None:
        # crdt-misc.go:43-55: elementwise max, src's tail appended.
        for i, n in enumerate(src):
            if i < len(self):
                if self[i] < n:
                    self[i] = n
            else:
                self.append(n)

    def Clone(self) -> "VersionVector":  # crdt-misc.go:70-74
        return VersionVector(self)

    def String(self) -> str:  # crdt-misc.go:57-68
        return "[" + ", ".join("(%s %d)" % (chr(ord("A") + i), n) for i, n in enumerate(self)) + "]"


def _go_printable(r: int) -> bool:
    # unicode.IsPrint, exact for ASCII; outside ASCII the same approximation as
    # csrc/serial.cpp (controls, format characters, separators, private use and
    # non-characters are not printable)
    if r < 0x20 or r == 0x7F:
        return False
    if r < 0x7F:
        return True
    if 0x80 <= r <= 0xA0 or r == 0xAD or 0x2000 <= r <= 0x200F or 0x2028 <= r <= 0x202F:
        return False
    if 0x205F <= r <= 0x206F or r in (0x3000, 0xFEFF) or 0xE000 <= r <= 0xF8FF:
        return False
    if (r & 0xFFFE) == 0xFFFE or 0xFDD0 <= r <= 0xFDEF or r >= 0xF0000:
        return False
    return True


def go_quote(s) -> str:
    """fmt %q of a Go string (strconv.Quote); s is str or bytes (bytes may hold
    invalid UTF-8, escaped as \\xNN)."""
    b = s.encode("utf-8", errors="surrogateescape") if isinstance(s, str) else bytes(s)
    out, i = ['"'], 0
    esc = {7: "\\a", 8: "\\b", 12: "\\f", 10: "\\n", 13: "\\r", 9: "\\t", 11: "\\v"}
    while i < len(b):
        c = b[i]
        n = 1 if c < 0x80 else 2 if c >> 5 == 6 else 3 if c >> 4 == 14 else 4 if c >> 3 == 30 else 0
        try:
            r = ord(b[i:i + n].decode("utf-8")) if n else None
        except UnicodeDecodeError:
            r = None
        if r is None:
            out.append("\\x%02x" % c)
            i += 1
            continue
        if r in (0x22, 0x5C):
            out.append("\\" + chr(r))
        elif _go_printable(r):
            out.append(chr(r))
        elif r in esc:
            out.append(esc[r])
        elif r < 0x20 or r == 0x7F:
            out.append("\\x%02x" % r)
        elif r < 0x10000:
            out.append("\\u%04x" % r)
        else:
            out.append("\\U%08x" % r)
        i += n
    out.append('"')
    return "".join(out)


class AWSet:
    """awset.go:55-59 -- ``{Actor, VersionVector, Entries map[string]Dot}``."""

    def __init__(self, actor: int = 0, vv=None, entries=None):
        self.Actor = actor
        self.VersionVector = VersionVector(vv if vv is not None else [])
        self.Entries: dict = dict(entries) if entries is not None else {}

    def SortedValues(self):  # awset.go:61-70
        return sorted(self.Entries)

    def Reset(self):  # awset.go:72-75
        self.VersionVector = VersionVector([0])
        self.Entries = {}

    def Clone(self) -> "AWSet":  # awset.go:77-85
        return AWSet(self.Actor, self.VersionVector.Clone(), self.Entries)

    def Has(self, k) -> bool:  # awset.go:87
        return k in self.Entries

    def Add(self, *keys) -> None:
        # awset.go:89-94: one fresh dot per key.
        for k in keys:
            if self.Actor >= len(self.VersionVector):
                raise GoPanic("Add: actor %d outside VersionVector" % self.Actor)
            self.VersionVector[self.Actor] += 1
            self.Entries[k] = Dot(self.Actor, self.VersionVector[self.Actor])

    def Del(self, *keys) -> None:
        # awset.go:96-101: no clock bump (the bump at :97 is commented out).
        for k in keys:
            self.Entries.pop(k, None)

    def Merge(self, src: "AWSet") -> None:  # awset.go:103-105
        self.merge(src.VersionVector, src.Entries)

    def merge(self, srcVV: VersionVector, srcEntries: dict) -> None:
        # awset.go:107-161, dst <- src.
        dst = self
        # phase 1 (awset.go:122-143): src dot wins on common keys; a src-only
        # key is added unless dst's clock already covers its dot.
        for k, srcDot in srcEntries.items():
            if k not in dst.Entries:
                if dst.VersionVector.HasDot(srcDot):
                    continue  # "skip"
            dst.Entries[k] = srcDot
        # phase 2 (awset.go:145-159): a dst-only key whose dot src has seen was
        # removed at src.
        for k in list(dst.Entries):
            dstDot = dst.Entries[k]
            if k in srcEntries:
                continue  # "keep"
            if srcVV.HasDot(dstDot):
                del dst.Entries[k]  # "remove"
        dst.VersionVector.Merge(srcVV)  # awset.go:160

    def deltaMerge(self, srcVV: VersionVector, srcChanges, srcDeleted) -> None:
        # awset-delta_test.go:107-166.
        dst = self
        for k, srcDot in (srcChanges or {}).items():  # :126-147, same rule as merge phase 1
            if k not in dst.Entries:
                if dst.VersionVector.HasDot(srcDot):
                    continue
            dst.Entries[k] = srcDot
        for k, srcDot in (srcDeleted or {}).items():  # :149-164
            if k in dst.Entries:
                if dst.VersionVector.HasDot(srcDot):
                    continue  # entry was updated in dst; keep it
                del dst.Entries[k]
            # absent: delete of a missing key is a no-op (:160-163)
        dst.VersionVector.Merge(srcVV)  # :165

    def String(self) -> str:  # awset.go:163-171: "\n  %s  %q" per value
        out = self.VersionVector.String()
        for v in self.SortedValues():
            out += "\n  %s  %s" % (self.Entries[v], go_quote(v))
        return out


class AWSetDelta(AWSet):
    """awset-delta_test.go:9-12 -- AWSet plus a tombstone map ``Deleted``."""

    def __init__(self, actor: int = 0, vv=None, entries=None, deleted=None):
        super().__init__(actor, vv, entries)
        self.Deleted = dict(deleted) if deleted else None  # nil map until first Del

    def Del(self, *keys) -> None:
        # awset-delta_test.go:14-33: ONE fresh dot per call, recorded for each
        # present key, which is then dropped.
        if self.Actor >= len(self.VersionVector):
            raise GoPanic("Del: actor %d outside VersionVector" % self.Actor)
        self.VersionVector[self.Actor] += 1
        dot2 = Dot(self.Actor, self.VersionVector[self.Actor])
        for k in keys:
            if k in self.Entries:
                if self.Deleted is None:
                    self.Deleted = {}
                self.Deleted[k] = dot2
                del self.Entries[k]

    def Clone(self) -> "AWSetDelta":  # awset-delta_test.go:35-49
        c = AWSetDelta(self.Actor, self.VersionVector.Clone(), self.Entries)
        if self.Deleted:
            c.Deleted = dict(self.Deleted)
        return c

    def Merge(self, src: "AWSetDelta") -> None:
        # awset-delta_test.go:51-65.
        dst = self
        if dst.VersionVector.Counter(src.Actor) <= 0:
            dst.merge(src.VersionVector, src.Entries)  # first contact: full merge, Deleted ignored
            return
        changed, deleted = src.MakeDeltaMergeData(dst.VersionVector)
        if changed is not None or deleted is not None:
            dst.deltaMerge(src.VersionVector, changed, deleted)
            dst.gcDeleted(src.VersionVector)
        # else: no-op -- dst keeps its version vector too (:60)

    def gcDeleted(self, srcVV) -> None:  # awset-delta_test.go:67-77: empty
        pass

    def MakeDeltaMergeData(self, dstVV: VersionVector):
        # awset-delta_test.go:79-105.  nil maps are returned as None.
        changed = None
        deleted = None
        for k, dot in self.Entries.items():  # :84-92 dot pruning
            if not dstVV.HasDot(dot):
                if changed is None:
                    changed = {}
                changed[k] = dot
        for k, dot in (self.Deleted or {}).items():  # :93-102, NOT pruned by dstVV
            m = self.Entries.get(k)
            if m is not None and (m.actor != dot.actor or m.counter > dot.counter):
                continue  # removed and then added again
            if deleted is None:
                deleted = {}
            deleted[k] = dot
        return changed, deleted


def snapshot(s: AWSet) -> dict:
    """JSON-able full state: sorted entries with dots, and the version vector."""
    d = {
        "actor": s.Actor,
        "vv": list(s.VersionVector),
        "entries": [[k, s.Entries[k].actor, s.Entries[k].counter] for k in sorted(s.Entries)],
    }
    if isinstance(s, AWSetDelta):
        dl = s.Deleted or {}
        d["deleted"] = [[k, dl[k].actor, dl[k].counter] for k in sorted(dl)]
    return d
