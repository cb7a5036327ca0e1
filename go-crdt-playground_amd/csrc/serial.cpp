// Fixture dumps and debug text for host-side batches.
//
//   crdt_awset_format   Go's (AWSet).String() of one document of a batch:
//                       awset.go:163-171 (VersionVector.String, then one line
//                       per entry in SortedValues order: "\n  %s  %q"), with
//                       Dot.String crdt-misc.go:17-19 and VersionVector.String
//                       crdt-misc.go:57-68
//   crdt_batch_dump / crdt_batch_info / crdt_batch_undump
//                       a self-checking binary image of a batch (live entries
//                       only, compact offsets), for fixtures and diffing
//
// Host buffers only; no GPU.
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/crdtgpu.h"

namespace {

// fmt's %c of a rune: UTF-8 encoding (Go writes U+FFFD for invalid runes)
void put_rune(std::string& s, uint32_t r) {
    if (r > 0x10FFFF || (r >= 0xD800 && r <= 0xDFFF)) r = 0xFFFD;
    if (r < 0x80) {
        s += (char)r;
    } else if (r < 0x800) {
        s += (char)(0xC0 | (r >> 6));
        s += (char)(0x80 | (r & 0x3F));
    } else if (r < 0x10000) {
        s += (char)(0xE0 | (r >> 12));
        s += (char)(0x80 | ((r >> 6) & 0x3F));
        s += (char)(0x80 | (r & 0x3F));
    } else {
        s += (char)(0xF0 | (r >> 18));
        s += (char)(0x80 | ((r >> 12) & 0x3F));
        s += (char)(0x80 | ((r >> 6) & 0x3F));
        s += (char)(0x80 | (r & 0x3F));
    }
}

// "(%c %d)" with 'A' + actor (crdt-misc.go:17-19, :65)
void put_dot(std::string& s, uint64_t actor, uint64_t counter) {
    s += '(';
    put_rune(s, (uint32_t)(actor > 0x10FFFF ? 0x110000 : 'A' + actor));
    s += ' ';
    s += std::to_string(counter);
    s += ')';
}

// Decode one UTF-8 rune at p (n bytes left); returns its length, 0 if invalid.
size_t utf8_rune(const unsigned char* p, size_t n, uint32_t& r) {
    const unsigned char c = p[0];
    size_t len;
    uint32_t min;
    if (c < 0x80) {
        r = c;
        return 1;
    } else if ((c & 0xE0) == 0xC0) {
        len = 2, r = c & 0x1F, min = 0x80;
    } else if ((c & 0xF0) == 0xE0) {
        len = 3, r = c & 0x0F, min = 0x800;
    } else if ((c & 0xF8) == 0xF0) {
        len = 4, r = c & 0x07, min = 0x10000;
    } else {
        return 0;
    }
    if (len > n) return 0;
    for (size_t i = 1; i < len; ++i) {
        if ((p[i] & 0xC0) != 0x80) return 0;
        r = (r << 6) | (p[i] & 0x3F);
    }
    if (r < min || r > 0x10FFFF || (r >= 0xD800 && r <= 0xDFFF)) return 0;
    return len;
}

// Printable runes of Go's unicode.IsPrint, approximated outside ASCII: the C1
// controls, the format characters of Latin-1/General Punctuation/BOM, line and
// paragraph separators and private-use/non-characters are not printable.
bool go_printable(uint32_t r) {
    if (r < 0x20 || r == 0x7F) return false;
    if (r < 0x7F) return true;
    if (r >= 0x80 && r <= 0xA0) return false;  // C1 controls, NBSP (Zs)
    if (r == 0xAD) return false;               // soft hyphen (Cf)
    if (r >= 0x2000 && r <= 0x200F) return false;
    if (r >= 0x2028 && r <= 0x202F) return false;
    if (r >= 0x205F && r <= 0x206F) return false;
    if (r == 0x3000 || r == 0xFEFF) return false;
    if (r >= 0xE000 && r <= 0xF8FF) return false;  // private use
    if ((r & 0xFFFE) == 0xFFFE || (r >= 0xFDD0 && r <= 0xFDEF)) return false;
    if (r >= 0xF0000) return false;
    return true;
}

// Go's %q of a string (strconv.Quote)
void put_quoted(std::string& s, const char* str, size_t n) {
    static const char hex[] = "0123456789abcdef";
    s += '"';
    const unsigned char* p = (const unsigned char*)str;
    size_t i = 0;
    while (i < n) {
        uint32_t r;
        const size_t len = utf8_rune(p + i, n - i, r);
        if (len == 0) {  // invalid byte
            s += "\\x";
            s += hex[p[i] >> 4];
            s += hex[p[i] & 15];
            ++i;
            continue;
        }
        if (r == '"' || r == '\\') {
            s += '\\';
            s += (char)r;
        } else if (go_printable(r)) {
            s.append((const char*)p + i, len);
        } else {
            switch (r) {
                case '\a': s += "\\a"; break;
                case '\b': s += "\\b"; break;
                case '\f': s += "\\f"; break;
                case '\n': s += "\\n"; break;
                case '\r': s += "\\r"; break;
                case '\t': s += "\\t"; break;
                case '\v': s += "\\v"; break;
                default:
                    if (r < 0x20 || r == 0x7F) {
                        s += "\\x";
                        s += hex[r >> 4];
                        s += hex[r & 15];
                    } else if (r < 0x10000) {
                        s += "\\u";
                        for (int k = 12; k >= 0; k -= 4) s += hex[(r >> k) & 15];
                    } else {
                        s += "\\U";
                        for (int k = 28; k >= 0; k -= 4) s += hex[(r >> k) & 15];
                    }
            }
        }
        i += len;
    }
    s += '"';
}

uint64_t fnv1a(const unsigned char* p, size_t n) {
    uint64_t h = 0xCBF29CE484222325ull;
    for (size_t i = 0; i < n; ++i) h = (h ^ p[i]) * 0x100000001B3ull;
    return h;
}

const char kMagic[8] = {'C', 'R', 'D', 'T', 'B', '0', '0', '1'};
constexpr size_t kHeader = 8 + 4 + 4 + 8;

// offsets region, padded to 8 bytes so the u64 arrays stay aligned
size_t offs_bytes(uint32_t n_docs) { return (4 * ((size_t)n_docs + 1) + 7) & ~(size_t)7; }

// entries region: keys (8n), counters (8n), actors (4n), padded to 8
size_t ents_bytes(uint64_t n) { return (20 * n + 7) & ~(size_t)7; }

uint32_t live_of(const crdt_awset_batch* b, uint32_t d) {
    return b->counts ? b->counts[d] : b->offsets[d + 1] - b->offsets[d];
}

}  // namespace

extern "C" {

int crdt_awset_format(const crdt_awset_batch* b, uint32_t doc, const char* const* names, char* buf, size_t cap,
                      size_t* len) {
    if (!b || !b->offsets || !b->vv || doc >= b->n_docs || (cap && !buf)) return CRDT_E_INVALID;
    std::string s = "[";
    for (uint32_t r = 0; r < b->R; ++r) {
        if (r) s += ", ";
        put_dot(s, r, b->vv[(size_t)doc * b->R + r]);
    }
    s += ']';
    const uint32_t o = b->offsets[doc], n = live_of(b, doc);
    for (uint32_t i = 0; i < n; ++i) {  // key ids are order-preserving: id order is SortedValues order
        s += "\n  ";
        put_dot(s, b->actors[o + i], b->counters[o + i]);
        s += "  ";
        const uint64_t id = b->keys[o + i];
        if (names) {
            const char* nm = names[id];
            put_quoted(s, nm, strlen(nm));
        } else {
            const std::string nm = "#" + std::to_string(id);
            put_quoted(s, nm.data(), nm.size());
        }
    }
    if (len) *len = s.size();
    if (cap) {
        const size_t m = s.size() < cap - 1 ? s.size() : cap - 1;
        memcpy(buf, s.data(), m);
        buf[m] = 0;
    }
    return CRDT_OK;
}

int crdt_batch_dump(const crdt_awset_batch* b, void* buf, size_t cap, size_t* len) {
    if (!b || !b->offsets || (b->n_docs && !b->vv) || !len) return CRDT_E_INVALID;
    uint64_t n = 0;
    for (uint32_t d = 0; d < b->n_docs; ++d) n += live_of(b, d);
    if (n >= (1ull << 32)) return CRDT_E_CAPACITY;  // per-doc offsets are u32 in the image
    const size_t need = kHeader + offs_bytes(b->n_docs) + ents_bytes(n) + 8 * (size_t)b->n_docs * b->R + 8;
    *len = need;
    if (!buf) return CRDT_OK;
    if (cap < need) return CRDT_E_CAPACITY;
    // built in an aligned scratch image, then copied: buf may sit at any address
    std::vector<uint64_t> img((need + 7) / 8);
    unsigned char* p = (unsigned char*)img.data();
    memcpy(p, kMagic, 8);
    memcpy(p + 8, &b->n_docs, 4);
    memcpy(p + 12, &b->R, 4);
    memcpy(p + 16, &n, 8);
    memset(p + kHeader, 0, need - kHeader);
    uint32_t* off = (uint32_t*)(p + kHeader);
    unsigned char* q = p + kHeader + offs_bytes(b->n_docs);
    uint64_t* keys = (uint64_t*)q;
    uint64_t* counters = (uint64_t*)(q + 8 * n);
    uint32_t* actors = (uint32_t*)(q + 16 * n);
    uint64_t* vv = (uint64_t*)(q + ents_bytes(n));
    uint64_t at = 0;
    for (uint32_t d = 0; d < b->n_docs; ++d) {
        off[d] = (uint32_t)at;
        const uint32_t o = b->offsets[d], c = live_of(b, d);
        memcpy(keys + at, b->keys + o, 8 * (size_t)c);
        memcpy(actors + at, b->actors + o, 4 * (size_t)c);
        memcpy(counters + at, b->counters + o, 8 * (size_t)c);
        at += c;
    }
    off[b->n_docs] = (uint32_t)at;
    memcpy(vv, b->vv, 8 * (size_t)b->n_docs * b->R);
    const uint64_t h = fnv1a(p, need - 8);
    memcpy(p + need - 8, &h, 8);
    memcpy(buf, p, need);
    return CRDT_OK;
}

int crdt_batch_info(const void* buf, size_t len, uint32_t* n_docs, uint32_t* R, uint64_t* n_entries) {
    if (!buf || len < kHeader + 12) return CRDT_E_INVALID;
    const unsigned char* p = (const unsigned char*)buf;
    if (memcmp(p, kMagic, 8)) return CRDT_E_INVALID;
    uint32_t nd, r;
    uint64_t n;
    memcpy(&nd, p + 8, 4);
    memcpy(&r, p + 12, 4);
    memcpy(&n, p + 16, 8);
    if (r == 0 || r > CRDT_MAX_R) return CRDT_E_INVALID;
    if (n >= (1ull << 32) || nd > (1u << 31)) return CRDT_E_INVALID;  // matches crdt_batch_dump
    const size_t need = kHeader + offs_bytes(nd) + ents_bytes(n) + 8 * (size_t)nd * r + 8;
    if (len != need) return CRDT_E_INVALID;
    uint64_t h;
    memcpy(&h, p + need - 8, 8);
    if (h != fnv1a(p, need - 8)) return CRDT_E_INVALID;
    if (n_docs) *n_docs = nd;
    if (R) *R = r;
    if (n_entries) *n_entries = n;
    return CRDT_OK;
}

int crdt_batch_undump(const void* buf, size_t len, const crdt_awset_out* out) {
    uint32_t nd, r;
    uint64_t n;
    int rc = crdt_batch_info(buf, len, &nd, &r, &n);
    if (rc != CRDT_OK) return rc;
    if (!out || !out->offsets || !out->counts || (n && (!out->keys || !out->actors || !out->counters)) ||
        (nd && !out->vv))
        return CRDT_E_INVALID;
    const unsigned char* p = (const unsigned char*)buf;
    const unsigned char* off = p + kHeader;  // u32 array; the image may sit at any address: memcpy reads
    const unsigned char* q = p + kHeader + offs_bytes(nd);
    auto off_at = [off](uint32_t d) {
        uint32_t v;
        memcpy(&v, off + 4 * (size_t)d, 4);
        return v;
    };
    if (off_at(0) != 0) return CRDT_E_INVALID;
    for (uint32_t d = 0; d < nd; ++d)
        if (off_at(d + 1) < off_at(d) || off_at(d + 1) > n) return CRDT_E_INVALID;
    if (off_at(nd) != n) return CRDT_E_INVALID;
    memcpy(out->offsets, off, 4 * ((size_t)nd + 1));
    for (uint32_t d = 0; d < nd; ++d) out->counts[d] = off_at(d + 1) - off_at(d);
    memcpy(out->keys, q, 8 * n);
    memcpy(out->counters, q + 8 * n, 8 * n);
    memcpy(out->actors, q + 16 * n, 4 * n);
    memcpy(out->vv, q + ents_bytes(n), 8 * (size_t)nd * r);
    return CRDT_OK;
}

}  // extern "C"
