// Host fuzz of the fixture image parser (crdt_batch_info / crdt_batch_undump,
// go-crdt-playground_amd/csrc/serial.cpp), which reads images a caller may
// not control.  Random batches are dumped, then mutated -- byte flips, header
// fields rewritten to edge values, offsets made non-monotone, lengths cut or
// extended -- and the checksum is re-signed, so that the parser's own checks
// (not the checksum) must reject each image or accept it safely.  Images are
// also parsed from misaligned addresses.  Built with
// -fsanitize=address,undefined (host/Makefile); tests/test_serial.py runs it.
// Exit code 0 = no sanitizer report and every accepted image well-formed.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "../../include/crdtgpu.h"

// FNV-1a 64 (the image's trailing checksum)
static uint64_t fnv1a(const unsigned char* p, size_t n) {
    uint64_t h = 0xCBF29CE484222325ull;
    for (size_t i = 0; i < n; ++i) h = (h ^ p[i]) * 0x100000001B3ull;
    return h;
}

static void resign(std::vector<unsigned char>& img) {
    if (img.size() < 8) return;
    const uint64_t h = fnv1a(img.data(), img.size() - 8);
    memcpy(img.data() + img.size() - 8, &h, 8);
}

int main(int argc, char** argv) {
    const long iters = argc > 1 ? atol(argv[1]) : 20000;
    std::mt19937_64 rng(argc > 2 ? strtoull(argv[2], nullptr, 10) : 1);
    auto rnd = [&](uint64_t n) { return n ? rng() % n : 0; };
    long accepted = 0, rejected = 0;
    for (long it = 0; it < iters; ++it) {
        // a random valid batch (slack slots, empty documents)
        const uint32_t nd = (uint32_t)rnd(7), R = 1 + (uint32_t)rnd(4);
        std::vector<uint32_t> off{0}, cnt;
        std::vector<uint64_t> keys, ctr, vv(std::max<size_t>((size_t)nd * R, 1));
        std::vector<uint32_t> act;
        for (uint32_t d = 0; d < nd; ++d) {
            const uint32_t live = (uint32_t)rnd(6), slack = (uint32_t)rnd(3);
            uint64_t k = rnd(5);
            for (uint32_t i = 0; i < live + slack; ++i) {
                keys.push_back(k);
                k += 1 + rnd(1000);
                act.push_back((uint32_t)rnd(R + 1));
                ctr.push_back(rng());
            }
            cnt.push_back(live);
            off.push_back(off.back() + live + slack);
        }
        for (auto& v : vv) v = rng();
        keys.push_back(0), act.push_back(0), ctr.push_back(0), cnt.push_back(0);
        const crdt_awset_batch b{nd, R, off.data(), cnt.data(), keys.data(), act.data(), ctr.data(), vv.data()};
        size_t len = 0;
        if (crdt_batch_dump(&b, nullptr, 0, &len) != CRDT_OK) return printf("dump size failed\n"), 1;
        std::vector<unsigned char> raw(len + 8);
        const size_t at = (size_t)rnd(8);  // dump to a misaligned address too
        if (crdt_batch_dump(&b, raw.data() + at, len, &len) != CRDT_OK) return printf("dump failed\n"), 1;
        std::vector<unsigned char> img(raw.begin() + at, raw.begin() + at + len);

        // mutate (it % 8 == 0: leave the image intact)
        const int kind = (int)(it % 8);
        if (kind == 1) {
            for (int m = 1 + (int)rnd(4); m > 0 && img.size() > 8; --m) img[rnd(img.size() - 8)] ^= (unsigned char)(1 + rnd(255));
        } else if (kind == 2 && img.size() >= 24) {  // header fields: n_docs, R, n to edge values
            const uint64_t edges[] = {0, 1, 2, 63, 64, 65, 0x7FFFFFFF, 0x80000000ull, 0xFFFFFFFFull, 1ull << 32,
                                      1ull << 40, ~0ull};
            const uint64_t v = edges[rnd(12)];
            const int field = (int)rnd(3);
            if (field == 0) memcpy(&img[8], &v, 4);
            if (field == 1) memcpy(&img[12], &v, 4);
            if (field == 2) memcpy(&img[16], &v, 8);
        } else if (kind == 3 && nd > 0) {  // offsets non-monotone / past the entry count
            const uint32_t v = (uint32_t)rnd(40);
            memcpy(&img[24 + 4 * rnd(nd + 1)], &v, 4);
        } else if (kind == 4) {  // cut or extend
            const size_t d = 1 + rnd(16);
            if (rnd(2) && img.size() > d)
                img.resize(img.size() - d);
            else
                img.resize(img.size() + d, (unsigned char)rnd(256));
        } else if (kind == 5 && img.size() > 8) {
            img[rnd(8)] ^= 0x20;  // magic
        }
        if (kind != 6) resign(img);  // kind 6: checksum left stale after a flip
        if (kind == 6 && img.size() > 8) img[rnd(img.size() - 8)] ^= 0x10;

        // parse from an aligned and from a misaligned copy
        for (size_t shift : {(size_t)0, (size_t)(1 + rnd(7))}) {
            std::vector<unsigned char> buf(img.size() + shift + 1);
            memcpy(buf.data() + shift, img.data(), img.size());
            const void* p = buf.data() + shift;
            uint32_t gd = 0, gr = 0;
            uint64_t gn = 0;
            if (crdt_batch_info(p, img.size(), &gd, &gr, &gn) != CRDT_OK) {
                ++rejected;
                continue;
            }
            if (gr == 0 || gr > CRDT_MAX_R || gn >= (1ull << 32)) return printf("info accepted a bad header\n"), 1;
            if ((uint64_t)gd * gr > (1u << 22) || gn > (1u << 22)) {  // a well-formed but huge image: skip
                ++accepted;
                continue;
            }
            std::vector<uint32_t> o(gd + 1), c(std::max<uint32_t>(gd, 1));
            std::vector<uint64_t> k(std::max<uint64_t>(gn, 1)), cc(std::max<uint64_t>(gn, 1)),
                v(std::max<uint64_t>((uint64_t)gd * gr, 1));
            std::vector<uint32_t> a(std::max<uint64_t>(gn, 1));
            const crdt_awset_out out{o.data(), c.data(), k.data(), a.data(), cc.data(), v.data()};
            if (crdt_batch_undump(p, img.size(), &out) != CRDT_OK) {
                ++rejected;
                continue;
            }
            ++accepted;
            if (o[0] != 0 || o[gd] != gn) return printf("undump accepted bad offsets\n"), 1;
            for (uint32_t d = 0; d < gd; ++d)
                if (o[d + 1] < o[d] || c[d] != o[d + 1] - o[d]) return printf("undump counts inconsistent\n"), 1;
            if (kind == 0 && (gd != nd || gr != R)) return printf("intact image read back wrong\n"), 1;
        }
    }
    printf("ok: %ld images accepted, %ld rejected\n", accepted, rejected);
    return 0;
}
