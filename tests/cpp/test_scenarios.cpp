// The reference's scenario tests, replayed through the C++ host mirror
// (go-crdt-playground_amd/host/crdt.hpp) whose Merge runs on the GPU.  Each
// function reads like its Go counterpart; besides the reference's own
// assertEntries checks it asserts the dots and clocks of SURVEY.md 4.1 (the
// same hand traces tests/golden/kat_scenarios.json holds).  Exit code 0 = all
// passed.  Built by __graft_entry__.build(); run by tests/test_host_cpp.py.
#include <cstdio>
#include <cstdlib>
#include <map>
#include <string>
#include <vector>

#include "../../go-crdt-playground_amd/host/crdt.hpp"

using namespace crdt;

static int failures = 0;
#define CHECK(cond)                                                        \
    do {                                                                   \
        if (!(cond)) {                                                     \
            std::printf("FAIL %s:%d: %s\n", __FILE__, __LINE__, #cond);    \
            ++failures;                                                    \
        }                                                                  \
    } while (0)

static void assertEntries(const AWSet& s, std::vector<std::string> want) {
    std::sort(want.begin(), want.end());
    auto got = s.SortedValues();
    if (got != want) {
        std::printf("FAIL entries: got");
        for (auto& g : got) std::printf(" %s", g.c_str());
        std::printf(" want");
        for (auto& w : want) std::printf(" %s", w.c_str());
        std::printf("\n");
        ++failures;
    }
}

static void expect(const AWSet& s, std::map<std::string, Dot> dots, VersionVector vv) {
    std::map<std::string, Dot> got(s.entries.begin(), s.entries.end());
    CHECK(got == dots);
    CHECK(s.versionVector == vv);
}

static const Actor A = 0, B = 1;

static void TestAWSetXXX() {  // awset_test.go:10-29
    AWSet a(0, {0, 0}), b(1, {0, 0});
    a.Add({"A", "B", "C"});
    b.Add({"A", "B", "C"});
    a.Merge(b);
    b.Merge(a);
    assertEntries(a, {"A", "B", "C"});
    assertEntries(b, {"A", "B", "C"});
    a.Del({"B"});
    b.Add({"B"});
    b.Merge(a);
    a.Merge(b);
    assertEntries(a, {"A", "B", "C"});
    assertEntries(b, {"A", "B", "C"});
    expect(a, {{"A", {B, 1}}, {"B", {B, 4}}, {"C", {B, 3}}}, {3, 4});
    expect(b, {{"A", {B, 1}}, {"B", {B, 4}}, {"C", {B, 3}}}, {3, 4});
}

static void TestAWSet() {  // awset_test.go:31-83
    AWSet a(0, {0, 0}), b(1, {0, 0});
    assertEntries(a, {});
    a.Add({"Shelly"});
    b.Merge(a);
    assertEntries(b, {"Shelly"});
    b.Add({"Bob", "Phil", "Pete"});
    a.Merge(b);
    assertEntries(a, {"Shelly", "Bob", "Phil", "Pete"});
    a.Del({"Phil"});
    a.Add({"Bob"});
    a.Add({"Anna"});
    b.Merge(a);
    assertEntries(b, {"Shelly", "Bob", "Pete", "Anna"});
    a.Del({"Bob", "Pete"});
    b.Del({"Bob", "Shelly"});
    a.Merge(b);
    b.Merge(a);
    assertEntries(a, {"Anna"});
    assertEntries(b, {"Anna"});
    a.Add({"A", "B", "C"});
    a.Del({"A"});
    a.Add({"A"});
    b.Merge(a);
    assertEntries(b, {"Anna", "A", "B", "C"});
    expect(b, {{"Anna", {A, 3}}, {"A", {A, 7}}, {"B", {A, 5}}, {"C", {A, 6}}}, {7, 3});
}

static void TestAWSetConcurrentAddWinsOverDelete() {  // awset_test.go:85-122
    AWSet a(0, {0, 0}), b(1, {0, 0});
    a.Add({"Anne", "Bob"});
    b.Add({"Anne"});
    {
        AWSet a2 = a.Clone(), b2 = b.Clone();
        b2.Add({"Bob"});
        a2.Del({"Bob"});
        b2.Merge(a2);
        a2.Merge(b2);
        assertEntries(b2, {"Anne", "Bob"});
        assertEntries(a2, {"Anne", "Bob"});
        expect(a2, {{"Anne", {A, 1}}, {"Bob", {B, 2}}}, {2, 2});
    }
    b.Add({"Bob"});
    b.Merge(a);
    expect(b, {{"Anne", {A, 1}}, {"Bob", {A, 2}}}, {2, 2});
    a.Del({"Bob"});
    b.Merge(a);
    a.Merge(b);
    assertEntries(b, {"Anne"});
    assertEntries(a, {"Anne"});
}

static void TestAWSetCommutativity() {  // awset_test.go:124-154
    AWSet a(0, {0, 0}), b(1, {0, 0});
    a.Add({"Shelly", "Bob", "Pete", "Anna"});
    b.Add({"Shelly", "Bob", "Pete", "Anna"});
    a.Del({"Anna"});
    b.Add({"Anna"});
    std::vector<std::string> want{"Shelly", "Bob", "Pete", "Anna"};
    {
        AWSet a2 = a.Clone(), b2 = b.Clone();
        b2.Merge(a2);
        a2.Merge(b2);
        assertEntries(a2, want);
        assertEntries(b2, want);
        expect(a2, {{"Shelly", {A, 1}}, {"Bob", {A, 2}}, {"Pete", {A, 3}}, {"Anna", {B, 5}}}, {4, 5});
    }
    a.Merge(b);
    b.Merge(a);
    assertEntries(a, want);
    assertEntries(b, want);
    expect(a, {{"Shelly", {B, 1}}, {"Bob", {B, 2}}, {"Pete", {B, 3}}, {"Anna", {B, 5}}}, {4, 5});
}

static void TestAWSetDelta() {  // awset-delta_test.go:168-189
    AWSetDelta a(0, {0, 0}), b(1, {0, 0});
    a.Add({"A", "B"});
    b.Add({"A", "C"});
    a.Merge(b);
    b.Merge(a);
    assertEntries(a, {"A", "B", "C"});
    assertEntries(b, {"A", "B", "C"});
    a.Del({"B"});
    a.Add({"D", "E"});
    b.Add({"E"});
    b.Merge(a);
    assertEntries(b, {"A", "C", "D", "E"});
    expect(b, {{"A", {B, 1}}, {"C", {B, 2}}, {"D", {A, 4}}, {"E", {A, 5}}}, {5, 3});
    a.Merge(b);  // no-op delta: A keeps its clock
    assertEntries(a, {"A", "C", "D", "E"});
    CHECK(a.versionVector == (VersionVector{5, 2}));
}

static void TestVersionVector() {  // crdt-misc_test.go:5-28
    VersionVector a{1, 1, 0, 4}, b{2, 0, 3, 0};
    a.Merge(b);
    CHECK(a == (VersionVector{2, 1, 3, 4}));
    b.Merge(a);
    CHECK(b == (VersionVector{2, 1, 3, 4}));
}

static void TestPanicsBecomeErrors() {
    AWSet a(0, {1, 1}), b(1, {1, 1});
    a.entries["x"] = Dot{2, 1};  // actor == len(vv): HasDot in phase 2 panics in Go
    bool threw = false;
    try {
        a.Merge(b);
    } catch (const Error& e) {
        threw = e.code == CRDT_E_ACTOR_RANGE;
    }
    CHECK(threw);
    CHECK(a.entries.size() == 1);  // untouched
}

// Version vectors of unequal lengths (zero-padded on the device): Go's panics
// at actor == len(vv) of the shorter vector, found by the host replay, and an
// exact result where Go does not panic.
static void TestRaggedVectors() {
    auto throws_range = [](auto&& fn) {
        try {
            fn();
        } catch (const Error& e) {
            return e.code == CRDT_E_ACTOR_RANGE;
        }
        return false;
    };
    {  // Counter(src.Actor) with src.Actor == len(dst VV)   awset-delta_test.go:53
        AWSetDelta d(0, {5, 5}), s(2, {1, 1, 1});
        CHECK(throws_range([&] { d.Merge(s); }));
        CHECK(d.versionVector == (VersionVector{5, 5}));
    }
    {  // tombstone HasDot on the shorter dst VV             awset-delta_test.go:153
        AWSetDelta d(0, {3, 3}), s(1, {1, 2, 1});
        d.entries["k"] = Dot{0, 1};
        s.deleted["k"] = Dot{2, 1};
        CHECK(throws_range([&] { d.Merge(s); }));
        CHECK(d.entries.size() == 1);
    }
    {  // no panic: a src-only key whose actor lies past the shorter dst VV is added
        AWSet d(0, {2}), s(2, {0, 0, 1});
        d.entries["a"] = Dot{0, 1};
        d.entries["b"] = Dot{0, 2};
        s.entries["c"] = Dot{2, 1};
        FoldBatch({&d}, {{&s}});
        expect(d, {{"a", {0, 1}}, {"b", {0, 2}}, {"c", {2, 1}}}, {2, 0, 1});
    }
}

static void TestBatches() {
    std::vector<AWSet> ds, ss;
    for (int i = 0; i < 40; ++i) {
        ds.emplace_back(0, VersionVector{0, 0});
        ss.emplace_back(1, VersionVector{0, 0});
        for (int j = 0; j < i % 7; ++j) ds.back().Add({"x" + std::to_string(j)});
        for (int j = 0; j < i % 5; ++j) ss.back().Add({"x" + std::to_string(j)});
    }
    std::vector<AWSet*> dp;
    std::vector<const AWSet*> sp;
    for (int i = 0; i < 40; ++i) {
        dp.push_back(&ds[i]);
        sp.push_back(&ss[i]);
    }
    MergeBatch(dp, sp);
    for (int i = 0; i < 40; ++i) {
        CHECK(ds[i].entries.size() == (size_t)std::max(i % 7, i % 5));
        CHECK(ds[i].versionVector == (VersionVector{(uint64_t)(i % 7), (uint64_t)(i % 5)}));
    }
    AWSet d(0, {0, 0, 0}), s1(1, {0, 0, 0}), s2(2, {0, 0, 0});
    s1.Add({"p", "q"});
    s2.Add({"q"});
    FoldBatch({&d}, {{&s1, &s2}});
    expect(d, {{"p", {1, 1}}, {"q", {2, 1}}}, {0, 2, 1});
}

// Aliased batches whose VersionVectors differ in length: every merge reads the
// pre-batch snapshot, so each result's VV width is that of the snapshot's
// states (crdt-misc.go:43-55 appends the longer tail), not of a source that
// another document of the same batch has already merged into.
static void TestAliasedRaggedWidths() {
    for (int rep = 0; rep < 20; ++rep) {  // the commits run on several threads: repeat
        std::vector<AWSet> s;
        std::vector<AWSet> want;
        for (int i = 0; i < 60; ++i) {  // chains a_i <- a_{i+1}, VV lengths 2,3,4,2,3,4,...
            AWSet x((uint32_t)(i % 2), VersionVector(2 + i % 3, 0));
            x.Add({"k" + std::to_string(i), "c"});
            if (i % 4 == 1) x.Del({"c"});
            s.push_back(x);
        }
        for (int i = 0; i + 1 < 60; ++i) {
            AWSet x = s[i];
            x.Merge(s[i + 1]);
            want.push_back(x);
        }
        std::vector<AWSet*> d;
        std::vector<const AWSet*> src;
        for (int i = 0; i + 1 < 60; ++i) d.push_back(&s[i]), src.push_back(&s[i + 1]);
        MergeBatch(d, src);
        for (int i = 0; i + 1 < 60; ++i)
            CHECK(s[i].entries == want[i].entries && s[i].versionVector == want[i].versionVector);
    }
    for (int rep = 0; rep < 20; ++rep) {
        std::vector<AWSetDelta> s;
        std::vector<AWSetDelta> want;
        for (int i = 0; i < 60; ++i) {
            AWSetDelta x((uint32_t)(i % 2), VersionVector(2 + i % 3, 0));
            x.Add({"k" + std::to_string(i), "c"});
            if (i % 4 == 1) x.Del({"c"});
            s.push_back(x);
        }
        for (int i = 0; i + 1 < 60; ++i) {
            AWSetDelta x = s[i];
            x.Merge(s[i + 1]);
            want.push_back(x);
        }
        std::vector<AWSetDelta*> d;
        std::vector<std::vector<const AWSetDelta*>> src;
        for (int i = 0; i + 1 < 60; ++i) d.push_back(&s[i]), src.push_back({&s[i + 1]});
        DeltaMergeBatch(d, src);
        for (int i = 0; i + 1 < 60; ++i)
            CHECK(s[i].entries == want[i].entries && s[i].versionVector == want[i].versionVector);
    }
}

// ExchangeBatch = the two merges of one snapshot, applied in place; an
// aliased MergeBatch (a <- b and b <- a in one batch) reads the snapshot too.
static void TestExchangeAndAliasing() {
    std::vector<AWSet> as, bs, xs, ys;
    for (int i = 0; i < 300; ++i) {
        AWSet a(0, {0, 0}), b(1, {0, 0});
        for (int j = 0; j < i % 11; ++j) a.Add({"k" + std::to_string(j)});
        b.Merge(a);
        for (int j = 0; j < i % 7; ++j) b.Add({"k" + std::to_string(2 * j + 1)});
        if (i % 3 == 0) a.Del({"k0", "k2"});
        if (i % 4 == 0) b.Del({"k1"});
        AWSet x = a, y = b;
        x.Merge(b);
        y.Merge(a);
        as.push_back(a), bs.push_back(b), xs.push_back(x), ys.push_back(y);
    }
    std::vector<AWSet*> pa, pb;
    for (size_t i = 0; i < as.size(); ++i) pa.push_back(&as[i]), pb.push_back(&bs[i]);
    ExchangeBatch(pa, pb);
    for (size_t i = 0; i < as.size(); ++i) {
        CHECK(as[i].entries == xs[i].entries && as[i].versionVector == xs[i].versionVector);
        CHECK(bs[i].entries == ys[i].entries && bs[i].versionVector == ys[i].versionVector);
    }
    AWSet a(0, {0, 0}), b(1, {0, 0});
    a.Add({"x", "y"});
    b.Add({"y", "z"});
    AWSet x = a, y = b;
    x.Merge(b);
    y.Merge(a);
    MergeBatch({&a, &b}, {&b, &a});
    CHECK(a.entries == x.entries && a.versionVector == x.versionVector);
    CHECK(b.entries == y.entries && b.versionVector == y.versionVector);
    bool threw = false;
    try {
        MergeBatch({&a, &a}, {&b, &b});
    } catch (const Error& e) {
        threw = e.code == CRDT_E_INVALID;
    }
    CHECK(threw);  // a destination twice
    TestAliasedRaggedWidths();
}

int main() {
    TestAWSetXXX();
    TestAWSet();
    TestAWSetConcurrentAddWinsOverDelete();
    TestAWSetCommutativity();
    TestAWSetDelta();
    TestVersionVector();
    TestPanicsBecomeErrors();
    TestRaggedVectors();
    TestBatches();
    TestExchangeAndAliasing();
    std::printf("%s: %d failure(s)\n", failures ? "FAILED" : "ok", failures);
    return failures ? 1 : 0;
}
