// lime_amd.hpp -- C++ host mirror of lime-core's operator API over the
// C-ABI (header-only).  Class names, constructor arguments and results follow
// lime-core/src/main/scala/org/bdgenomics/lime/set_theory/:
//
//   DistributedIntersection<T,U>(left, right, partitionMap, threshold = 0).compute()
//       -> vector<pair<ReferenceRegion, pair<T,U>>>          Intersection.scala:45-69
//   DistributedMerge<T>(rdd, partitionMap, threshold = 0).compute()
//       -> vector<pair<ReferenceRegion, vector<T>>>           Merge.scala:34-36
//   DistributedSubtract<T,U>(left, right, partitionMap, threshold = 0).compute()
//       -> vector<pair<ReferenceRegion, pair<T, optional<U>>>> Subtract.scala:78-116
//   DistributedComplement<T>(rdd, partitionMap, referenceNameBounds, threshold = 0).compute()
//       -> vector<pair<ReferenceRegion, vector<T>>>           Complement.scala:131-134
//
// An "RDD" is a host vector of (ReferenceRegion, value).  `partitionMap` is
// accepted for signature parity and ignored: results equal the reference's
// single-partition execution, in its emission order.
// Errors are thrown as lime::Error (status code + message); a complement
// contig missing from referenceNameBounds throws lime::NoSuchElement, as the
// reference's referenceNameBounds(name) does (Complement.scala:106,118).
#pragma once

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <map>
#include <memory>
#include <numeric>
#include <optional>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

#include "lime_amd.h"

namespace lime {

enum class Strand : int8_t { Independent = 0, Forward = 1, Reverse = 2, Unknown = 3 };
// RegionOrdering compares bdg-formats' Strand enum ordinals (FORWARD,
// REVERSE, INDEPENDENT, UNKNOWN)
inline int strand_ord(Strand s) {
    static const int ord[4] = {2, 0, 1, 3};
    return ord[(int)s & 3];
}

struct ReferenceRegion {
    std::string referenceName;
    int64_t start = 0, end = 0;
    Strand strand = Strand::Independent;
    ReferenceRegion() = default;
    ReferenceRegion(std::string n, int64_t s, int64_t e, Strand st = Strand::Independent)
        : referenceName(std::move(n)), start(s), end(e), strand(st) {}
    bool operator==(const ReferenceRegion &o) const {
        return referenceName == o.referenceName && start == o.start && end == o.end &&
               strand == o.strand;
    }
};

struct Error : std::runtime_error {
    int code;
    Error(int c, const std::string &m) : std::runtime_error(m), code(c) {}
};
struct NoSuchElement : Error {
    explicit NoSuchElement(const std::string &m) : Error(LIME_ERR_CONTIG, m) {}
};

inline void check(int rc) {
    if (rc != LIME_OK) throw Error(rc, lime_last_error());
}

template <class T>
using RDD = std::vector<std::pair<ReferenceRegion, T>>;
using PartitionMap = std::vector<std::optional<std::pair<ReferenceRegion, ReferenceRegion>>>;

// One device context shared by the operators of a thread.
class Engine {
   public:
    explicit Engine(int device = 0) {
        // the header and the loaded library must agree on the C-ABI contract
        if (lime_abi_version() != LIME_ABI_VERSION)
            throw std::runtime_error("liblime_amd C-ABI version " +
                                     std::to_string(lime_abi_version()) + ", header " +
                                     std::to_string(LIME_ABI_VERSION));
        check(lime_ctx_create(device, &ctx_));
    }
    ~Engine() { lime_ctx_destroy(ctx_); }
    Engine(const Engine &) = delete;
    Engine &operator=(const Engine &) = delete;
    lime_ctx *ctx() const { return ctx_; }
    static Engine &thread_default() {
        thread_local Engine e(0);
        return e;
    }

   private:
    lime_ctx *ctx_ = nullptr;
};

namespace detail {

struct Space {
    std::vector<std::string> names;  // Java String order
    std::vector<int64_t> lengths;
    std::unordered_map<std::string, int32_t> index;
    lime_space *h = nullptr;
    Space(std::vector<std::string> nm, std::vector<int64_t> len) {
        std::vector<const char *> p;
        for (auto &s : nm) p.push_back(s.c_str());
        std::vector<int32_t> rank(nm.size());
        check(lime_contig_rank((int32_t)nm.size(), p.data(), rank.data()));
        std::vector<size_t> ord(nm.size());
        std::iota(ord.begin(), ord.end(), 0);
        std::stable_sort(ord.begin(), ord.end(), [&](size_t a, size_t b) { return rank[a] < rank[b]; });
        for (size_t i : ord) {
            index[nm[i]] = (int32_t)names.size();
            names.push_back(nm[i]);
            lengths.push_back(len[i]);
        }
        check(lime_space_create((int32_t)names.size(), lengths.data(), &h));
    }
    ~Space() { lime_space_destroy(h); }
    Space(const Space &) = delete;
};

// A space holds u32 global coordinates (span sum(len + 1) <= 2^32 - 1).  A
// larger genome is cut, in Java String order, into consecutive spaces below
// the cap; every operator but closest is contig-local and runs space by
// space, closest chains its sweep liveness (lime_closest_count_chained).
// LIME_SPAN_CAP lowers the cap (tests cut small genomes the same way).
inline int64_t span_cap() {
    const char *e = std::getenv("LIME_SPAN_CAP");
    const int64_t v = e ? std::atoll(e) : 0;
    return v > 0 && v < 0xFFFFFFFFll ? v : 0xFFFFFFFFll;
}

struct Genome {
    std::vector<std::unique_ptr<Space>> spaces;
    std::unordered_map<std::string, int> group;
    Genome(const std::vector<std::string> &nm, const std::vector<int64_t> &len) {
        std::vector<const char *> p;
        for (auto &x : nm) p.push_back(x.c_str());
        std::vector<int32_t> rank(nm.size());
        if (!nm.empty()) check(lime_contig_rank((int32_t)nm.size(), p.data(), rank.data()));
        std::vector<size_t> ord(nm.size());
        std::iota(ord.begin(), ord.end(), 0);
        std::stable_sort(ord.begin(), ord.end(), [&](size_t a, size_t b) { return rank[a] < rank[b]; });
        const int64_t cap = span_cap();
        std::vector<std::string> cn;
        std::vector<int64_t> cl;
        int64_t span = 0;
        for (size_t i : ord) {
            if (len[i] + 1 > cap)
                throw Error(LIME_ERR_RANGE, "contig " + nm[i] + " is longer than a space can hold");
            if (!cn.empty() && span + len[i] + 1 > cap) {
                spaces.push_back(std::make_unique<Space>(cn, cl));
                cn.clear();
                cl.clear();
                span = 0;
            }
            group[nm[i]] = (int)spaces.size();
            cn.push_back(nm[i]);
            cl.push_back(len[i]);
            span += len[i] + 1;
        }
        if (!cn.empty() || spaces.empty()) spaces.push_back(std::make_unique<Space>(cn, cl));
    }
    // rows (indices into rdd) per space, in their given order
    template <class T>
    std::vector<std::vector<size_t>> split(const RDD<T> &rdd, const std::vector<size_t> &rows) const {
        std::vector<std::vector<size_t>> out(spaces.size());
        for (size_t i : rows) {
            auto it = group.find(rdd[i].first.referenceName);
            if (it == group.end()) throw NoSuchElement("key not found: " + rdd[i].first.referenceName);
            out[(size_t)it->second].push_back(i);
        }
        return out;
    }
};

template <class T>
std::unique_ptr<Genome> space_of(std::initializer_list<const RDD<T> *> rdds) {
    std::map<std::string, int64_t> ext;
    for (auto *r : rdds)
        for (auto &kv : *r) {
            auto &e = ext[kv.first.referenceName];
            e = std::max(e, kv.first.end);
        }
    std::vector<std::string> n;
    std::vector<int64_t> l;
    for (auto &kv : ext) {
        n.push_back(kv.first);
        l.push_back(kv.second);
    }
    return std::make_unique<Genome>(n, l);
}

inline std::vector<size_t> all_rows(size_t n) {
    std::vector<size_t> r(n);
    std::iota(r.begin(), r.end(), 0);
    return r;
}

struct SetHandle {
    lime_set *h = nullptr;
    ~SetHandle() { lime_set_destroy(h); }
};

template <class T>
void upload(lime_ctx *ctx, const Space &sp, const RDD<T> &rdd, const std::vector<size_t> &rows,
            SetHandle &out, bool stranded = false) {
    std::vector<int32_t> c(rows.size());
    std::vector<int64_t> s(rows.size()), e(rows.size());
    std::vector<int8_t> st(rows.size());
    for (size_t k = 0; k < rows.size(); ++k) {
        const auto &r = rdd[rows[k]].first;
        auto it = sp.index.find(r.referenceName);
        if (it == sp.index.end()) throw NoSuchElement("key not found: " + r.referenceName);
        c[k] = it->second;
        s[k] = r.start;
        e[k] = r.end;
        st[k] = (int8_t)r.strand;
    }
    if (stranded)
        check(lime_set_create_host_stranded(ctx, sp.h, (int64_t)rows.size(), c.data(), s.data(),
                                            e.data(), st.data(), &out.h));
    else
        check(lime_set_create_host(ctx, sp.h, (int64_t)rows.size(), c.data(), s.data(),
                                   e.data(), &out.h));
}

// more than one distinct strand among the rows
template <class T>
bool mixed_strands(const RDD<T> &rdd) {
    for (size_t i = 1; i < rdd.size(); ++i)
        if (rdd[i].first.strand != rdd[0].first.strand) return true;
    return false;
}

template <class T>
std::map<Strand, std::vector<size_t>> strand_groups(const RDD<T> &rdd) {
    std::map<Strand, std::vector<size_t>> g;
    for (size_t i = 0; i < rdd.size(); ++i) g[rdd[i].first.strand].push_back(i);
    return g;
}

inline std::u16string u16(const std::string &s) {  // for Java String order
    std::u16string o;
    for (size_t i = 0; i < s.size();) {
        unsigned char b = (unsigned char)s[i];
        uint32_t cp;
        int k = b < 0x80 ? 1 : (b >> 5) == 6 ? 2 : (b >> 4) == 14 ? 3 : (b >> 3) == 30 ? 4 : 1;
        cp = k == 1 ? b : k == 2 ? b & 0x1f : k == 3 ? b & 0x0f : b & 0x07;
        for (int j = 1; j < k && i + j < s.size(); ++j) cp = (cp << 6) | ((unsigned char)s[i + j] & 0x3f);
        i += k;
        if (cp >= 0x10000) {
            cp -= 0x10000;
            o.push_back((char16_t)(0xD800 + (cp >> 10)));
            o.push_back((char16_t)(0xDC00 + (cp & 0x3ff)));
        } else {
            o.push_back((char16_t)cp);
        }
    }
    return o;
}

// rank of each row in RegionOrdering (name, start, end, strand), stable
template <class T>
std::vector<size_t> sorted_rank(const RDD<T> &rdd) {
    std::vector<size_t> idx(rdd.size());
    std::iota(idx.begin(), idx.end(), 0);
    std::vector<std::u16string> key(rdd.size());
    for (size_t i = 0; i < rdd.size(); ++i) key[i] = u16(rdd[i].first.referenceName);
    std::stable_sort(idx.begin(), idx.end(), [&](size_t a, size_t b) {
        const auto &x = rdd[a].first, &y = rdd[b].first;
        if (key[a] != key[b]) return key[a] < key[b];
        if (x.start != y.start) return x.start < y.start;
        if (x.end != y.end) return x.end < y.end;
        return strand_ord(x.strand) < strand_ord(y.strand);
    });
    std::vector<size_t> rank(rdd.size());
    for (size_t k = 0; k < idx.size(); ++k) rank[idx[k]] = k;
    return rank;
}

}  // namespace detail

namespace detail {
// the contigs of both sides, each as long as its furthest end
template <class T, class U>
std::unique_ptr<Genome> join_space(const RDD<T> &left, const RDD<U> &right) {
    std::map<std::string, int64_t> ext;
    for (auto &kv : left) {
        auto &e = ext[kv.first.referenceName];
        e = std::max(e, kv.first.end);
    }
    for (auto &kv : right) {
        auto &e = ext[kv.first.referenceName];
        e = std::max(e, kv.first.end);
    }
    std::vector<std::string> n;
    std::vector<int64_t> l;
    for (auto &kv : ext) {
        n.push_back(kv.first);
        l.push_back(kv.second);
    }
    return std::make_unique<Genome>(n, l);
}

struct PairHit {
    size_t a, b;
    int64_t s, e;
};
// Pairwise join of two keyed RDDs through the engine, one strand group at a
// time (ReferenceRegion.overlaps / distance need equal strands), returned in
// the reference's P = 1 emission order: left in sorted order, then cache
// (= sorted right) order (SetTheory.scala:181-186).
template <typename T, typename U, typename PlanFn>
std::vector<PairHit> pair_join(const RDD<T> &left, const RDD<U> &right, Engine &eng,
                               PlanFn make_plan) {
    auto gn = join_space(left, right);
    auto lg = strand_groups(left);
    auto rg = strand_groups(right);
    std::vector<PairHit> hits;
    for (auto &g : lg) {
        auto it = rg.find(g.first);
        if (it == rg.end()) continue;
        auto ls = gn->split(left, g.second), rs = gn->split(right, it->second);
        for (size_t k = 0; k < gn->spaces.size(); ++k) {
            if (ls[k].empty() || rs[k].empty()) continue;
            SetHandle A, B;
            upload(eng.ctx(), *gn->spaces[k], left, ls[k], A);
            upload(eng.ctx(), *gn->spaces[k], right, rs[k], B);
            lime_pairs *plan = nullptr;
            int64_t n = 0;
            check(make_plan(eng.ctx(), A.h, B.h, &plan, &n));
            std::vector<lime_pair> p((size_t)n);
            int rc = lime_intersect_fill_host(plan, 0, n, p.data());
            lime_pairs_destroy(plan);
            check(rc);
            for (auto &x : p) hits.push_back({ls[k][x.a_row], rs[k][x.b_row], x.start, x.end});
        }
    }
    auto lr = sorted_rank(left);
    auto rr = sorted_rank(right);
    std::sort(hits.begin(), hits.end(), [&](const PairHit &x, const PairHit &y) {
        return lr[x.a] != lr[y.a] ? lr[x.a] < lr[y.a] : rr[x.b] < rr[y.b];
    });
    return hits;
}
}  // namespace detail

// DistributedWindow (Window.scala:71-95): every right row nearby each left
// row (ADAM isNearby, default distance 1000), keyed by the left region.
template <typename T, typename U>
class DistributedWindow {
   public:
    DistributedWindow(RDD<T> left, RDD<U> right, PartitionMap partitionMap = {},
                      int64_t threshold = 1000, Engine &eng = Engine::thread_default())
        : left_(std::move(left)), right_(std::move(right)), pm_(std::move(partitionMap)),
          threshold_(threshold), eng_(eng) {}

    std::vector<std::pair<ReferenceRegion, std::pair<T, U>>> compute() {
        auto hits = detail::pair_join(left_, right_, eng_, [&](lime_ctx *c, lime_set *a,
                                                              lime_set *b, lime_pairs **pl,
                                                              int64_t *n) {
            return lime_window_count(c, a, b, threshold_, pl, n);
        });
        std::vector<std::pair<ReferenceRegion, std::pair<T, U>>> out;
        out.reserve(hits.size());
        for (auto &h : hits)
            out.push_back({left_[h.a].first, {left_[h.a].second, right_[h.b].second}});
        return out;
    }

   private:
    RDD<T> left_;
    RDD<U> right_;
    PartitionMap pm_;
    int64_t threshold_;
    Engine &eng_;
};

// SingleClosest (Closest.scala:34-214, the CLI's closest): for each left row
// in RegionOrdering, the cached right rows at the same unstrandedDistance as
// the sweep's currentClosest, keyed by the left region; the reference's sweep
// on one partition (lime_closest_count).  Rows of every strand go into one
// stranded set per side (the order includes strand, the distance ignores it).
template <typename T, typename U, int MODE = LIME_CLOSEST>
class ClosestOp {
   public:
    ClosestOp(RDD<T> left, RDD<U> right, PartitionMap partitionMap = {},
              Engine &eng = Engine::thread_default())
        : left_(std::move(left)), right_(std::move(right)), pm_(std::move(partitionMap)),
          eng_(eng) {}

    std::vector<std::pair<ReferenceRegion, std::pair<T, U>>> compute() {
        auto gn = detail::join_space(left_, right_);
        auto ls = gn->split(left_, detail::all_rows(left_.size()));
        auto rs = gn->split(right_, detail::all_rows(right_.size()));
        std::vector<std::pair<ReferenceRegion, std::pair<T, U>>> out;
        int32_t live = 1;  // the sweep's liveness, carried from space to space
        for (size_t k = 0; k < gn->spaces.size(); ++k) {
            detail::SetHandle A, B;
            detail::upload(eng_.ctx(), *gn->spaces[k], left_, ls[k], A, true);
            detail::upload(eng_.ctx(), *gn->spaces[k], right_, rs[k], B, true);
            lime_pairs *plan = nullptr;
            int64_t n = 0;
            int32_t next = 0;
            check(lime_closest_count_chained(eng_.ctx(), A.h, B.h, MODE, live, &next, &plan, &n));
            live = next;
            std::vector<lime_pair> p((size_t)n);
            int rc = lime_intersect_fill_host(plan, 0, n, p.data());
            lime_pairs_destroy(plan);
            check(rc);
            for (auto &x : p) {
                const size_t a = ls[k][x.a_row], b = rs[k][x.b_row];
                out.push_back({left_[a].first, {left_[a].second, right_[b].second}});
            }
        }
        return out;
    }

   private:
    RDD<T> left_;
    RDD<U> right_;
    PartitionMap pm_;
    Engine &eng_;
};
template <typename T, typename U>
using SingleClosest = ClosestOp<T, U, LIME_CLOSEST>;
// Closest.scala:216-268 (the suite's variant: covered lengths compared too)
template <typename T, typename U>
using SingleClosestSingleOverlap = ClosestOp<T, U, LIME_CLOSEST_SINGLE_OVERLAP>;

template <class T, class U>
class DistributedIntersection {
   public:
    DistributedIntersection(RDD<T> left, RDD<U> right, PartitionMap partitionMap = {},
                            int64_t threshold = 0, Engine &eng = Engine::thread_default())
        : left_(std::move(left)), right_(std::move(right)), pm_(std::move(partitionMap)),
          threshold_(threshold), eng_(eng) {}

    std::vector<std::pair<ReferenceRegion, std::pair<T, U>>> compute() {
        auto hits = detail::pair_join(left_, right_, eng_, [&](lime_ctx *c, lime_set *a,
                                                              lime_set *b, lime_pairs **pl,
                                                              int64_t *n) {
            return lime_intersect_count(c, a, b, threshold_, pl, n);
        });
        std::vector<std::pair<ReferenceRegion, std::pair<T, U>>> out;
        out.reserve(hits.size());
        for (auto &h : hits) {
            const auto &a = left_[h.a].first;
            out.push_back({ReferenceRegion(a.referenceName, h.s, h.e, a.strand),
                           {left_[h.a].second, right_[h.b].second}});
        }
        return out;
    }

   private:
    RDD<T> left_;
    RDD<U> right_;
    PartitionMap pm_;
    int64_t threshold_;
    Engine &eng_;
};

template <class T, class U>
class DistributedSubtract {
   public:
    DistributedSubtract(RDD<T> left, RDD<U> right, PartitionMap partitionMap = {},
                        int64_t threshold = 0, int mode = LIME_SUBTRACT_LIME,
                        Engine &eng = Engine::thread_default())
        : left_(std::move(left)), right_(std::move(right)), pm_(std::move(partitionMap)),
          threshold_(threshold), mode_(mode), eng_(eng) {}

    std::vector<std::pair<ReferenceRegion, std::pair<T, std::optional<U>>>> compute() {
        auto gn = detail::join_space(left_, right_);
        auto lg = detail::strand_groups(left_);
        auto rg = detail::strand_groups(right_);
        struct Rem { size_t a; int64_t k; int64_t b; int64_t s, e; };
        std::vector<Rem> rem;
        for (auto &g : lg) {
            static const std::vector<size_t> none;
            auto it = rg.find(g.first);
            auto ls = gn->split(left_, g.second);
            auto rs = gn->split(right_, it == rg.end() ? none : it->second);
            for (size_t q = 0; q < gn->spaces.size(); ++q) {
                if (ls[q].empty()) continue;
                detail::SetHandle A, B;
                detail::upload(eng_.ctx(), *gn->spaces[q], left_, ls[q], A);
                detail::upload(eng_.ctx(), *gn->spaces[q], right_, rs[q], B);
                lime_result *res = nullptr;
                int64_t cnt = 0;
                check(lime_subtract(eng_.ctx(), A.h, B.h, threshold_, mode_, &res, &cnt));
                std::vector<int32_t> c((size_t)cnt);
                std::vector<int64_t> s((size_t)cnt), e((size_t)cnt), ar((size_t)cnt), br((size_t)cnt);
                int rc = lime_result_fill_host(res, c.data(), s.data(), e.data(), ar.data(), br.data());
                lime_result_destroy(res);
                check(rc);
                for (int64_t k = 0; k < cnt; ++k)
                    rem.push_back({ls[q][ar[k]], k, br[k] < 0 ? -1 : (int64_t)rs[q][br[k]], s[k], e[k]});
            }
        }
        auto lr = detail::sorted_rank(left_);
        std::stable_sort(rem.begin(), rem.end(), [&](const Rem &x, const Rem &y) {
            return lr[x.a] != lr[y.a] ? lr[x.a] < lr[y.a] : x.k < y.k;
        });
        std::vector<std::pair<ReferenceRegion, std::pair<T, std::optional<U>>>> out;
        for (auto &r : rem) {
            const auto &a = left_[r.a].first;
            std::optional<U> u;
            if (r.b >= 0) u = right_[r.b].second;
            out.push_back({ReferenceRegion(a.referenceName, r.s, r.e, a.strand), {left_[r.a].second, u}});
        }
        return out;
    }

   private:
    RDD<T> left_;
    RDD<U> right_;
    PartitionMap pm_;
    int64_t threshold_;
    int mode_;
    Engine &eng_;
};

template <class T>
class DistributedMerge {
   public:
    DistributedMerge(RDD<T> rdd, PartitionMap partitionMap = {}, int64_t threshold = 0,
                     Engine &eng = Engine::thread_default())
        : rdd_(std::move(rdd)), pm_(std::move(partitionMap)), threshold_(threshold), eng_(eng) {}

    // the SetTheory.scala:208-225 fold; mixed strands run as ONE stranded set
    // (RegionOrdering order, a run break at every strand change)
    std::vector<std::pair<ReferenceRegion, std::vector<T>>> compute() {
        auto gn = detail::space_of<T>({&rdd_});
        auto rank = detail::sorted_rank(rdd_);
        const bool mixed = detail::mixed_strands(rdd_);
        auto parts = gn->split(rdd_, detail::all_rows(rdd_.size()));
        std::vector<std::pair<ReferenceRegion, std::vector<T>>> out;
        for (size_t q = 0; q < gn->spaces.size(); ++q) {
            const auto &rows = parts[q];
            if (rows.empty()) continue;
            const auto &sp = *gn->spaces[q];
            detail::SetHandle A;
            detail::upload(eng_.ctx(), sp, rdd_, rows, A, mixed);
            lime_result *res = nullptr;
            int64_t cnt = 0;
            check(lime_merge(eng_.ctx(), A.h, &res, &cnt));
            std::vector<int32_t> c((size_t)cnt);
            std::vector<int64_t> s((size_t)cnt), e((size_t)cnt), rid(rows.size());
            int rc = lime_result_fill_host(res, c.data(), s.data(), e.data(), nullptr, nullptr);
            if (rc == LIME_OK) rc = lime_result_run_of_row(res, rid.data());
            lime_result_destroy(res);
            check(rc);
            std::vector<std::vector<size_t>> members((size_t)cnt);
            std::vector<size_t> order(rows.size());
            std::iota(order.begin(), order.end(), 0);
            std::sort(order.begin(), order.end(),
                      [&](size_t x, size_t y) { return rank[rows[x]] < rank[rows[y]]; });
            for (size_t m : order) members[(size_t)rid[m]].push_back(rows[m]);
            for (int64_t k = 0; k < cnt; ++k) {
                const Strand st = members[k].empty() ? Strand::Independent
                                                     : rdd_[members[k][0]].first.strand;
                std::vector<T> v;
                for (size_t m : members[k]) v.push_back(rdd_[m].second);
                out.push_back({ReferenceRegion(sp.names[c[k]], s[k], e[k], st), std::move(v)});
            }
        }
        return out;
    }

   private:
    RDD<T> rdd_;
    PartitionMap pm_;
    int64_t threshold_;
    Engine &eng_;
};

// Cluster.scala:8-121: Merge's fold, keyed by each cluster's FIRST member
// region (postProcess :33-35).  The fold passes no threshold (quirk Q6), so
// every variant is the strict-overlap fold: strand-blind (covers) for the
// unstranded variants; overlaps (a run break at every strand change, one
// stranded set) for the stranded ones.
template <class T, bool STRANDED>
class ClusterOp {
   public:
    ClusterOp(RDD<T> rdd, PartitionMap partitionMap = {}, int64_t threshold = 0,
              Engine &eng = Engine::thread_default())
        : rdd_(std::move(rdd)), pm_(std::move(partitionMap)), threshold_(threshold), eng_(eng) {}

    std::vector<std::pair<ReferenceRegion, std::vector<T>>> compute() {
        auto gn = detail::space_of<T>({&rdd_});
        auto rank = detail::sorted_rank(rdd_);
        const bool mixed = STRANDED && detail::mixed_strands(rdd_);
        auto parts = gn->split(rdd_, detail::all_rows(rdd_.size()));
        std::vector<std::vector<size_t>> clusters;  // member rows in fold order
        for (size_t q = 0; q < gn->spaces.size(); ++q) {
            const auto &rows = parts[q];
            if (rows.empty()) continue;
            detail::SetHandle A;
            detail::upload(eng_.ctx(), *gn->spaces[q], rdd_, rows, A, mixed);
            lime_result *res = nullptr;
            int64_t cnt = 0;
            check(lime_merge(eng_.ctx(), A.h, &res, &cnt));
            std::vector<int64_t> rid(rows.size());
            int rc = lime_result_run_of_row(res, rid.data());
            lime_result_destroy(res);
            check(rc);
            std::vector<size_t> order(rows.size());
            std::iota(order.begin(), order.end(), 0);
            std::sort(order.begin(), order.end(),
                      [&](size_t x, size_t y) { return rank[rows[x]] < rank[rows[y]]; });
            const size_t base = clusters.size();
            clusters.resize(base + (size_t)cnt);
            for (size_t m : order) clusters[base + (size_t)rid[m]].push_back(rows[m]);
        }
        std::sort(clusters.begin(), clusters.end(),
                  [&](const std::vector<size_t> &x, const std::vector<size_t> &y) {
                      return rank[x[0]] < rank[y[0]];
                  });
        std::vector<std::pair<ReferenceRegion, std::vector<T>>> out;
        for (auto &c : clusters) {
            std::vector<T> v;
            for (size_t i : c) v.push_back(rdd_[i].second);
            out.push_back({rdd_[c[0]].first, std::move(v)});
        }
        return out;
    }

   private:
    RDD<T> rdd_;
    PartitionMap pm_;
    int64_t threshold_;
    Engine &eng_;
};
template <class T>
using UnstrandedCluster = ClusterOp<T, false>;
template <class T>
using UnstrandedClusterWithMinimumOverlap = ClusterOp<T, false>;
template <class T>
using StrandedCluster = ClusterOp<T, true>;
template <class T>
using StrandedClusterWithMinimumOverlap = ClusterOp<T, true>;

template <class T>
class DistributedComplement {
   public:
    DistributedComplement(RDD<T> rdd, PartitionMap partitionMap,
                          std::map<std::string, ReferenceRegion> referenceNameBounds,
                          int64_t threshold = 0, Engine &eng = Engine::thread_default())
        : rdd_(std::move(rdd)), pm_(std::move(partitionMap)),
          bounds_(std::move(referenceNameBounds)), threshold_(threshold), eng_(eng) {}

    std::vector<std::pair<ReferenceRegion, std::vector<T>>> compute() {
        std::vector<std::string> n;
        std::vector<int64_t> l;
        for (auto &kv : bounds_) {
            n.push_back(kv.first);
            l.push_back(kv.second.end);
        }
        detail::Genome gn(n, l);
        auto parts = gn.split(rdd_, detail::all_rows(rdd_.size()));  // throws NoSuchElement
        std::vector<std::pair<ReferenceRegion, std::vector<T>>> out;
        for (size_t q = 0; q < gn.spaces.size(); ++q) {
            const auto &sp = *gn.spaces[q];
            detail::SetHandle A;
            detail::upload(eng_.ctx(), sp, rdd_, parts[q], A);
            lime_result *res = nullptr;
            int64_t cnt = 0;
            check(lime_complement(eng_.ctx(), sp.h, A.h, &res, &cnt));
            std::vector<int32_t> c((size_t)cnt);
            std::vector<int64_t> s((size_t)cnt), e((size_t)cnt);
            int rc = lime_result_fill_host(res, c.data(), s.data(), e.data(), nullptr, nullptr);
            lime_result_destroy(res);
            check(rc);
            for (int64_t k = 0; k < cnt; ++k)
                out.push_back({ReferenceRegion(sp.names[c[k]], s[k], e[k]), {}});
        }
        return out;
    }

   private:
    RDD<T> rdd_;
    PartitionMap pm_;
    std::map<std::string, ReferenceRegion> bounds_;
    int64_t threshold_;
    Engine &eng_;
};

}  // namespace lime
