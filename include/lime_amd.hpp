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
    explicit Engine(int device = 0) { check(lime_ctx_create(device, &ctx_)); }
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

template <class T>
std::unique_ptr<Space> space_of(std::initializer_list<const RDD<T> *> rdds) {
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
    return std::make_unique<Space>(n, l);
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
std::unique_ptr<Space> join_space(const RDD<T> &left, const RDD<U> &right) {
    auto sp = space_of<T>({&left});
    std::map<std::string, int64_t> ext;
    for (size_t c = 0; c < sp->names.size(); ++c) ext[sp->names[c]] = sp->lengths[c];
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
    return std::make_unique<Space>(n, l);
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
    auto sp = join_space(left, right);
    auto lg = strand_groups(left);
    auto rg = strand_groups(right);
    std::vector<PairHit> hits;
    for (auto &g : lg) {
        auto it = rg.find(g.first);
        if (it == rg.end()) continue;
        SetHandle A, B;
        upload(eng.ctx(), *sp, left, g.second, A);
        upload(eng.ctx(), *sp, right, it->second, B);
        lime_pairs *plan = nullptr;
        int64_t n = 0;
        check(make_plan(eng.ctx(), A.h, B.h, &plan, &n));
        std::vector<lime_pair> p((size_t)n);
        int rc = lime_intersect_fill_host(plan, 0, n, p.data());
        lime_pairs_destroy(plan);
        check(rc);
        for (auto &x : p) hits.push_back({g.second[x.a_row], it->second[x.b_row], x.start, x.end});
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
        auto sp = detail::join_space(left_, right_);
        std::vector<size_t> la(left_.size()), ra(right_.size());
        for (size_t i = 0; i < la.size(); ++i) la[i] = i;
        for (size_t i = 0; i < ra.size(); ++i) ra[i] = i;
        detail::SetHandle A, B;
        detail::upload(eng_.ctx(), *sp, left_, la, A, true);
        detail::upload(eng_.ctx(), *sp, right_, ra, B, true);
        lime_pairs *plan = nullptr;
        int64_t n = 0;
        check(lime_closest_count(eng_.ctx(), A.h, B.h, MODE, &plan, &n));
        std::vector<lime_pair> p((size_t)n);
        int rc = lime_intersect_fill_host(plan, 0, n, p.data());
        lime_pairs_destroy(plan);
        check(rc);
        std::vector<std::pair<ReferenceRegion, std::pair<T, U>>> out;
        out.reserve(p.size());
        for (auto &x : p)
            out.push_back({left_[x.a_row].first, {left_[x.a_row].second, right_[x.b_row].second}});
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
        std::map<std::string, int64_t> ext;
        for (auto &kv : left_) ext[kv.first.referenceName] = std::max(ext[kv.first.referenceName], kv.first.end);
        for (auto &kv : right_) ext[kv.first.referenceName] = std::max(ext[kv.first.referenceName], kv.first.end);
        std::vector<std::string> n;
        std::vector<int64_t> l;
        for (auto &kv : ext) {
            n.push_back(kv.first);
            l.push_back(kv.second);
        }
        detail::Space sp(n, l);
        auto lg = detail::strand_groups(left_);
        auto rg = detail::strand_groups(right_);
        struct Rem { size_t a; int64_t k; int64_t b; int64_t s, e; };
        std::vector<Rem> rem;
        for (auto &g : lg) {
            static const std::vector<size_t> none;
            auto it = rg.find(g.first);
            const auto &rrows = it == rg.end() ? none : it->second;
            detail::SetHandle A, B;
            detail::upload(eng_.ctx(), sp, left_, g.second, A);
            detail::upload(eng_.ctx(), sp, right_, rrows, B);
            lime_result *res = nullptr;
            int64_t cnt = 0;
            check(lime_subtract(eng_.ctx(), A.h, B.h, threshold_, mode_, &res, &cnt));
            std::vector<int32_t> c((size_t)cnt);
            std::vector<int64_t> s((size_t)cnt), e((size_t)cnt), ar((size_t)cnt), br((size_t)cnt);
            int rc = lime_result_fill_host(res, c.data(), s.data(), e.data(), ar.data(), br.data());
            lime_result_destroy(res);
            check(rc);
            for (int64_t k = 0; k < cnt; ++k)
                rem.push_back({g.second[ar[k]], k, br[k] < 0 ? -1 : (int64_t)rrows[br[k]], s[k], e[k]});
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
        auto sp = detail::space_of<T>({&rdd_});
        auto rank = detail::sorted_rank(rdd_);
        std::vector<size_t> all(rdd_.size());
        std::iota(all.begin(), all.end(), 0);
        detail::SetHandle A;
        detail::upload(eng_.ctx(), *sp, rdd_, all, A, detail::mixed_strands(rdd_));
        lime_result *res = nullptr;
        int64_t cnt = 0;
        check(lime_merge(eng_.ctx(), A.h, &res, &cnt));
        std::vector<int32_t> c((size_t)cnt);
        std::vector<int64_t> s((size_t)cnt), e((size_t)cnt), rid(all.size());
        int rc = lime_result_fill_host(res, c.data(), s.data(), e.data(), nullptr, nullptr);
        if (rc == LIME_OK) rc = lime_result_run_of_row(res, rid.data());
        lime_result_destroy(res);
        check(rc);
        std::vector<std::vector<size_t>> members((size_t)cnt);
        std::vector<size_t> order(all);
        std::sort(order.begin(), order.end(), [&](size_t x, size_t y) { return rank[x] < rank[y]; });
        for (size_t m : order) members[(size_t)rid[m]].push_back(m);
        std::vector<std::pair<ReferenceRegion, std::vector<T>>> out;
        for (int64_t k = 0; k < cnt; ++k) {
            const Strand st = members[k].empty() ? Strand::Independent
                                                 : rdd_[members[k][0]].first.strand;
            std::vector<T> v;
            for (size_t m : members[k]) v.push_back(rdd_[m].second);
            out.push_back({ReferenceRegion(sp->names[c[k]], s[k], e[k], st), std::move(v)});
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
        auto sp = detail::space_of<T>({&rdd_});
        auto rank = detail::sorted_rank(rdd_);
        std::vector<size_t> all(rdd_.size());
        std::iota(all.begin(), all.end(), 0);
        std::vector<std::vector<size_t>> clusters;  // member rows in fold order
        if (!all.empty()) {
            detail::SetHandle A;
            detail::upload(eng_.ctx(), *sp, rdd_, all, A, STRANDED && detail::mixed_strands(rdd_));
            lime_result *res = nullptr;
            int64_t cnt = 0;
            check(lime_merge(eng_.ctx(), A.h, &res, &cnt));
            std::vector<int64_t> rid(all.size());
            int rc = lime_result_run_of_row(res, rid.data());
            lime_result_destroy(res);
            check(rc);
            std::vector<size_t> order(all);
            std::sort(order.begin(), order.end(),
                      [&](size_t x, size_t y) { return rank[x] < rank[y]; });
            clusters.resize((size_t)cnt);
            for (size_t m : order) clusters[(size_t)rid[m]].push_back(m);
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
        detail::Space sp(n, l);
        std::vector<size_t> rows(rdd_.size());
        std::iota(rows.begin(), rows.end(), 0);
        detail::SetHandle A;
        detail::upload(eng_.ctx(), sp, rdd_, rows, A);  // throws NoSuchElement
        lime_result *res = nullptr;
        int64_t cnt = 0;
        check(lime_complement(eng_.ctx(), sp.h, A.h, &res, &cnt));
        std::vector<int32_t> c((size_t)cnt);
        std::vector<int64_t> s((size_t)cnt), e((size_t)cnt);
        int rc = lime_result_fill_host(res, c.data(), s.data(), e.data(), nullptr, nullptr);
        lime_result_destroy(res);
        check(rc);
        std::vector<std::pair<ReferenceRegion, std::vector<T>>> out;
        for (int64_t k = 0; k < cnt; ++k)
            out.push_back({ReferenceRegion(sp.names[c[k]], s[k], e[k]), {}});
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
