/*
 * lime_oracle.c -- CPU restatement of LIME's per-partition set-theory
 * algorithms.  TEST INFRASTRUCTURE ONLY: this file is the parity checker for
 * the HIP engine (tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
 * leg).  It is never linked into, loaded by, or called from the product path
 * (lime_amd/liblime_amd.so).
 *
 * What it restates (all paths relative to /root/reference):
 *   - region order + predicates: ADAM 0.23 ReferenceRegion (3rd-party, not
 *     vendored; restated from its call sites):
 *       compareTo at OverlapBasedSetTheory.scala:23,37
 *       covers(o)  = same name && a.end > o.start && a.start < o.end (strand-blind)
 *       overlaps(o)= covers(o) && same strand
 *       overlapsBy = min(end) - max(start) if overlaps, else None
 *   - sweep-line join: SetTheory.scala:131-187 (pruneCache :131-141 incl. the
 *     Q8 "index <= 0 -> trim nothing" quirk, advanceCache :150-155,
 *     makeIterator :175-187) with OverlapBasedSetTheory.scala:21-38 predicates.
 *   - intersection: Intersection.scala:19-24 (primitive), :37-42 (condition,
 *     uses the *field* threshold), :58-69 (processHits).
 *   - subtract: Subtract.scala:19-24 (condition), :53-75 (subtract), :91-116
 *     (processHits: filter, reverse-order fold into blocks, per-block
 *     remnants -- quirk Q5).  Mode LO_SUB_SET additionally restates the
 *     set-difference definition of SURVEY.md Appendix A.3.
 *   - merge: SetTheory.scala:208-225 (localCompute fold; condition/primitive
 *     called without threshold -> 0, quirk Q6), Merge.scala:8-31.
 *   - window: Window.scala:51-95 (cache predicates and processHits) over the
 *     same sweep, with ADAM's isNearby / distance (gap + 1) restated.
 *   - closest: Closest.scala:10-268 (SingleClosest, SingleClosestSingleOverlap)
 *     with its mutable currentClosest over the same sweep, pinned by the
 *     arrays of ClosestSuite.scala:21-45,64-85.
 *   - complement: Complement.scala:11-128 as pinned by ComplementSuite.scala
 *     (canonical P=1-independent form): gaps of
 *     merge(A) per genome contig in String order, zero-width gaps dropped,
 *     contigs without data emitted whole.
 *
 * Every op runs the reference's algorithm as a single partition (P = 1); the
 * partition-count artefacts Q1/Q2 of SURVEY.md Appendix B are deliberately not
 * reproduced (they make Spark's own output P-dependent).
 *
 * Output arrays use the two-call protocol: each op returns the exact output
 * count and writes min(count, cap) records, so callers ask with cap = 0 first.
 */
#define _POSIX_C_SOURCE 200809L
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
    int32_t contig; /* rank of the contig name in Java String order */
    int64_t start;
    int64_t end;
    int8_t strand; /* 0 = unstranded / independent */
    int64_t row;   /* original input row: the payload T / U */
} lo_region;

/* ------------------------------------------------------------------ order */

/* Strand codes are 0 independent, 1 forward, 2 reverse, 3 unknown; the
 * ordering compares bdg-formats' Strand enum ordinals (FORWARD, REVERSE,
 * INDEPENDENT, UNKNOWN -- 3rd-party schema, restated). */
static int lo_strand_ord(int8_t c) {
    static const int ord[4] = {2, 0, 1, 3};
    return (c >= 0 && c < 4) ? ord[(int)c] : 4;
}

/* RegionOrdering: (referenceName, start, end, strand); ties by input row so
 * that equal regions keep input order (Spark's sort is stable per partition). */
static int lo_cmp(const lo_region *a, const lo_region *b) {
    if (a->contig != b->contig) return a->contig < b->contig ? -1 : 1;
    if (a->start != b->start) return a->start < b->start ? -1 : 1;
    if (a->end != b->end) return a->end < b->end ? -1 : 1;
    if (a->strand != b->strand)
        return lo_strand_ord(a->strand) < lo_strand_ord(b->strand) ? -1 : 1;
    return 0;
}
static int lo_qsort_cmp(const void *x, const void *y) {
    const lo_region *a = (const lo_region *)x, *b = (const lo_region *)y;
    int c = lo_cmp(a, b);
    if (c) return c;
    return a->row < b->row ? -1 : (a->row > b->row ? 1 : 0);
}

static int lo_covers(const lo_region *a, const lo_region *o) {
    return a->contig == o->contig && a->end > o->start && a->start < o->end;
}
static int lo_overlaps(const lo_region *a, const lo_region *o) {
    return lo_covers(a, o) && a->strand == o->strand;
}
/* overlapsBy(o).exists(_ >= t) */
static int lo_overlaps_by_at_least(const lo_region *a, const lo_region *o, int64_t t) {
    if (!lo_overlaps(a, o)) return 0;
    int64_t e = a->end < o->end ? a->end : o->end;
    int64_t s = a->start > o->start ? a->start : o->start;
    return e - s >= t;
}

static lo_region *lo_load(int64_t n, const int32_t *c, const int64_t *s, const int64_t *e,
                          const int8_t *strand) {
    lo_region *r = (lo_region *)malloc(sizeof(lo_region) * (size_t)(n > 0 ? n : 1));
    for (int64_t i = 0; i < n; ++i) {
        r[i].contig = c[i];
        r[i].start = s[i];
        r[i].end = e[i];
        r[i].strand = strand ? strand[i] : 0;
        r[i].row = i;
    }
    qsort(r, (size_t)n, sizeof(lo_region), lo_qsort_cmp);
    return r;
}

/* ------------------------------------------------------- output buffering */

typedef struct {
    int64_t count, cap;
    int32_t *contig;
    int64_t *start, *end, *lrow, *rrow;
    /* hash: also fold lo_pair_hash(start, end, lrow, rrow) into (hsum, hxor),
     * the order-independent checksum of SURVEY.md 8(d) (hash == 2: the result
     * form, mix64(lo_pair_hash(...) + contig), absent rows as 0xffffffff, as
     * the engine's lime_result_checksum); grow: the arrays are owned and
     * doubled on demand (the contig-sharded drivers below) */
    int hash, grow;
    uint64_t hsum, hxor;
} lo_out;

uint64_t lo_pair_hash(uint32_t start, uint32_t end, uint32_t a, uint32_t b);
static uint64_t lo_mix64(uint64_t z);

static void lo_out_grow(lo_out *o) {
    int64_t cap = o->cap ? 2 * o->cap : 1024;
    o->contig = (int32_t *)realloc(o->contig, sizeof(int32_t) * (size_t)cap);
    o->start = (int64_t *)realloc(o->start, sizeof(int64_t) * (size_t)cap);
    o->end = (int64_t *)realloc(o->end, sizeof(int64_t) * (size_t)cap);
    o->lrow = (int64_t *)realloc(o->lrow, sizeof(int64_t) * (size_t)cap);
    o->rrow = (int64_t *)realloc(o->rrow, sizeof(int64_t) * (size_t)cap);
    o->cap = cap;
}

static void lo_emit(lo_out *o, int32_t c, int64_t s, int64_t e, int64_t lr, int64_t rr) {
    if (o->hash) {
        uint64_t h = lo_pair_hash((uint32_t)s, (uint32_t)e, (uint32_t)lr, (uint32_t)rr);
        if (o->hash == 2) h = lo_mix64(h + (uint64_t)(uint32_t)c);
        o->hsum += h;
        o->hxor ^= h;
    }
    if (o->grow && o->count == o->cap) lo_out_grow(o);
    if (o->count < o->cap) {
        int64_t k = o->count;
        if (o->contig) o->contig[k] = c;
        if (o->start) o->start[k] = s;
        if (o->end) o->end[k] = e;
        if (o->lrow) o->lrow[k] = lr;
        if (o->rrow) o->rrow[k] = rr;
    }
    o->count++;
}

/* ----------------------------------------------------- sweep-line machinery */

/* The right-side cache: SetTheory.scala:83 ListBuffer, append at the tail
 * (advanceCache) and trimStart at the head (pruneCache). */
typedef struct {
    const lo_region **v;
    int64_t head, tail, cap;
} lo_cache;

static void cache_push(lo_cache *c, const lo_region *r) {
    if (c->tail == c->cap) {
        if (c->head > 0) { /* compact */
            memmove(c->v, c->v + c->head, sizeof(*c->v) * (size_t)(c->tail - c->head));
            c->tail -= c->head;
            c->head = 0;
        }
        if (c->tail == c->cap) {
            c->cap = c->cap ? c->cap * 2 : 64;
            c->v = (const lo_region **)realloc(c->v, sizeof(*c->v) * (size_t)c->cap);
        }
    }
    c->v[c->tail++] = r;
}

/* OverlapBasedSetTheory.scala:21-24: cached < to && !cached.covers(to) */
static int prune_cond(const lo_region *cached, const lo_region *to) {
    return lo_cmp(cached, to) < 0 && !lo_covers(cached, to);
}
/* OverlapBasedSetTheory.scala:35-38: cand <= until || cand.covers(until) */
static int advance_cond(const lo_region *cand, const lo_region *until) {
    return lo_cmp(cand, until) <= 0 || lo_covers(cand, until);
}

/* SetTheory.scala:131-141.  indexWhere(!prune) == -1 (everything prunable)
 * maps to 0, i.e. nothing is trimmed (quirk Q8, performance only). */
static void prune_cache(lo_cache *c, const lo_region *to) {
    int64_t index = -1;
    for (int64_t i = c->head; i < c->tail; ++i)
        if (!prune_cond(c->v[i], to)) { index = i - c->head; break; }
    if (index > 0) c->head += index;
}

/* SetTheory.scala:150-155 */
static void advance_cache(lo_cache *c, const lo_region *right, int64_t nr, int64_t *rpos,
                          const lo_region *until) {
    while (*rpos < nr && advance_cond(&right[*rpos], until)) cache_push(c, &right[(*rpos)++]);
}

/* ------------------------------------------------------------- intersect */

/* Intersection.scala:58-69 processHits: every cached R with
 * overlapsBy(L, R) >= threshold, in cache order, emits
 * (L.intersection(R), (L.value, R.value)). */
static void lo_intersect_sorted(const lo_region *L, int64_t nl, const lo_region *R, int64_t nr,
                                int64_t threshold, lo_out *o) {
    lo_cache cache = {0};
    int64_t rpos = 0;
    for (int64_t i = 0; i < nl; ++i) { /* SetTheory.scala:181-186 */
        const lo_region *cur = &L[i];
        advance_cache(&cache, R, nr, &rpos, cur);
        prune_cache(&cache, cur);
        for (int64_t k = cache.head; k < cache.tail; ++k) {
            const lo_region *r = cache.v[k];
            if (lo_overlaps_by_at_least(cur, r, threshold)) {
                int64_t s = cur->start > r->start ? cur->start : r->start;
                int64_t e = cur->end < r->end ? cur->end : r->end;
                lo_emit(o, cur->contig, s, e, cur->row, r->row);
            }
        }
    }
    free(cache.v);
}

int64_t lo_intersect(int64_t nl, const int32_t *lc, const int64_t *ls, const int64_t *le,
                     const int8_t *lstr, int64_t nr, const int32_t *rc, const int64_t *rs,
                     const int64_t *re, const int8_t *rstr, int64_t threshold, int64_t cap,
                     int32_t *oc, int64_t *os, int64_t *oe, int64_t *olrow, int64_t *orrow) {
    lo_region *L = lo_load(nl, lc, ls, le, lstr);
    lo_region *R = lo_load(nr, rc, rs, re, rstr);
    lo_out out = {0, cap, oc, os, oe, olrow, orrow};
    lo_intersect_sorted(L, nl, R, nr, threshold, &out);
    free(L);
    free(R);
    return out.count;
}

/* ---------------------------------------------------------------- window */

/* ADAM ReferenceRegion.distance (3rd-party, restated):
 * None across contigs (or strands, as overlaps), 0 if overlapping, else the
 * gap + 1 ("abutting regions are at distance 1").  isNearby(o, d) =
 * distance(o).exists(_ <= d).  The +1 and the strand test are not pinned by
 * WindowSuite (its pairs are all within a few bases or overlapping). */
static int lo_nearby(const lo_region *a, const lo_region *o, int64_t d) {
    if (a->contig != o->contig || a->strand != o->strand) return 0;
    if (lo_overlaps(a, o)) return 0 <= d;
    int64_t dist = o->start >= a->end ? o->start - a->end + 1 : a->start - o->end + 1;
    return dist <= d;
}

/* Window.scala:71-95 over the SetTheory.scala:131-187 sweep, with Window's
 * own cache predicates (:51-68): prune <=> cached < to && !to.isNearby(cached,
 * threshold); advance <=> cand <= until || until.isNearby(cand, threshold).
 * processHits (:84-95) emits (L, (L.value, R.value)) for every cached R with
 * L.isNearby(R, threshold), in cache order. */
int64_t lo_window(int64_t nl, const int32_t *lc, const int64_t *ls, const int64_t *le,
                  const int8_t *lstr, int64_t nr, const int32_t *rc, const int64_t *rs,
                  const int64_t *re, const int8_t *rstr, int64_t d, int64_t cap, int32_t *oc,
                  int64_t *os, int64_t *oe, int64_t *olrow, int64_t *orrow) {
    lo_region *L = lo_load(nl, lc, ls, le, lstr);
    lo_region *R = lo_load(nr, rc, rs, re, rstr);
    lo_out out = {0, cap, oc, os, oe, olrow, orrow};
    lo_cache cache = {0};
    int64_t rpos = 0;
    for (int64_t i = 0; i < nl; ++i) {
        const lo_region *cur = &L[i];
        while (rpos < nr && (lo_cmp(&R[rpos], cur) <= 0 || lo_nearby(cur, &R[rpos], d)))
            cache_push(&cache, &R[rpos++]);
        int64_t index = -1; /* pruneCache, Q8: all prunable -> trim nothing */
        for (int64_t k = cache.head; k < cache.tail; ++k)
            if (!(lo_cmp(cache.v[k], cur) < 0 && !lo_nearby(cur, cache.v[k], d))) {
                index = k - cache.head;
                break;
            }
        if (index > 0) cache.head += index;
        for (int64_t k = cache.head; k < cache.tail; ++k) {
            const lo_region *r = cache.v[k];
            if (lo_nearby(cur, r, d)) lo_emit(&out, cur->contig, cur->start, cur->end, cur->row, r->row);
        }
    }
    free(cache.v);
    free(L);
    free(R);
    return out.count;
}

/* --------------------------------------------------------------- closest */

#define LO_CLOSEST 0        /* SingleClosest (Closest.scala:34-214), the CLI's op */
#define LO_CLOSEST_SINGLE 1 /* SingleClosestSingleOverlap (Closest.scala:216-268) */
#define LO_NONE INT64_MAX   /* Option.None (different reference names) */

/* ADAM unstrandedDistance (3rd-party, restated like distance above but
 * strand-blind): None across contigs, 0 if covering, else gap + 1. */
static int64_t lo_udist(const lo_region *a, const lo_region *o) {
    if (a->contig != o->contig) return LO_NONE;
    if (lo_covers(a, o)) return 0;
    return o->start >= a->end ? o->start - a->end + 1 : a->start - o->end + 1;
}
/* ADAM coversBy: the covered length when covering, else None (restated as
 * the overlap length, like overlapsBy in Appendix A.2; the suite's arrays do
 * not tell it apart from other readings). */
static int64_t lo_covers_by(const lo_region *a, const lo_region *o) {
    if (!lo_covers(a, o)) return LO_NONE;
    int64_t e = a->end < o->end ? a->end : o->end;
    int64_t s = a->start > o->start ? a->start : o->start;
    return e - s;
}
static int64_t lo_or(int64_t v, int64_t dflt) { return v == LO_NONE ? dflt : v; }

/* Closest.scala, over the SetTheory.scala:131-187 sweep with its mutable
 * currentClosest (:12, initially ReferenceRegion("", 0, 0): contig -1 here).
 *   advance (:179-192 / :251-267) sets currentClosest = candidate on success;
 *   prune   (:160-169 / :230-241) with the Q8 "index <= 0 -> trim nothing";
 *   processHits (:202-213): every cached R with unstrandedDistance(L, R)
 *   .contains(unstrandedDistance(L, C).getOrElse(Long.MaxValue)), emitted as
 *   (L, (L.value, R.value)) in cache order.
 * One partition holding every row (P = 1), as for the other ops. */
int64_t lo_closest(int64_t nl, const int32_t *lc, const int64_t *ls, const int64_t *le,
                   const int8_t *lstr, int64_t nr, const int32_t *rc, const int64_t *rs,
                   const int64_t *re, const int8_t *rstr, int mode, int64_t cap, int32_t *oc,
                   int64_t *os, int64_t *oe, int64_t *olrow, int64_t *orrow) {
    lo_region *L = lo_load(nl, lc, ls, le, lstr);
    lo_region *R = lo_load(nr, rc, rs, re, rstr);
    lo_out out = {0, cap, oc, os, oe, olrow, orrow};
    lo_cache cache = {0};
    lo_region dummy = {-1, 0, 0, 0, -1};
    const lo_region *C = &dummy;
    int64_t rpos = 0;
    for (int64_t i = 0; i < nl; ++i) {
        const lo_region *u = &L[i];
        /* advanceCache */
        while (rpos < nr) {
            const lo_region *c = &R[rpos];
            int adv;
            if (c->contig != u->contig)
                adv = 0;
            else if (u->contig != C->contig)
                adv = 1;
            else if (mode == LO_CLOSEST)
                adv = lo_udist(u, c) <= lo_or(lo_udist(u, C), INT64_MAX);
            else
                adv = (lo_covers(u, c) && lo_covers_by(u, c) >= lo_or(lo_covers_by(u, C), 0)) ||
                      (!lo_covers(u, c) && lo_udist(u, c) <= lo_or(lo_udist(u, C), INT64_MAX));
            if (!adv) break;
            C = c;
            cache_push(&cache, &R[rpos++]);
        }
        /* pruneCache */
        int64_t index = -1;
        for (int64_t k = cache.head; k < cache.tail; ++k) {
            const lo_region *c = cache.v[k];
            int prune;
            if (c->contig != u->contig)
                prune = 1;
            else {
                prune = lo_udist(u, c) > lo_or(lo_udist(u, C), 0);
                if (mode == LO_CLOSEST_SINGLE)
                    prune = prune || (lo_covers(u, c) &&
                                      lo_covers_by(u, c) < lo_or(lo_covers_by(u, C), INT64_MAX));
            }
            if (!prune) {
                index = k - cache.head;
                break;
            }
        }
        if (index > 0) cache.head += index;
        /* processHits */
        int64_t target = lo_or(lo_udist(u, C), INT64_MAX);
        for (int64_t k = cache.head; k < cache.tail; ++k) {
            const lo_region *r = cache.v[k];
            int64_t d = lo_udist(u, r);
            if (d != LO_NONE && d == target)
                lo_emit(&out, u->contig, u->start, u->end, u->row, r->row);
        }
    }
    free(cache.v);
    free(L);
    free(R);
    return out.count;
}

/* -------------------------------------------------------------- subtract */

#define LO_SUB_LIME 0 /* Subtract.scala:103-114 exactly: per-block remnants (Q5) */
#define LO_SUB_SET 1  /* a \ union(hits): SURVEY.md Appendix A.3 'set' mode */

typedef struct {
    int64_t start, end, rrow;
} lo_block;

/* Subtract.scala:91-116 processHits over the SetTheory.scala:131-187 sweep,
 * on one sorted partition */
static void lo_subtract_sorted(const lo_region *L, int64_t nl, const lo_region *R, int64_t nr,
                               int64_t threshold, int mode, lo_out *o) {
    lo_cache cache = {0};
    int64_t rpos = 0;
    lo_block *blocks = NULL;
    int64_t bcap = 0;
    for (int64_t i = 0; i < nl; ++i) {
        const lo_region *cur = &L[i];
        advance_cache(&cache, R, nr, &rpos, cur);
        prune_cache(&cache, cur);
        /* Subtract.scala:95-98: filteredCache */
        int64_t nb = 0;
        int first = 1;
        for (int64_t k = cache.head; k < cache.tail; ++k) {
            const lo_region *r = cache.v[k];
            if (!lo_overlaps_by_at_least(cur, r, threshold)) continue;
            /* :103-108 fold: foldLeft(List(filteredCache.head)) over the WHOLE
             * filtered cache, so the head is visited twice: a no-op hull for a
             * non-empty head, a duplicated block for a zero-width one.
             * b.head overlaps a -> hull, keep head's value; otherwise start a
             * new block.  (The fold's List is built in reverse; we keep blocks
             * in forward order and emit reversed.) */
            if (first) {
                first = 0;
                if (nb == bcap) {
                    bcap = bcap ? bcap * 2 : 16;
                    blocks = (lo_block *)realloc(blocks, sizeof(lo_block) * (size_t)bcap);
                }
                blocks[0].start = r->start;
                blocks[0].end = r->end;
                blocks[0].rrow = r->row;
                nb = 1;
            }
            if (nb > 0) {
                lo_block *h = &blocks[nb - 1];
                lo_region hr = {cur->contig, h->start, h->end, r->strand, 0};
                if (lo_overlaps(&hr, r)) {
                    if (r->start < h->start) h->start = r->start;
                    if (r->end > h->end) h->end = r->end;
                    continue;
                }
            }
            if (nb == bcap) {
                bcap = bcap ? bcap * 2 : 16;
                blocks = (lo_block *)realloc(blocks, sizeof(lo_block) * (size_t)bcap);
            }
            blocks[nb].start = r->start;
            blocks[nb].end = r->end;
            blocks[nb].rrow = r->row;
            nb++;
        }
        if (nb == 0) { /* :100-101 (L, (v, None)) */
            lo_emit(o, cur->contig, cur->start, cur->end, cur->row, -1);
            continue;
        }
        if (mode == LO_SUB_LIME) {
            /* :109-114 over the reversed block list; subtract() :53-75 */
            for (int64_t b = nb - 1; b >= 0; --b) {
                if (blocks[b].start > cur->start)
                    lo_emit(o, cur->contig, cur->start, blocks[b].start, cur->row, blocks[b].rrow);
                if (cur->end > blocks[b].end)
                    lo_emit(o, cur->contig, blocks[b].end, cur->end, cur->row, blocks[b].rrow);
            }
        } else {
            /* a \ (B_0 u ... u B_{nb-1}); blocks are disjoint, sorted */
            int64_t pos = cur->start;
            for (int64_t b = 0; b < nb; ++b) {
                if (blocks[b].start > pos)
                    lo_emit(o, cur->contig, pos, blocks[b].start, cur->row, blocks[b].rrow);
                if (blocks[b].end > pos) pos = blocks[b].end;
            }
            if (cur->end > pos) lo_emit(o, cur->contig, pos, cur->end, cur->row, blocks[nb - 1].rrow);
        }
    }
    free(blocks);
    free(cache.v);
}

int64_t lo_subtract(int64_t nl, const int32_t *lc, const int64_t *ls, const int64_t *le,
                    const int8_t *lstr, int64_t nr, const int32_t *rc, const int64_t *rs,
                    const int64_t *re, const int8_t *rstr, int64_t threshold, int mode,
                    int64_t cap, int32_t *oc, int64_t *os, int64_t *oe, int64_t *olrow,
                    int64_t *orrow) {
    lo_region *L = lo_load(nl, lc, ls, le, lstr);
    lo_region *R = lo_load(nr, rc, rs, re, rstr);
    lo_out out = {0, cap, oc, os, oe, olrow, orrow};
    lo_subtract_sorted(L, nl, R, nr, threshold, mode, &out);
    free(L);
    free(R);
    return out.count;
}

/* ----------------------------------------------------------------- merge */

/* SetTheory.scala:208-225 localCompute with Merge.scala condition/primitive:
 * fold over the sorted partition keeping the running hull at the list head;
 * condition(head, next) = head.overlaps(next) (threshold not passed -> 0);
 * primitive = hull.  run_of_row[row] receives the index of the run the input
 * row was folded into (the Iterable[T] grouping). */
static int64_t lo_merge_sorted(const lo_region *A, int64_t n, int64_t cap, int32_t *oc,
                               int64_t *os, int64_t *oe, int8_t *ostrand, int64_t *run_of_row) {
    int64_t count = 0;
    lo_region head;
    for (int64_t i = 0; i < n; ++i) {
        const lo_region *a = &A[i];
        if (i > 0 && lo_overlaps(&head, a)) {
            if (a->start < head.start) head.start = a->start;
            if (a->end > head.end) head.end = a->end;
        } else {
            if (i > 0) {
                if (count - 1 < cap) {
                    if (oc) oc[count - 1] = head.contig;
                    if (os) os[count - 1] = head.start;
                    if (oe) oe[count - 1] = head.end;
                    if (ostrand) ostrand[count - 1] = head.strand;
                }
            }
            head = *a;
            count++;
        }
        if (run_of_row) run_of_row[a->row] = count - 1;
    }
    if (count > 0 && count - 1 < cap) {
        if (oc) oc[count - 1] = head.contig;
        if (os) os[count - 1] = head.start;
        if (oe) oe[count - 1] = head.end;
        if (ostrand) ostrand[count - 1] = head.strand;
    }
    return count;
}

int64_t lo_merge(int64_t n, const int32_t *c, const int64_t *s, const int64_t *e,
                 const int8_t *strand, int64_t cap, int32_t *oc, int64_t *os, int64_t *oe,
                 int8_t *ostrand, int64_t *run_of_row) {
    lo_region *A = lo_load(n, c, s, e, strand);
    int64_t count = lo_merge_sorted(A, n, cap, oc, os, oe, ostrand, run_of_row);
    free(A);
    return count;
}

/* ------------------------------------------------------------ complement */

/* Complement.scala:59-128 getComplement + :33-50 postProcess, in the
 * partition-count-independent form pinned by ComplementSuite.scala:19-114
 * (SURVEY.md Appendix A.3): contigs in String order (= contig rank order);
 * for a contig with merged runs r_0..r_k emit [0, r_0.s), [r_i.e, r_{i+1}.s),
 * [r_k.e, len); a contig without data emits [0, len); zero-width gaps (quirk
 * Q4) are dropped.  Strand is ignored (the gap regions carry none).
 * Returns -1 if a data contig is outside [0, n_genome) (the reference throws
 * NoSuchElementException from referenceNameBounds(name), :106,118). */
/* the gaps of one contig g (its rows A[0..n), sorted) */
static void lo_complement_contig(const lo_region *A, int64_t n, int32_t g, int64_t glen,
                                 lo_out *o) {
    int64_t pos = 0;
    int have = 0;
    lo_region head;
    for (int64_t i = 0; i < n; ++i) {
        const lo_region *a = &A[i];
        if (have && lo_overlaps(&head, a)) {
            if (a->end > head.end) head.end = a->end;
            continue;
        }
        if (have) { /* close the previous run: gap before the new one */
            if (head.start > pos) lo_emit(o, g, pos, head.start, -1, -1);
            if (head.end > pos) pos = head.end;
        }
        head = *a;
        have = 1;
    }
    if (have) {
        if (head.start > pos) lo_emit(o, g, pos, head.start, -1, -1);
        if (head.end > pos) pos = head.end;
    }
    if (glen > pos) lo_emit(o, g, pos, glen, -1, -1);
}

int64_t lo_complement(int64_t n, const int32_t *c, const int64_t *s, const int64_t *e,
                      int32_t n_genome, const int64_t *genome_len, int64_t cap, int32_t *oc,
                      int64_t *os, int64_t *oe) {
    for (int64_t i = 0; i < n; ++i)
        if (c[i] < 0 || c[i] >= n_genome) return -1;
    lo_region *A = lo_load(n, c, s, e, NULL);
    lo_out out = {0, cap, oc, os, oe, NULL, NULL};
    int64_t i = 0;
    for (int32_t g = 0; g < n_genome; ++g) {
        const int64_t i0 = i;
        while (i < n && A[i].contig == g) ++i;
        lo_complement_contig(A + i0, i - i0, g, genome_len[g], &out);
    }
    free(A);
    return out.count;
}

/* ---------------------------------------------------- order-free checksum */

/* splitmix64 finaliser: the order-independent checksum of SURVEY.md 8(d)
 * (sum and xor of mix64 over each output tuple), shared with the engine's
 * verification kernels so full-size runs can be compared without sorting. */
static uint64_t lo_mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    return z ^ (z >> 31);
}
uint64_t lo_pair_hash(uint32_t start, uint32_t end, uint32_t a, uint32_t b) {
    uint64_t x = ((uint64_t)start << 32) | end;
    uint64_t y = ((uint64_t)a << 32) | b;
    return lo_mix64(x ^ lo_mix64(y));
}

/* ------------------------------------------- contig-sharded drivers (MT) */

/* The reference runs one Spark task per range partition; every op here is
 * contig-local (no predicate holds across reference names), so sharding the
 * rows by contig and running the same per-partition code (lo_intersect_sorted,
 * lo_merge_sorted) on each contig in its own thread gives exactly the P = 1
 * result, with outputs concatenated in contig (String) order.  These drivers
 * take the device's u32 contig-local coordinates so that full-size inputs
 * (1e8-5e8 rows) need no int64 copy; rows keep their input index.  They
 * serve the size-independent parity checks of SURVEY.md 8(d) ("Verification
 * at scale": count plus order-independent checksum) and the CPU baseline. */

typedef struct {
    int64_t n;
    const int32_t *c;
    const uint32_t *s, *e;
    int64_t *off; /* n_contigs + 1: rows of contig k are idx[off[k] .. off[k+1]) */
    int64_t *idx;
} lo_groups;

static void lo_group(lo_groups *g, int32_t nc, int64_t n, const int32_t *c, const uint32_t *s,
                     const uint32_t *e) {
    g->n = n;
    g->c = c;
    g->s = s;
    g->e = e;
    g->off = (int64_t *)calloc((size_t)nc + 2, sizeof(int64_t));
    g->idx = (int64_t *)malloc(sizeof(int64_t) * (size_t)(n > 0 ? n : 1));
    for (int64_t i = 0; i < n; ++i) g->off[c[i] + 1]++;
    for (int32_t k = 0; k < nc; ++k) g->off[k + 1] += g->off[k];
    int64_t *pos = (int64_t *)malloc(sizeof(int64_t) * ((size_t)nc + 1));
    memcpy(pos, g->off, sizeof(int64_t) * ((size_t)nc + 1));
    for (int64_t i = 0; i < n; ++i) g->idx[pos[c[i]]++] = i;
    free(pos);
}

static void lo_ungroup(lo_groups *g) {
    free(g->off);
    free(g->idx);
}

/* stable LSD radix sort of (key, id) pairs by key, 16-bit digits; passes
 * whose digit is constant over the input are skipped */
static void lo_radix_pairs(uint64_t *key, int64_t *id, int64_t n) {
    if (n < 2) return;
    uint64_t *k2 = (uint64_t *)malloc(sizeof(uint64_t) * (size_t)n);
    int64_t *i2 = (int64_t *)malloc(sizeof(int64_t) * (size_t)n);
    int64_t *cnt = (int64_t *)malloc(sizeof(int64_t) * 65536);
    for (int shift = 0; shift < 64; shift += 16) {
        memset(cnt, 0, sizeof(int64_t) * 65536);
        for (int64_t j = 0; j < n; ++j) cnt[(key[j] >> shift) & 0xffff]++;
        if (cnt[(key[0] >> shift) & 0xffff] == n) continue;
        int64_t run = 0;
        for (int d = 0; d < 65536; ++d) {
            const int64_t c = cnt[d];
            cnt[d] = run;
            run += c;
        }
        for (int64_t j = 0; j < n; ++j) {
            const int64_t at = cnt[(key[j] >> shift) & 0xffff]++;
            k2[at] = key[j];
            i2[at] = id[j];
        }
        memcpy(key, k2, sizeof(uint64_t) * (size_t)n);
        memcpy(id, i2, sizeof(int64_t) * (size_t)n);
    }
    free(k2);
    free(i2);
    free(cnt);
}

/* the rows of contig k as sorted regions (RegionOrdering, ties by row).  All
 * rows of a group share the contig and strand 0 and come in ascending row
 * order, so lo_qsort_cmp's order is the STABLE order by (start, end): one
 * radix sort of start << 32 | end (the contig-sharded drivers' 1e9-row inputs
 * would spend minutes in qsort; lo_load keeps qsort, and the drivers are
 * checked against it by tests/test_oracle.py) */
static lo_region *lo_load_group(const lo_groups *g, int32_t k, int64_t *n_out) {
    const int64_t a = g->off[k], b = g->off[k + 1], n = b - a;
    lo_region *r = (lo_region *)malloc(sizeof(lo_region) * (size_t)(n > 0 ? n : 1));
    uint64_t *key = (uint64_t *)malloc(sizeof(uint64_t) * (size_t)(n > 0 ? n : 1));
    int64_t *id = (int64_t *)malloc(sizeof(int64_t) * (size_t)(n > 0 ? n : 1));
    for (int64_t j = 0; j < n; ++j) {
        const int64_t i = g->idx[a + j];
        key[j] = ((uint64_t)g->s[i] << 32) | (uint64_t)g->e[i];
        id[j] = i;
    }
    lo_radix_pairs(key, id, n);
    for (int64_t j = 0; j < n; ++j) {
        lo_region *x = &r[j];
        x->contig = k;
        x->start = (int64_t)(key[j] >> 32);
        x->end = (int64_t)(key[j] & 0xffffffffu);
        x->strand = 0;
        x->row = id[j];
    }
    free(key);
    free(id);
    *n_out = n;
    return r;
}

typedef struct {
    int op; /* 0 intersect, 1 merge, 2 subtract, 3 complement */
    int32_t nc;
    lo_groups L, R;
    int64_t threshold;
    int mode;                  /* subtract */
    const int64_t *genome_len; /* complement */
    int keep;            /* buffer the records (else count + checksum only) */
    int32_t *order;      /* contigs, largest first */
    int next;            /* work-queue head (atomic) */
    lo_out *res;         /* per contig */
    int64_t *run_of_row; /* merge: local run id per input row */
} lo_mt;

static void *lo_mt_worker(void *arg) {
    lo_mt *m = (lo_mt *)arg;
    for (;;) {
        const int q = __sync_fetch_and_add(&m->next, 1);
        if (q >= m->nc) break;
        const int32_t k = m->order[q];
        lo_out *o = &m->res[k];
        int64_t nl = 0, nr = 0;
        lo_region *L = lo_load_group(&m->L, k, &nl);
        if (m->op == 0 || m->op == 2) {
            lo_region *R = lo_load_group(&m->R, k, &nr);
            o->hash = m->op == 0 ? 1 : 2;
            o->grow = m->keep;
            if (m->op == 0)
                lo_intersect_sorted(L, nl, R, nr, m->threshold, o);
            else
                lo_subtract_sorted(L, nl, R, nr, m->threshold, m->mode, o);
            free(R);
        } else if (m->op == 3) {
            o->hash = 2;
            lo_complement_contig(L, nl, k, m->genome_len[k], o);
        } else {
            /* at most one run per row: the buffers are sized by the rows */
            o->cap = nl;
            o->start = (int64_t *)malloc(sizeof(int64_t) * (size_t)(nl > 0 ? nl : 1));
            o->end = (int64_t *)malloc(sizeof(int64_t) * (size_t)(nl > 0 ? nl : 1));
            o->count = lo_merge_sorted(L, nl, nl, NULL, o->start, o->end, NULL, m->run_of_row);
        }
        free(L);
    }
    return NULL;
}

static void lo_mt_run(lo_mt *m, int nthreads) {
    /* contigs largest first, so the long shards start early */
    m->order = (int32_t *)malloc(sizeof(int32_t) * (size_t)(m->nc > 0 ? m->nc : 1));
    for (int32_t k = 0; k < m->nc; ++k) m->order[k] = k;
    for (int32_t a = 1; a < m->nc; ++a) { /* insertion sort: nc is small */
        const int32_t k = m->order[a];
        const int64_t w = (m->L.off[k + 1] - m->L.off[k]) + (m->R.off ? m->R.off[k + 1] - m->R.off[k] : 0);
        int32_t b = a - 1;
        while (b >= 0) {
            const int32_t j = m->order[b];
            const int64_t wj = (m->L.off[j + 1] - m->L.off[j]) +
                               (m->R.off ? m->R.off[j + 1] - m->R.off[j] : 0);
            if (wj >= w) break;
            m->order[b + 1] = j;
            --b;
        }
        m->order[b + 1] = k;
    }
    m->next = 0;
    m->res = (lo_out *)calloc((size_t)(m->nc > 0 ? m->nc : 1), sizeof(lo_out));
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    pthread_t th[256];
    int started = 0;
    for (int t = 1; t < nthreads; ++t)
        if (pthread_create(&th[started], NULL, lo_mt_worker, m) == 0) ++started;
    lo_mt_worker(m);
    for (int t = 0; t < started; ++t) pthread_join(th[t], NULL);
    free(m->order);
}

static void lo_out_free(lo_out *o) {
    free(o->contig);
    free(o->start);
    free(o->end);
    free(o->lrow);
    free(o->rrow);
}

/* intersect (Intersection.scala:58-69 over the SetTheory.scala:131-187 sweep)
 * sharded by contig over `nthreads` threads.  Returns the pair count; *sum /
 * *xr receive the order-independent checksum (sum and xor of lo_pair_hash of
 * (start, end, a_row, b_row), contig-local start / end as the engine hashes
 * them).  With cap >= count the records are also written in the reference's
 * P = 1 emission order. */
int64_t lo_intersect_mt(int32_t n_contigs, int64_t nl, const int32_t *lc, const uint32_t *ls,
                        const uint32_t *le, int64_t nr, const int32_t *rc, const uint32_t *rs,
                        const uint32_t *re, int64_t threshold, int nthreads, int64_t cap,
                        int32_t *oc, int64_t *os, int64_t *oe, int64_t *olrow, int64_t *orrow,
                        uint64_t *sum, uint64_t *xr) {
    for (int64_t i = 0; i < nl; ++i)
        if (lc[i] < 0 || lc[i] >= n_contigs) return -1;
    for (int64_t i = 0; i < nr; ++i)
        if (rc[i] < 0 || rc[i] >= n_contigs) return -1;
    lo_mt m;
    memset(&m, 0, sizeof(m));
    m.op = 0;
    m.nc = n_contigs;
    m.threshold = threshold;
    m.keep = cap > 0;
    lo_group(&m.L, n_contigs, nl, lc, ls, le);
    lo_group(&m.R, n_contigs, nr, rc, rs, re);
    lo_mt_run(&m, nthreads);
    int64_t total = 0;
    uint64_t hs = 0, hx = 0;
    for (int32_t k = 0; k < n_contigs; ++k) {
        total += m.res[k].count;
        hs += m.res[k].hsum;
        hx ^= m.res[k].hxor;
    }
    if (cap >= total) {
        int64_t at = 0;
        for (int32_t k = 0; k < n_contigs; ++k) {
            const lo_out *o = &m.res[k];
            for (int64_t j = 0; j < o->count; ++j, ++at) {
                if (oc) oc[at] = o->contig[j];
                if (os) os[at] = o->start[j];
                if (oe) oe[at] = o->end[j];
                if (olrow) olrow[at] = o->lrow[j];
                if (orrow) orrow[at] = o->rrow[j];
            }
        }
    }
    for (int32_t k = 0; k < n_contigs; ++k) lo_out_free(&m.res[k]);
    free(m.res);
    lo_ungroup(&m.L);
    lo_ungroup(&m.R);
    if (sum) *sum = hs;
    if (xr) *xr = hx;
    return total;
}

/* merge (SetTheory.scala:208-225 + Merge.scala) sharded by contig.  Returns
 * the run count; with cap >= count writes the runs in order.  run_of_row
 * (optional, n entries) receives every input row's global run index, and
 * (*gsum, *gxr) the checksum of that grouping: sum / xor over rows r of
 * mix64(r << 32 | run_of_row[r]) -- the Iterable[T] of every run. */
static uint64_t lo_mix64(uint64_t z);

int64_t lo_merge_mt(int32_t n_contigs, int64_t n, const int32_t *c, const uint32_t *s,
                    const uint32_t *e, int nthreads, int64_t cap, int32_t *oc, int64_t *os,
                    int64_t *oe, int64_t *run_of_row, uint64_t *gsum, uint64_t *gxr) {
    for (int64_t i = 0; i < n; ++i)
        if (c[i] < 0 || c[i] >= n_contigs) return -1;
    lo_mt m;
    memset(&m, 0, sizeof(m));
    m.op = 1;
    m.nc = n_contigs;
    int64_t *rid = run_of_row ? run_of_row : (int64_t *)malloc(sizeof(int64_t) * (size_t)(n > 0 ? n : 1));
    m.run_of_row = rid;
    lo_group(&m.L, n_contigs, n, c, s, e);
    lo_mt_run(&m, nthreads);
    int64_t *base = (int64_t *)malloc(sizeof(int64_t) * ((size_t)n_contigs + 1));
    int64_t total = 0;
    for (int32_t k = 0; k < n_contigs; ++k) {
        base[k] = total;
        total += m.res[k].count;
    }
    uint64_t hs = 0, hx = 0;
    for (int64_t i = 0; i < n; ++i) {
        rid[i] += base[c[i]];
        const uint64_t h = lo_mix64(((uint64_t)i << 32) | (uint64_t)(uint32_t)rid[i]);
        hs += h;
        hx ^= h;
    }
    if (cap >= total) {
        for (int32_t k = 0; k < n_contigs; ++k) {
            const lo_out *o = &m.res[k];
            for (int64_t j = 0; j < o->count; ++j) {
                const int64_t at = base[k] + j;
                if (oc) oc[at] = k;
                if (os) os[at] = o->start[j];
                if (oe) oe[at] = o->end[j];
            }
        }
    }
    for (int32_t k = 0; k < n_contigs; ++k) lo_out_free(&m.res[k]);
    free(m.res);
    free(base);
    lo_ungroup(&m.L);
    if (!run_of_row) free(rid);
    if (gsum) *gsum = hs;
    if (gxr) *gxr = hx;
    return total;
}

/* subtract (Subtract.scala:91-116 over the sweep) sharded by contig, both
 * modes.  Returns the region count; (*sum, *xr) receive the result checksum
 * of every region -- sum / xor of mix64(lo_pair_hash(start, end, a_row,
 * b_row) + contig), an absent b_row (None) as 0xffffffff -- the form of the
 * engine's lime_result_checksum. */
int64_t lo_subtract_mt(int32_t n_contigs, int64_t nl, const int32_t *lc, const uint32_t *ls,
                       const uint32_t *le, int64_t nr, const int32_t *rc, const uint32_t *rs,
                       const uint32_t *re, int64_t threshold, int mode, int nthreads,
                       uint64_t *sum, uint64_t *xr) {
    for (int64_t i = 0; i < nl; ++i)
        if (lc[i] < 0 || lc[i] >= n_contigs) return -1;
    for (int64_t i = 0; i < nr; ++i)
        if (rc[i] < 0 || rc[i] >= n_contigs) return -1;
    lo_mt m;
    memset(&m, 0, sizeof(m));
    m.op = 2;
    m.nc = n_contigs;
    m.threshold = threshold;
    m.mode = mode;
    lo_group(&m.L, n_contigs, nl, lc, ls, le);
    lo_group(&m.R, n_contigs, nr, rc, rs, re);
    lo_mt_run(&m, nthreads);
    int64_t total = 0;
    uint64_t hs = 0, hx = 0;
    for (int32_t k = 0; k < n_contigs; ++k) {
        total += m.res[k].count;
        hs += m.res[k].hsum;
        hx ^= m.res[k].hxor;
        lo_out_free(&m.res[k]);
    }
    free(m.res);
    lo_ungroup(&m.L);
    lo_ungroup(&m.R);
    if (sum) *sum = hs;
    if (xr) *xr = hx;
    return total;
}

/* complement (Complement.scala:59-128 in the ComplementSuite-pinned form)
 * sharded by contig: the genome has n_contigs contigs (String order), every
 * row's contig among them.  Returns the gap count and the result checksum
 * (as lo_subtract_mt, both rows absent). */
int64_t lo_complement_mt(int32_t n_contigs, const int64_t *genome_len, int64_t n,
                         const int32_t *c, const uint32_t *s, const uint32_t *e, int nthreads,
                         uint64_t *sum, uint64_t *xr) {
    for (int64_t i = 0; i < n; ++i)
        if (c[i] < 0 || c[i] >= n_contigs) return -1;
    lo_mt m;
    memset(&m, 0, sizeof(m));
    m.op = 3;
    m.nc = n_contigs;
    m.genome_len = genome_len;
    lo_group(&m.L, n_contigs, n, c, s, e);
    lo_mt_run(&m, nthreads);
    int64_t total = 0;
    uint64_t hs = 0, hx = 0;
    for (int32_t k = 0; k < n_contigs; ++k) {
        total += m.res[k].count;
        hs += m.res[k].hsum;
        hx ^= m.res[k].hxor;
        lo_out_free(&m.res[k]);
    }
    free(m.res);
    lo_ungroup(&m.L);
    if (sum) *sum = hs;
    if (xr) *xr = hx;
    return total;
}
