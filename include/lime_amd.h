/*
 * lime_amd.h -- C-ABI of the MI355X (gfx950) engine for LIME's genomic
 * set-theory hot path: intersection, merge (union), subtract (difference)
 * and complement over ReferenceRegion-keyed interval sets.
 *
 * Plain C types only (no HIP/torch types in signatures); every function
 * returns an int status (LIME_OK = 0) and leaves a thread-local message in
 * lime_last_error().  One HIP stream per context; contexts are independent,
 * so concurrent calls from N executor threads each use their own context
 * (SURVEY.md 8(b) "Threading").
 *
 * Reference interface each entry point replaces (paths under gman90/lime):
 *   lime_set_create_host    ADAM loadBed(...).repartitionAndSort() +
 *                           OverlapBasedSetTheory.prepare()'s sort
 *                           (cli/Intersection.scala:42-48,
 *                            OverlapBasedSetTheory.scala:45-86)
 *   lime_intersect_count /  DistributedIntersection(left, right, partitionMap,
 *   lime_intersect_fill_*     threshold).compute()  (Intersection.scala:45-69,
 *                            SetTheory.scala:162-187)
 *   lime_merge              DistributedMerge(rdd, partitionMap).compute()
 *                            (Merge.scala:34-36, SetTheory.scala:202-282)
 *   lime_subtract           DistributedSubtract(left, right, partitionMap,
 *                            threshold).compute()  (Subtract.scala:78-116)
 *   lime_complement         DistributedComplement(rdd, partitionMap,
 *                            referenceNameBounds).compute()
 *                            (Complement.scala:33-134)
 *   lime_bed_read           ADAM sc.loadBed(path) (3rd-party; BED3-6 text)
 *   lime_contig_rank        ReferenceRegion ordering by referenceName
 *                            (java.lang.String.compareTo)
 *
 * Semantics are SURVEY.md Appendix A (strict half-open overlap, sort order
 * (contig, start, end), zero-width gaps dropped in complement).  Strand is
 * handled by the host layer (lime_amd.hpp / lime_amd python package), which
 * partitions rows by strand before calling this ABI; the engine itself sees
 * unstranded contigs.
 */
#ifndef LIME_AMD_H
#define LIME_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2: lime_set_lower_bound / _first_reaching return -(LIME_ERR_*) on error
 *    (was -1); lime_pairs_checksum_device and the sharded-path helpers added
 * 6: lime_route_rows_interleaved, lime_deinterleave_u32 (the routed
 *    exchange without per-column repacking) */
#define LIME_ABI_VERSION 6

/* status codes */
#define LIME_OK 0
#define LIME_ERR_ARG 1      /* bad argument (null pointer, negative count, ...)          */
#define LIME_ERR_RANGE 2    /* coordinate outside [0, 2^32) / contig length / span > 2^32 */
#define LIME_ERR_DEVICE 3   /* HIP runtime error (or no device)                          */
#define LIME_ERR_NOMEM 4    /* device or host allocation failed                          */
#define LIME_ERR_CONTIG 5   /* contig id not in the space (NoSuchElementException)       */
#define LIME_ERR_IO 6       /* file could not be read / parsed                           */
#define LIME_ERR_OVERFLOW 7 /* an output count does not fit the engine's index types     */

/* subtract modes */
#define LIME_SUBTRACT_LIME 0 /* Subtract.scala:103-114 exactly (per-block remnants, Q5) */
#define LIME_SUBTRACT_SET 1  /* a minus union(hits)                                     */

typedef struct lime_ctx lime_ctx;       /* device + stream + memory pool            */
typedef struct lime_space lime_space;   /* contigs (String order) and their lengths */
typedef struct lime_set lime_set;       /* sorted, device-resident interval set     */
typedef struct lime_pairs lime_pairs;   /* intersect plan: pair count + fill state  */
typedef struct lime_result lime_result; /* merge / subtract / complement output     */
typedef struct lime_bed lime_bed;       /* parsed BED file (host memory)            */
typedef struct lime_dbed lime_dbed;     /* parsed BED text (device memory)          */
typedef struct lime_bitset lime_bitset; /* bit-per-base set over a space            */

/* One intersect output record: the intersection region in contig-local
 * coordinates (contig = contig of left row a_row) and the two input rows. */
typedef struct {
    uint32_t start, end, a_row, b_row;
} lime_pair;

const char *lime_last_error(void);
int lime_abi_version(void);

/* ----------------------------------------------------------------- context */
int lime_ctx_create(int device, lime_ctx **out);
int lime_ctx_destroy(lime_ctx *ctx);
/* Run subsequent work on a caller-owned hipStream_t (e.g. torch's current
 * stream); NULL restores the context's own stream. */
int lime_ctx_set_stream(lime_ctx *ctx, void *hip_stream);
int lime_ctx_synchronize(lime_ctx *ctx);
/* bytes currently held by the context's device pool (live blocks and the
 * cached free ones) */
int64_t lime_ctx_pool_bytes(const lime_ctx *ctx);
/* bytes of the pool's LIVE blocks (what the context's objects and any call
 * in flight hold); *peak (may be NULL) = their high-water mark since the
 * last reset, reset to the live bytes when reset_peak != 0 */
int64_t lime_ctx_pool_live_bytes(lime_ctx *ctx, int32_t reset_peak, int64_t *peak);

/* ------------------------------------------------------------------- space */
/* Contig ids are 0..n-1 in the caller's order, which must be Java String
 * order of the names for output order to match the reference (use
 * lime_contig_rank).  Internally contig c occupies global coordinates
 * [off[c], off[c] + len[c]] with off[c+1] = off[c] + len[c] + 1, so the total
 * span sum(len + 1) must stay below 2^32 (hg19/hg38: ~3.1e9). */
int lime_space_create(int32_t n_contigs, const int64_t *lengths, lime_space **out);
int lime_space_destroy(lime_space *space);
int32_t lime_space_contigs(const lime_space *space);
int64_t lime_space_span(const lime_space *space);
int64_t lime_space_offset(const lime_space *space, int32_t contig);

/* --------------------------------------------------------------------- sets */
/* Host arrays (JVM Long coordinates): upload, validate and sort on device.
 * Rows keep their input index (0..n-1) as the payload handle. */
int lime_set_create_host(lime_ctx *ctx, const lime_space *space, int64_t n, const int32_t *contig,
                         const int64_t *start, const int64_t *end, lime_set **out);
/* Stranded set (the CLI keys ReferenceRegion.stranded): strand codes per row
 * (0 independent, 1 forward, 2 reverse, 3 unknown).  Sorted in the full
 * RegionOrdering (start, end, strand); lime_merge on it follows the
 * reference fold exactly: a run breaks where the strand changes
 * (Merge.condition = overlaps, which requires equal strands). */
int lime_set_create_host_stranded(lime_ctx *ctx, const lime_space *space, int64_t n,
                                  const int32_t *contig, const int64_t *start,
                                  const int64_t *end, const int8_t *strand, lime_set **out);
/* Device arrays (u32 contig-local coordinates) already resident in HBM:
 * validated and sorted on the context's stream, inputs are not modified.
 * Device inputs (here and in every call below that takes them) are read on
 * the context's stream: on the context's own stream a call returns once they
 * are consumed; on a caller stream (lime_ctx_set_stream) they must stay valid
 * until that stream has passed the call -- a stream-ordered allocator on the
 * same stream (e.g. PyTorch's) gives exactly that. */
int lime_set_create_device(lime_ctx *ctx, const lime_space *space, int64_t n,
                           const int32_t *d_contig, const uint32_t *d_start,
                           const uint32_t *d_end, lime_set **out);
/* Same with strand codes in HBM (NULL = every row independent): sorted in the
 * full RegionOrdering (start, end, strand), as lime_set_create_host_stranded. */
int lime_set_create_device_stranded(lime_ctx *ctx, const lime_space *space, int64_t n,
                                    const int32_t *d_contig, const uint32_t *d_start,
                                    const uint32_t *d_end, const int8_t *d_strand,
                                    lime_set **out);
/* Device arrays already in the space's GLOBAL coordinates (gstart, gend) with
 * caller-chosen row ids -- e.g. a coordinate shard's own sorted rows followed
 * by its halo.  Validated (gend >= gstart, inside the span) and sorted only if
 * not already in canonical order. */
int lime_set_create_global(lime_ctx *ctx, const lime_space *space, int64_t n,
                           const uint32_t *d_gstart, const uint32_t *d_gend,
                           const uint32_t *d_row, lime_set **out);
/* The same with strand codes (device, one per input row, as
 * lime_set_create_device_stranded): sorted in the full RegionOrdering; a
 * coordinate shard's stranded rows (merge breaks runs at strand changes). */
int lime_set_create_global_stranded(lime_ctx *ctx, const lime_space *space, int64_t n,
                                    const uint32_t *d_gstart, const uint32_t *d_gend,
                                    const uint32_t *d_row, const int8_t *d_strand,
                                    lime_set **out);
int lime_set_destroy(lime_set *set);
int64_t lime_set_size(const lime_set *set);
/* first sorted row with gstart >= gkey; on error -(LIME_ERR_*) */
int64_t lime_set_lower_bound(const lime_set *set, uint32_t gkey);
/* first sorted row j with max(gend[0..j]) > gkey, i.e. every row from there
 * on may reach past gkey and none before does (a coordinate shard's rows that
 * can overlap a later shard: the left halo of pairwise ops); n if none;
 * on error -(LIME_ERR_*) */
int64_t lime_set_first_reaching(const lime_set *set, uint32_t gkey);
/* The same for k keys at once (host arrays; one launch, one read-back):
 * the per-shard bounds of the sharded halos. */
int lime_set_lower_bounds(const lime_set *set, int32_t k, const uint32_t *gkeys, int64_t *out);
int lime_set_first_reachings(const lime_set *set, int32_t k, const uint32_t *gkeys, int64_t *out);
/* device-to-device copy of sorted rows [first, first + count) */
int lime_set_copy_rows_device(const lime_set *set, int64_t first, int64_t count, uint32_t *d_gstart,
                              uint32_t *d_gend, uint32_t *d_row);
/* Width statistics gathered when the set was built: min and max of end -
 * start, and whether any row has zero width. */
int lime_set_stats(const lime_set *set, uint32_t *min_width, uint32_t *max_width,
                   int32_t *has_zero_width);
/* A new plain set: the rows of `set` followed by n more rows (device arrays
 * in global coordinates and caller row ids) that the CALLER guarantees to be
 * in canonical order and to start at or after the set's last row -- a
 * coordinate shard's own rows followed by its right halo (rows of later
 * shards).  Nothing is sorted or validated and nothing is read back (no
 * stream drain): the rows are copied device-to-device, and the width
 * statistics are `set`'s combined with the caller's bounds for the added rows
 * (min_width / max_width / has_zero_width of those rows, or bounds of them).
 * Replaces rebuilding the shard's set (lime_set_create_global: a validating
 * pass and a read-back) in the sharded pairwise step.  With the environment
 * variable LIME_CHECK_EXTEND=1 the contract is checked on the device (order
 * at the join and among the added rows, width bounds, zero-width flag: one
 * pass and a read-back) and a violation fails with LIME_ERR_ARG. */
int lime_set_extend_sorted(lime_ctx *ctx, const lime_set *set, int64_t n, const uint32_t *d_gstart,
                           const uint32_t *d_gend, const uint32_t *d_row, uint32_t min_width,
                           uint32_t max_width, int32_t has_zero_width, lime_set **out);
/* The same with rows on both sides: n_before rows that precede every row of
 * `set`, then `set`, then n_after rows that follow it -- a coordinate shard's
 * left halo (rows of earlier shards reaching into it), own rows and right
 * halo, which the sharded subtract needs (Subtract.scala:78-116 over the
 * replication of OverlapBasedSetTheory.scala:75-80).  The width bounds cover
 * all added rows.  ABI 4. */
int lime_set_concat_sorted(lime_ctx *ctx, const lime_set *set, int64_t n_before,
                           const uint32_t *b_gstart, const uint32_t *b_gend, const uint32_t *b_row,
                           int64_t n_after, const uint32_t *a_gstart, const uint32_t *a_gend,
                           const uint32_t *a_row, uint32_t min_width, uint32_t max_width,
                           int32_t has_zero_width, lime_set **out);
/* Device pointers of the sorted set: global start, global end, input row. */
int lime_set_device_arrays(const lime_set *set, const uint32_t **gstart, const uint32_t **gend,
                           const uint32_t **row);
/* Host copy of the sorted set in contig-local coordinates. */
int lime_set_fill_host(const lime_set *set, int32_t *contig, int64_t *start, int64_t *end,
                       int64_t *row);

/* ---------------------------------------------------------------- intersect */
/* Count pass: exact number of qualifying pairs (overlapsBy >= threshold). */
int lime_intersect_count(lime_ctx *ctx, const lime_set *a, const lime_set *b, int64_t threshold,
                         lime_pairs **plan, int64_t *n_pairs);
/* Same with ownership for a coordinate shard that carries its right
 * neighbours' boundary rows ("halo") after its own: only the first a_owned
 * rows of a and b_owned rows of b own output pairs (a pair is owned by the
 * row whose start is the smaller, ties to a); the halo rows act as partners
 * only, so shard outputs are disjoint.  -1 = all rows. */
int lime_intersect_count_owned(lime_ctx *ctx, const lime_set *a, const lime_set *b,
                               int64_t threshold, int64_t a_owned, int64_t b_owned,
                               lime_pairs **plan, int64_t *n_pairs);
/* Fill pass: write pairs [first, first + count) of the plan's output order
 * into a caller-owned DEVICE buffer (chunked emission for outputs larger
 * than HBM).  Asynchronous on the context stream. */
int lime_intersect_fill_device(lime_pairs *plan, int64_t first, int64_t count, lime_pair *d_out);
/* Same into a caller-owned HOST buffer (synchronous). */
int lime_intersect_fill_host(lime_pairs *plan, int64_t first, int64_t count, lime_pair *out);
/* Order-independent checksum (sum and xor of lime_pair_hash over every pair)
 * computed on device without materialising the pairs. */
int lime_intersect_checksum(lime_pairs *plan, uint64_t *sum, uint64_t *xr);
/* The same checksum over `count` records already STORED in a device buffer
 * (e.g. a chunk lime_intersect_fill_device wrote): verifies the bytes a fill
 * wrote, not only the fill's arithmetic. */
int lime_pairs_checksum_device(lime_ctx *ctx, const lime_pair *d_pairs, int64_t count,
                               uint64_t *sum, uint64_t *xr);
int lime_pairs_destroy(lime_pairs *plan);

/* ------------------------------------------------------------------- window */
/* DistributedWindow(left, right, partitionMap, threshold = distance).compute()
 * (lime-core Window.scala:71-95, CLI cli/Window.scala:42-55): every pair
 * (a, b) with ADAM a.isNearby(b, distance) (overlapping, or a gap of at most
 * distance - 1 bases: ADAM's distance is gap + 1).  The records carry a's own
 * region (Window.primitive returns the first region) and the two rows; fill
 * and checksum them with lime_intersect_fill_* / lime_intersect_checksum. */
int lime_window_count(lime_ctx *ctx, const lime_set *a, const lime_set *b, int64_t distance,
                      lime_pairs **plan, int64_t *n_pairs);

/* ------------------------------------------------------------------ closest */
#define LIME_CLOSEST 0 /* SingleClosest (lime-core Closest.scala:34-214), the CLI's op */
#define LIME_CLOSEST_SINGLE_OVERLAP 1 /* SingleClosestSingleOverlap (Closest.scala:216-268) */

/* SingleClosest(left = a, right = b, partitionMap).compute() (Closest.scala
 * :34-214, CLI cli/Closest.scala:45-58) as the reference's sweep computes it on
 * one partition, mutable currentClosest included: for each left row the right
 * rows of its cache at the same unstrandedDistance as the current closest,
 * in cache order.  Both sets must be in full RegionOrdering (built with
 * lime_set_create_host_stranded; strand codes 0 when unstranded).  The records
 * carry a's own region (primitive returns the first region) and the two rows;
 * fill and checksum them with lime_intersect_fill_* / lime_intersect_checksum. */
int lime_closest_count(lime_ctx *ctx, const lime_set *a, const lime_set *b, int mode,
                       lime_pairs **plan, int64_t *n_pairs);
/* Diagnostics of a closest plan: the Jacobi rounds its cache-head fixed point
 * ran (capped at 32; LIME_CLOSEST_MAX_ROUNDS overrides) and whether the
 * in-order per-contig recursion finished it (same fixed point: the head
 * function is monotone). */
int lime_closest_rounds(const lime_pairs *plan, int32_t *rounds, int32_t *sequential);
/* closest over a genome cut into several spaces (spans >= 2^32: the host
 * splits the contigs, in order, into spaces below 2^32).  The reference's
 * sweep carries its liveness across contigs (a contig's lefts are reached
 * only from the end of the previous contig's rights), so the spaces chain:
 * alive_in = 1 for the first space, then the previous call's *alive_out. */
int lime_closest_count_chained(lime_ctx *ctx, const lime_set *a, const lime_set *b, int mode,
                               int32_t alive_in, int32_t *alive_out, lime_pairs **plan,
                               int64_t *n_pairs);

/* ------------------------------------------------------------ merge et al. */
int lime_merge(lime_ctx *ctx, const lime_set *a, lime_result **out, int64_t *n_runs);
/* DistributedSubtract of b from a (Subtract.scala:78-116), mode
 * LIME_SUBTRACT_LIME or LIME_SUBTRACT_SET.  At threshold <= 0 the blocks are
 * b's merge runs; when b has no zero-width rows and every 2048-row tile of a
 * sees at most 3072 rows of b, one pass derives them from b's rows in its
 * window (no merge scan of b); else b's merge scan runs first.  The
 * environment variable LIME_SUB_NO_LS (any value) forces the latter (tests
 * compare the two). */
int lime_subtract(lime_ctx *ctx, const lime_set *a, const lime_set *b, int64_t threshold,
                  int mode, lime_result **out, int64_t *n_regions);
int lime_complement(lime_ctx *ctx, const lime_space *genome_space, const lime_set *a,
                    lime_result **out, int64_t *n_regions);
/* Gaps of sorted, disjoint runs already in HBM (global coordinates, e.g. a
 * coordinate shard's merged runs after the cross-shard carry) over the genome,
 * keeping only the gaps whose START lies in [lo, hi) -- a shard's share of
 * the complement (Complement.scala:59-128 per partition, :67-73 / :112-122
 * at partition bounds, :39-45 for contigs without data).  The shard passes
 * its runs framed by the previous shards' last run end (a zero-width run at
 * it) and the next shards' first run start, so the gaps at its bounds end
 * where the unsharded result's do; lo = 0, hi = span gives lime_complement
 * of the runs. */
int lime_complement_runs(lime_ctx *ctx, const lime_space *genome, int64_t n,
                         const uint32_t *d_gstart, const uint32_t *d_gend, int64_t lo, int64_t hi,
                         lime_result **out, int64_t *n_regions);
int64_t lime_result_size(const lime_result *res);
/* Host copy of a result: regions in contig-local coordinates plus the
 * left/right input rows (-1 where the reference has None / no payload). */
int lime_result_fill_host(const lime_result *res, int32_t *contig, int64_t *start, int64_t *end,
                          int64_t *a_row, int64_t *b_row);
/* merge only: run index of every input row (the Iterable[T] grouping). */
int lime_result_run_of_row(const lime_result *res, int64_t *run_of_row);
/* merge only: the run of every SORTED input row and that row's id, copied
 * to caller DEVICE buffers (as many as the merged set has rows) -- the
 * Iterable[T] grouping on the device, which a sharded merge maps to global
 * run ids after the cross-shard carry */
int lime_result_copy_run_ids_device(const lime_result *res, uint32_t *d_run, uint32_t *d_row);
/* device-to-device copy of regions [first, first + count) (global) */
int lime_result_copy_rows_device(const lime_result *res, int64_t first, int64_t count,
                                 uint32_t *d_gstart, uint32_t *d_gend);
/* merge of a stranded set: strand codes of runs [first, first + count) to a
 * host array (0 for every run of an unstranded merge) -- the sharded merge
 * carry continues a run across a shard bound only on the same strand */
int lime_result_run_strands(const lime_result *res, int64_t first, int64_t count, int8_t *out);
int lime_result_device_arrays(const lime_result *res, const uint32_t **gstart,
                              const uint32_t **gend);
/* host copy of regions [first, first + count) in global coordinates */
int lime_result_copy_range(const lime_result *res, int64_t first, int64_t count, uint32_t *gstart,
                           uint32_t *gend);
int lime_result_destroy(lime_result *res);
/* Order-independent checksum of a result on the device (verification at
 * scale): reg = sum / xor over regions of
 * mix64(lime_pair_hash(start, end, a_row, b_row) + contig) with contig-local
 * start / end and 0xffffffff for an absent row; grp (merge results, else 0) =
 * sum / xor over input rows r of mix64(r << 32 | run of r), the Iterable[T]
 * grouping.  grp_sum / grp_xor may be NULL. */
int lime_result_checksum(const lime_result *res, uint64_t *reg_sum, uint64_t *reg_xor,
                         uint64_t *grp_sum, uint64_t *grp_xor);
/* BED writer on the device (the output side of loadBed, SURVEY.md 8(f) row
 * 1): the rows of a sorted set (in sorted order) or of a result, as
 * "chrom<TAB>start<TAB>end\n" lines in contig-local coordinates, into a
 * caller-owned HOST buffer.  names[c] = name of contig c of the object's
 * space (String order).  Two-call protocol: with cap < *len (e.g. out =
 * NULL, cap = 0) only the byte count *len is returned. */
int lime_set_format_bed(const lime_set *set, const char *const *names, char *out, int64_t cap,
                        int64_t *len);
int lime_result_format_bed(const lime_result *res, const char *const *names, char *out,
                           int64_t cap, int64_t *len);

/* ----------------------------------------------------- bit-per-base path */
/* The bit-per-base set straight from UNSORTED device rows (u32 contig-local
 * coordinates, as lime_set_create_device): rows are only grouped by 2^23-base
 * bin and then by 2^19-base paint tile (two counting scatters) -- no sort and
 * no merge.  Same bits as lime_bitset_from_set on the sorted set.
 * Memory (this and every *_from_device / *_from_global entry point below):
 * the bitset KEEPS its input rows in binned form for its lifetime, so that
 * an op's runs come straight from the bins (one paint per tile, no stored
 * words): 4 B per row (packed start / length, paint-tile order) + 16 B per
 * cross piece (a row crossing a paint tile, ~len / 2^19 of rows) + ~16 B per
 * 2^19-base paint tile, per input set.  The words (window bits / 8 B, 386 MB
 * over hg38) are painted on first need (popcount, an op whose other operand
 * is not binned, an AND past 16 sets) and are then held as well.  C5's
 * 8 x 1.25e8 rows: 4.0 GB of bins (against 386 MB of words);
 * lime_bitset_drop_bins trades them for the words. */
int lime_bitset_from_device(lime_ctx *ctx, const lime_space *space, int64_t n,
                            const int32_t *d_contig, const uint32_t *d_start,
                            const uint32_t *d_end, lime_bitset **out);
int lime_bitset_from_set(lime_ctx *ctx, const lime_set *a, lime_bitset **out);
/* A coordinate shard's bitset: global bits [lo, hi) of the space only
 * (lo % 64 == 0), from device rows in GLOBAL coordinates (gstart, gend, e.g.
 * the rows lime_route_rows delivered to this shard), clipped to the window.
 * Ops combine bitsets of the same window; their runs are in global
 * coordinates (SURVEY.md 8(e) "Bitset ops": clip at shard bounds, no halo). */
int lime_bitset_from_global(lime_ctx *ctx, const lime_space *space, int64_t lo, int64_t hi,
                            int64_t n, const uint32_t *d_gstart, const uint32_t *d_gend,
                            lime_bitset **out);
/* The AND of k row sets' bits straight from their unsorted device rows
 * (C5's k-way intersection, SURVEY.md 8(d) and Appendix A.4: the fold of the
 * reference's pairwise intersect, cli/Intersection.scala:41-54, over merged
 * operands): every set is binned as above, then one
 * kernel paints each tile of every set in LDS and ANDs them in registers --
 * one bitset stored, no per-set bitsets (past 16 sets, each group of 16
 * ANDs into the words of the earlier ones).  n, d_contig, d_start, d_end: k
 * entries each (host arrays of device pointers).  Same bits as
 * lime_bitset_and_runs over the k sets' bitsets. */
int lime_bitset_and_from_device(lime_ctx *ctx, const lime_space *space, int32_t k,
                                const int64_t *n, const int32_t *const *d_contig,
                                const uint32_t *const *d_start, const uint32_t *const *d_end,
                                lime_bitset **out);
/* The same over a coordinate shard's window [lo, hi) from GLOBAL rows (as
 * lime_bitset_from_global). */
int lime_bitset_and_from_global(lime_ctx *ctx, const lime_space *space, int64_t lo, int64_t hi,
                                int32_t k, const int64_t *n, const uint32_t *const *d_gstart,
                                const uint32_t *const *d_gend, lime_bitset **out);
int lime_bitset_window(const lime_bitset *bs, int64_t *lo, int64_t *n_words);
/* op: 0 = a, 1 = not a (within contigs), 2 = a and b, 3 = a and not b */
int lime_bitset_runs(lime_ctx *ctx, int op, const lime_bitset *a, const lime_bitset *b,
                     lime_result **out, int64_t *n_runs);
/* k-way AND of k bitsets, runs extracted (any k: past 16 the words are ANDed
 * group by group into a temporary bitset first) */
int lime_bitset_and_runs(lime_ctx *ctx, int k, const lime_bitset *const *sets, lime_result **out,
                         int64_t *n_runs);
int64_t lime_bitset_popcount(lime_ctx *ctx, const lime_bitset *a);
/* Paint the words (if not yet painted) and free the binned rows a bitset
 * built from rows keeps: it then holds window bits / 8 bytes, and every op
 * reads its words (same bits, same runs).  No-op for a bitset without bins. */
int lime_bitset_drop_bins(lime_ctx *ctx, lime_bitset *bs);
int lime_bitset_destroy(lime_bitset *bs);

/* ------------------------------------------------------ range sharding */
/* Route unsorted device rows to coordinate shards (the
 * Spark shuffles of ADAM repartitionAndSort, cli/Intersection.scala:42-43,
 * and OverlapBasedSetTheory.scala:75-84 with Partitioners.scala:10-20's
 * explicit-destination partitioner).  Shard r owns global coordinates
 * [splits[r], splits[r+1]) (host array, n_shards + 1 entries, splits[0] = 0,
 * splits[n_shards] = span, n_shards <= 64).  d_contig == NULL: d_start /
 * d_end are already global.  clip = 0: every row goes to the shard of its
 * start, whole; clip = 1: to every shard it overlaps, clipped to it.
 * counts[r] receives the rows for shard r; when their total is <= cap the
 * rows are also written grouped by shard (shard order, input order within a
 * shard) as global (d_gs, d_ge) and row id row_base + input index (d_row may
 * be NULL); d_strand_in (per input row, may be NULL) travels with its rows
 * to d_strand_out (stranded sets: the CLI's ReferenceRegion.stranded keys).
 * Validation and error codes as lime_set_create_device. */
int lime_route_rows(lime_ctx *ctx, const lime_space *space, int64_t n, const int32_t *d_contig,
                    const uint32_t *d_start, const uint32_t *d_end, uint32_t row_base,
                    int32_t n_shards, const uint32_t *splits, int clip, int64_t cap,
                    uint32_t *d_gs, uint32_t *d_ge, uint32_t *d_row, int64_t *counts,
                    const int8_t *d_strand_in, int8_t *d_strand_out);
/* The same routing with the pieces written INTERLEAVED into one device
 * array: piece p occupies d_rows[p * k .. p * k + k) = global start, global
 * end and (k = 3) row id row_base + input index -- the send buffer of ONE
 * all_to_all as it stands (no per-column repacking before the exchange).
 * k = 2 (clipped rows for bit-per-base shards) or 3.  No strand codes.
 * Errors, counts and cap as lime_route_rows.  ABI 6. */
int lime_route_rows_interleaved(lime_ctx *ctx, const lime_space *space, int64_t n,
                                const int32_t *d_contig, const uint32_t *d_start,
                                const uint32_t *d_end, uint32_t row_base, int32_t n_shards,
                                const uint32_t *splits, int clip, int64_t cap, int32_t k,
                                uint32_t *d_rows, int64_t *counts);
/* Interleaved rows (n rows of k = 2 or 3 u32 words, as exchanged) into k
 * device column arrays (d_dst2 unused for k = 2): one pass, stream-ordered,
 * no sync -- the receiving side of the routed exchange.  ABI 6. */
int lime_deinterleave_u32(lime_ctx *ctx, int64_t n, int32_t k, const uint32_t *d_src,
                          uint32_t *d_dst0, uint32_t *d_dst1, uint32_t *d_dst2);
/* k evenly spaced rows' global starts (rows i * n / k, i < k) into the
 * device array d_out, for count-balanced splitters (lime_amd.dist
 * sample_splits: the sampled range partitioner behind ADAM
 * repartitionAndSort, cli/Intersection.scala:41-42, Partitioners.scala:10-20).
 * d_contig == NULL: d_start is already global.  Stream-ordered, no sync.
 * ABI 4. */
int lime_sample_starts(lime_ctx *ctx, const lime_space *space, int64_t n, const int32_t *d_contig,
                       const uint32_t *d_start, int32_t k, uint32_t *d_out);

/* ------------------------------------------------------ synthetic inputs */
/* Counter-based generators (splitmix64 keyed by (seed, row)) identical to
 * lime_amd/synth.py, written to caller-owned device arrays. */
int lime_synth_uniform(lime_ctx *ctx, const lime_space *space, int64_t n, uint64_t seed,
                       uint32_t len_lo, uint32_t len_hi, int32_t *d_contig, uint32_t *d_start,
                       uint32_t *d_end);
int lime_synth_pileup(lime_ctx *ctx, const lime_space *space, int64_t n, uint64_t seed,
                      int64_t n_centres, uint32_t sigma, uint32_t len_lo, uint32_t len_hi,
                      int32_t *d_contig, uint32_t *d_start, uint32_t *d_end);
/* Rows [first, first + n) of the same sequences (a rank's slice of one
 * input: every shard count sees the same rows). */
int lime_synth_uniform_rows(lime_ctx *ctx, const lime_space *space, int64_t first, int64_t n,
                            uint64_t seed, uint32_t len_lo, uint32_t len_hi, int32_t *d_contig,
                            uint32_t *d_start, uint32_t *d_end);
int lime_synth_pileup_rows(lime_ctx *ctx, const lime_space *space, int64_t first, int64_t n,
                           uint64_t seed, int64_t n_centres, uint32_t sigma, uint32_t len_lo,
                           uint32_t len_hi, int32_t *d_contig, uint32_t *d_start,
                           uint32_t *d_end);

/* ------------------------------------------------------ host-only helpers */
/* rank_out[i] = position of names[i] in Java String order of the distinct
 * names (UTF-16 code-unit order; equal to byte order for ASCII). */
int lime_contig_rank(int32_t n, const char *const *names, int32_t *rank_out);
int lime_bed_read(const char *path, lime_bed **out);
int64_t lime_bed_rows(const lime_bed *bed);
int32_t lime_bed_contigs(const lime_bed *bed);
const char *lime_bed_contig_name(const lime_bed *bed, int32_t i);
/* per-row arrays, valid until lime_bed_free; contig = index into the BED's
 * own name table (first-seen order); strand: 0 '.', 1 '+', 2 '-', 3 '?' */
const int32_t *lime_bed_contig_ids(const lime_bed *bed);
const int64_t *lime_bed_starts(const lime_bed *bed);
const int64_t *lime_bed_ends(const lime_bed *bed);
const int8_t *lime_bed_strands(const lime_bed *bed);
const char *lime_bed_name(const lime_bed *bed, int64_t row); /* 4th column or "" */
void lime_bed_free(lime_bed *bed);
/* genome file: "name<TAB>length" per line (cli/Complement.scala:43-44) */

/* BED text parsed ON THE DEVICE (ADAM sc.loadBed replacement, cli/
 * Intersection.scala:42-45): `text` holds nbytes of BED in host memory; the
 * records stay in HBM as contig id (order of first appearance, names via
 * lime_dbed_contig_name), u32 start / end, strand code, and the byte offset +
 * length of the 4th column in `text`.  Same record rules and error codes as
 * lime_bed_read; coordinates outside [0, 2^32) are LIME_ERR_RANGE. */
int lime_bed_parse_device(lime_ctx *ctx, const char *text, int64_t nbytes, lime_dbed **out);
int64_t lime_dbed_rows(const lime_dbed *bed);
int32_t lime_dbed_contigs(const lime_dbed *bed);
const char *lime_dbed_contig_name(const lime_dbed *bed, int32_t i);
int lime_dbed_device_arrays(const lime_dbed *bed, const int32_t **contig, const uint32_t **start,
                            const uint32_t **end, const int8_t **strand);
int lime_dbed_fill_host(const lime_dbed *bed, int32_t *contig, int64_t *start, int64_t *end,
                        int8_t *strand, int64_t *name_off, int32_t *name_len);
/* Rewrite the device contig ids in place: id i -> new_id_of_contig[i] (n =
 * lime_dbed_contigs), e.g. to a lime_space's String-order ids before
 * lime_set_create_device.  Once per handle. */
int lime_dbed_remap_contigs(lime_dbed *bed, const int32_t *new_id_of_contig, int32_t n);
void lime_dbed_free(lime_dbed *bed);
int lime_genome_read(const char *path, int32_t *n_out, char ***names_out, int64_t **lengths_out);
void lime_genome_free(int32_t n, char **names, int64_t *lengths);
uint64_t lime_pair_hash(uint32_t start, uint32_t end, uint32_t a_row, uint32_t b_row);

#ifdef __cplusplus
}
#endif
#endif /* LIME_AMD_H */
