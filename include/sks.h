/*
 * sks.h — C ABI of the MI355X spaced-k-mer sketch + ANI engine (libsks.so).
 *
 * Plain pointers and sizes only.  "d_" arguments are device (HBM) pointers on
 * the context's device; everything else is host memory owned by the caller.
 * Every entry point returns an sks_status (0 = OK); the message of the last
 * failure on the calling thread is available from sks_last_error().
 *
 * Each entry point names the reference interface it replaces
 * (bensonlzl/spaced-kmer-sketching @ 2024-10-22, paths under src/).
 * The reference is a source-level C++ API with no FFI; the C++ facade in
 * spaced-kmer-sketching_amd/cpp/ re-exposes the reference names on top of
 * this ABI (see INTEGRATION.md for the binding a maintainer would add).
 */
#ifndef SKS_H
#define SKS_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SKS_ABI_VERSION 3  /* 3: a join layout's boff row ends with one more word, the log2 of
                              the buckets per region, which the join reads: layouts built by
                              an ABI-2 library (rows without that word) must not be joined by
                              this one (round 5).  2: deduplicated join layout (masks, region
                              ends), elem_words on the layout entry points,
                              sks_ctx_set_join_check; later additions within 2 (new symbols
                              only): sks_ani_rows, sks_intersect_layout_ani, sks_host_alloc,
                              sks_host_free, sks_join_layout_stat_copy, sks_sketches_export,
                              sks_all_pairs_ani, sks_ctx_set_layout_blocks_hint,
                              sks_ctx_ani_table */

typedef enum sks_status {
  SKS_OK = 0,
  SKS_E_ARG = 1,         /* invalid argument (the reference has UB here)        */
  SKS_E_HIP = 2,         /* HIP runtime error / no device                        */
  SKS_E_IO = 3,          /* unreadable FASTA (reference: stderr + exit(1))       */
  SKS_E_NOMEM = 4,       /* host or device allocation failed                    */
  SKS_E_UNSUPPORTED = 5, /* valid in the reference, not implemented here (yet)   */
  SKS_E_LENGTH = 6       /* pair lists of different lengths (kmer_set.cpp:147)   */
} sks_status;

/* Sketch selection policy: the device-side replacement for the reference's
 * std::function<bool(const kmer)> sketching_cond (kmer.hpp:97, kmer_sliding.cpp:183),
 * which is a host callback and cannot run in a kernel. */
typedef enum sks_policy_kind {
  SKS_FRAC_MOD = 0, /* keep iff frac_min_hash(k) % param == 0 (kmer-sketching.cpp:30-34) */
  SKS_BOTTOM_S = 1  /* the `param` distinct k-mers with the smallest frac_min_hash
                       (ties by k-mer value) — build-defined, no reference equivalent */
} sks_policy_kind;

/* boost::hash_value(dynamic_bitset) flavour used by frac_min_hash (kmer.hpp:137-146).
 * The reference does not pin its Boost version; see DESIGN.md "hash parity". */
typedef enum sks_hash_flavour {
  SKS_HASH_BOOST_MIX = 0,   /* Boost >= 1.81: hash_combine = hash_mix(seed + 0x9e3779b9 + v) */
  SKS_HASH_BOOST_LEGACY = 1 /* Boost 1.71-1.80: MurmurHash2-style hash_combine_impl          */
} sks_hash_flavour;

typedef struct sks_policy {
  int32_t kind;    /* sks_policy_kind                                   */
  int32_t flavour; /* sks_hash_flavour                                  */
  uint64_t param;  /* SKS_FRAC_MOD: c (> 0); SKS_BOTTOM_S: s (> 0)       */
  int64_t nonce;   /* frac_min_hash nonce; the reference uses fmh(1)     */
} sks_policy;

/* ---- library ---------------------------------------------------------------- */
int sks_abi_version(void);
const char* sks_last_error(void);
/* "src:<16 hex digits>": hash of the sources this library was linked from
 * (spaced-kmer-sketching_amd/srchash.py); no reference counterpart. */
const char* sks_build_info(void);

/* ---- host helpers (no device needed) ---------------------------------------------- */
/* generate_random_spaced_seed_mask(w, k, seed) — kmer_bitset.cpp:132-152.
 * mask[0] = bits 0..63, mask[1] = bits 64..127.  1 <= k <= w <= 64. */
int sks_mask_generate(int window, int k, uint64_t seed, uint64_t mask[2]);
/* contiguous_kmer(l) — kmer_bitset.cpp:50-56 (l > 64 -> SKS_E_ARG like its runtime_error). */
int sks_mask_contiguous(int length, uint64_t mask[2]);
/* frac_min_hash::operator() — kmer.hpp:144-148 (kmer = masked canonical bits). */
uint64_t sks_frac_min_hash(const uint64_t kmer[2], const uint64_t mask[2], int window,
                           int64_t nonce, int flavour);
/* containment / binomial_estimator — ani_estimation.cpp:24-28, :38-42. */
double sks_containment(int intersection, int set_size);
double sks_binomial_estimator(double containment, int kmer_num_ones);
/* Vector form of kmer-sketching.cpp:195-200: cont[i] = containment(inter[i], size_first[i]),
 * ani[i] = binomial_estimator(cont[i], kmer_num_ones).  Either output may be NULL. */
int sks_ani_from_counts(const int32_t* inter, const int32_t* size_first, uint64_t n,
                        int kmer_num_ones, double* cont, double* ani);

/* ---- FASTA ingress (host) — fasta_processing.cpp:79-211 ----------------------------- */
typedef struct sks_fasta sks_fasta;
/* strings_from_fasta(): parses the file with the reference's record rules.
 * Unreadable file -> SKS_E_IO (the reference prints to stderr and exit(1)s). */
int sks_fasta_open(const char* path, sks_fasta** out);
void sks_fasta_close(sks_fasta* f);
uint64_t sks_fasta_num_records(const sks_fasta* f);
/* Record i's raw content (the i-th string of strings_from_fasta). */
int sks_fasta_record(const sks_fasta* f, uint64_t i, const uint8_t** data, uint64_t* len);
/* The record stream handed to the device: every record followed by one '\n'
 * separator (a non-ACGT byte, so k-mers never span records). */
const uint8_t* sks_fasta_stream(const sks_fasta* f);
uint64_t sks_fasta_stream_bytes(const sks_fasta* f);
/* cut_nucleotide_strings(): ACGT runs as codes 0..3 (one byte each).  Call with
 * NULL buffers to get *n_codes / *n_runs, then again with buffers that large. */
int sks_fasta_runs(const sks_fasta* f, uint8_t* codes, uint64_t* run_lens, uint64_t* n_codes,
                   uint64_t* n_runs);

/* ---- device context ---------------------------------------------------------------- */
typedef struct sks_ctx sks_ctx;
/* stream: a hipStream_t (may be NULL = the default stream).  Creating a context
 * loads every code object of the library on its device (one empty kernel per HIP
 * translation unit; ~30 ms the first time in a process), so that the first build
 * or join does not pay it inside the caller's timing. */
int sks_ctx_create(int device, void* stream, sks_ctx** out);
int sks_ctx_destroy(sks_ctx* ctx);
int sks_ctx_set_stream(sks_ctx* ctx, void* stream);
/* The device index the context was created on (-1 for NULL). */
int sks_ctx_device(const sks_ctx* ctx);
int sks_ctx_synchronize(sks_ctx* ctx);

/* Per-phase device times of the last sketch build / intersection on this
 * context, measured with hipEvents on the context's stream. */
typedef struct sks_timings {
  float scan_ms;      /* fused extract/canonicalise/hash/select kernel(s) */
  float post_ms;      /* sort + unique + bottom-s selection               */
  float total_ms;     /* whole call, first launch to last                 */
  uint64_t windows;   /* k-mer windows hashed                             */
  uint64_t scan_launches;
  uint64_t survivors; /* records emitted by the scan kernel               */
} sks_timings;
int sks_ctx_last_timings(const sks_ctx* ctx, sks_timings* out);

/* ---- sketch build: kmer_sliding.cpp:112-238 + kmer.hpp:135-190 + kmer_set.cpp:54-133 ---
 * d_seq: n_bytes of sequence bytes in device memory.  Non-ACGT bytes split runs
 * exactly as fasta_processing.cpp:144-179 does, so an sks_fasta stream can be
 * uploaded as is.  The bytes are cut into n_seg segments (genomes) by the host
 * array seg_off[n_seg + 1]; one sketch is built per segment (the reference
 * builds one kmer_set per FASTA file, kmer_set.cpp:112-133).
 * Result: an opaque device-resident sketch set (sorted unique canonical masked
 * k-mers per segment; one u64 word per k-mer when window <= 32, two (lo, hi)
 * when 32 < window <= 64). */
typedef struct sks_sketch_set sks_sketch_set;
int sks_sketch_build(sks_ctx* ctx, const uint8_t* d_seq, uint64_t n_bytes, const uint64_t* seg_off,
                     uint32_t n_seg, int window, const uint64_t mask[2], const sks_policy* policy,
                     sks_sketch_set** out);
/* Frees the set. Like hipFree, it first waits for all work queued on the
 * device; the arrays then go to a per-process block cache for later builds. */
int sks_sketch_set_free(sks_sketch_set* set);
/* Stream-ordered free (the hipFreeAsync contract): every use of the set must
 * be ordered before the current end of `stream` (a hipStream_t, NULL = the
 * null stream). Does not wait; the arrays are reused only once that point of
 * `stream` has completed. Lets several host threads build and free
 * concurrently without the device-wide wait of sks_sketch_set_free. */
int sks_sketch_set_free_on_stream(sks_sketch_set* set, void* stream);
uint32_t sks_sketch_set_num(const sks_sketch_set* set);
int sks_sketch_set_elem_words(const sks_sketch_set* set); /* 1 or 2 */
/* Host copies of per-sketch sizes (kmer_set::kmer_set_size, kmer.hpp:186-189)
 * and windows hashed per sketch. */
int sks_sketch_set_sizes(const sks_sketch_set* set, uint32_t* sizes);
int sks_sketch_set_windows(const sks_sketch_set* set, uint64_t* windows);
/* Device layout: sketch i = d_data()[start[i]*elem_words ...], sizes[i] elements. */
const uint64_t* sks_sketch_set_device_data(const sks_sketch_set* set);
const uint64_t* sks_sketch_set_device_starts(const sks_sketch_set* set);
const uint32_t* sks_sketch_set_device_sizes(const sks_sketch_set* set);
int sks_sketch_set_starts(const sks_sketch_set* set, uint64_t* starts);
/* Copy sketch i to host (sizes[i] * elem_words u64). */
int sks_sketch_set_copy(const sks_sketch_set* set, uint32_t i, uint64_t* out);
/* Write all sketches into a caller-owned fixed-stride device layout
 * (d_dst[i * stride * elem_words ...], d_sizes[i]) — the all-gather shape. */
int sks_sketch_set_export(const sks_sketch_set* set, uint64_t* d_dst, uint64_t stride,
                          uint32_t* d_sizes);

/* ---- persisted sketches (no reference equivalent) ------------------
 * A sketch set remembers how it was made; sks_sketch_set_save writes it with
 * that description to a self-checking file (format: csrc/persist.cpp) and
 * sks_sketch_set_load brings it back onto the context's device, ready for
 * sks_intersect_*.  A missing, truncated or corrupt file -> SKS_E_IO. */
typedef struct sks_sketch_info {
  int32_t window;
  int32_t elem_words;
  uint64_t mask[2];
  sks_policy policy;
  uint32_t n;
  int32_t has_names;
} sks_sketch_info;
int sks_sketch_set_info(const sks_sketch_set* set, sks_sketch_info* info);
/* names: n strings (e.g. the FASTA file names), or NULL to clear. */
int sks_sketch_set_set_names(sks_sketch_set* set, const char* const* names);
/* Name of sketch i, or NULL when the set has no names. */
const char* sks_sketch_set_name(const sks_sketch_set* set, uint32_t i);
int sks_sketch_set_save(const sks_sketch_set* set, const char* path);
int sks_sketch_set_load(sks_ctx* ctx, const char* path, sks_sketch_set** out);
/* One set holding the sketches of sets[0], sets[1], ... in order (e.g. shards
 * sketched on different ranks or at different times).  All sets must share
 * window, mask and policy. */
int sks_sketch_set_concat(sks_ctx* ctx, const sks_sketch_set* const* sets, uint32_t n_sets,
                          sks_sketch_set** out);

/* ---- ordered k-mer lists: nucleotide_string_list_to_kmers (kmer_sliding.cpp:112-238) ---
 * Every selected window of every segment, in stream order, duplicates kept —
 * the reference's vector<kmer>.  Same inputs as sks_sketch_build; the policy
 * must be SKS_FRAC_MOD (the per-k-mer predicate; param 1 keeps every window).
 * Element i: window start byte positions[i] and bits[4i..4i+3] = kmer_bits
 * (lo, hi), masked_bits (lo, hi) of the reference's `kmer` (kmer.hpp:75-86):
 * kmer_bits is the chosen strand's window register — R (2w bits), or F, which
 * in the reference keeps up to 64 bases of the run ending at the window. */
typedef struct sks_kmer_list sks_kmer_list;
int sks_kmer_list_build(sks_ctx* ctx, const uint8_t* d_seq, uint64_t n_bytes, const uint64_t* seg_off,
                        uint32_t n_seg, int window, const uint64_t mask[2], const sks_policy* policy,
                        sks_kmer_list** out);
int sks_kmer_list_free(sks_kmer_list* list);
uint64_t sks_kmer_list_total(const sks_kmer_list* list);
/* counts[n_seg]: k-mers per segment (the list is segment 0's, then segment 1's, ...). */
int sks_kmer_list_counts(const sks_kmer_list* list, uint64_t* counts);
const uint64_t* sks_kmer_list_device_positions(const sks_kmer_list* list);
const uint64_t* sks_kmer_list_device_bits(const sks_kmer_list* list);
/* Host copies; either pointer may be NULL. */
int sks_kmer_list_copy(const sks_kmer_list* list, uint64_t* positions, uint64_t* bits);

/* Every window of a record-stream piece, dense by start position, for a HOST
 * predicate: the window sequence nucleotide_string_to_kmers hands to its
 * std::function<bool(const kmer)> (kmer_sliding.cpp:144-183), without any
 * selection.  Row i describes the window starting at byte first + i of d_seq
 * (i < n_windows): {kmer_bits lo, hi, masked_bits lo} for window <= 32 (3
 * words), {kmer_bits lo, hi, masked_bits lo, hi} for window > 32 (4 words);
 * bit i % 64 of d_valid[i / 64] is set when all its bytes are ACGT (case-
 * insensitive; any other byte ends a run, fasta_processing.cpp:144-179) — the
 * rows of invalid windows are unspecified.  kmer_bits is the canonical window
 * with the reference's 128-bit history (up to 64 bases of the run), so a caller
 * cutting a stream into pieces passes min(first_of_piece, 64 - window) bytes
 * of history before `first`.  Queued on the context stream (no host sync). */
int sks_windows_dense(sks_ctx* ctx, const uint8_t* d_seq, uint64_t n_bytes, uint64_t first, uint64_t n_windows,
                      int window, const uint64_t mask[2], uint64_t* d_rows, uint64_t* d_valid);
/* Words per row of sks_windows_dense: 3 (window <= 32) or 4. */
int sks_windows_dense_row_words(int window);

/* ---- intersection: kmer_set.cpp:23-41, :143-184 ----------------------------------
 * Sketches in device memory: sketch i = d_data[d_starts[i]*elem_words ...],
 * d_sizes[i] elements, each sorted ascending and unique (as built above). */
/* Pair list (compute_pairwise_kmer_set_intersections): d_out[p] = |S[a[p]] ∩ S[b[p]]|. */
int sks_intersect_pairs(sks_ctx* ctx, const uint64_t* d_data, const uint64_t* d_starts,
                        const uint32_t* d_sizes, int elem_words, const int32_t* d_a,
                        const int32_t* d_b, uint64_t n_pairs, int32_t* d_out);
/* All ordered pairs of a row block (generate_all_pairs_from_vector, generators.hpp:44-58):
 * d_out[(i - row_begin) * n + j] = |S[i] ∩ S[j]| for row_begin <= i < row_end, 0 <= j < n. */
int sks_intersect_all(sks_ctx* ctx, const uint64_t* d_data, const uint64_t* d_starts,
                      const uint32_t* d_sizes, int elem_words, uint32_t n, uint32_t row_begin,
                      uint32_t row_end, int32_t* d_out);

/* Symmetric all-vs-all for sharding across devices: the n x n matrix is cut
 * into 64 x 64 tiles and the upper-triangle tiles (I <= J, row-major, count
 * sks_intersect_sym_tiles(n)) in [tile_begin, tile_end) are computed; each
 * count is written to both d_out[i * n + j] and d_out[j * n + i] of the n x n
 * int32 matrix, which the call zeroes first.  Summing the matrices of calls
 * that together cover [0, sks_intersect_sym_tiles(n)) gives the full
 * generate_all_pairs_from_vector result (e.g. an all-reduce over ranks). */
uint64_t sks_intersect_sym_tiles(uint32_t n);
int sks_intersect_sym(sks_ctx* ctx, const uint64_t* d_data, const uint64_t* d_starts,
                      const uint32_t* d_sizes, int elem_words, uint32_t n, uint64_t tile_begin,
                      uint64_t tile_end, int32_t* d_out);

/* ---- sketch union (no reference equivalent) --------------------------------------------
 * Sorted unique union of n u64 k-mers (any order, duplicates allowed): e.g. the
 * FracMinHash sketches of chunks of one genome cut with (w-1)-base halos, whose
 * union is the genome's sketch (FracMinHash keeps a k-mer on its own hash).
 * d_out holds n values; *n_out (host) = distinct values.  Narrow (w <= 32) only. */
int sks_sketch_union(sks_ctx* ctx, const uint64_t* d_in, uint64_t n, uint64_t* d_out,
                     uint64_t* n_out);
/* The same for 32 < w <= 64: n 128-bit k-mers as (lo, hi) word pairs (2n words),
 * ordered by the 128-bit value like the reference's operator< on kmer_bitset.
 * d_in / d_out 16-byte aligned (SKS_E_ARG otherwise). */
int sks_sketch_union_wide(sks_ctx* ctx, const uint64_t* d_in, uint64_t n, uint64_t* d_out,
                          uint64_t* n_out);

/* ---- join layout: all-vs-all across GPUs ------------------------------------------------
 * The all-pairs join kernel (sks_intersect_all / _sym, SKS_INTERSECT_JOIN) reads
 * a "join layout": blocks of 64 consecutive sketches, each DISTINCT value of a
 * block stored once with a 64-bit mask of the block's sketches holding it
 * (bit s = sketch 64 * block + s).  Buckets are two-level: G =
 * sks_join_layout_groups(log_b) value groups cut by bounds (G + 1 values of
 * elem_words words each, non-decreasing, bounds[0] = 0, bounds[G] = the
 * largest value), each split into 8 (or 2^log_b when log_b < 3) hash buckets;
 * 2^rg consecutive groups form a region (NR = regions per block; the build
 * picks rg in 1..3 by its size: 8-group regions when the blocks give >= 1024
 * of them, smaller ones for small builds).  A region's entries start at its
 * raw offset in the block (the block's sketch elements in earlier regions),
 * so its tail up to the next region is unused.  Exposing the
 * layout lets a multi-GPU caller build the layout of its own sketches only and
 * all-gather layouts instead of raw sketches (no replicated build):
 *   vals   u64[total * elem_words]  entry values, block-major (total = sum of sizes)
 *   masks  u64[total]               sketch mask of each entry
 *   boff   u32[nb * sks_join_layout_boff_words(log_b)]  per block (nb = ceil(n/64)):
 *          2^log_b bucket starts, then NR region ends, relative to bstart[block]
 *          (room for G), and in the row's last word log2 of the buckets per region
 *   bstart u64[nb + 1]              raw block starts (prefix of the sizes); [nb] = total
 * Layouts of consecutive sketch ranges that each start at a multiple of 64 can
 * be concatenated (append vals/masks/boff and add the data offset to bstart)
 * when they were built with the same bounds.  elem_words: 1 (u64 k-mers,
 * w <= 32) or 2 ((lo, hi) k-mers, 32 < w <= 64). */
/* log_b for a largest sketch of max_sketch_size elements (all ranks must agree). */
uint32_t sks_join_layout_log_b(uint32_t max_sketch_size);
/* Block-bucket population (entries) one join chunk holds; larger buckets are
 * joined in sub-chunks (exact, slower). */
uint32_t sks_join_layout_capacity(void);
/* Value groups of a layout with 2^log_b buckets (bounds hold groups + 1 values). */
uint32_t sks_join_layout_groups(uint32_t log_b);
/* Words of one block's boff row: 2^log_b bucket starts + room for the region
 * ends + the region size word (the row's last word, log2 of the buckets per
 * region; added in ABI 3 — rows of ABI-2 layouts are one word shorter). */
uint32_t sks_join_layout_boff_words(uint32_t log_b);
/* Group bounds fixed by the mask alone (host array of (groups + 1) * elem_words
 * words): the quantiles of min(F & M, R & M) for random sequence, so every rank
 * of a multi-GPU all-vs-all uses the same bounds without sampling or
 * exchanging anything.  Any bounds give exact counts; these balance groups for
 * genome-like (near-uniform) k-mers. */
int sks_join_layout_bounds_for_mask(const uint64_t mask[2], uint32_t log_b, int elem_words, uint64_t* bounds);
/* Group bounds balanced for the set (quantiles averaged over up to 64 sample
 * sketches), queued on the context stream.  Any bounds give exact counts. */
int sks_join_layout_bounds(sks_ctx* ctx, const uint64_t* d_data, const uint64_t* d_starts,
                           const uint32_t* d_sizes, int elem_words, uint32_t n, uint32_t log_b,
                           uint64_t* d_bounds);
/* Builds the layout of sketches (d_data, d_starts, d_sizes)[0, n) into caller
 * buffers (three launches: bounds + block starts, group positions, placement).
 * d_bounds: the group bounds (NULL: the set's own, sks_join_layout_bounds).
 * *max_block_bucket (host) receives the largest block-bucket population in
 * entries, or UINT32_MAX when the build could not place a group (only for
 * adversarial 128-bit values; the layout is then invalid) — it waits for the
 * build; NULL skips that read-back.  total_hint: the n sizes' sum when the
 * caller knows it (the build then never waits for the stream), UINT64_MAX to
 * have the sizes read back. */
int sks_join_layout_build(sks_ctx* ctx, const uint64_t* d_data, const uint64_t* d_starts,
                          const uint32_t* d_sizes, int elem_words, uint32_t n, uint64_t total_hint,
                          uint32_t log_b, const uint64_t* d_bounds, uint64_t* d_out_vals,
                          uint64_t* d_out_masks, uint32_t* d_out_boff, uint64_t* d_out_bstart,
                          uint32_t* max_block_bucket);
/* Queues a copy of the last sks_join_layout_build's two status words on this
 * context — [0] the largest block-bucket population, [1] non-zero when the
 * layout is invalid (see max_block_bucket) — into d_dst (2 x u32, device), so
 * a caller that skips the read-back can check the layout after the join
 * without a stream round trip.  Call it right after the build. */
/* Region-size hint for the next sks_join_layout_build calls on this context:
 * the number of 64-sketch blocks that actually hold sketches (0, the default:
 * every block does).  A build over a buffer with many empty rows — a rank's
 * exchange buffer, a slot per rank — then picks the region size (workgroups
 * per block) for its real work.  The layout's content does not depend on it. */
int sks_ctx_set_layout_blocks_hint(sks_ctx* ctx, uint32_t blocks);
int sks_join_layout_stat_copy(sks_ctx* ctx, uint32_t* d_dst);
/* sks_intersect_sym over a join layout of n sketches: upper-triangle 64x64 tiles
 * [tile_begin, tile_end) into the n x n int32 matrix d_out (zeroed first). */
int sks_intersect_sym_layout(sks_ctx* ctx, uint32_t n, uint32_t log_b, int elem_words, const uint64_t* d_vals,
                             const uint64_t* d_masks, const uint32_t* d_boff, const uint64_t* d_bstart,
                             uint64_t tile_begin, uint64_t tile_end, int32_t* d_out);

/* Tiles of the n x n matrix over a join layout whose block 0 is global block
 * blk0 (a rank's own blocks, or a gathered layout with blk0 = 0); every tile's
 * two blocks must lie in the layout.  Tiles: d_tiles == NULL -> upper-triangle
 * tiles [tile_begin, tile_end) (row-major, sks_intersect_sym_tiles; blk0 must
 * be 0, else SKS_E_ARG); else the list d_tiles[2t] = I, d_tiles[2t + 1] = J
 * (I <= J, global block indices) for t in [tile_begin, tile_end).  packed == 0:
 * counts are ADDED to the n x n int32 matrix d_out at (i, j) and (j, i);
 * packed != 0: to d_out[(t - tile_begin) * 4096 + r * 64 + c] for row I*64 + r,
 * column J*64 + c (a diagonal tile holds both triangles).  The caller zeroes
 * d_out.  A multi-GPU caller counts the tiles of its own blocks on its own
 * layout while the others' layouts are still being gathered. */
int sks_intersect_layout_tiles(sks_ctx* ctx, uint32_t n, uint32_t log_b, int elem_words, const uint64_t* d_vals,
                               const uint64_t* d_masks, const uint32_t* d_boff, const uint64_t* d_bstart,
                               uint32_t blk0, const uint32_t* d_tiles, uint64_t tile_begin,
                               uint64_t tile_end, int packed, int32_t* d_out);

/* sks_intersect_layout_tiles with the row blocks and the column blocks in two
 * layouts (built with the same bounds): tile (I, J) of the list joins row block
 * I of the row layout (whose block 0 is global block r_blk0) with column block
 * J of the column layout (block 0 = c_blk0).  A multi-GPU caller joins its own
 * layout with each peer's as the peer's sketches arrive. */
int sks_intersect_layout_pair_tiles(sks_ctx* ctx, uint32_t n, uint32_t log_b, int elem_words,
                                    const uint64_t* d_rvals, const uint64_t* d_rmasks, const uint32_t* d_rboff,
                                    const uint64_t* d_rbstart, uint32_t r_blk0, const uint64_t* d_cvals,
                                    const uint64_t* d_cmasks, const uint32_t* d_cboff, const uint64_t* d_cbstart,
                                    uint32_t c_blk0, const uint32_t* d_tiles, uint64_t tile_begin,
                                    uint64_t tile_end, int packed, int32_t* d_out);
/* sks_intersect_layout_pair_tiles fused with containment / ANI — the count
 * loop, the containment / binomial_estimator loop and the host result vector of
 * kmer-sketching.cpp:185-200 (ani_estimation.cpp:24-42) in one launch: counts
 * are added to d_out as there (packed or both halves of the n x n matrix; the
 * caller zeroes d_out), and as each tile's last workgroup finishes, it writes
 *   ani[i * n + j] = binomial_estimator(containment(|S_i ∩ S_j|, d_sizes[i]), kmer_num_ones)
 * for both orientations (i, j) and (j, i) of every pair of the tile (the
 * diagonal tile's own pairs once).  d_sizes[i] = |S_i| (int32, n entries, by
 * global genome index).  ani: n * n doubles in device memory, or pinned host
 * memory (sks_host_alloc, or any hipHostMalloc'd buffer): the kernel then
 * writes the host matrix itself, so the transfer runs while later tiles are
 * counted.  Cells of tiles not in the list are left untouched.  d_tiles ==
 * NULL: the upper-triangle tiles [tile_begin, tile_end) of ONE layout
 * (rows == cols, r_blk0 = c_blk0 = 0). */
int sks_intersect_layout_ani(sks_ctx* ctx, uint32_t n, uint32_t log_b, int elem_words,
                             const uint64_t* d_rvals, const uint64_t* d_rmasks, const uint32_t* d_rboff,
                             const uint64_t* d_rbstart, uint32_t r_blk0, const uint64_t* d_cvals,
                             const uint64_t* d_cmasks, const uint32_t* d_cboff, const uint64_t* d_cbstart,
                             uint32_t c_blk0, const uint32_t* d_tiles, uint64_t tile_begin, uint64_t tile_end,
                             int packed, int32_t* d_out, const int32_t* d_sizes, int kmer_num_ones, double* ani);
/* sks_sketch_set_export for sketches given as device arrays (e.g. a received
 * shard): d_dst[i * stride * elem_words ...] = sketch i padded with ~0 words,
 * d_dst_sizes[i] = d_sizes[i]; queued on the context stream, no wait.  Every
 * d_sizes[i] must be <= stride (the caller's bound; larger sketches are cut). */
int sks_sketches_export(sks_ctx* ctx, const uint64_t* d_data, const uint64_t* d_starts, const uint32_t* d_sizes,
                        int elem_words, uint32_t n, uint64_t* d_dst, uint64_t stride, uint32_t* d_dst_sizes);
/* The whole "comparison" of kmer-sketching.cpp:185-200 in one call, for one
 * process and one device: every ordered pair of the n sketches (d_data,
 * d_starts, d_sizes — e.g. a set's device arrays) counted over a join layout
 * of all of them (built in context scratch), and, when ani != NULL, their
 * containment / ANI written by the join as in sks_intersect_layout_ani
 * (ani[i * n + j], n * n doubles in device or pinned host memory).
 * d_counts: the packed upper-triangle tiles [sks_intersect_sym_tiles(n)][64][64]
 * int32 (sks_intersect_layout_tiles' packed format; the call clears them, the
 * caller need not), or NULL to keep them in scratch.  max_size: the largest sketch (sizes the buckets); total: the sizes'
 * sum (or an upper bound).  d_status (device, 2 x u32, may be NULL) receives the
 * layout's status words (sks_join_layout_stat_copy).  Queued on the context
 * stream; nothing waits.  sks_ctx_last_intersect_ms then times the join launch
 * alone. */
int sks_all_pairs_ani(sks_ctx* ctx, const uint64_t* d_data, const uint64_t* d_starts, const uint32_t* d_sizes,
                      int elem_words, uint32_t n, uint32_t max_size, uint64_t total, int kmer_num_ones,
                      double* ani, int32_t* d_counts, uint32_t* d_status);
/* One rank's step of a multi-GPU all-vs-all (sks_dist.all_vs_all_join) in one
 * call: the join layout of the n sketches (context scratch; group bounds
 * d_bounds, or sampled when NULL; blocks_hint as sks_ctx_set_layout_blocks_hint)
 * whose block 0 is global block blk0, then the join of the n_tiles global
 * (I, J) tiles of d_tiles (u32 pairs, both blocks in this set) into the packed
 * d_counts[n_tiles][64][64], and — ani non-NULL — containment / ANI of both
 * orientations written into the n_global x n_global matrix ani (device or
 * mapped pinned host memory), with |S_g| = d_sizes_global[g] for global genome
 * g.  The counts, the tiles' finisher counters and the two status words
 * (d_status, as sks_join_layout_build's: max block bucket, invalid) are
 * cleared by the build itself: four launches, no memset, no host sync.
 * Replaces per tile kmer_set.cpp:23-41 over kmer_set.cpp:167-184's pairs. */
int sks_layout_tiles_ani(sks_ctx* ctx, const uint64_t* d_data, const uint64_t* d_starts, const uint32_t* d_sizes,
                         int elem_words, uint32_t n, uint64_t total, uint32_t log_b, const uint64_t* d_bounds,
                         uint32_t blocks_hint, uint32_t blk0, const uint32_t* d_tiles, uint64_t n_tiles,
                         uint32_t n_global, const int32_t* d_sizes_global, int kmer_num_ones, double* ani,
                         int32_t* d_counts, uint32_t* d_status);
/* Pinned host memory the device reads and writes directly (mapped into every
 * device's address space): the destination of a fused ANI matrix.  coherent:
 * fine-grained (every device store goes to the host as issued); 0: coarse-
 * grained (device stores are cached and written back by the end of the kernel,
 * in whole lines).  No reference counterpart (the reference's result vectors
 * are plain host vectors, kmer-sketching.cpp:193). */
int sks_host_alloc(uint64_t bytes, int coherent, void** out);
/* ANI by shared-element count for sets of `size` elements, kept on the context:
 * table[x] = binomial_estimator(containment(x, size), kmer_num_ones) for x in
 * [0, size] (the same device function as the fused conversion, so the same
 * doubles).  The fused ANI of sks_intersect_layout_ani / sks_all_pairs_ani then
 * reads a row whose set holds `size` elements from the table instead of
 * evaluating pow (bottom-s sets: every row).  Queued on the context stream;
 * rebuilt only when (size, kmer_num_ones) changes; sizes above
 * SKS_ANI_TABLE_MAX (or 0) drop the table.  sks_all_pairs_ani calls it with its
 * max_size. */
#define SKS_ANI_TABLE_MAX (1u << 20)
int sks_ctx_ani_table(sks_ctx* ctx, uint32_t size, int kmer_num_ones);
int sks_host_free(void* p);
/* The set's sketches back to back (sizes[i] * elem_words words each, in order)
 * and its sizes, copied into caller device buffers (a send buffer). */
int sks_sketch_set_export_csr(const sks_sketch_set* set, uint64_t* d_data, uint32_t* d_sizes);

/* ---- containment / ANI on the device: kmer-sketching.cpp:195-200 + ani_estimation.cpp:24-42 ----
 * d_ani[i * n + j] = binomial_estimator(containment(counts[i][j], |S_i|), kmer_num_ones)
 * for the n x n count matrix (|S_i| = counts[i][i]); d_cont (may be NULL) the
 * containments.  Queued on the context stream. */
int sks_ani_matrix(sks_ctx* ctx, const int32_t* d_counts, uint32_t n, int kmer_num_ones, double* d_cont,
                   double* d_ani);
/* Rows [row_begin, row_end) of sks_ani_matrix (same addressing: d_ani[i * n + j]),
 * so a caller can convert and copy out the rows an all-pairs call has finished
 * (rows of tile rows [0, I) are final once those tile rows are counted) while
 * later tiles are still being counted. */
int sks_ani_rows(sks_ctx* ctx, const int32_t* d_counts, uint32_t n, uint32_t row_begin, uint32_t row_end,
                 int kmer_num_ones, double* d_cont, double* d_ani);
/* Packed tiles (d_packed [n_tiles][64][64] of tiles d_tiles[2t] = I,
 * d_tiles[2t + 1] = J, as sks_intersect_layout_tiles writes them):
 * d_ani[t][0][r][c] = ANI of (64 I + r, 64 J + c), d_ani[t][1][c][r] = ANI of
 * (64 J + c, 64 I + r); d_sizes[i] = |S_i| (int32). */
int sks_ani_tiles(sks_ctx* ctx, const int32_t* d_packed, const uint32_t* d_tiles, uint64_t n_tiles, uint32_t n,
                  const int32_t* d_sizes, int kmer_num_ones, double* d_ani);

/* ---- FASTA ingress (device) — fasta_processing.cpp:79-133 on the GPU ------------------
 * d_raw: the n_raw bytes of one FASTA file in device memory (the host only reads
 * the file).  Writes to d_stream exactly the bytes sks_fasta_stream() holds for
 * the same file (records in order, each followed by one '\n'), and, when
 * d_rec_end is non-NULL, the stream position of record i's '\n' to d_rec_end[i].
 * *stream_bytes / *n_records always receive the sizes; d_stream == NULL is a
 * size query.  Capacity too small -> SKS_E_LENGTH, nothing written.  Output is
 * at most n_raw + 1 bytes.  Returns after the sizes are known; the copy kernels
 * are queued on the context stream. */
int sks_fasta_parse_device(sks_ctx* ctx, const uint8_t* d_raw, uint64_t n_raw, uint8_t* d_stream,
                           uint64_t stream_cap, uint64_t* d_rec_end, uint64_t rec_cap,
                           uint64_t* stream_bytes, uint64_t* n_records);
/* Device time (ms) of the last sks_fasta_parse_device call (waits for it). */
int sks_ctx_last_ingress_ms(sks_ctx* ctx, float* ms);

/* ---- diagnostics / tuning ------------------------------------------------------------- */
/* Device time (ms) between the first and last launch of the last
 * sks_intersect_* call on this context (waits for it to finish). */
int sks_ctx_last_intersect_ms(sks_ctx* ctx, float* ms);
/* Fix the scan kernel's persistent grid size (0 = derive from occupancy). */
int sks_ctx_set_scan_grid(sks_ctx* ctx, int grid);
/* Kernel used by sks_intersect_all / sks_intersect_sym for u64 sketches.  All
 * give identical counts; AUTO (default) = the LDS hash join when the bucket
 * sizes allow it, else the LDS merge tiles, else one wavefront per pair.
 * (Round 3's block-postings and range-join kernels were measured slower than
 * the hash join on every workload and removed) */
enum {
  SKS_INTERSECT_AUTO = 0,
  SKS_INTERSECT_MERGE = 1,    /* 64x64 tiles of pairwise LDS merges */
  SKS_INTERSECT_JOIN = 2,     /* 64x64 tiles, LDS hash join of the two blocks */
  SKS_INTERSECT_GLOBAL = 3    /* one wavefront per pair, straight from HBM */
};
int sks_ctx_set_intersect_kernel(sks_ctx* ctx, int kind);
/* Diagnostics: on != 0 switches the context's join-layout builds and join
 * launches to instrumented kernels that check, per element, the invariants the
 * counts rest on (the layout's deduplication: every element's representative
 * holds its value; the join table: every inserted value is found naming its
 * own entry).  sks_ctx_join_check_violations waits for the context's stream
 * and returns (and resets) the violations counted on the device since the
 * last call; a correct build counts 0. */
int sks_ctx_set_join_check(sks_ctx* ctx, int on);
int sks_ctx_join_check_violations(sks_ctx* ctx, uint64_t* violations);

/* ---- synthetic genomes (bench / test utility; no reference equivalent) ----------------- */
/* Fills d_out[0..n) with ACGT bytes: base(p) = splitmix64(seed ^ (p * golden)) >> 62;
 * if mut_rate > 0 a position mutates with probability mut_rate. */
int sks_synth_bases(sks_ctx* ctx, uint8_t* d_out, uint64_t n, uint64_t seed, uint64_t mut_seed,
                    double mut_rate, uint64_t pos_offset);

#ifdef __cplusplus
}
#endif
#endif /* SKS_H */
