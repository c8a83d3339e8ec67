// Internal declarations shared by the kernels and the C-ABI layer.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>
#include <vector>

namespace sks {

// Small host<->device copies through a per-thread pinned staging buffer,
// synchronous on `s` only. A pageable hipMemcpyAsync goes through the
// runtime's shared staging path: with two contexts building on two streams, one
// context's 1 KB count read-back waited for the other stream's scan
// (--hip-trace), serialising the concurrent builds.
hipError_t pinned_d2h(void* dst, const void* src, size_t bytes, hipStream_t s);
hipError_t pinned_h2d(void* dst, const void* src, size_t bytes, hipStream_t s);
// Staging buffers parked by exited threads, ready for reuse (diagnostics).
size_t pinned_pool_size();

// The process's device block cache (api.cpp): a parked block of at least
// `bytes` on the current device, or a fresh hipMalloc; and a stream-ordered
// release (the block is handed out again only once `s` has passed the point of
// the call).  Neither waits for the device.
hipError_t cache_alloc(void** p, size_t bytes);
void cache_release_after(void* p, size_t bytes, hipStream_t s);

constexpr int kModeFrac = 0;
constexpr int kModeBottom = 1;
constexpr int kModeList = 2;  // FracMinHash test, emits window start positions

// Arguments of the fused scan kernel (scan.hip).  All per-segment arrays are
// device arrays indexed by the launch-local segment index.
struct ScanParams {
  const uint8_t* seq;
  const uint64_t* seg_begin;    // [n_seg] first byte of each segment
  const uint64_t* seg_end;      // [n_seg] end byte (exclusive)
  const uint64_t* tile_prefix;  // [n_seg + 1] tiles before each segment
  uint32_t n_seg;
  uint64_t n_tiles;
  int w;
  uint64_t mask_lo, mask_hi;
  uint64_t kconst;              // H(mask) ^ w ^ nonce
  // FracMinHash divisibility test (sks_hash.hpp DivTest)
  uint32_t low_mask, high_mask;  // x mod 2^s == 0 test (words)
  uint64_t dinv, dlim;           // odd part: x * d^-1 <= (2^64 - 1) / d
  // bottom-s pre-filter: keep fmh <= seg_thresh[seg]
  const uint64_t* seg_thresh;
  // output records: frac narrow key=C; frac wide key=lo val=hi;
  // bottom narrow key=C (fmh filled in by launch_fmh_narrow) val=C;
  // bottom wide key=fmh val=lo hi=hi
  uint64_t* out_key;
  uint64_t* out_val;
  uint64_t* out_hi;
  const uint64_t* seg_out_off;  // [n_seg] first record slot
  const uint64_t* seg_out_cap;  // [n_seg] record capacity
  unsigned long long* seg_count;    // [n_seg] records emitted (may exceed capacity)
  unsigned long long* seg_windows;  // [n_seg] valid windows hashed
  // dynamic tile queue (narrow scan): a zeroed counter, or null for static
  // per-workgroup tile ranges; `chunk` (set by launch_scan) tiles per grab
  unsigned long long* tile_queue;
  uint32_t chunk;
};

uint64_t scan_tiles_for(uint64_t seg_bytes);
hipError_t launch_scan(const ScanParams& p, int mode, int flavour, bool wide, int device,
                       hipStream_t stream, int grid_override);

// ---- post-processing (post.hip) -------------------------------------------------
// Grow-only device scratch owned by a context.  With `owner` set (the
// context's stream; every use of the buffer is ordered on it) a grown buffer's
// old block goes back to the block cache after the stream's queued work, with
// no device-wide wait; without it, growth waits for the whole device.
struct Scratch {
  void* ptr = nullptr;
  size_t bytes = 0;
  const hipStream_t* owner = nullptr;
  hipError_t reserve(size_t n);
  void release();
};

// Sort each CSR segment of keys ascending (optionally carrying values).
// keys/vals are sorted in place via the alt buffers; results land in `*_out`.
hipError_t seg_sort_keys(const uint64_t* keys_in, uint64_t* keys_out, uint64_t total,
                         const std::vector<uint64_t>& host_off, const uint64_t* d_off,
                         int end_bit, Scratch& tmp, hipStream_t s);
hipError_t seg_sort_pairs(const uint64_t* keys_in, uint64_t* keys_out, const uint64_t* vals_in,
                          uint64_t* vals_out, uint64_t total, const std::vector<uint64_t>& host_off,
                          const uint64_t* d_off, int end_bit, Scratch& tmp, hipStream_t s);

// Maximal runs of set bits of a 64-bit k-mer mask. Masked k-mers only have
// mask bits set, so gathering those bits into the low popcount(mask) bits
// (a pext) is order-preserving and injective: the post-scan sorts then run
// ceil(popcount / 8) radix passes instead of ceil(top bit / 8)
// (config 3, w=31/k=21: 42 bits instead of 62, 6 passes instead of 8).
// The gather runs as Hacker's Delight's compress / expand butterfly (7-4,
// 7-5): six masks of bits moving right by 1, 2, 4, ... 32, computed on the host,
// so a pack is at most six and/xor/shift/or steps on SGPR constants (a
// 2-bit-granular k-mer mask never moves a bit by an odd amount: five).
struct BitRuns {
  uint32_t n = 0;    // runs of set bits of the mask; 0: not packed (identity)
  uint64_t mask = 0;
  uint64_t mv[6] = {0, 0, 0, 0, 0, 0};
};
BitRuns bit_runs(uint64_t mask);
hipError_t launch_bits_expand(uint64_t* keys, uint64_t n, const BitRuns& runs, hipStream_t s);
// Bottom-s post-processing per genome in one workgroup (post.hip
// k_bottom_fused): genomes of <= bottom_fused_capacity() candidates.
// d_res[g] = sketch size; ~0: fewer than s distinct candidates under a finite
// threshold (retry); kBottomOverflow: d_cnt[g] > d_cap[g] (the scan dropped
// records; d_cap may be null when the counts are known to fit).  max_cnt: a
// bound of every d_cnt[g] (or of d_cap[g]) below the capacity.  set_sizes /
// set_starts (may be null): the sketch set's device arrays, written per genome
// (size, dst_off[g]) so a build needs no host round trip before them.
constexpr uint64_t kBottomOverflow = ~1ull;
uint32_t bottom_fused_capacity();
hipError_t launch_bottom_fused(uint64_t* rec, const uint64_t* d_src_off, const uint64_t* d_cnt,
                               const uint64_t* d_retry_ok, const uint64_t* d_dst_off,
                               uint32_t n_seg, uint64_t max_cnt, uint64_t s_param, int key_bits,
                               const BitRuns& runs, uint64_t kconst, int flavour, uint64_t* out,
                               uint64_t* d_res, hipStream_t s, const uint64_t* d_cap = nullptr,
                               uint32_t* set_sizes = nullptr, uint64_t* set_starts = nullptr);

// Compact sparse survivor regions [off[g], off[g] + cnt[g]) into dense CSR,
// packing each value's mask bits when `pack` is given.  tag_shift >= 0 ORs the
// segment index in above the key bits, (g << tag_shift) | key: the segments of a
// many-genome build then sort as ONE device-wide radix sort over
// tag_shift + seg_tag_bits(n_seg) bits (each segment keeps its CSR range, as the
// counts per tag are the segment sizes) instead of a segmented sort, whose one
// workgroup per segment left most of the chip idle (64 genomes of 25k keys:
// 0.5 ms per sort).  The tag is dropped on output (seg_unique_scatter's keep
// masks; runs_expand keeps only the packed width).
hipError_t compact_regions(const uint64_t* src, uint64_t* dst, const uint64_t* d_src_off,
                           const uint64_t* d_dst_off, uint32_t n_seg, uint64_t max_len,
                           hipStream_t s, const BitRuns* pack = nullptr, int tag_shift = -1);
int seg_tag_bits(uint32_t n_seg);  // ceil(log2(n_seg))
// out[off[g] .. off[g+1]) = g: the segment of every element (a segment tag
// that does not fit above the key rides as a sort value instead)
hipError_t launch_seg_ids(uint64_t* out, const uint64_t* d_off, uint32_t n_seg, uint64_t max_len, hipStream_t s);

// Per-segment unique of sorted keys (optionally by a (key, key2) pair):
// writes d_flag_pos (exclusive scan of "first of run" flags) and per-segment
// unique counts d_uniq[g].  Keys equal in key (and key2 when non-null) are
// one element.
// max_len: longest segment (sizes the grid; segments are grid-strided).
hipError_t seg_unique_scan(const uint64_t* keys, const uint64_t* keys2, uint64_t total,
                           uint64_t max_len, const uint64_t* d_off, uint32_t n_seg, uint32_t* d_flag,
                           uint64_t* d_pos, uint64_t* d_uniq, Scratch& tmp, hipStream_t s);
// Scatter the first `limit[g]` unique elements of each segment:
// out[dst_off[g] + rank] = vals[i] (and out2 from vals2 when non-null).
// limit == nullptr keeps every unique element; dst_off == nullptr places
// segment g at pos[off[g]] (the global unique rank, i.e. dense CSR output).
hipError_t sort_unique_u64(const uint64_t* in, uint64_t n, uint64_t* out, uint64_t* n_out,
                           Scratch& tmp, hipStream_t s);
hipError_t sort_unique_u128(const uint64_t* in, uint64_t n, uint64_t* out, uint64_t* n_out,
                            Scratch& tmp, hipStream_t s);
hipError_t seg_unique_scatter(const uint64_t* vals, const uint64_t* vals2, uint64_t total,
                              uint64_t max_len, const uint64_t* d_off, uint32_t n_seg,
                              const uint32_t* d_flag,
                              const uint64_t* d_pos, const uint64_t* d_limit,
                              const uint64_t* d_dst_off, uint64_t* out, uint64_t* out2,
                              hipStream_t s, const BitRuns* expand = nullptr, uint64_t keep = ~0ull,
                              uint64_t keep2 = ~0ull);

// Every window of a piece dense by start (windows.hip): rows[i] = {kmer_bits
// lo, hi, masked lo(, masked hi for w > 32)} of the window starting at
// first + i, valid[i / 64] bit i % 64 set when that window is all ACGT.
hipError_t launch_windows_dense(const uint8_t* seq, uint64_t n_bytes, uint64_t first, uint64_t n_win, int w,
                                uint64_t m_lo, uint64_t m_hi, uint64_t* rows, uint64_t* valid, hipStream_t s);

// ---- intersection (intersect.hip) ---------------------------------------------------
hipError_t launch_intersect_pairs(const uint64_t* data, const uint64_t* starts,
                                  const uint32_t* sizes, int elem_words, const int32_t* a,
                                  const int32_t* b, uint64_t n_pairs, int32_t* out, hipStream_t s);
hipError_t launch_intersect_all_global(const uint64_t* data, const uint64_t* starts,
                                       const uint32_t* sizes, int elem_words, uint32_t n,
                                       uint32_t row_begin, uint32_t row_end, int32_t* out,
                                       hipStream_t s);
// Tiled all-pairs (intersect.hip + join.hip): ew = 1 (u64) or 2 (128-bit)
// k-mers.  sym: upper-triangle tiles [tile_begin, tile_end) written to both
// halves of an n x n matrix; otherwise rows [row_begin, row_end) x n.  Zeroes
// `out` first.  *used_tiles = false means no tiled kernel could take the set
// (extreme value skew, or 128-bit k-mers without a join layout): use the
// global kernel.  check: the invariant-checking kernel builds.
hipError_t launch_intersect_tiled(const uint64_t* data, const uint64_t* starts, const uint32_t* sizes,
                                  uint32_t n, bool sym, uint32_t row_begin, uint32_t row_end,
                                  uint64_t tile_begin, uint64_t tile_end, int32_t* out,
                                  Scratch& work, hipStream_t s, bool* used_tiles, int algo, int ew,
                                  bool check);
// intersection kernel choice (sks_ctx_set_intersect_kernel)
constexpr int kIntersectAuto = 0;    // join when the bucket sizes allow, else merge tiles
constexpr int kIntersectMerge = 1;   // k_tiles (pairwise LDS merges)
constexpr int kIntersectJoin = 2;    // k_join (LDS hash join), merge tiles if infeasible
constexpr int kIntersectGlobal = 3;  // one wavefront per pair from global memory
uint64_t intersect_sym_tiles(uint32_t n);
// Common value-range bucket bounds[0..B] (quantiles averaged over up to 64
// sample sketches; any non-decreasing bounds give exact counts) and
// pos[i][b] = first element of sketch i that is >= bounds[b] (pos[i][B] = size).
hipError_t launch_value_bounds(const uint64_t* data, const uint64_t* starts, const uint32_t* sizes,
                               uint32_t n, uint32_t B, uint64_t* bounds, hipStream_t s);
hipError_t launch_bucket_pos(const uint64_t* data, const uint64_t* starts, const uint32_t* sizes,
                             uint32_t n, uint32_t B, const uint64_t* bounds, uint32_t* pos,
                             hipStream_t s);

// Join layout (layout.hip builds it, join.hip's k_join reads it; format in
// join_common.hpp): per 64-sketch block, each distinct value once with the mask
// of the block's sketches holding it, in value groups x hash buckets, regions
// of groups at their raw offsets.
struct JoinLayout {
  const uint64_t* vals;    // [T * ew] entry values
  const uint64_t* masks;   // [T] sketch masks
  const uint32_t* boff;    // [nb * (B + NR)] bucket starts, then region ends (block-relative)
  const uint64_t* bstart;  // [nb + 1] raw block starts
};
uint32_t join_cap();                       // entries per join chunk (table capacity)
uint32_t join_log_b(uint32_t max_size);    // bucket count for a largest sketch of max_size
// G = 2^log_b / 8 value groups (>= 1); bounds: (G + 1) values of ew words.
// join_layout_bounds computes the group bounds of a set (the median over up
// to 64 sample sketches of their quantiles).  join_layout_build: the layout of sketches (data,
// starts, sizes)[0, count) with the caller's bounds, or (d_bounds null)
// bounds computed from these sketches; temp: join_layout_temp_bytes;
// d_stat[0] is raised to the largest block-bucket population (entries),
// d_stat[1] counts groups the build could not place (layout invalid).  Three
// launches, no host synchronisation.  `zero`: up to three word spans the build's
// second launch clears before the placement runs (the caller's status words,
// count tiles, tile counters: no memset launches of their own).
// Code objects: HIP loads each .hip translation unit's code object on a device
// at the first launch of one of its kernels (post.hip's, with the rocPRIM sorts,
// is 14 MB and takes ~30 ms), so sks_ctx_create launches one empty kernel per
// unit (load_code_objects, api.cpp) and a context's first build does not pay it.
#define SKS_TU_LIST(X) X(ani) X(ingress) X(intersect) X(join) X(layout) X(post) X(scan) X(windows)
#define SKS_DECLARE_HOOK(tu) hipError_t code_object_hook_##tu(hipStream_t s);
SKS_TU_LIST(SKS_DECLARE_HOOK)
#undef SKS_DECLARE_HOOK
#define SKS_CODE_OBJECT_HOOK(tu)                                    \
  __global__ void k_code_object_##tu() {}                           \
  hipError_t code_object_hook_##tu(hipStream_t s) {                 \
    hipLaunchKernelGGL(k_code_object_##tu, dim3(1), dim3(1), 0, s); \
    return hipGetLastError();                                       \
  }
uint32_t join_layout_groups(uint32_t log_b);
// log2 of the value groups per region a build of n_blk blocks uses (1..3)
uint32_t join_layout_region_log(uint32_t n_blk, uint32_t log_b);
uint32_t join_layout_boff_words(uint32_t log_b);  // B + NR: one block's boff row
hipError_t join_layout_bounds(const uint64_t* data, const uint64_t* starts, const uint32_t* sizes,
                              uint32_t count, uint32_t log_b, int ew, uint64_t* bounds, hipStream_t s);
size_t join_layout_temp_bytes(uint32_t count, uint32_t log_b, int ew);
struct ZeroSpans {
  uint32_t* p[3];     // 4-byte aligned, null: unused
  uint64_t words[3];
};
hipError_t join_layout_build(const uint64_t* data, const uint64_t* starts, const uint32_t* sizes,
                             uint32_t count, uint32_t log_b, int ew, const uint64_t* d_bounds, void* temp,
                             uint64_t* out_vals, uint64_t* out_masks, uint32_t* out_boff,
                             uint64_t* out_bstart, uint32_t* d_stat, bool check, hipStream_t s,
                             const ZeroSpans* zero = nullptr, uint32_t blocks_hint = 0);
// Tiles of the n x n (sym: upper-triangle range [tile_begin, tile_end), or
// with d_tiles the (I, J) list entries [tile_begin, tile_end), both halves
// written) or rows x n matrix; tile (I, J) reads row block r_blk0 + I of
// `rows` and column block c_blk0 + J of `cols` (uint32 arithmetic: 0 - blk0
// maps global block indices onto a layout whose block 0 is blk0).  packed:
// out = [tile - tile_begin][64][64].  Counts are added to `out`.
// Fused containment / ANI (sym / tile-list launches only): the last workgroup
// of each tile reads the tile's finished counts back and writes
// ani[i * n + j] = binomial_estimator(containment(count, sizes[i]), k) for both
// orientations of the tile, so the conversion (and, when `ani` is pinned host
// memory, its PCIe transfer) runs under the join instead of after it.
struct JoinAni {
  double* ani;            // n x n row-major: HBM, or host memory mapped for the device
  const int32_t* sizes;   // [n] |S_i| by global genome index
  int kmer_num_ones;      // k of binomial_estimator
  uint32_t* tile_done;    // [tile_end - tile_begin] workgroups finished per tile, zeroed
  const double* root = nullptr;  // optional: root[i] = ANI of i shared elements for a set of root_size
  uint32_t root_size = 0;
};
hipError_t join_launch(const JoinLayout& rows, uint32_t r_blk0, const JoinLayout& cols, uint32_t c_blk0,
                       uint32_t n, uint32_t log_b, int ew, bool sym, uint32_t row_begin, uint32_t row_end,
                       uint64_t tile_begin, uint64_t tile_end, const uint32_t* d_tiles, bool packed,
                       int32_t* out, bool check, hipStream_t s, const JoinAni* ani = nullptr,
                       int layout_rg = -1);
// (layout_rg >= 0: rows and cols are ONE layout built with that region log, so a
// tile list needs no cross-region windows when its regions hold 64 buckets)
// SKS check builds: invariant violations counted since the last call (and reset)
unsigned long long join_check_take();
unsigned long long layout_check_take();

// ---- containment / ANI (ani.hip) ------------------------------------------------------------
// Dense: ani[i * n + j] from the n x n count matrix (|S_i| on its diagonal).
hipError_t launch_ani_matrix(const int32_t* counts, uint32_t n, int kmer_num_ones, double* cont, double* ani,
                             hipStream_t s);
// Packed symmetric tiles (I, J) = tiles[2t], tiles[2t + 1]: out [t][2][64][64]
// (both orientations of each pair); sizes[i] = |S_i|.
hipError_t launch_ani_tiles(const int32_t* packed, const uint32_t* tiles, uint64_t n_tiles, uint32_t n,
                            const int32_t* sizes, int kmer_num_ones, double* out, hipStream_t s);

// ---- device FASTA ingress (ingress.hip) -------------------------------------------------
// strings_from_fasta on the device: writes the host parser's record stream
// (fasta.cpp) to `out` and each record's '\n' position to rec_end (optional).
// out == nullptr: size query only.  *too_small: a capacity was short (nothing
// written).  Synchronises `s` twice (sizes are read back).
hipError_t fasta_parse_device(const uint8_t* raw, uint64_t n, uint8_t* out, uint64_t out_cap,
                              uint64_t* rec_end, uint64_t rec_cap, Scratch& work, Scratch& tmp,
                              hipStream_t s, uint64_t* out_bytes, uint64_t* n_records,
                              bool* too_small);

// ---- misc kernels (post.hip) -------------------------------------------------------------
hipError_t launch_synth(uint8_t* out, uint64_t n, uint64_t seed, uint64_t mut_seed,
                        uint64_t mut_thresh, uint64_t pos_offset, hipStream_t s);
hipError_t launch_export(const uint64_t* data, const uint64_t* starts, const uint32_t* sizes,
                         uint32_t n, int elem_words, uint64_t* dst, uint64_t stride,
                         uint32_t* dst_sizes, hipStream_t s);
// nucleotide_string_to_kmers' `kmer` for each selected window start pos[i]
// (kmer_sliding.cpp:112-186): out[4i..4i+3] = kmer_bits (lo, hi), masked_bits
// (lo, hi).  kmer_bits is the chosen strand's window register: R (2w bits), or
// F holding up to 64 bases of the run ending at the window (the reference
// never clears F's older bases).  seg_begin: [n_seg] sorted segment starts.
hipError_t launch_materialise(const uint8_t* seq, const uint64_t* seg_begin, uint32_t n_seg,
                              const uint64_t* pos, uint64_t n, int w, uint64_t mask_lo,
                              uint64_t mask_hi, uint64_t* out, hipStream_t s);
hipError_t launch_iota(uint64_t* out, uint64_t n, hipStream_t s);
// Bottom-s from C-sorted distinct candidates (uk, segment g at [uoff[g], uoff[g+1])):
// writes the min(limit[g], n_g) k-mers with the smallest (fmh, k-mer), in k-mer
// order, to out + dst[g].  Needs every n_g with limit[g] > 0 to be at most
// bottom_select_capacity().
uint32_t bottom_select_capacity();
hipError_t launch_bottom_select(const uint64_t* uk, const uint64_t* d_uoff, const uint64_t* d_dst,
                                const uint64_t* d_lim, uint32_t n_seg, uint64_t kconst,
                                int flavour, uint64_t* out, hipStream_t s);
// keys[i] = frac_min_hash of the narrow canonical k-mer keys[i] (in place).
hipError_t launch_fmh_narrow(uint64_t* keys, uint64_t n, uint64_t kconst, int flavour, hipStream_t s);
hipError_t launch_gather(const uint64_t* src, const uint64_t* idx, uint64_t n, uint64_t* out,
                         hipStream_t s);
hipError_t launch_interleave(const uint64_t* lo, const uint64_t* hi, uint64_t n, uint64_t* out,
                             hipStream_t s);

}  // namespace sks
