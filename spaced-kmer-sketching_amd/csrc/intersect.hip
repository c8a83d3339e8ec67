// Kernel 2 — pairwise sketch intersection counts.
//
// The reference counts |A ∩ B| by iterating the smaller kmer_set and probing
// the larger hash map (kmer_set.cpp:23-41), one pair per cilk_for iteration
// (kmer_set.cpp:167-184).  Sketches here are sorted unique arrays, so a pair
// is a sorted-merge count — the same integer the reference computes.
//   * k_tiles: the all-pairs path for u64 sketches (bucketed, LDS-tiled; see
//     the comment above it).
//   * k_pairs / k_all: one 64-lane wavefront per pair straight from global
//     memory — pair lists, 128-bit k-mers, and the fallback for pathological
//     value skew.  The smaller sketch is split evenly over the lanes, each lane
//     lower_bounds its first element in the larger one and merges forward.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <cstdint>
#include <vector>

#include <rocprim/rocprim.hpp>

#include "join_common.hpp"
#include "sks_internal.hpp"

namespace sks {

namespace {

using jc::fp_slot;
using jc::fp_tag;
using jc::join_chain;
using jc::kFFree;
using jc::kFLog;
using jc::kFSlots;
using jc::sym_tile;

constexpr int kB = 256;
constexpr int kWavesPerBlock = kB / 64;
// workgroups per launch at most (HIP caps a grid at 2^32 - 1 work-items);
// larger grids are cut into slices
constexpr uint64_t kMaxGrid = 1ull << 22;

struct U128 {
  uint64_t lo, hi;
};

template <int EW>
__device__ __forceinline__ U128 load_elem(const uint64_t* p, uint64_t i) {
  if constexpr (EW == 1) return U128{p[i], 0};
  else return U128{p[2 * i], p[2 * i + 1]};
}

__device__ __forceinline__ bool lt(const U128& a, const U128& b) {
  return a.hi < b.hi || (a.hi == b.hi && a.lo < b.lo);
}
__device__ __forceinline__ bool eq(const U128& a, const U128& b) { return a.hi == b.hi && a.lo == b.lo; }

template <int EW>
__device__ __forceinline__ int32_t wave_pair_count(const uint64_t* __restrict__ data,
                                                   uint64_t sa, uint32_t na, uint64_t sb,
                                                   uint32_t nb) {
  const int lane = threadIdx.x & 63;
  // iterate the smaller sketch
  if (na > nb) {
    uint64_t ts = sa; sa = sb; sb = ts;
    uint32_t tn = na; na = nb; nb = tn;
  }
  const uint64_t* A = data + sa * EW;
  const uint64_t* B = data + sb * EW;
  const uint32_t i0 = (uint32_t)(((uint64_t)na * lane) >> 6);
  const uint32_t i1 = (uint32_t)(((uint64_t)na * (lane + 1)) >> 6);
  int32_t cnt = 0;
  if (i0 < i1) {
    U128 x = load_elem<EW>(A, i0);
    // lower_bound of x in B
    uint32_t lo = 0, hi = nb;
    while (lo < hi) {
      uint32_t mid = (lo + hi) >> 1;
      if (lt(load_elem<EW>(B, mid), x)) lo = mid + 1; else hi = mid;
    }
    uint32_t j = lo;
    uint32_t i = i0;
    U128 y = j < nb ? load_elem<EW>(B, j) : U128{~0ull, ~0ull};
    while (i < i1 && j < nb) {
      if (lt(y, x)) {
        ++j;
        if (j < nb) y = load_elem<EW>(B, j);
      } else {
        if (eq(x, y)) {
          ++cnt;
          ++j;
          if (j < nb) y = load_elem<EW>(B, j);
        }
        ++i;
        if (i < i1) x = load_elem<EW>(A, i);
      }
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o, 64);
  return cnt;
}

template <int EW>
__global__ __launch_bounds__(kB) void k_pairs(const uint64_t* __restrict__ data,
                                              const uint64_t* __restrict__ starts,
                                              const uint32_t* __restrict__ sizes,
                                              const int32_t* __restrict__ a,
                                              const int32_t* __restrict__ b, uint64_t p0,
                                              uint64_t n_pairs, int32_t* __restrict__ out) {
  const uint64_t p = p0 + (uint64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
  if (p >= n_pairs) return;
  const int32_t ia = a[p], ib = b[p];
  int32_t c = wave_pair_count<EW>(data, starts[ia], sizes[ia], starts[ib], sizes[ib]);
  if ((threadIdx.x & 63) == 0) out[p] = c;
}

template <int EW>
__global__ __launch_bounds__(kB) void k_all(const uint64_t* __restrict__ data,
                                            const uint64_t* __restrict__ starts,
                                            const uint32_t* __restrict__ sizes, uint32_t n,
                                            uint32_t row_begin, uint64_t p0, uint64_t n_pairs,
                                            int32_t* __restrict__ out) {
  const uint64_t p = p0 + (uint64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
  if (p >= n_pairs) return;
  const uint32_t i = row_begin + (uint32_t)(p / n), j = (uint32_t)(p % n);
  int32_t c = wave_pair_count<EW>(data, starts[i], sizes[i], starts[j], sizes[j]);
  if ((threadIdx.x & 63) == 0) out[p] = c;
}

// ---- tiled all-pairs kernel (u64 sketches) ---------------------------------------------
//
// The value range is cut into B buckets by common boundaries (quantiles of the
// largest sketch), so |S_i ∩ S_j| = Σ_b |S_i[b] ∩ S_j[b]|.  A workgroup owns a
// 64 x 64 tile of (row, column) sketches and a group of buckets; per bucket it
// stages the 128 bucket parts in LDS interleaved as lds[pos][slot] (slot =
// sketch within the tile), then every lane merges one pair.  Lane l of a wave
// always handles row l and column (l + k) mod 64, so the 32 lanes of each
// ds_read_b64 group touch 32 distinct slots -> bank-conflict-free reads at any
// merge positions.  Counts accumulate in registers across the bucket group and
// leave with one atomicAdd per pair.
constexpr int kTile = 64;
constexpr int kSlots = 2 * kTile;
constexpr int kMaxPart = 150;   // LDS: 150 * 128 * 8 = 153,600 B (one workgroup per CU)
constexpr int kGoodPart = 60;   // <= 60 keeps LDS <= 61.4 KB: two workgroups per CU
constexpr int kDiagPerWave = kTile / kWavesPerBlock;  // 16
constexpr int kRowBytes = kSlots * 8;                  // one LDS position across all slots

struct TileArgs {
  const uint64_t* data;
  const uint64_t* starts;
  const uint32_t* sizes;
  const uint32_t* pos;  // [n][B + 1] bucket boundaries (element index within sketch)
  uint32_t n, B, P, buckets_per_group, n_groups;
  uint32_t row_begin, row_end;  // rows mode: rows [row_begin, row_end) x all n columns
  uint32_t n_col_blocks, n_row_blocks;
  int sym;                      // 1: upper-triangle tiles, write both (i, j) and (j, i)
  uint64_t tile_begin;
  int32_t* out;
  uint64_t ld;
};

// Common bucket bounds: bounds[b] = mean over K sample sketches (spread over the
// collection) of each one's b/B quantile.  A single sketch's quantiles are
// noisy — its wide gaps become buckets that hold several times the mean part
// of every unrelated sketch — and averaging K of them shrinks that noise by
// sqrt(K).  Any non-decreasing bounds give exact counts; these only have to
// balance the parts.  Each quantile sequence is non-decreasing and rounded
// addition / division are monotonic, so the bounds are too.
__global__ void k_bounds(const uint64_t* __restrict__ data, const uint64_t* __restrict__ starts,
                         const uint32_t* __restrict__ sizes, uint32_t n, uint32_t K, uint32_t B,
                         uint64_t* __restrict__ bounds) {
  uint32_t b = blockIdx.x * kB + threadIdx.x;
  if (b > B) return;
  if (b == 0) { bounds[0] = 0; return; }
  if (b == B) { bounds[B] = ~0ull; return; }
  double acc = 0.0;
  uint32_t used = 0;
  for (uint32_t k = 0; k < K; ++k) {
    const uint32_t i = (uint32_t)((uint64_t)k * n / K);
    const uint32_t sz = sizes[i];
    if (!sz) continue;
    acc += (double)data[starts[i] + (uint64_t)b * sz / B];
    ++used;
  }
  const double m = used ? acc / (double)used : 0.0;
  bounds[b] = m >= 18446744073709549568.0 ? ~0ull : (uint64_t)m;
}

__global__ void k_bucket_pos(const uint64_t* __restrict__ data, const uint64_t* __restrict__ starts,
                             const uint32_t* __restrict__ sizes, uint32_t n, uint32_t B,
                             const uint64_t* __restrict__ bounds, uint32_t* __restrict__ pos) {
  uint64_t idx = (uint64_t)blockIdx.x * kB + threadIdx.x;
  uint32_t i = (uint32_t)(idx / (B + 1)), b = (uint32_t)(idx % (B + 1));
  if (i >= n) return;
  uint32_t size = sizes[i];
  uint32_t r;
  if (b == 0) r = 0;
  else if (b == B) r = size;
  else {
    const uint64_t* S = data + starts[i];
    const uint64_t v = bounds[b];
    uint32_t lo = 0, hi = size;
    while (lo < hi) {
      uint32_t mid = (lo + hi) >> 1;
      if (S[mid] < v) lo = mid + 1; else hi = mid;
    }
    r = lo;
  }
  pos[(uint64_t)i * (B + 1) + b] = r;
}

// Largest part over all (sketch, bucket), and largest bucket population of one
// 64-sketch block (the join's hash-table load).  One thread per (block, bucket).
__global__ void k_part_stats(const uint32_t* __restrict__ pos, uint32_t n, uint32_t B, uint32_t n_cb,
                             uint32_t* __restrict__ stats) {
  const uint64_t idx = (uint64_t)blockIdx.x * kB + threadIdx.x;
  if (idx >= (uint64_t)n_cb * B) return;
  const uint32_t cb = (uint32_t)(idx / B), b = (uint32_t)(idx % B);
  uint32_t mx = 0, sum = 0;
  for (uint32_t i = cb * 64; i < min(n, cb * 64 + 64); ++i) {
    const uint32_t* q = pos + (uint64_t)i * (B + 1) + b;
    const uint32_t part = q[1] - q[0];
    mx = max(mx, part);
    sum += part;
  }
  atomicMax(&stats[0], mx);
  atomicMax(&stats[1], sum);
}

__global__ __launch_bounds__(kB) void k_tiles(TileArgs a) {
  // lds[pos * kSlots + slot], pos < a.P (dynamic: sized to the largest part)
  // (the only LDS object, so its base is LDS address 0 and element offsets
  // need no base add); part lengths follow the P x 128 element block
  extern __shared__ uint64_t lds[];
  uint32_t* s_len = reinterpret_cast<uint32_t*>(lds + (size_t)a.P * kSlots);
  const uint64_t t = a.tile_begin + blockIdx.x / a.n_groups;
  const uint32_t grp = blockIdx.x % a.n_groups;
  uint32_t I, J;
  if (a.sym) {
    sym_tile(t, a.n_col_blocks, I, J);
  } else {
    I = (uint32_t)(t / a.n_col_blocks);
    J = (uint32_t)(t % a.n_col_blocks);
  }
  const uint32_t row0 = (a.sym ? 0 : a.row_begin) + I * kTile;
  const uint32_t row_lim = a.sym ? a.n : a.row_end;
  const uint32_t col0 = J * kTile;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;

  // loader role: slot = sketch within the tile, par = which half of the positions
  const uint32_t slot = tid & (kSlots - 1), par = tid >> 7;
  const uint32_t sid = slot < kTile ? row0 + slot : col0 + (slot - kTile);
  const bool sv = slot < kTile ? (sid < row_lim) : (sid < a.n);
  const uint64_t sstart = sv ? a.starts[sid] : 0;
  const uint32_t* spos = a.pos + (uint64_t)(sv ? sid : 0) * (a.B + 1);

  uint32_t cnt[kDiagPerWave];
#pragma unroll
  for (int q = 0; q < kDiagPerWave; ++q) cnt[q] = 0;

  const uint32_t b0 = grp * a.buckets_per_group;
  const uint32_t b1 = min(a.B, b0 + a.buckets_per_group);
  for (uint32_t b = b0; b < b1; ++b) {
    uint32_t beg = 0, len = 0;
    if (sv) {
      beg = spos[b];
      len = spos[b + 1] - beg;
    }
    if (par == 0) s_len[slot] = len;
    // 8 independent loads in flight per thread
    const uint64_t* src = a.data + sstart + beg;
    for (uint32_t j0 = par; j0 < len; j0 += 16) {
      uint64_t v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const uint32_t j = j0 + 2 * u;
        v[u] = j < len ? src[j] : 0;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const uint32_t j = j0 + 2 * u;
        if (j < len) lds[j * kSlots + slot] = v[u];
      }
    }
    __syncthreads();
    // Lane = row `lane`; 16 columns (lane + 16*wave + q) mod 64.  The 16
    // merges advance together with no per-step branches: indices are LDS byte
    // offsets clamped to the last element, every step reads both sides, and
    // i += (x <= y), j += (y <= x), m += (x == y).  Once one side is exhausted
    // its clamped element was already consumed, so it can match again only
    // when BOTH sides sit on equal last elements; each such step advances both
    // offsets, and those extra counts are subtracted after the bucket.
    const uint32_t na = s_len[lane];
    // raw LDS byte addresses: dynamic LDS begins after the static allocation
    const uint32_t lds0 = __builtin_amdgcn_groupstaticsize();
    const uint32_t a_base = lds0 + lane * 8u;
    const uint32_t a_last = a_base + (na ? na - 1 : 0) * kRowBytes;
    uint32_t io[kDiagPerWave], jo[kDiagPerWave], b_last[kDiagPerWave];
#pragma unroll
    for (int q = 0; q < kDiagPerWave; ++q) {
      const uint32_t c = (lane + wave * kDiagPerWave + q) & (kTile - 1);
      const uint32_t nb = s_len[kTile + c];
      const uint32_t b_base = lds0 + c * 8u;  // column slots start kTile * 8 bytes in
      io[q] = a_base;
      jo[q] = b_base;
      b_last[q] = b_base + (nb ? nb - 1 : 0) * kRowBytes;
    }
    typedef __attribute__((address_space(3))) const uint64_t lds_u64;
    // Matches are not counted per step: every step advances i, j or both, so
    // over T steps  matches = (i advances + j advances) - T.
    uint32_t steps = 0;
    for (;;) {
      uint32_t live = 0;
#pragma unroll
      for (int q = 0; q < kDiagPerWave; ++q) live |= (io[q] <= a_last) & (jo[q] <= b_last[q]);
      if (!__any(live)) break;
#pragma unroll 1
      for (int rep = 0; rep < 4; ++rep) {
        uint64_t xs[kDiagPerWave], ys[kDiagPerWave];
#pragma unroll
        for (int q = 0; q < kDiagPerWave; ++q) {
          xs[q] = *reinterpret_cast<lds_u64*>((size_t)min(io[q], a_last));
          ys[q] = *reinterpret_cast<lds_u64*>((size_t)(min(jo[q], b_last[q]) + kTile * 8));
        }
#pragma unroll
        for (int q = 0; q < kDiagPerWave; ++q) {
          io[q] += xs[q] > ys[q] ? 0u : (uint32_t)kRowBytes;
          jo[q] += xs[q] < ys[q] ? 0u : (uint32_t)kRowBytes;
        }
      }
      steps += 4;
    }
#pragma unroll
    for (int q = 0; q < kDiagPerWave; ++q) {
      const uint32_t c = (lane + wave * kDiagPerWave + q) & (kTile - 1);
      const uint32_t nb = s_len[kTile + c];
      const int32_t ia = (int32_t)((io[q] - a_base) / kRowBytes);
      const int32_t jb = (int32_t)((jo[q] - lds0 - c * 8u) / kRowBytes);
      // steps taken with both sides past their ends (equal last elements)
      const int32_t spurious = max(0, min(ia - (int32_t)na, jb - (int32_t)nb));
      if (na && nb) cnt[q] += (uint32_t)(ia + jb - (int32_t)steps - spurious);
    }
    __syncthreads();
  }
  const uint32_t r = row0 + lane;
  if (r >= row_lim) return;
#pragma unroll
  for (int q = 0; q < kDiagPerWave; ++q) {
    const uint32_t c = col0 + ((lane + wave * kDiagPerWave + q) & (kTile - 1));
    if (c >= a.n || cnt[q] == 0) continue;
    const uint64_t orow = a.sym ? r : (r - a.row_begin);
    atomicAdd(&a.out[orow * a.ld + c], (int32_t)cnt[q]);
    if (a.sym && I != J) atomicAdd(&a.out[(uint64_t)c * a.ld + r], (int32_t)cnt[q]);
  }
}


// ---- join all-pairs kernel (u64 sketches) ----------------------------------------------
//
// Same 64 x 64 tiles as k_tiles, but a workgroup joins the two blocks instead
// of merging 4096 pairs: the column block's elements go into an LDS hash table
// value -> 64-bit mask of the columns holding it, every row element probes it
// once, and a hit with mask m adds 1 to cnt[row][c] for each set bit c
// (ds_add into an LDS 64 x 65 matrix).  Work per tile is
// (row + column elements) + Σ_pairs |S_i ∩ S_j| instead of
// Σ_pairs (|S_i| + |S_j|): 64x fewer steps for unrelated sketches and still
// fewer when every pair is identical.
//
// Layout (built per call by k_hb_count / scan / k_hb_scatter): elements are
// hash-bucketed — masked k-mers sit on a lattice (the mask's don't-care bits
// are 0), so value-range buckets are lumpy, while a hash of the value gives
// Poisson parts — and stored block-major: for each 64-sketch block, bucket by
// bucket, sketch by sketch, with the sketch's slot in the block in a u8 id
// array.  A run of buckets of one block is one contiguous range, so a
// workgroup streams the column block in coalesced chunks of whole buckets
// that fit the table (<= kJCap elements; a larger bucket is cut into
// sub-chunks) and the row block's same buckets with them.  off[(blk * B + b) * 64 + slot] = start of (blk, b, slot).
#ifndef SKS_JOIN_DIAG  // diagnostics only (wrong counts): 1 no probes / hit adds,
#define SKS_JOIN_DIAG 0  // 2 no count flush, 4 probes without hit adds
#endif
// 512 threads (8 waves): with the table's LDS allowing 3 workgroups per CU,
// 24 waves per CU instead of 12 hide the LDS round trips of the insert and
// probe chains (config 4: k_join 0.86 -> 0.69 ms; 1024 threads 0.72)
#ifndef SKS_JOIN_THREADS
#define SKS_JOIN_THREADS 512
#endif
constexpr int kJB = SKS_JOIN_THREADS;       // threads per k_join workgroup
constexpr int kJCap = 1024;                  // column elements per chunk
constexpr int kJMade = kJCap / kJB;         // column elements per thread per chunk
constexpr int kJWin = 256;                  // bucket offsets staged per window
constexpr uint32_t kJMaxLogB = 14;          // B <= 16384 (LDS histogram of k_hb_count)
// Hit counts as bit-sliced counters: plane b of
// tile row r is the 64-bit word of bit b of the row's 64 column counts, and a
// hit with column mask m is a carry chain of atomic XORs (m &= old after each
// plane: a plane bit that was set carries).  A mask of k columns then costs
// about log2(k) + 2 LDS atomics instead of k (a 32-bit count matrix with one
// ds_add per set bit, rounds 1-2: 0.653 -> 0.604 ms on config 4).
constexpr int kPlanes = 32;
constexpr uint32_t kNoSlot = 0xFFFFFFFFu;

struct JoinArgs {
  JoinLayout r, c;  // row blocks (tile row I = block r_blk0 + I) and column blocks
  uint32_t r_blk0, c_blk0;  // (tile column J = block c_blk0 + J; uint32 arithmetic, -blk0 works)
  uint32_t B, n, n_col_blocks, n_groups, buckets_per_group;
  int sym;
  uint32_t row_begin, row_end;
  uint64_t tile_begin;
  const uint32_t* tiles;  // optional (I, J) list (global block indices), sym semantics
  int32_t* out;
  uint64_t ld;
  uint32_t cap;  // column elements per chunk (<= kJCap): table load <= cap / kFSlots
  int packed;    // out = [tile - tile_begin][64][64]
};

// Elements of one chunk held in registers: column elements k = cs + tid + kJB * u
// (u < kJMade: a chunk holds <= kJCap) and the first kJRowPf * kJB row elements;
// the rest of a (rare) larger row range is read in the probe loop.
constexpr int kJRowPf = 1536 / kJB;
// s_waitcnt immediate for gfx9 "vmcnt(0)" with expcnt / lgkmcnt left at their
// maxima: vmcnt = imm[3:0] | imm[15:14] << 4, expcnt = imm[6:4], lgkmcnt = imm[11:8]
constexpr int kWaitVmcnt0 = 0x0F70;
struct JoinChunk {
  uint64_t cv[kJMade];
  uint32_t cid[kJMade];
  uint64_t rv[kJRowPf];
  uint32_t rid[kJRowPf];
};

__device__ __forceinline__ void join_fetch(const uint64_t* __restrict__ cdata,
                                           const uint8_t* __restrict__ cids,
                                           const uint64_t* __restrict__ rdata,
                                           const uint8_t* __restrict__ rids, uint32_t cs,
                                           uint32_t ce, uint32_t rs, uint32_t re, int tid,
                                           JoinChunk& c) {
#pragma unroll
  for (int u = 0; u < kJMade; ++u) {
    const uint32_t k = cs + tid + kJB * u;
    c.cv[u] = k < ce ? cdata[k] : 0;
    c.cid[u] = k < ce ? cids[k] : 0xFFu;
  }
#pragma unroll
  for (int u = 0; u < kJRowPf; ++u) {
    const uint32_t k = rs + tid + kJB * u;
    c.rv[u] = k < re ? rdata[k] : 0;
    c.rid[u] = k < re ? rids[k] : 0xFFu;
  }
}

#ifdef SKS_JOIN_STAMPS  // diagnostic build: cycles per k_join phase, wave 0 of each workgroup
__device__ unsigned long long g_join_stamps[8];
#define JSTAMP(i)                                              \
  do {                                                         \
    const uint64_t t_ = __builtin_amdgcn_s_memtime();          \
    st_acc[i] += t_ - st_last;                                 \
    st_last = t_;                                              \
  } while (0)
#else
#define JSTAMP(i) do {} while (0)
#endif

// ---- k_join: the join kernel ----------------------------------------------------------------
//
// Each chunk's column elements are first staged as entries {value, column
// bit} in LDS (plain stores); the hash table then holds 32-bit slots
// (fingerprint << 10 | entry index).  An insert is one 32-bit compare-swap
// (the 64-bit one runs at about half its rate) and, for a value already present,
// a check of the entry it names plus an OR of the column bit into that entry;
// a probe reads 32-bit slots and, on a fingerprint match, the 16-byte entry.
// Values need no reserved "empty" key (the empty marker lives in the slot), and
// the entries need no reset: the next chunk's staging overwrites them.
static_assert(kJCap == 1024, "entry index: 10 bits; join_chain reads entry x & 1023 of any slot word");

__global__ __launch_bounds__(kJB) void k_join(JoinArgs a) {
#ifdef SKS_JOIN_STAMPS
  uint64_t st_acc[6] = {0, 0, 0, 0, 0, 0};
  uint64_t st_last = __builtin_amdgcn_s_memtime();
#endif
  __shared__ uint32_t s_slot[kFSlots];
  __shared__ ulonglong2 s_ent[kJCap];  // {value, mask of the columns holding it}
  __shared__ unsigned long long s_pl[kPlanes * kTile];  // plane b of row r at [b * 64 + r]
  __shared__ uint32_t s_roff[kJWin + 1], s_coff[kJWin + 1];
  __shared__ uint16_t s_next[kJWin];

  const uint64_t t = a.tile_begin + blockIdx.x / a.n_groups;
  const uint32_t grp = blockIdx.x % a.n_groups;
  uint32_t I, J;
  if (a.tiles) {
    I = a.tiles[2 * t];
    J = a.tiles[2 * t + 1];
  } else if (a.sym) {
    sym_tile(t, a.n_col_blocks, I, J);
  } else {
    I = (uint32_t)(t / a.n_col_blocks);
    J = (uint32_t)(t % a.n_col_blocks);
  }
  const bool rows_mode = !a.sym && !a.tiles;
  const uint32_t row0 = (rows_mode ? a.row_begin : 0) + I * kTile;
  const uint32_t row_lim = rows_mode ? a.row_end : a.n;
  const uint32_t col0 = J * kTile;
  const int tid = threadIdx.x, lane = tid & 63;
  const uint32_t rblk = a.r_blk0 + I, cblk = a.c_blk0 + J;
  const uint64_t rb = a.r.bstart[rblk], cb = a.c.bstart[cblk];
  const uint64_t* rdata = a.r.data + rb;
  const uint8_t* rids = a.r.ids + rb;
  const uint64_t* cdata = a.c.data + cb;
  const uint8_t* cids = a.c.ids + cb;
  const uint32_t* roff = a.r.boff + (uint64_t)rblk * (a.B + 1);
  const uint32_t* coff = a.c.boff + (uint64_t)cblk * (a.B + 1);
  const uint32_t r_valid = min<uint32_t>(kTile, row_lim - row0);

  for (int i = tid; i < kFSlots / 4; i += kJB)
    reinterpret_cast<uint4*>(s_slot)[i] = make_uint4(kFFree, kFFree, kFFree, kFFree);
  // a tile on the diagonal: row block = column block, in the same layout (rows
  // taken from a separate layout start off a block boundary, so never match)
  const bool self_tile = row0 == col0;
  for (int i = tid; i < kPlanes * kTile / 2; i += kJB) reinterpret_cast<uint4*>(s_pl)[i] = make_uint4(0, 0, 0, 0);
  __shared__ uint32_t s_top;  // planes used (the highest carry chain)
  // A tile on the diagonal (row block = column block) finds every row element in
  // its own column: those self-hits are counted per row with plain adds, outside
  // the carry chains (unrelated sketches would otherwise run a chain per element)
  __shared__ uint32_t s_self[kTile];
  if (tid < kTile) s_self[tid] = 0;
  if (tid == 0) s_top = 0;
  uint32_t top = 0;
  auto add_hits = [&](uint32_t r, unsigned long long m) {
    if (self_tile && ((m >> r) & 1ull)) {  // (a sub-chunk of a large bucket may not hold it)
      atomicAdd(&s_self[r], 1u);
      m &= ~(1ull << r);
    }
    unsigned long long* p = &s_pl[r];
    uint32_t b = 0;
    for (; m && b < kPlanes; ++b) m &= atomicXor(p + b * kTile, m);
    top = max(top, b);
  };
  // columns holding v (0 if none)
  auto lookup = [&](uint64_t v, uint32_t h, uint32_t x) -> unsigned long long {
    if (x != kFFree) x = join_chain(x, h, fp_tag(v), v, 0u, s_slot, s_ent, false);
    return x == kFFree ? 0ull : s_ent[x & 1023u].y;
  };

  uint32_t diag_acc = 0;  // SKS_JOIN_DIAG & 4: hits counted, not added
  uint32_t made[kJMade];  // slots this thread created in the current chunk
#pragma unroll
  for (int u = 0; u < kJMade; ++u) made[u] = kNoSlot;

  const uint32_t b0 = grp * a.buckets_per_group;
  const uint32_t b1 = min(a.B, b0 + a.buckets_per_group);
  for (uint32_t wb = b0; wb < b1; wb += kJWin) {
    const uint32_t we = min(b1, wb + kJWin);
    __syncthreads();  // previous window fully consumed
    for (uint32_t i = tid; i <= we - wb; i += kJB) {
      s_roff[i] = roff[wb + i];
      s_coff[i] = coff[wb + i];
    }
    __syncthreads();
    for (uint32_t i = tid; i < we - wb; i += kJB) {
      const uint32_t cs = s_coff[i];
      uint32_t lo = i + 1, hi = we - wb;
      while (lo < hi) {
        const uint32_t mid = (lo + hi + 1) >> 1;
        if (s_coff[mid] - cs <= a.cap) lo = mid; else hi = mid - 1;
      }
      s_next[i] = (uint16_t)lo;
    }
    __syncthreads();
    JSTAMP(0);
    // chunks and oversized-bucket sub-chunks exactly as in k_join
    auto chunk_end = [&](uint32_t bs) { return wb + (uint32_t)s_next[bs - wb]; };
    uint32_t bs = wb, be = chunk_end(wb);
    uint32_t cs = s_coff[0], ce = min(s_coff[be - wb], cs + a.cap);
    // a chunk of whole buckets of a diagonal tile needs no row elements: its
    // rows are its columns (step 2 below)
    auto rows_end = [&](uint32_t bs_, uint32_t be_, uint32_t cs_, uint32_t ce_) {
      const bool whole = cs_ == s_coff[bs_ - wb] && ce_ == s_coff[be_ - wb];
      return self_tile && whole ? s_roff[bs_ - wb] : s_roff[be_ - wb];
    };
    JoinChunk cur;
    join_fetch(cdata, cids, rdata, rids, cs, ce, s_roff[0], rows_end(bs, be, cs, ce), tid, cur);
    while (bs < we) {
      const uint32_t rs = s_roff[bs - wb], re = s_roff[be - wb];
      __builtin_amdgcn_s_waitcnt(kWaitVmcnt0);  // this chunk's elements have landed
      uint32_t nbs, nbe, ncs, nce;
      if (ce < s_coff[be - wb]) {
        nbs = bs;
        nbe = be;
        ncs = ce;
      } else {
        nbs = be;
        nbe = nbs < we ? chunk_end(nbs) : nbs;
        ncs = s_coff[nbs - wb];
      }
      nce = min(s_coff[nbe - wb], ncs + a.cap);
      JoinChunk nxt;
      if (nbs < we)
        join_fetch(cdata, cids, rdata, rids, ncs, nce, s_roff[nbs - wb], rows_end(nbs, nbe, ncs, nce), tid,
                   nxt);

      // 0) free the previous chunk's slots (its probes are done: barrier below
      //    the probe loop) and stage this chunk's entries
#pragma unroll
      for (int u = 0; u < kJMade; ++u) {
        if (made[u] != kNoSlot) s_slot[made[u]] = kFFree;
        made[u] = kNoSlot;
        const uint32_t e = tid + kJB * u;
        if (cs + e < ce) s_ent[e] = make_ulonglong2(cur.cv[u], 1ull << cur.cid[u]);
      }
      __syncthreads();
      // 1) insert: one 32-bit compare-swap per element; a value already
      //    present adds its column bit to the entry the slot names
      uint32_t hs[kJMade], prev[kJMade], tags[kJMade], ent[kJMade];
#pragma unroll
      for (int u = 0; u < kJMade; ++u) {
        hs[u] = kNoSlot;
        ent[u] = 0;
        const uint32_t e = tid + kJB * u;
        if (cs + e < ce) {
          hs[u] = fp_slot(cur.cv[u]);
          tags[u] = fp_tag(cur.cv[u]);
          prev[u] = atomicCAS(&s_slot[hs[u]], kFFree, (tags[u] << 10) | e);
        }
      }
#pragma unroll
      for (int u = 0; u < kJMade; ++u) {
        if (hs[u] == kNoSlot) continue;
        const uint64_t v = cur.cv[u];
        const uint32_t e = tid + kJB * u;
        uint32_t h = hs[u], x = prev[u];
        if (x != kFFree) x = join_chain(x, h, tags[u], v, (tags[u] << 10) | e, s_slot, s_ent, true);
        if (x == kFFree) {  // created slot h naming entry e
          made[u] = h;
          ent[u] = e;
        } else {  // v is present: add the column bit to its entry
          ent[u] = x & 1023u;
          atomicOr(&s_ent[ent[u]].y, 1ull << cur.cid[u]);
        }
      }
      __syncthreads();
      JSTAMP(1);
      // 2) probe with the row elements: first slots read together. A diagonal
      //    tile's chunk of whole buckets has the column elements as its row
      //    elements: each one's hits are the final mask of the entry it joined
      if (self_tile && cs == s_coff[bs - wb] && ce == s_coff[be - wb]) {
#pragma unroll
        for (int u = 0; u < kJMade; ++u) {
          const uint32_t r = cur.cid[u];
          if (hs[u] == kNoSlot || r >= r_valid) continue;
          const unsigned long long m = s_ent[ent[u]].y;
#ifdef SKS_JOIN_CHECK  // diagnostic build: an element's entry holds its value and its column bit
          if (s_ent[ent[u]].x != cur.cv[u] || !((m >> r) & 1ull))
            printf("join check: tile %u,%u buckets [%u,%u) cols [%u,%u) e=%u ent=%u v=%llx entv=%llx m=%llx r=%u "
                   "slot=%u made=%u prev=%x\n", I, J, bs, be, cs, ce, (uint32_t)(tid + kJB * u), ent[u],
                   (unsigned long long)cur.cv[u], (unsigned long long)s_ent[ent[u]].x, m, r, hs[u], made[u],
                   prev[u]);
#endif
          if (SKS_JOIN_DIAG & 1) continue;
          if (SKS_JOIN_DIAG & 4) { diag_acc += __popcll(m); continue; }
          add_hits(r, m);
        }
        __syncthreads();
        JSTAMP(2);
        cur = nxt;
        bs = nbs;
        be = nbe;
        cs = ncs;
        ce = nce;
        continue;
      }
      uint32_t sl[kJRowPf], sh[kJRowPf];
#pragma unroll
      for (int u = 0; u < kJRowPf; ++u) {
        sl[u] = kFFree;
        sh[u] = 0;
        if (cur.rid[u] < r_valid) {
          sh[u] = fp_slot(cur.rv[u]);
          sl[u] = s_slot[sh[u]];
        }
      }
#pragma unroll
      for (int u = 0; u < kJRowPf; ++u) {
        const uint32_t r = cur.rid[u];
        if (r >= r_valid) continue;
        const unsigned long long m = lookup(cur.rv[u], sh[u], sl[u]);
        if (SKS_JOIN_DIAG & 1) continue;
        if (SKS_JOIN_DIAG & 4) { diag_acc += __popcll(m); continue; }
        if (m) add_hits(r, m);
      }
      for (uint32_t k = rs + tid + kJB * kJRowPf; k < re; k += kJB) {
        const uint32_t r = rids[k];
        if (r >= r_valid) continue;
        const uint64_t v = rdata[k];
        const uint32_t h = fp_slot(v);
        const unsigned long long m = lookup(v, h, s_slot[h]);
        if (SKS_JOIN_DIAG & 4) { diag_acc += __popcll(m); continue; }
        if (m) add_hits(r, m);
      }
      __syncthreads();
      JSTAMP(2);
      cur = nxt;
      bs = nbs;
      be = nbe;
      cs = ncs;
      ce = nce;
    }
  }
  __syncthreads();
  JSTAMP(5);
  if (SKS_JOIN_DIAG & 4) atomicAdd(&s_slot[0], diag_acc);
  if (SKS_JOIN_DIAG & 2) return;
  // planes the carry chains reached (unrelated tiles: none or one)
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) top = max(top, (uint32_t)__shfl_xor(top, o, 64));
  if (lane == 0 && top) atomicMax(&s_top, top);
  __syncthreads();
  const int np = (int)s_top;
  for (uint32_t r = tid >> 6; r < kTile; r += kJB / 64) {  // a wave per row, a lane per column
    const uint32_t c = lane;
    uint32_t cnt = 0;
    for (int b = 0; b < np; ++b) cnt |= (uint32_t)((s_pl[b * kTile + r] >> c) & 1ull) << b;
    if (self_tile && c == r) cnt += s_self[r];
    if (!cnt) continue;
    const uint32_t gr = row0 + r, gc = col0 + c;
    if (gr >= row_lim || gc >= a.n) continue;
    if (a.packed) {
      atomicAdd(&a.out[(t - a.tile_begin) * (kTile * kTile) + r * kTile + c], (int32_t)cnt);
      continue;
    }
    const uint64_t orow = rows_mode ? (gr - a.row_begin) : gr;
    atomicAdd(&a.out[orow * a.ld + gc], (int32_t)cnt);
  }
  // the mirror (j, i) of an off-diagonal symmetric tile: a wave per column, a lane
  // per row, so each wave's atomics fall on one output row (contiguous), as above.
  // (Round 2 added it in the loop above, lanes over columns: 64 rows, 64 lines
  // per wave instruction.  Config 5, 200 related genomes, every tile dense: whole
  // call 0.180 -> 0.125 ms; config 4 unchanged, 0.671 ms, most tiles sparse.)
  if (!a.packed && !rows_mode && I != J) {
    for (uint32_t c = tid >> 6; c < kTile; c += kJB / 64) {
      const uint32_t r = lane;
      uint32_t cnt = 0;
      for (int b = 0; b < np; ++b) cnt |= (uint32_t)((s_pl[b * kTile + r] >> c) & 1ull) << b;
      const uint32_t gr = row0 + r, gc = col0 + c;
      if (!cnt || gr >= row_lim || gc >= a.n) continue;
      atomicAdd(&a.out[(uint64_t)gc * a.ld + gr], (int32_t)cnt);
    }
  }
#ifdef SKS_JOIN_STAMPS
  JSTAMP(4);
  if (tid == 0)
    for (int i = 0; i < 6; ++i) atomicAdd(&g_join_stamps[i], (unsigned long long)st_acc[i]);
#endif
}

}  // namespace

hipError_t launch_intersect_pairs(const uint64_t* data, const uint64_t* starts,
                                  const uint32_t* sizes, int elem_words, const int32_t* a,
                                  const int32_t* b, uint64_t n_pairs, int32_t* out, hipStream_t s) {
  const uint64_t per = kMaxGrid * kWavesPerBlock;  // pairs per launch slice
  for (uint64_t p0 = 0; p0 < n_pairs; p0 += per) {
    const uint64_t blocks = (std::min(per, n_pairs - p0) + kWavesPerBlock - 1) / kWavesPerBlock;
    if (elem_words == 1)
      hipLaunchKernelGGL(k_pairs<1>, dim3((unsigned)blocks), dim3(kB), 0, s, data, starts, sizes, a,
                         b, p0, n_pairs, out);
    else
      hipLaunchKernelGGL(k_pairs<2>, dim3((unsigned)blocks), dim3(kB), 0, s, data, starts, sizes, a,
                         b, p0, n_pairs, out);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

hipError_t launch_intersect_all_global(const uint64_t* data, const uint64_t* starts,
                                       const uint32_t* sizes, int elem_words, uint32_t n,
                                       uint32_t row_begin, uint32_t row_end, int32_t* out,
                                       hipStream_t s) {
  const uint64_t n_pairs = (uint64_t)(row_end - row_begin) * n;
  const uint64_t per = kMaxGrid * kWavesPerBlock;
  for (uint64_t p0 = 0; p0 < n_pairs; p0 += per) {
    const uint64_t blocks = (std::min(per, n_pairs - p0) + kWavesPerBlock - 1) / kWavesPerBlock;
    if (elem_words == 1)
      hipLaunchKernelGGL(k_all<1>, dim3((unsigned)blocks), dim3(kB), 0, s, data, starts, sizes, n,
                         row_begin, p0, n_pairs, out);
    else
      hipLaunchKernelGGL(k_all<2>, dim3((unsigned)blocks), dim3(kB), 0, s, data, starts, sizes, n,
                         row_begin, p0, n_pairs, out);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

}  // namespace sks

namespace sks {

uint32_t join_cap() {  // SKS_JOIN_CAP (diagnostics) is clamped to [64, kJCap]
  static const uint32_t cap = std::max<uint32_t>(
      64, std::min<uint32_t>(kJCap, getenv("SKS_JOIN_CAP") ? (uint32_t)atoi(getenv("SKS_JOIN_CAP"))
                                                           : kJCap));
  return cap;
}

// Bucket count for the join: mean block-bucket population ~ cap / 6, so a
// chunk holds several whole buckets.
uint32_t join_log_b(uint32_t max_size) {
  uint32_t log_b = 0;
  while ((1ull << log_b) * (join_cap() / 6) < 64ull * max_size && log_b < kJMaxLogB) ++log_b;
  return log_b;
}

hipError_t join_launch(const JoinLayout& rows, uint32_t r_blk0, const JoinLayout& cols, uint32_t c_blk0,
                       uint32_t n, uint32_t log_b, bool sym, uint32_t row_begin, uint32_t row_end,
                       uint64_t tile_begin, uint64_t tile_end, const uint32_t* d_tiles, bool packed,
                       int32_t* out, hipStream_t s) {
  const uint32_t n_cb = (n + kTile - 1) / kTile;
  const uint32_t n_rb = sym ? n_cb : (row_end - row_begin + kTile - 1) / kTile;
  if (!d_tiles) {
    const uint64_t all_tiles = sym ? (uint64_t)n_cb * (n_cb + 1) / 2 : (uint64_t)n_rb * n_cb;
    if (!sym) { tile_begin = 0; tile_end = all_tiles; }
    tile_end = std::min(tile_end, all_tiles);
  }
  if (tile_begin >= tile_end) return hipSuccess;
  const uint64_t tiles = tile_end - tile_begin;
  const uint32_t B = 1u << log_b;
  JoinArgs ja{};
  ja.r = rows;
  ja.c = cols;
  ja.r_blk0 = r_blk0;
  ja.c_blk0 = c_blk0;
  ja.tiles = d_tiles;
  ja.packed = packed ? 1 : 0;
  ja.B = B;
  ja.n = n;
  ja.n_col_blocks = n_cb;
  ja.sym = (sym || d_tiles) ? 1 : 0;
  ja.row_begin = row_begin;
  ja.row_end = row_end;
  ja.tile_begin = tile_begin;
  ja.out = out;
  ja.ld = n;
  ja.cap = join_cap();
  // bucket groups per tile: ~128 buckets per workgroup (a workgroup's start-up —
  // clearing its table and count planes — and its count flush, up to 4096 global
  // atomics on a tile of related genomes, are then small beside its chunks), at
  // least ~1024 workgroups in all, at least 16 buckets each.  Config 4 (136
  // tiles, B = 4096), round 3 sweep of SKS_JOIN_WGS, whole call family /
  // unrelated genomes: 1088 workgroups 0.870 / 0.792 ms, 2176 0.705 / 0.691,
  // 4352 (this rule) 0.681 / 0.674, 8704 (round 2's ~64 buckets) 0.742 / 0.681,
  // 17408 0.900 / 0.734.  Config 5 (10 tiles): the 1024 floor, 1030.
  // SKS_JOIN_WGS (diagnostics) sets the total instead.
  // The ~128-buckets floor only applies while the grid is small (<= 64K
  // workgroups); with very many tiles a tile gets fewer, larger groups (down to
  // one), and the launch is cut into tile slices of at most kMaxGrid workgroups
  // (HIP caps a grid at 2^32 - 1 work-items).
  static const uint64_t wgs_env = getenv("SKS_JOIN_WGS") ? strtoull(getenv("SKS_JOIN_WGS"), 0, 10) : 0;
  uint64_t want = wgs_env ? (wgs_env + tiles - 1) / tiles
                          : std::max<uint64_t>(std::min<uint64_t>((B + 127) / 128, (65536 + tiles - 1) / tiles),
                                               (1024 + tiles - 1) / tiles);
  if (!wgs_env) want = std::min<uint64_t>(want, std::max<uint32_t>(1, B / 16));
  const uint32_t groups = (uint32_t)std::min<uint64_t>(B, std::max<uint64_t>(1, want));
  ja.buckets_per_group = (B + groups - 1) / groups;
  ja.n_groups = (B + ja.buckets_per_group - 1) / ja.buckets_per_group;
  const uint64_t tiles_per_launch = std::max<uint64_t>(1, kMaxGrid / ja.n_groups);
  for (uint64_t t0 = tile_begin; t0 < tile_end; t0 += tiles_per_launch) {
    const uint64_t nt = std::min(tiles_per_launch, tile_end - t0);
    ja.tile_begin = t0;
    if (packed) ja.out = out + (t0 - tile_begin) * (uint64_t)(kTile * kTile);
    hipLaunchKernelGGL(k_join, dim3((unsigned)(nt * ja.n_groups)), dim3(kJB), 0, s, ja);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
#ifdef SKS_JOIN_STAMPS
  {
    unsigned long long h[8] = {0};
    (void)hipStreamSynchronize(s);
    (void)hipMemcpyFromSymbol(h, HIP_SYMBOL(g_join_stamps), sizeof h);
    const unsigned long long z[8] = {0};
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_join_stamps), z, sizeof z);
    const double wgs = (double)(tile_end - tile_begin) * ja.n_groups;
    fprintf(stderr, "[k_join stamps] cycles per workgroup: setup %.0f insert %.0f probe %.0f reset %.0f "
            "flush %.0f tail-barrier %.0f (%.0f workgroups)\n", h[0] / wgs, h[1] / wgs, h[2] / wgs,
            h[3] / wgs, h[4] / wgs, h[5] / wgs, wgs);
  }
#endif
  return hipSuccess;
}

// Tiled all-pairs for u64 sketches.  Host-synchronous (reads sizes and bucket
// positions back to pick the bucket count).  mode: sym (upper-triangle tiles
// [tile_begin, tile_end) into a full n x n matrix) or rows.
hipError_t launch_intersect_tiled(const uint64_t* data, const uint64_t* starts, const uint32_t* sizes,
                                  uint32_t n, bool sym, uint32_t row_begin, uint32_t row_end,
                                  uint64_t tile_begin, uint64_t tile_end, int32_t* out,
                                  Scratch& work, hipStream_t s, bool* used_tiles, int algo) {
  *used_tiles = false;
  hipError_t e;
  const uint64_t out_words = sym ? (uint64_t)n * n : (uint64_t)(row_end - row_begin) * n;
  if ((e = hipMemsetAsync(out, 0, out_words * sizeof(int32_t), s)) != hipSuccess) return e;
  if (n == 0 || out_words == 0) { *used_tiles = true; return hipSuccess; }
  std::vector<uint32_t> h_sizes(n);
  if ((e = pinned_d2h(h_sizes.data(), sizes, n * sizeof(uint32_t), s)) != hipSuccess) return e;
  const uint32_t max_size = *std::max_element(h_sizes.begin(), h_sizes.end());
  if (max_size == 0) { *used_tiles = true; return hipSuccess; }

  const uint32_t n_cb = (n + kTile - 1) / kTile;
  const uint32_t n_rb = sym ? n_cb : (row_end - row_begin + kTile - 1) / kTile;
  const uint64_t all_tiles = sym ? (uint64_t)n_cb * (n_cb + 1) / 2 : (uint64_t)n_rb * n_cb;
  if (!sym) { tile_begin = 0; tile_end = all_tiles; }
  tile_end = std::min(tile_end, all_tiles);
  if (tile_begin >= tile_end) { *used_tiles = true; return hipSuccess; }
  const uint64_t tiles = tile_end - tile_begin;
  static const bool dbg = getenv("SKS_DEBUG_INTERSECT") != nullptr;

  auto launch = [&](const uint64_t* d, const uint64_t* st, const uint32_t* pos, uint32_t B,
                    uint32_t P) -> hipError_t {
    TileArgs a{};
    a.data = d;
    a.starts = st;
    a.sizes = sizes;
    a.pos = pos;
    a.n = n;
    a.B = B;
    a.P = P;
    a.sym = sym ? 1 : 0;
    a.n_col_blocks = n_cb;
    a.row_begin = row_begin;
    a.row_end = row_end;
    a.n_row_blocks = n_rb;
    uint32_t groups = (uint32_t)std::min<uint64_t>(B, std::max<uint64_t>(1, (2048 + tiles - 1) / tiles));
    a.buckets_per_group = (B + groups - 1) / groups;
    a.n_groups = (B + a.buckets_per_group - 1) / a.buckets_per_group;
    a.tile_begin = tile_begin;
    a.out = out;
    a.ld = n;
    if (dbg)
      fprintf(stderr, "[sks intersect] merge tiles n=%u B=%u P=%u tiles=%llu groups=%u\n", n, B, P,
              (unsigned long long)tiles, a.n_groups);
    const size_t lds_bytes = (size_t)std::max<uint32_t>(P, 1) * kSlots * sizeof(uint64_t) +
                             kSlots * sizeof(uint32_t);
    static const hipError_t attr = hipFuncSetAttribute(
        reinterpret_cast<const void*>(k_tiles), hipFuncAttributeMaxDynamicSharedMemorySize,
        (int)(kMaxPart * kSlots * sizeof(uint64_t) + kSlots * sizeof(uint32_t)));
    if (attr != hipSuccess) return attr;
    const uint64_t per = std::max<uint64_t>(1, kMaxGrid / a.n_groups);  // tiles per slice
    for (uint64_t t0 = tile_begin; t0 < tile_end; t0 += per) {
      a.tile_begin = t0;
      hipLaunchKernelGGL(k_tiles, dim3((unsigned)(std::min(per, tile_end - t0) * a.n_groups)), dim3(kB),
                         lds_bytes, s, a);
      hipError_t le = hipGetLastError();
      if (le != hipSuccess) return le;
    }
    *used_tiles = true;
    return hipSuccess;
  };
  auto align16 = [](size_t x) { return (x + 15) & ~(size_t)15; };

  uint64_t total = 0;
  for (uint32_t i = 0; i < n; ++i) total += h_sizes[i];
  // the layout's bucket starts are u32 (< 2^32 elements per layout)
  const bool join_fits = total < (1ull << 32);
  if (algo != kIntersectMerge && join_fits) {
    // hash-bucketed block-major copy of the column sketches (and of the row
    // range when its blocks are not aligned with the column blocks), then k_join
    const bool sep_rows = !sym && (row_begin % kTile) != 0;
    const uint32_t rn = row_end - row_begin;
    uint64_t r_total = 0;
    if (sep_rows)
      for (uint32_t i = row_begin; i < row_end; ++i) r_total += h_sizes[i];
    uint32_t log_b = join_log_b(max_size);
    for (;;) {
      const uint32_t B = 1u << log_b;
      const size_t tmp_c = join_layout_temp_bytes(n, log_b);
      const size_t tmp_r = !sep_rows ? 0 : join_layout_temp_bytes(rn, log_b);
      size_t o = 0;
      const size_t o_cdat = o; o = align16(o + total * 8);
      const size_t o_cids = o; o = align16(o + total);
      const size_t o_cbof = o; o = align16(o + (size_t)n_cb * (B + 1) * 4);
      const size_t o_cbst = o; o = align16(o + (size_t)(n_cb + 1) * 8);
      const size_t o_rdat = o; o = align16(o + r_total * 8);
      const size_t o_rids = o; o = align16(o + r_total);
      const size_t o_rbof = o; o = align16(o + (sep_rows ? (size_t)n_rb * (B + 1) * 4 : 0));
      const size_t o_rbst = o; o = align16(o + (sep_rows ? (size_t)(n_rb + 1) * 8 : 0));
      const size_t o_stat = o; o = align16(o + 16);
      const size_t o_bnd = o; o = align16(o + (size_t)(B + 1) * 8);
      const size_t o_tmp = o; o = align16(o + std::max(tmp_c, tmp_r));
      if ((e = work.reserve(o)) != hipSuccess) return e;
      char* w = static_cast<char*>(work.ptr);
      JoinLayout cl{reinterpret_cast<uint64_t*>(w + o_cdat), reinterpret_cast<uint8_t*>(w + o_cids),
                    reinterpret_cast<uint32_t*>(w + o_cbof), reinterpret_cast<uint64_t*>(w + o_cbst)};
      JoinLayout rl = cl;
      uint32_t* stat = reinterpret_cast<uint32_t*>(w + o_stat);
      if ((e = hipMemsetAsync(stat, 0, 4, s)) != hipSuccess) return e;
      // a separate row layout shares the column set's group bounds; a single
      // layout computes its own in the build's first launch (three in all)
      uint64_t* gbounds = sep_rows ? reinterpret_cast<uint64_t*>(w + o_bnd) : nullptr;
      if (sep_rows && (e = join_layout_bounds(data, starts, sizes, n, log_b, gbounds, s)) != hipSuccess)
        return e;
      auto build_layout = [&](uint32_t first, uint32_t cnt, uint64_t tot, const JoinLayout& L,
                              size_t tmp_bytes) -> hipError_t {
        return join_layout_build(data, starts + first, sizes + first, cnt, log_b, gbounds, w + o_tmp,
                                 const_cast<uint64_t*>(L.data), const_cast<uint8_t*>(L.ids),
                                 const_cast<uint32_t*>(L.boff), const_cast<uint64_t*>(L.bstart), stat, s);
      };
      if ((e = build_layout(0, n, total, cl, tmp_c)) != hipSuccess) return e;
      if (sep_rows) {
        rl = JoinLayout{reinterpret_cast<uint64_t*>(w + o_rdat), reinterpret_cast<uint8_t*>(w + o_rids),
                        reinterpret_cast<uint32_t*>(w + o_rbof), reinterpret_cast<uint64_t*>(w + o_rbst)};
        if ((e = build_layout(row_begin, rn, r_total, rl, tmp_r)) != hipSuccess) return e;
      }
      uint32_t h_stat = 0;
      if ((e = pinned_d2h(&h_stat, stat, 4, s)) != hipSuccess) return e;
      if (dbg)
        fprintf(stderr, "[sks intersect] join n=%u B=%u max block bucket %u tiles=%llu\n", n, B,
                h_stat, (unsigned long long)tiles);
      // buckets above the table's capacity are joined in sub-chunks (exact, but
      // the bucket's row elements are probed once per sub-chunk), so more
      // buckets are tried first while the count matrix allows
      if (h_stat <= join_cap() || log_b >= kJMaxLogB) {
        const uint32_t r_blk0 = sep_rows ? 0 : (sym ? 0 : row_begin / kTile);
        if ((e = join_launch(rl, r_blk0, cl, 0, n, log_b, sym, row_begin, row_end, tile_begin, tile_end, nullptr, false,
                             out, s)) != hipSuccess)
          return e;
        *used_tiles = true;
        return hipSuccess;
      }
      ++log_b;
    }
  }

  // merge tiles: value-range buckets (parts must stay sorted)
  uint32_t B = 1;
  while ((uint64_t)B * 32 < max_size) B <<= 1;  // mean part <= 32 elements
  for (;;) {
    const size_t o_bounds = 0, o_pos = align16(o_bounds + (size_t)(B + 1) * 8);
    const size_t o_stats = align16(o_pos + (size_t)n * (B + 1) * 4);
    if ((e = work.reserve(o_stats + 16)) != hipSuccess) return e;
    char* w = static_cast<char*>(work.ptr);
    uint64_t* bounds = reinterpret_cast<uint64_t*>(w + o_bounds);
    uint32_t* pos = reinterpret_cast<uint32_t*>(w + o_pos);
    uint32_t* stats = reinterpret_cast<uint32_t*>(w + o_stats);
    if ((e = hipMemsetAsync(stats, 0, 2 * sizeof(uint32_t), s)) != hipSuccess) return e;
    hipLaunchKernelGGL(k_bounds, dim3((B + 1 + kB - 1) / kB), dim3(kB), 0, s, data, starts, sizes,
                       n, std::min<uint32_t>(n, 64), B, bounds);
    const uint64_t items = (uint64_t)n * (B + 1);
    hipLaunchKernelGGL(k_bucket_pos, dim3((unsigned)((items + kB - 1) / kB)), dim3(kB), 0, s, data,
                       starts, sizes, n, B, bounds, pos);
    const uint64_t cells = (uint64_t)n_cb * B;
    hipLaunchKernelGGL(k_part_stats, dim3((unsigned)((cells + kB - 1) / kB)), dim3(kB), 0, s, pos,
                       n, B, n_cb, stats);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    uint32_t h_stats[2];
    if ((e = pinned_d2h(h_stats, stats, sizeof(h_stats), s)) != hipSuccess) return e;
    const uint32_t P = h_stats[0];
    if (P <= (uint32_t)kGoodPart) return launch(data, starts, pos, B, P);
    if (B >= (1u << 16) || (uint64_t)B * 8 > max_size) {
      if (P <= (uint32_t)kMaxPart) return launch(data, starts, pos, B, P);
      return hipSuccess;  // pathological skew: caller falls back to the global kernel
    }
    B <<= 1;
  }
}

hipError_t launch_value_bounds(const uint64_t* data, const uint64_t* starts, const uint32_t* sizes,
                               uint32_t n, uint32_t B, uint64_t* bounds, hipStream_t s) {
  hipLaunchKernelGGL(k_bounds, dim3((B + 1 + kB - 1) / kB), dim3(kB), 0, s, data, starts, sizes, n,
                     std::min<uint32_t>(n, 64), B, bounds);
  return hipGetLastError();
}

hipError_t launch_bucket_pos(const uint64_t* data, const uint64_t* starts, const uint32_t* sizes,
                             uint32_t n, uint32_t B, const uint64_t* bounds, uint32_t* pos,
                             hipStream_t s) {
  const uint64_t items = (uint64_t)n * (B + 1);
  if (!items) return hipSuccess;
  hipLaunchKernelGGL(k_bucket_pos, dim3((unsigned)((items + kB - 1) / kB)), dim3(kB), 0, s, data, starts,
                     sizes, n, B, bounds, pos);
  return hipGetLastError();
}

uint64_t intersect_sym_tiles(uint32_t n) {
  uint64_t nb = (n + kTile - 1) / kTile;
  return nb * (nb + 1) / 2;
}

}  // namespace sks
