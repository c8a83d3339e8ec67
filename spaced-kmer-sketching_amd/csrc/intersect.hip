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
#include <cstdint>
#include <vector>

#include "sks_internal.hpp"

namespace sks {

namespace {

constexpr int kB = 256;
constexpr int kWavesPerBlock = kB / 64;

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
                                              const int32_t* __restrict__ b, uint64_t n_pairs,
                                              int32_t* __restrict__ out) {
  const uint64_t p = (uint64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
  if (p >= n_pairs) return;
  const int32_t ia = a[p], ib = b[p];
  int32_t c = wave_pair_count<EW>(data, starts[ia], sizes[ia], starts[ib], sizes[ib]);
  if ((threadIdx.x & 63) == 0) out[p] = c;
}

template <int EW>
__global__ __launch_bounds__(kB) void k_all(const uint64_t* __restrict__ data,
                                            const uint64_t* __restrict__ starts,
                                            const uint32_t* __restrict__ sizes, uint32_t n,
                                            uint32_t row_begin, uint64_t n_pairs,
                                            int32_t* __restrict__ out) {
  const uint64_t p = (uint64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
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

__global__ void k_bounds(const uint64_t* __restrict__ data, uint64_t ref_start, uint32_t ref_size,
                         uint32_t B, uint64_t* __restrict__ bounds) {
  uint32_t b = blockIdx.x * kB + threadIdx.x;
  if (b > B) return;
  if (b == 0) bounds[0] = 0;
  else if (b == B) bounds[B] = ~0ull;
  else bounds[b] = data[ref_start + (uint64_t)b * ref_size / B];
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

__device__ __forceinline__ void sym_tile(uint64_t t, uint32_t nb, uint32_t& I, uint32_t& J) {
  uint32_t i = 0;
  uint64_t rem = t;
  while (rem >= nb - i) {  // row i of the upper triangle holds nb - i tiles
    rem -= nb - i;
    ++i;
  }
  I = i;
  J = i + (uint32_t)rem;
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
// Same tiles and buckets as k_tiles, but instead of merging 64 x 64 pairs a
// workgroup joins the two blocks: per bucket, the 64 column parts go into an
// LDS hash table value -> 64-bit mask of the columns holding it, and every
// row element probes it once; a hit with mask m adds 1 to cnt[row][c] for each
// set bit c (ds_add in an LDS 64 x 65 matrix).  Work per tile is
// (row elements + column elements) + Σ_pairs |S_i ∩ S_j| instead of
// Σ_pairs (|S_i| + |S_j|) — 64x fewer steps for unrelated sketches and still
// fewer when every pair is identical.  Lane l of every wave owns row l, so the
// ds_adds of one instruction hit 64 different rows (stride 65: distinct banks
// for equal columns).
constexpr int kJSlots = 2048;               // hash slots (load <= 1/2, see host)
constexpr int kJLog = 11;
constexpr int kJMaxPart = 32;               // largest part a join launch accepts
constexpr int kJMaxCol = kJSlots / 2;       // largest column-block bucket population
constexpr int kJPer = kJMaxPart / kWavesPerBlock;  // elements per thread per part (8)
constexpr int kCntLd = kTile + 1;
constexpr uint64_t kEmpty = ~0ull;
constexpr uint32_t kNoSlot = 0xFFFFFFFFu;

__device__ __forceinline__ uint32_t join_hash(uint64_t v) {
  return (((uint32_t)v ^ (uint32_t)(v >> 32)) * 0x9E3779B1u) >> (32 - kJLog);
}

__global__ __launch_bounds__(kB) void k_join(TileArgs a) {
  __shared__ uint64_t s_key[kJSlots];
  __shared__ uint64_t s_msk[kJSlots];
  __shared__ uint64_t s_row[kJMaxPart * kTile];
  __shared__ uint32_t s_cnt[kTile * kCntLd];
  __shared__ uint32_t s_len[kTile];
  __shared__ unsigned long long s_special;  // columns holding the value ~0 (== kEmpty)

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

  for (int i = tid; i < kJSlots; i += kB) {
    s_key[i] = kEmpty;
    s_msk[i] = 0;
  }
  for (int i = tid; i < kTile * kCntLd; i += kB) s_cnt[i] = 0;
  if (tid == 0) s_special = 0;

  // lane = sketch slot within the block (row `lane` and column `lane`)
  const uint32_t rid = row0 + lane, cid = col0 + lane;
  const bool rv = rid < row_lim, cv = cid < a.n;
  const uint64_t rstart = rv ? a.starts[rid] : 0, cstart = cv ? a.starts[cid] : 0;
  const uint32_t* rpos = a.pos + (uint64_t)(rv ? rid : 0) * (a.B + 1);
  const uint32_t* cpos = a.pos + (uint64_t)(cv ? cid : 0) * (a.B + 1);
  const unsigned long long cbit = 1ull << lane;

  const uint32_t b0 = grp * a.buckets_per_group;
  const uint32_t b1 = min(a.B, b0 + a.buckets_per_group);
  __syncthreads();
  for (uint32_t b = b0; b < b1; ++b) {
    // 1) stage the row parts (lds[pos][row]) and insert the column parts
    uint32_t rbeg = 0, rlen = 0, cbeg = 0, clen = 0;
    if (rv) { rbeg = rpos[b]; rlen = rpos[b + 1] - rbeg; }
    if (cv) { cbeg = cpos[b]; clen = cpos[b + 1] - cbeg; }
    if (wave == 0) s_len[lane] = rlen;
    uint64_t rvals[kJPer], cvals[kJPer];
#pragma unroll
    for (int u = 0; u < kJPer; ++u) {
      const uint32_t e = wave + kWavesPerBlock * u;
      rvals[u] = e < rlen ? a.data[rstart + rbeg + e] : 0;
      cvals[u] = e < clen ? a.data[cstart + cbeg + e] : 0;
    }
    uint32_t made[kJPer];
#pragma unroll
    for (int u = 0; u < kJPer; ++u) {
      const uint32_t e = wave + kWavesPerBlock * u;
      made[u] = kNoSlot;
      if (e < rlen) s_row[e * kTile + lane] = rvals[u];
      if (e < clen) {
        const uint64_t v = cvals[u];
        if (v == kEmpty) {
          atomicOr(&s_special, cbit);
        } else {
          uint32_t h = join_hash(v);
          for (;;) {
            const unsigned long long prev = atomicCAS(
                reinterpret_cast<unsigned long long*>(&s_key[h]), (unsigned long long)kEmpty,
                (unsigned long long)v);
            if (prev == kEmpty || prev == v) {
              if (prev == kEmpty) made[u] = h;
              atomicOr(reinterpret_cast<unsigned long long*>(&s_msk[h]), cbit);
              break;
            }
            h = (h + 1) & (kJSlots - 1);
          }
        }
      }
    }
    __syncthreads();
    // 2) probe: lane = row, this wave takes positions wave, wave + 4, ...
    const uint32_t nrow = s_len[lane];
    const unsigned long long special = s_special;
#pragma unroll
    for (int u = 0; u < kJPer; ++u) {
      const uint32_t e = wave + kWavesPerBlock * u;
      if (e < nrow) {
        const uint64_t v = s_row[e * kTile + lane];
        unsigned long long m = 0;
        if (v == kEmpty) {
          m = special;
        } else {
          uint32_t h = join_hash(v);
          for (;;) {
            const uint64_t k = s_key[h];
            if (k == v) { m = s_msk[h]; break; }
            if (k == kEmpty) break;
            h = (h + 1) & (kJSlots - 1);
          }
        }
        while (m) {
          const uint32_t c = (uint32_t)__builtin_ctzll(m);
          m &= m - 1;
          atomicAdd(&s_cnt[lane * kCntLd + c], 1u);
        }
      }
    }
    __syncthreads();
    // 3) reset the slots this thread created (and the ~0 mask)
#pragma unroll
    for (int u = 0; u < kJPer; ++u) {
      if (made[u] != kNoSlot) {
        s_key[made[u]] = kEmpty;
        s_msk[made[u]] = 0;
      }
    }
    if (tid == 0) s_special = 0;
    __syncthreads();
  }
  // counts -> global (one atomic per nonzero pair; both halves for sym off-diagonal)
  for (int i = tid; i < kTile * kTile; i += kB) {
    const uint32_t r = i >> 6, c = i & 63;
    const uint32_t cnt = s_cnt[r * kCntLd + c];
    if (!cnt) continue;
    const uint32_t gr = row0 + r, gc = col0 + c;
    if (gr >= row_lim || gc >= a.n) continue;
    const uint64_t orow = a.sym ? gr : (gr - a.row_begin);
    atomicAdd(&a.out[orow * a.ld + gc], (int32_t)cnt);
    if (a.sym && I != J) atomicAdd(&a.out[(uint64_t)gc * a.ld + gr], (int32_t)cnt);
  }
}

}  // namespace

hipError_t launch_intersect_pairs(const uint64_t* data, const uint64_t* starts,
                                  const uint32_t* sizes, int elem_words, const int32_t* a,
                                  const int32_t* b, uint64_t n_pairs, int32_t* out, hipStream_t s) {
  if (n_pairs == 0) return hipSuccess;
  uint64_t blocks = (n_pairs + kWavesPerBlock - 1) / kWavesPerBlock;
  if (elem_words == 1)
    hipLaunchKernelGGL(k_pairs<1>, dim3((unsigned)blocks), dim3(kB), 0, s, data, starts, sizes, a, b,
                       n_pairs, out);
  else
    hipLaunchKernelGGL(k_pairs<2>, dim3((unsigned)blocks), dim3(kB), 0, s, data, starts, sizes, a, b,
                       n_pairs, out);
  return hipGetLastError();
}

hipError_t launch_intersect_all_global(const uint64_t* data, const uint64_t* starts,
                                       const uint32_t* sizes, int elem_words, uint32_t n,
                                       uint32_t row_begin, uint32_t row_end, int32_t* out,
                                       hipStream_t s) {
  uint64_t n_pairs = (uint64_t)(row_end - row_begin) * n;
  if (n_pairs == 0) return hipSuccess;
  uint64_t blocks = (n_pairs + kWavesPerBlock - 1) / kWavesPerBlock;
  if (elem_words == 1)
    hipLaunchKernelGGL(k_all<1>, dim3((unsigned)blocks), dim3(kB), 0, s, data, starts, sizes, n,
                       row_begin, n_pairs, out);
  else
    hipLaunchKernelGGL(k_all<2>, dim3((unsigned)blocks), dim3(kB), 0, s, data, starts, sizes, n,
                       row_begin, n_pairs, out);
  return hipGetLastError();
}

}  // namespace sks

namespace sks {

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
  std::vector<uint64_t> h_starts(n);
  if ((e = hipMemcpyAsync(h_sizes.data(), sizes, n * sizeof(uint32_t), hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
  if ((e = hipMemcpyAsync(h_starts.data(), starts, n * sizeof(uint64_t), hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
  if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
  uint32_t ref = 0;
  for (uint32_t i = 1; i < n; ++i) if (h_sizes[i] > h_sizes[ref]) ref = i;
  const uint32_t max_size = h_sizes[ref];
  if (max_size == 0) { *used_tiles = true; return hipSuccess; }
  uint32_t B = 1;
  while ((uint64_t)B * 32 < max_size) B <<= 1;  // mean part <= 32 elements
  std::vector<uint32_t> h_pos;
  uint32_t P = 0;
  bool use_join = false;
  const uint32_t n_cb = (n + kTile - 1) / kTile;
  for (;;) {
    size_t bytes = sizeof(uint64_t) * (B + 1) + sizeof(uint32_t) * (uint64_t)n * (B + 1) + 64;
    if ((e = work.reserve(bytes)) != hipSuccess) return e;
    uint64_t* bounds = reinterpret_cast<uint64_t*>(work.ptr);
    uint32_t* pos = reinterpret_cast<uint32_t*>(bounds + B + 1);
    hipLaunchKernelGGL(k_bounds, dim3((B + 1 + kB - 1) / kB), dim3(kB), 0, s, data, h_starts[ref],
                       max_size, B, bounds);
    uint64_t items = (uint64_t)n * (B + 1);
    hipLaunchKernelGGL(k_bucket_pos, dim3((unsigned)((items + kB - 1) / kB)), dim3(kB), 0, s, data,
                       starts, sizes, n, B, bounds, pos);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    h_pos.resize(items);
    if ((e = hipMemcpyAsync(h_pos.data(), pos, items * sizeof(uint32_t), hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
    if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
    P = 0;
    for (uint32_t i = 0; i < n; ++i)
      for (uint32_t b = 0; b < B; ++b)
        P = std::max(P, h_pos[(uint64_t)i * (B + 1) + b + 1] - h_pos[(uint64_t)i * (B + 1) + b]);
    if (algo != kIntersectMerge && P <= (uint32_t)kJMaxPart) {
      // largest bucket population of one 64-sketch column block (hash-table load)
      uint32_t colmax = 0;
      std::vector<uint32_t> acc(B);
      for (uint32_t cb = 0; cb < n_cb && colmax <= (uint32_t)kJMaxCol; ++cb) {
        std::fill(acc.begin(), acc.end(), 0u);
        for (uint32_t i = cb * kTile; i < std::min(n, cb * kTile + kTile); ++i) {
          const uint32_t* q = &h_pos[(uint64_t)i * (B + 1)];
          for (uint32_t b = 0; b < B; ++b) acc[b] += q[b + 1] - q[b];
        }
        for (uint32_t b = 0; b < B; ++b) colmax = std::max(colmax, acc[b]);
      }
      if (colmax <= (uint32_t)kJMaxCol) { use_join = true; break; }
    }
    if (algo == kIntersectMerge && P <= (uint32_t)kGoodPart) break;
    const bool grow = B < (1u << 16) &&
                      (uint64_t)B * (algo == kIntersectMerge ? 8 : 2) <= max_size;
    if (!grow) {
      if (P <= (uint32_t)kMaxPart) break;  // merge tiles
      return hipSuccess;  // pathological skew: caller falls back to the global kernel
    }
    B <<= 1;
  }
  TileArgs a{};
  a.data = data;
  a.starts = starts;
  a.sizes = sizes;
  a.pos = reinterpret_cast<uint32_t*>(reinterpret_cast<uint64_t*>(work.ptr) + B + 1);
  a.n = n;
  a.B = B;
  a.P = P;
  a.sym = sym ? 1 : 0;
  a.n_col_blocks = (n + kTile - 1) / kTile;
  a.row_begin = row_begin;
  a.row_end = row_end;
  a.n_row_blocks = sym ? a.n_col_blocks : (row_end - row_begin + kTile - 1) / kTile;
  const uint64_t all_tiles = sym ? (uint64_t)a.n_col_blocks * (a.n_col_blocks + 1) / 2
                                 : (uint64_t)a.n_row_blocks * a.n_col_blocks;
  if (!sym) { tile_begin = 0; tile_end = all_tiles; }
  tile_end = std::min(tile_end, all_tiles);
  if (tile_begin >= tile_end) { *used_tiles = true; return hipSuccess; }
  const uint64_t tiles = tile_end - tile_begin;
  uint32_t groups = (uint32_t)std::min<uint64_t>(B, std::max<uint64_t>(1, (2048 + tiles - 1) / tiles));
  a.buckets_per_group = (B + groups - 1) / groups;
  a.n_groups = (B + a.buckets_per_group - 1) / a.buckets_per_group;
  a.tile_begin = tile_begin;
  a.out = out;
  a.ld = n;
  if (use_join) {
    hipLaunchKernelGGL(k_join, dim3((unsigned)(tiles * a.n_groups)), dim3(kB), 0, s, a);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    *used_tiles = true;
    return hipSuccess;
  }
  const size_t lds_bytes = (size_t)std::max<uint32_t>(P, 1) * kSlots * sizeof(uint64_t) +
                           kSlots * sizeof(uint32_t);
  static const hipError_t attr = hipFuncSetAttribute(
      reinterpret_cast<const void*>(k_tiles), hipFuncAttributeMaxDynamicSharedMemorySize,
      (int)(kMaxPart * kSlots * sizeof(uint64_t) + kSlots * sizeof(uint32_t)));
  if (attr != hipSuccess) return attr;
  hipLaunchKernelGGL(k_tiles, dim3((unsigned)(tiles * a.n_groups)), dim3(kB), lds_bytes, s, a);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  *used_tiles = true;
  return hipSuccess;
}

uint64_t intersect_sym_tiles(uint32_t n) {
  uint64_t nb = (n + kTile - 1) / kTile;
  return nb * (nb + 1) / 2;
}

}  // namespace sks
