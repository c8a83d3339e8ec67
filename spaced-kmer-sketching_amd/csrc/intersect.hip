// Kernel 2 — pairwise sketch intersection counts.
//
// The reference counts |A ∩ B| by iterating the smaller kmer_set and probing
// the larger hash map (kmer_set.cpp:23-41), one pair per cilk_for iteration
// (kmer_set.cpp:167-184).  Sketches here are sorted unique arrays, so a pair
// is a sorted-merge count — the same integer the reference computes.
//   * k_join (join.hip, over the join layout of layout.hip): the all-pairs
//     path (u64 and 128-bit k-mers); launch_intersect_tiled below builds the
//     layout and dispatches.
//   * k_tiles: 64 x 64 tiles of pairwise LDS merges (u64; SKS_INTERSECT_MERGE,
//     and the fallback when a join layout cannot be built).
//   * k_pairs / k_all: one 64-lane wavefront per pair straight from global
//     memory — pair lists, and the fallback for pathological value skew.  The smaller sketch is split evenly over the lanes, each lane
//     lower_bounds its first element in the larger one and merges forward.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <cstdint>
#include <mutex>
#include <unordered_map>
#include <vector>

#include <rocprim/rocprim.hpp>

#include "join_common.hpp"
#include "sks_internal.hpp"

namespace sks {

namespace {

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

// bucket counts learned per largest-sketch size: a join whose layout had
// buckets above the table's capacity makes later calls on that size start with
// more buckets (the call itself keeps its exact sub-chunked counts)
static std::mutex g_log_b_mu;
static std::unordered_map<uint32_t, uint32_t> g_log_b_min;
static uint32_t start_log_b(uint32_t max_size) {
  std::lock_guard<std::mutex> lk(g_log_b_mu);
  const auto it = g_log_b_min.find(max_size);
  return std::max(join_log_b(max_size), it == g_log_b_min.end() ? 0u : it->second);
}
static void bump_log_b(uint32_t max_size, uint32_t log_b) {
  std::lock_guard<std::mutex> lk(g_log_b_mu);
  uint32_t& x = g_log_b_min[max_size];
  x = std::max(x, log_b);
}

// Tiled all-pairs (ew = 1: u64 k-mers, join or merge tiles; ew = 2: 128-bit
// k-mers, join only).  Host-synchronous (reads the sizes and the layout's
// statistics back to pick the bucket count).  mode: sym (upper-triangle tiles
// [tile_begin, tile_end) into a full n x n matrix) or rows.  check: the
// invariant-checking kernel builds (sks_ctx_set_join_check).
hipError_t launch_intersect_tiled(const uint64_t* data, const uint64_t* starts, const uint32_t* sizes,
                                  uint32_t n, bool sym, uint32_t row_begin, uint32_t row_end,
                                  uint64_t tile_begin, uint64_t tile_end, int32_t* out,
                                  Scratch& work, hipStream_t s, bool* used_tiles, int algo, int ew,
                                  bool check) {
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
  if ((algo != kIntersectMerge || ew == 2) && join_fits) {
    // the join layout of the column sketches (and of the row range when its
    // blocks are not aligned with the column blocks), then k_join
    const bool sep_rows = !sym && (row_begin % kTile) != 0;
    const uint32_t rn = row_end - row_begin;
    uint64_t r_total = 0;
    if (sep_rows)
      for (uint32_t i = row_begin; i < row_end; ++i) r_total += h_sizes[i];
    uint32_t log_b = start_log_b(max_size);
    for (;;) {
      const uint32_t BW = jc::lay_boff_words(log_b), G = jc::lay_groups(log_b);
      const size_t tmp_c = join_layout_temp_bytes(n, log_b, ew);
      const size_t tmp_r = !sep_rows ? 0 : join_layout_temp_bytes(rn, log_b, ew);
      size_t o = 0;
      const size_t o_cval = o; o = align16(o + total * 8 * ew);
      const size_t o_cmsk = o; o = align16(o + total * 8);
      const size_t o_cbof = o; o = align16(o + (size_t)n_cb * BW * 4);
      const size_t o_cbst = o; o = align16(o + (size_t)(n_cb + 1) * 8);
      const size_t o_rval = o; o = align16(o + r_total * 8 * ew);
      const size_t o_rmsk = o; o = align16(o + r_total * 8);
      const size_t o_rbof = o; o = align16(o + (sep_rows ? (size_t)n_rb * BW * 4 : 0));
      const size_t o_rbst = o; o = align16(o + (sep_rows ? (size_t)(n_rb + 1) * 8 : 0));
      const size_t o_stat = o; o = align16(o + 16);
      const size_t o_bnd = o; o = align16(o + (size_t)(G + 1) * 8 * ew);
      const size_t o_tmp = o; o = align16(o + std::max(tmp_c, tmp_r));
      if ((e = work.reserve(o)) != hipSuccess) return e;
      char* w = static_cast<char*>(work.ptr);
      auto lay_at = [&](size_t ov, size_t om, size_t ob, size_t os) {
        return JoinLayout{reinterpret_cast<uint64_t*>(w + ov), reinterpret_cast<uint64_t*>(w + om),
                          reinterpret_cast<uint32_t*>(w + ob), reinterpret_cast<uint64_t*>(w + os)};
      };
      const JoinLayout cl = lay_at(o_cval, o_cmsk, o_cbof, o_cbst);
      const JoinLayout rl = sep_rows ? lay_at(o_rval, o_rmsk, o_rbof, o_rbst) : cl;
      uint32_t* stat = reinterpret_cast<uint32_t*>(w + o_stat);
      if ((e = hipMemsetAsync(stat, 0, 8, s)) != hipSuccess) return e;
      // a separate row layout shares the column set's group bounds; a single
      // layout computes its own in the build's first launch (three in all)
      uint64_t* gbounds = sep_rows ? reinterpret_cast<uint64_t*>(w + o_bnd) : nullptr;
      if (sep_rows && (e = join_layout_bounds(data, starts, sizes, n, log_b, ew, gbounds, s)) != hipSuccess)
        return e;
      auto build_layout = [&](uint32_t first, uint32_t cnt, const JoinLayout& L) -> hipError_t {
        return join_layout_build(data, starts + first, sizes + first, cnt, log_b, ew, gbounds, w + o_tmp,
                                 const_cast<uint64_t*>(L.vals), const_cast<uint64_t*>(L.masks),
                                 const_cast<uint32_t*>(L.boff), const_cast<uint64_t*>(L.bstart), stat, check, s);
      };
      if ((e = build_layout(0, n, cl)) != hipSuccess) return e;
      if (sep_rows && (e = build_layout(row_begin, rn, rl)) != hipSuccess) return e;
      // the join runs right behind the build (no host round trip between them);
      // the build's status words are read back after it: an invalid layout (a
      // group the build could not place: adversarial 128-bit values) discards
      // the counts and retries with more buckets.  Buckets above the table's
      // capacity are joined in sub-chunks (exact; their row entries are probed
      // once per sub-chunk) and only make the next call on these sizes start
      // with more buckets.
      const uint32_t r_blk0 = sep_rows ? 0 : (sym ? 0 : row_begin / kTile);
      if ((e = join_launch(rl, r_blk0, cl, 0, n, log_b, ew, sym, row_begin, row_end, tile_begin, tile_end,
                           nullptr, false, out, check, s)) != hipSuccess)
        return e;
      uint32_t h_stat[2] = {0, 0};
      if ((e = pinned_d2h(h_stat, stat, 8, s)) != hipSuccess) return e;
      if (dbg)
        fprintf(stderr, "[sks intersect] join n=%u ew=%d B=%u max block bucket %u invalid %u tiles=%llu\n", n, ew,
                1u << log_b, h_stat[0], h_stat[1], (unsigned long long)tiles);
      if (h_stat[1]) {
        if ((e = hipMemsetAsync(out, 0, out_words * sizeof(int32_t), s)) != hipSuccess) return e;
        if (log_b < jc::kMaxLogB) { ++log_b; continue; }
        break;
      }
      if (h_stat[0] > join_cap() && log_b < jc::kMaxLogB) bump_log_b(max_size, log_b + 1);
      *used_tiles = true;
      return hipSuccess;
    }
  }
  if (ew != 1) return hipSuccess;  // the merge tiles take u64 k-mers: one wavefront per pair

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

SKS_CODE_OBJECT_HOOK(intersect)

}  // namespace sks
