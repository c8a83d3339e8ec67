// Kernel 2 (default) — all-pairs intersection over block postings.
//
// The reference counts |A ∩ B| by probing the larger hash map for every
// element of the smaller set (kmer_set.cpp:23-41), one pair per cilk_for
// iteration (kmer_set.cpp:167-184).  Here the N x N matrix is cut into 64 x 64
// tiles of (row block, column block) of sketches, and a tile is a join of its
// two blocks' POSTINGS:
//
//   postings of a block = for every value held by any of its 64 sketches, the
//   value and a 64-bit mask of the sketches holding it, hash-bucketed (B
//   buckets of (v * φ) >> (64 - log_b)).
//
// Related genomes share most of their values, so a block holds each shared
// value once (config 4: ~2x fewer entries than elements), and the counts of a
// tile are a binary matrix product
//
//   count[r][c] = Σ_v R_v[r] · C_v[c]      (R_v, C_v: the value's row / column masks)
//
// over the values present in both blocks — GEMM-shaped, so it runs on the
// matrix cores: v_mfma_i32_32x32x32_i8 over 0/1 operands expanded from the
// masks.  The join itself only finds the shared values: the column block's
// postings of a chunk of buckets are scattered into an LDS hash table at
// positions the layout build precomputed (plain stores, no compare-swap), and
// every row posting probes it once.
//
// Layout (postings_build, three launches):
//   k_pl_sort    one workgroup per sketch: counting sort of its elements by
//                layout group (16 consecutive buckets) into `stage`
//   k_pl_groups  one workgroup per block: where each (block, group) starts
//   k_pl_place   one workgroup per (block, group): its elements from the 64
//                sketches' runs, deduplicated in an LDS hash table (masks OR-ed),
//                counted per bucket, and placed: every bucket's postings get a
//                linear-probing table of 2 slots per posting and each posting
//                its slot there (`pos`), written in bucket order.
// Per block k and bucket b: bkt[(k * B + b) * 2] = {first posting (relative to
// bstart[k]), count}; postings of one group are contiguous.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <vector>

#include "sks_internal.hpp"

namespace sks {

namespace {

constexpr int kPB = 256;                  // threads of the layout kernels
constexpr int kGLog = 4;                  // 16 buckets per layout group
constexpr int kGBK = 1 << kGLog;
constexpr uint32_t kPlMax = 4096;         // elements of one (block, group) k_pl_place holds
constexpr uint32_t kPlTab = 2 * kPlMax;   // its dedupe table (power of two)
constexpr uint32_t kPMaxLogB = 14;
constexpr int kJB = 512;                  // k_pjoin threads (8 waves)
constexpr uint32_t kTCap = 2048;          // LDS table slots of the join (16 B each)
constexpr uint32_t kPMaxDistinct = kTCap / 2;  // a bucket's table must fit one chunk
constexpr uint32_t kHCap = 1024;          // hit list entries (16 B each)
constexpr uint32_t kEmpty = 0xFFFFFFFFu;
constexpr uint64_t kMaxGrid = 1ull << 22;  // workgroups per launch slice

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

__host__ __device__ inline uint32_t pl_groups(uint32_t log_b) {
  return log_b > kGLog ? 1u << (log_b - kGLog) : 1u;
}
__host__ __device__ inline uint32_t pl_group_buckets(uint32_t log_b) {
  return log_b > kGLog ? (uint32_t)kGBK : 1u << log_b;
}
__device__ __forceinline__ uint32_t pbucket(uint64_t v, uint32_t log_b) {
  return log_b ? (uint32_t)((v * 0x9E3779B97F4A7C15ull) >> (64 - log_b)) : 0u;
}
// home slot of v in a bucket table of T slots (independent bits of another product)
__device__ __forceinline__ uint32_t phome(uint64_t v, uint32_t T) {
  const uint32_t h = (uint32_t)((v * 0xD6E8FEB86659FD93ull) >> 32);
  return (uint32_t)(((uint64_t)h * T) >> 32);
}
__device__ __forceinline__ uint32_t dedupe_home(uint64_t v) {
  return (uint32_t)((v * 0xC2B2AE3D27D4EB4Full) >> 40);
}
__device__ __forceinline__ uint32_t ptab(uint32_t d) { return 2 * d; }

// exclusive scan of n <= 4 * kPB values in LDS `a` (kPB threads); returns the total
__device__ uint32_t block_scan_excl(uint32_t* a, uint32_t n, uint32_t* s_wsum) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  uint32_t v[4], local = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const uint32_t i = 4 * tid + q;
    v[q] = i < n ? a[i] : 0;
    local += v[q];
  }
  uint32_t incl = local;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t t = __shfl_up(incl, o, 64);
    if (lane >= o) incl += t;
  }
  if (lane == 63) s_wsum[wave] = incl;
  __syncthreads();
  uint32_t before = 0, total = 0;
  for (int w = 0; w < kPB / 64; ++w) {
    if (w < wave) before += s_wsum[w];
    total += s_wsum[w];
  }
  uint32_t run = before + incl - local;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const uint32_t i = 4 * tid + q;
    if (i < n) a[i] = run;
    run += v[q];
  }
  __syncthreads();
  return total;
}

// One workgroup per sketch i = first + blockIdx.x: counting sort of its
// elements by layout group into stage[S[i] ..): gcnt / goff[(i - first) * G + g].
__global__ __launch_bounds__(kPB) void k_pl_sort(const uint64_t* __restrict__ data,
                                                 const uint64_t* __restrict__ starts,
                                                 const uint32_t* __restrict__ sizes, uint32_t first,
                                                 const uint64_t* __restrict__ S, uint32_t log_b,
                                                 uint64_t* __restrict__ stage,
                                                 uint32_t* __restrict__ gcnt,
                                                 uint32_t* __restrict__ goff) {
  __shared__ uint32_t s_h[1u << (kPMaxLogB - kGLog)];
  __shared__ uint32_t s_wsum[kPB / 64];
  const uint32_t G = pl_groups(log_b);
  const uint32_t gshift = log_b > kGLog ? kGLog : log_b;
  const uint32_t li = blockIdx.x, i = first + li;
  const uint32_t sz = sizes[i];
  const uint64_t* src = data + starts[i];
  for (uint32_t g = threadIdx.x; g < G; g += kPB) s_h[g] = 0;
  __syncthreads();
  uint32_t e = threadIdx.x;
  for (; e + 3 * kPB < sz; e += 4 * kPB) {
    uint64_t v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = src[e + u * kPB];
#pragma unroll
    for (int u = 0; u < 4; ++u) atomicAdd(&s_h[pbucket(v[u], log_b) >> gshift], 1u);
  }
  for (; e < sz; e += kPB) atomicAdd(&s_h[pbucket(src[e], log_b) >> gshift], 1u);
  __syncthreads();
  uint32_t* oc = gcnt + (uint64_t)li * G;
  for (uint32_t g = threadIdx.x; g < G; g += kPB) oc[g] = s_h[g];
  block_scan_excl(s_h, G, s_wsum);
  const uint64_t base = S[li];
  uint32_t* oo = goff + (uint64_t)li * G;
  for (uint32_t g = threadIdx.x; g < G; g += kPB) oo[g] = (uint32_t)(base + s_h[g]);
  __syncthreads();
  for (uint32_t g = threadIdx.x; g < G; g += kPB) s_h[g] += (uint32_t)base;  // cursors
  __syncthreads();
  e = threadIdx.x;
  for (; e + 3 * kPB < sz; e += 4 * kPB) {
    uint64_t v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = src[e + u * kPB];
#pragma unroll
    for (int u = 0; u < 4; ++u) stage[atomicAdd(&s_h[pbucket(v[u], log_b) >> gshift], 1u)] = v[u];
  }
  for (; e < sz; e += kPB) {
    const uint64_t v = src[e];
    stage[atomicAdd(&s_h[pbucket(v, log_b) >> gshift], 1u)] = v;
  }
}

// One workgroup per block k: gbase[k * G + g] = bstart[k] + elements of the
// block's groups before g (where group g's postings start).
__global__ __launch_bounds__(kPB) void k_pl_groups(const uint32_t* __restrict__ gcnt, uint32_t count,
                                                   uint32_t G, const uint64_t* __restrict__ bstart,
                                                   uint32_t* __restrict__ gbase) {
  __shared__ uint32_t s_c[1u << (kPMaxLogB - kGLog)];
  __shared__ uint32_t s_wsum[kPB / 64];
  const uint32_t k = blockIdx.x;
  const uint32_t s_end = min(64u, count - 64u * k);
  for (uint32_t g = threadIdx.x; g < G; g += kPB) {
    uint32_t t = 0;
    for (uint32_t s = 0; s < s_end; ++s) t += gcnt[(uint64_t)(64u * k + s) * G + g];
    s_c[g] = t;
  }
  __syncthreads();
  block_scan_excl(s_c, G, s_wsum);
  const uint32_t b0 = (uint32_t)bstart[k];
  for (uint32_t g = threadIdx.x; g < G; g += kPB) gbase[(uint64_t)k * G + g] = b0 + s_c[g];
}

// One workgroup per (block k, group g): dedupe + per-bucket tables.
// stat[0]: largest postings count of one bucket; stat[1]: largest (block,
// group) element count (the build is only valid while it is <= kPlMax).
__global__ __launch_bounds__(kPB) void k_pl_place(const uint64_t* __restrict__ stage,
                                                  const uint32_t* __restrict__ gcnt,
                                                  const uint32_t* __restrict__ goff,
                                                  const uint32_t* __restrict__ gbase,
                                                  const uint64_t* __restrict__ bstart, uint32_t count,
                                                  uint32_t log_b, uint64_t* __restrict__ ent,
                                                  uint16_t* __restrict__ pos,
                                                  uint32_t* __restrict__ bkt,
                                                  uint32_t* __restrict__ stat) {
  __shared__ uint64_t s_val[kPlMax];
  __shared__ unsigned long long s_msk[kPlMax];
  __shared__ uint32_t s_tab[kPlTab];
  __shared__ uint8_t s_sid[kPlMax];
  __shared__ uint32_t s_roff[64], s_rbeg[65];
  __shared__ uint32_t s_bcnt[kGBK], s_bbeg[kGBK + 1], s_tbeg[kGBK + 1];
  const uint32_t G = pl_groups(log_b), GB = pl_group_buckets(log_b);
  const uint32_t B = 1u << log_b;
  const uint32_t k = blockIdx.x / G, g = blockIdx.x % G;
  const uint32_t s_end = min(64u, count - 64u * k);
  const int tid = threadIdx.x, lane = tid & 63;
  // the 64 sketches' runs of this group (wave 0)
  if (tid < 64) {
    const uint32_t s = (uint32_t)tid;
    const uint64_t gi = (uint64_t)(64u * k + s) * G + g;
    const uint32_t c = s < s_end ? gcnt[gi] : 0;
    s_roff[s] = s < s_end ? goff[gi] : 0;
    uint32_t incl = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t t = __shfl_up(incl, o, 64);
      if (lane >= o) incl += t;
    }
    s_rbeg[s] = incl - c;
    if (s == 63) s_rbeg[64] = incl;
  }
  if (tid < kGBK) s_bcnt[tid] = 0;
  __syncthreads();
  const uint32_t n = s_rbeg[64];
  const uint64_t blk0 = bstart[k];
  const uint32_t gb = gbase[(uint64_t)k * G + g];  // first posting of the group
  uint32_t* bd = bkt + ((uint64_t)k * B + (uint64_t)g * GB) * 2;
  if (n > kPlMax) {  // the caller raises log_b and rebuilds
    if (tid == 0) atomicMax(&stat[1], n);
    for (uint32_t b = tid; b < GB; b += kPB) {
      bd[2 * b] = gb - (uint32_t)blk0;
      bd[2 * b + 1] = 0;
    }
    return;
  }
  // slot ids of the elements (a wave per run), then the elements themselves
  for (uint32_t s = tid >> 6; s < s_end; s += kPB / 64)
    for (uint32_t e = s_rbeg[s] + lane; e < s_rbeg[s + 1]; e += 64) s_sid[e] = (uint8_t)s;
  uint32_t TS = 64;  // dedupe table size: power of two >= 2n
  while (TS < 2 * n) TS <<= 1;
  for (uint32_t t = tid; t < TS; t += kPB) s_tab[t] = kEmpty;
  __syncthreads();
  for (uint32_t e = tid; e < n; e += kPB) {
    const uint32_t s = s_sid[e];
    s_val[e] = stage[s_roff[s] + (e - s_rbeg[s])];
    s_msk[e] = 1ull << s;
  }
  __syncthreads();
  // 1) dedupe: the first element to claim a value's slot owns it; the others OR
  //    their sketch bit into the owner's mask
  constexpr int kPer = kPlMax / kPB;  // elements per thread at most
  uint32_t own = 0;                   // bit u: element tid + u * kPB owns its value
#pragma unroll
  for (int u = 0; u < kPer; ++u) {
    const uint32_t e = tid + u * kPB;
    if (e >= n) break;
    const uint64_t v = s_val[e];
    uint32_t h = dedupe_home(v) & (TS - 1);
    // (the loop carries only h and x; the outcome is taken from x after it —
    // see k_join's lookup in intersect.hip)
    uint32_t x = atomicCAS(&s_tab[h], kEmpty, e);
    while (x != kEmpty && s_val[x] != v) {
      h = (h + 1) & (TS - 1);
      x = atomicCAS(&s_tab[h], kEmpty, e);
    }
    if (x == kEmpty)
      own |= 1u << u;
    else
      atomicOr(&s_msk[x], s_msk[e]);
  }
  __syncthreads();
  // 2) postings per bucket of the group
  uint32_t rank[kPer];
#pragma unroll
  for (int u = 0; u < kPer; ++u) {
    rank[u] = 0;
    if (own & (1u << u)) {
      const uint32_t e = tid + u * kPB;
      rank[u] = atomicAdd(&s_bcnt[pbucket(s_val[e], log_b) & (GB - 1)], 1u);
    }
  }
  __syncthreads();
  if (tid == 0) {
    uint32_t a = 0, t = 0, mx = 0;
    for (uint32_t b = 0; b < GB; ++b) {
      s_bbeg[b] = a;
      s_tbeg[b] = t;
      a += s_bcnt[b];
      t += ptab(s_bcnt[b]);
      mx = max(mx, s_bcnt[b]);
    }
    s_bbeg[GB] = a;
    s_tbeg[GB] = t;
    if (mx) atomicMax(&stat[0], mx);
  }
  __syncthreads();
  const uint32_t tabn = s_tbeg[GB];  // <= 2 * n <= TS
  for (uint32_t t = tid; t < tabn; t += kPB) s_tab[t] = kEmpty;
  for (uint32_t b = tid; b < GB; b += kPB) {
    bd[2 * b] = gb - (uint32_t)blk0 + s_bbeg[b];
    bd[2 * b + 1] = s_bcnt[b];
  }
  __syncthreads();
  // 3) each posting's slot in its bucket's linear-probing table (T = 2 d)
#pragma unroll
  for (int u = 0; u < kPer; ++u) {
    if (!(own & (1u << u))) continue;
    const uint32_t e = tid + u * kPB;
    const uint64_t v = s_val[e];
    const uint32_t lb = pbucket(v, log_b) & (GB - 1);
    const uint32_t T = ptab(s_bcnt[lb]), tb = s_tbeg[lb];
    uint32_t p = phome(v, T);
    while (atomicCAS(&s_tab[tb + p], kEmpty, 0u) != kEmpty) p = (p + 1 == T) ? 0 : p + 1;
    const uint64_t o = (uint64_t)gb + s_bbeg[lb] + rank[u];
    ent[2 * o] = v;
    ent[2 * o + 1] = s_msk[e];
    pos[o] = (uint16_t)p;
  }
}

// ---- k_pjoin ------------------------------------------------------------------------------
struct PJoinArgs {
  PostingsLayout r, c;  // row blocks (tile row I = block r_blk0 + I) and column blocks
  uint32_t r_blk0;
  uint32_t log_b, n, n_col_blocks, groups_per_wg, n_wg_per_tile;
  int sym;
  uint32_t row_begin, row_end;
  uint64_t tile_begin;
  const uint32_t* tiles;  // optional explicit tile list: tiles[2t] = I, tiles[2t + 1] = J
  int32_t* out;
  uint64_t ld;
  int packed;  // 1: out = [tile][64][64] (tile index relative to tile_begin)
};

// v_mfma_i32_32x32x32_i8 operand map (tools/microbench/mfma_i8_layout.hip):
// lane l holds A[row l & 31][k = 16 (l >> 5) + j] and B[k][col l & 31] in byte j.
__device__ __forceinline__ int mfma_k(int lane, int j) { return 16 * (lane >> 5) + j; }

__global__ __launch_bounds__(kJB) void k_pjoin(PJoinArgs a) {
  __shared__ ulonglong2 s_tab[kTCap];          // {value, column mask}; mask 0 = empty
  __shared__ ulonglong2 s_hit[kHCap];          // {row mask, column mask}
  __shared__ uint32_t s_cb[kGBK], s_cc[kGBK], s_rb[kGBK], s_rc[kGBK], s_tb[kGBK + 1];
  __shared__ uint32_t s_chunk[kGBK + 1], s_nchunk, s_nhit;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint64_t t = a.tile_begin + blockIdx.x / a.n_wg_per_tile;
  const uint32_t wg = blockIdx.x % a.n_wg_per_tile;
  uint32_t I, J;
  if (a.tiles) {
    I = a.tiles[2 * t];
    J = a.tiles[2 * t + 1];
  } else if (a.sym) {
    uint32_t i = 0;
    uint64_t rem = t;
    while (rem >= a.n_col_blocks - i) {
      rem -= a.n_col_blocks - i;
      ++i;
    }
    I = i;
    J = i + (uint32_t)rem;
  } else {
    I = (uint32_t)(t / a.n_col_blocks);
    J = (uint32_t)(t % a.n_col_blocks);
  }
  const bool rows_mode = !a.sym && !a.tiles;
  const uint32_t row0 = (rows_mode ? a.row_begin : 0) + I * 64;
  const uint32_t row_lim = rows_mode ? a.row_end : a.n;
  const uint32_t col0 = J * 64;
  const uint32_t r_valid = min(64u, row_lim - row0);
  const unsigned long long rmask = r_valid >= 64 ? ~0ull : ((1ull << r_valid) - 1);
  const uint32_t rblk = a.r_blk0 + I;
  // a diagonal tile joins a block with itself: its hits are the postings
  const bool self_tile = row0 == col0 && a.r.ent == a.c.ent;
  const uint32_t B = 1u << a.log_b, G = pl_groups(a.log_b), GB = pl_group_buckets(a.log_b);
  const uint64_t* cent = a.c.ent + 2 * a.c.bstart[J];
  const uint16_t* cpos = a.c.pos + a.c.bstart[J];
  const uint64_t* rent = a.r.ent + 2 * a.r.bstart[rblk];
  const uint32_t* cbkt = a.c.bkt + (uint64_t)J * B * 2;
  const uint32_t* rbkt = a.r.bkt + (uint64_t)rblk * B * 2;

  for (uint32_t i = tid; i < kTCap; i += kJB) s_tab[i] = make_ulonglong2(0, 0);
  if (tid == 0) s_nhit = 0;
  v16i acc = {};
  const int q = wave & 3, kh = wave >> 2;  // MFMA: quadrant (row half, column half), K half
  const int rh = q >> 1, ch = q & 1;

  // counts += Σ hits (rows ⊗ columns) on the matrix cores; nh hits in s_hit
  auto accumulate = [&](uint32_t nh) {
    const uint32_t npad = (nh + 63) & ~63u;
    for (uint32_t i = nh + tid; i < npad; i += kJB) s_hit[i] = make_ulonglong2(0, 0);
    __syncthreads();
    const uint32_t* hw = reinterpret_cast<const uint32_t*>(s_hit);
    const uint32_t bit = lane & 31;
    for (uint32_t kb = kh; kb * 32 < npad; kb += 2) {
      v4i fa, fb;
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        uint32_t wa = 0, wbv = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const uint32_t k = kb * 32 + mfma_k(lane, 4 * d + j);
          const uint32_t xr = hw[4 * k + rh], xc = hw[4 * k + 2 + ch];
          wa |= ((xr >> bit) & 1u) << (8 * j);
          wbv |= ((xc >> bit) & 1u) << (8 * j);
        }
        fa[d] = (int)wa;
        fb[d] = (int)wbv;
      }
      acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa, fb, acc, 0, 0, 0);
    }
    __syncthreads();
    if (tid == 0) s_nhit = 0;
    __syncthreads();
  };
  // append a hit (wave-aggregated); call from all lanes of the wave
  auto append = [&](bool hit, unsigned long long R, unsigned long long C) {
    const uint64_t bal = __ballot(hit);
    if (!bal) return;
    const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32),
                                                     __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
    uint32_t base = 0;
    if (lane == 0) base = atomicAdd(&s_nhit, (uint32_t)__popcll(bal));
    base = __shfl(base, 0, 64);
    if (hit) s_hit[base + below] = make_ulonglong2(R, C);
  };

  const uint32_t g0 = wg * a.groups_per_wg, g1 = min(G, g0 + a.groups_per_wg);
  for (uint32_t g = g0; g < g1; ++g) {
    __syncthreads();
    if (tid < (int)GB) {
      const uint32_t b = g * GB + tid;
      s_cb[tid] = cbkt[2 * b];
      s_cc[tid] = cbkt[2 * b + 1];
      s_rb[tid] = rbkt[2 * b];
      s_rc[tid] = rbkt[2 * b + 1];
    }
    __syncthreads();
    if (tid == 0) {  // chunks of whole buckets whose tables fit kTCap slots
      uint32_t nc = 0, tot = 0;
      s_chunk[0] = 0;
      for (uint32_t b = 0; b < GB; ++b) {
        // a bucket over the table (an invalid layout: the caller checks the
        // build's stat and redoes the call) is skipped, never overflows LDS
        if (ptab(s_cc[b]) > kTCap) s_cc[b] = 0;
        const uint32_t T = ptab(s_cc[b]);
        if (tot + T > kTCap) {
          s_chunk[++nc] = b;
          tot = 0;
        }
        s_tb[b] = tot;
        tot += T;
      }
      s_chunk[++nc] = GB;
      s_nchunk = nc;
    }
    __syncthreads();
    const uint32_t nchunk = s_nchunk;
    for (uint32_t ci = 0; ci < nchunk; ++ci) {
      const uint32_t bs = s_chunk[ci], be = s_chunk[ci + 1];
      const uint32_t cs = s_cb[bs], ce = s_cb[be - 1] + s_cc[be - 1];
      if (self_tile) {
        // rows = columns: every posting (v, M) is a hit M ⊗ M
        for (uint32_t base = cs; base < ce; base += kJB) {
          const uint32_t e = base + tid;
          unsigned long long M = 0;
          if (e < ce) M = cent[2 * e + 1];
          append(e < ce && (M & rmask), M & rmask, M);
          __syncthreads();
          const uint32_t nh = s_nhit;
          __syncthreads();
          if (nh > kHCap - kJB) accumulate(nh);
        }
        continue;
      }
      const uint32_t rs = s_rb[bs], re = s_rb[be - 1] + s_rc[be - 1];
      if (rs == re || cs == ce) continue;
      // column postings into the table at their precomputed slots
      uint32_t made[kTCap / 2 / kJB];
#pragma unroll
      for (int u = 0; u < (int)(kTCap / 2 / kJB); ++u) {
        made[u] = kEmpty;
        const uint32_t e = cs + tid + u * kJB;
        if (e < ce) {
          const uint64_t v = cent[2 * e];
          const unsigned long long M = cent[2 * e + 1];
          const uint32_t lb = pbucket(v, a.log_b) & (GB - 1);
          made[u] = s_tb[lb] + cpos[e];
          s_tab[made[u]] = make_ulonglong2(v, M);
        }
      }
      __syncthreads();
      // row postings probe
      for (uint32_t base = rs; base < re; base += kJB) {
        const uint32_t e = base + tid;
        bool hit = false;
        unsigned long long R = 0, C = 0;
        if (e < re) {
          const uint64_t v = rent[2 * e];
          R = rent[2 * e + 1] & rmask;
          const uint32_t lb = pbucket(v, a.log_b) & (GB - 1);
          const uint32_t T = ptab(s_cc[lb]);
          if (R && T) {
            const uint32_t tb = s_tb[lb];
            uint32_t p = phome(v, T);
            ulonglong2 x = s_tab[tb + p];
            while (x.y != 0 && x.x != v) {
              p = (p + 1 == T) ? 0 : p + 1;
              x = s_tab[tb + p];
            }
            hit = x.y != 0;
            C = x.y;
          }
        }
        append(hit, R, C);
        __syncthreads();
        const uint32_t nh = s_nhit;
        __syncthreads();
        if (nh > kHCap - kJB) accumulate(nh);
      }
      // free the chunk's slots (its probes are done: barrier above) before the
      // next chunk writes its own
#pragma unroll
      for (int u = 0; u < (int)(kTCap / 2 / kJB); ++u)
        if (made[u] != kEmpty) s_tab[made[u]].y = 0;
      __syncthreads();
    }
  }
  __syncthreads();
  const uint32_t nh_last = s_nhit;
  __syncthreads();
  if (nh_last) accumulate(nh_last);
  // flush: the K-half-1 waves hand their sums to the K-half-0 waves via LDS
  int* s_red = reinterpret_cast<int*>(s_tab);  // [quadrant][reg][lane]
  if (kh == 1)
#pragma unroll
    for (int r = 0; r < 16; ++r) s_red[(q * 16 + r) * 64 + lane] = acc[r];
  __syncthreads();
  if (kh == 1) return;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int v = acc[r] + s_red[(q * 16 + r) * 64 + lane];
    if (!v) continue;
    const uint32_t lr = 32 * rh + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
    const uint32_t lc = 32 * ch + (lane & 31);
    if (a.packed) {
      atomicAdd(&a.out[(t - a.tile_begin) * 4096 + lr * 64 + lc], v);
      continue;
    }
    const uint32_t gr = row0 + lr, gc = col0 + lc;
    if (gr >= row_lim || gc >= a.n) continue;
    const uint64_t orow = rows_mode ? gr - a.row_begin : gr;
    atomicAdd(&a.out[orow * a.ld + gc], v);
    if (!rows_mode && I != J) atomicAdd(&a.out[(uint64_t)gc * a.ld + gr], v);
  }
}

}  // namespace

uint32_t postings_log_b(uint32_t max_size) {
  // mean block-bucket population <= 128 elements
  uint32_t log_b = 0;
  while ((64ull * max_size >> log_b) > 128 && log_b < kPMaxLogB) ++log_b;
  return log_b;
}

uint32_t postings_max_distinct() { return kPMaxDistinct; }

size_t postings_bytes(uint32_t count, uint32_t log_b, uint64_t total) {
  const uint64_t n_blk = (count + 63) / 64, B = 1ull << log_b;
  auto al = [](uint64_t x) { return (x + 255) & ~(uint64_t)255; };
  return al(total * 16) + al(total * 2) + al(n_blk * B * 8) + al((n_blk + 1) * 8);
}

size_t postings_temp_bytes(uint32_t count, uint32_t log_b, uint64_t total) {
  const uint64_t n_blk = (count + 63) / 64, G = pl_groups(log_b);
  auto al = [](uint64_t x) { return (x + 255) & ~(uint64_t)255; };
  return al(total * 8) + 2 * al((uint64_t)count * G * 4) + al(n_blk * G * 4) + al((uint64_t)count * 8) +
         al(16);
}

hipError_t postings_build(const uint64_t* data, const uint64_t* starts, const uint32_t* sizes,
                          const uint32_t* h_sizes, uint32_t first, uint32_t count, uint32_t log_b,
                          void* out, void* temp, uint32_t* d_stat, PostingsLayout* L, hipStream_t s) {
  const uint64_t n_blk = (count + 63) / 64, B = 1ull << log_b, G = pl_groups(log_b);
  uint64_t total = 0;
  for (uint32_t i = 0; i < count; ++i) total += h_sizes[first + i];
  auto al = [](uint64_t x) { return (x + 255) & ~(uint64_t)255; };
  char* o = static_cast<char*>(out);
  uint64_t* ent = reinterpret_cast<uint64_t*>(o);
  o += al(total * 16);
  uint16_t* pos = reinterpret_cast<uint16_t*>(o);
  o += al(total * 2);
  uint32_t* bkt = reinterpret_cast<uint32_t*>(o);
  o += al(n_blk * B * 8);
  uint64_t* bstart = reinterpret_cast<uint64_t*>(o);
  char* w = static_cast<char*>(temp);
  uint64_t* stage = reinterpret_cast<uint64_t*>(w);
  w += al(total * 8);
  uint32_t* gcnt = reinterpret_cast<uint32_t*>(w);
  w += al((uint64_t)count * G * 4);
  uint32_t* goff = reinterpret_cast<uint32_t*>(w);
  w += al((uint64_t)count * G * 4);
  uint32_t* gbase = reinterpret_cast<uint32_t*>(w);
  w += al(n_blk * G * 4);
  uint64_t* S = reinterpret_cast<uint64_t*>(w);
  // host offsets: each sketch's stage run and each block's postings region
  std::vector<uint64_t> hs(count + n_blk + 1);
  uint64_t acc = 0;
  for (uint32_t i = 0; i < count; ++i) {
    if (i % 64 == 0) hs[count + i / 64] = acc;
    hs[i] = acc;
    acc += h_sizes[first + i];
  }
  hs[count + n_blk] = acc;
  hipError_t e;
  // S and bstart are uploaded together: S = hs[0, count), bstart = hs[count, ..)
  if ((e = pinned_h2d(S, hs.data(), count * 8, s)) != hipSuccess) return e;
  if ((e = pinned_h2d(bstart, hs.data() + count, (n_blk + 1) * 8, s)) != hipSuccess) return e;
  if (L) *L = PostingsLayout{ent, pos, bkt, bstart};
  if (count == 0) return hipSuccess;
  hipLaunchKernelGGL(k_pl_sort, dim3(count), dim3(kPB), 0, s, data, starts, sizes, first, S, log_b,
                     stage, gcnt, goff);
  hipLaunchKernelGGL(k_pl_groups, dim3((unsigned)n_blk), dim3(kPB), 0, s, gcnt, count, (uint32_t)G,
                     bstart, gbase);
  hipLaunchKernelGGL(k_pl_place, dim3((unsigned)(n_blk * G)), dim3(kPB), 0, s, stage, gcnt, goff,
                     gbase, bstart, count, log_b, ent, pos, bkt, d_stat);
  return hipGetLastError();
}

hipError_t postings_join(const PostingsLayout& rows, uint32_t r_blk0, const PostingsLayout& cols,
                         uint32_t n, uint32_t log_b, bool sym, uint32_t row_begin, uint32_t row_end,
                         uint64_t tile_begin, uint64_t tile_end, const uint32_t* d_tiles,
                         bool packed, int32_t* out, hipStream_t s) {
  const uint32_t n_cb = (n + 63) / 64;
  const uint32_t n_rb = sym ? n_cb : (row_end - row_begin + 63) / 64;
  if (!d_tiles) {
    const uint64_t all = sym ? (uint64_t)n_cb * (n_cb + 1) / 2 : (uint64_t)n_rb * n_cb;
    if (!sym) {
      tile_begin = 0;
      tile_end = all;
    }
    tile_end = std::min(tile_end, all);
  }
  if (tile_begin >= tile_end) return hipSuccess;
  const uint64_t tiles = tile_end - tile_begin;
  const uint32_t G = pl_groups(log_b);
  PJoinArgs ja{};
  ja.r = rows;
  ja.c = cols;
  ja.r_blk0 = r_blk0;
  ja.log_b = log_b;
  ja.n = n;
  ja.n_col_blocks = n_cb;
  ja.sym = sym ? 1 : 0;
  ja.row_begin = row_begin;
  ja.row_end = row_end;
  ja.tiles = d_tiles;
  ja.out = out;
  ja.ld = n;
  ja.packed = packed ? 1 : 0;
  // groups per workgroup: ~4 groups (64 buckets) each while the grid is small,
  // at least ~1024 workgroups in all (SKS_PJOIN_WGS: total, diagnostics)
  static const uint64_t wgs_env = getenv("SKS_PJOIN_WGS") ? strtoull(getenv("SKS_PJOIN_WGS"), 0, 10) : 0;
  uint64_t per_tile = wgs_env ? (wgs_env + tiles - 1) / tiles
                              : std::max<uint64_t>(std::min<uint64_t>((G + 3) / 4, (65536 + tiles - 1) / tiles),
                                                   (1024 + tiles - 1) / tiles);
  per_tile = std::min<uint64_t>(std::max<uint64_t>(per_tile, 1), G);
  ja.groups_per_wg = (uint32_t)((G + per_tile - 1) / per_tile);
  ja.n_wg_per_tile = (G + ja.groups_per_wg - 1) / ja.groups_per_wg;
  const uint64_t tiles_per_launch = std::max<uint64_t>(1, kMaxGrid / ja.n_wg_per_tile);
  for (uint64_t t0 = tile_begin; t0 < tile_end; t0 += tiles_per_launch) {
    const uint64_t nt = std::min(tiles_per_launch, tile_end - t0);
    ja.tile_begin = t0;
    if (packed && t0 != tile_begin) ja.out = out + (t0 - tile_begin) * 4096;
    if (packed) ja.tile_begin = t0;  // packed index is relative to this slice's first tile
    hipLaunchKernelGGL(k_pjoin, dim3((unsigned)(nt * ja.n_wg_per_tile)), dim3(kJB), 0, s, ja);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

}  // namespace sks
