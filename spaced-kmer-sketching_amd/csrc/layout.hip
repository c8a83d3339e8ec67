// The join layout (input of k_join, intersect.hip): for every block of 64
// consecutive sketches, its elements bucket by bucket, sketch by sketch, with
// each element's slot in the block in a u8 id array, the per-block bucket
// starts boff[blk][0..B] and the block starts bstart[0..n_blk].
//
// Buckets are two-level.  The value range is cut into G = B / 16 groups by
// common bounds (quantiles averaged over up to 64 sample sketches), and a
// group's 16 buckets are chosen by a hash of the value.  The two levels serve
// two masters:
//   * every sketch is sorted, so its part of a value group is ONE contiguous
//     range (two binary searches): the build reads each sketch's part straight
//     from the sketch, with no counting or staging pass over the whole set
//     (round 2's all-hash build: count, column sums, scan, offsets, staging
//     copy, placement — six launches and ~0.19 ms for config 4);
//   * within a group the buckets are hashed, so a block's bucket populations are
//     Poisson.  Fine value-range buckets are lumpy for related sketches (a
//     bucket that is large for one member of a family is large for all 64 of
//     its block: k_join over a value-range layout ran 1.2 instead of 0.6 ms,
//     DESIGN.md §5), while a group of ~2.7k block elements averages that out.
// Counts are exact for any non-decreasing bounds; all layouts whose blocks are
// joined with each other (a multi-GPU gather) must share one bounds array.
//
// Build (join_layout_build), three launches: k_gl_prep (the group bounds when
// the caller gives none, and the block starts), k_gl_pos (every sketch's group
// starts: a workgroup per sketch), then k_gl_place, one workgroup per
// (block, group): the group's elements read once into registers, a (bucket x
// slot) histogram in LDS, its scans (the block's bucket starts and each
// (bucket, slot) cursor), and the scatter into LDS, copied out to the group's
// own contiguous part of the layout with contiguous stores.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

#include "sks_internal.hpp"

namespace sks {

namespace {

constexpr int kTile = 64;
constexpr int kGB = 16;    // hash buckets per value group
constexpr int kGLog = 4;
// a (block, group) of at most this many elements is assembled in LDS and
// written out with contiguous stores; a larger one (skewed values) scatters
// straight to global memory
constexpr uint32_t kGCap = 4096;
constexpr int kPT = 256;   // threads of the layout kernels
constexpr uint32_t kMaxLogB = 14;

__device__ __forceinline__ uint32_t group_bucket(uint64_t v, uint32_t gb_log) {
  return gb_log ? (uint32_t)((v * 0x9E3779B97F4A7C15ull) >> (64 - gb_log)) : 0u;
}

// inclusive prefix sum over the 64 lanes of a wave (DPP; no LDS)
__device__ __forceinline__ uint32_t wave_scan(uint32_t v) {
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false);  // row_shr:1
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false);  // row_shr:2
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false);  // row_shr:4
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false);  // row_shr:8
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);  // row_bcast:15
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);  // row_bcast:31
  return v;
}

// Workgroups [0, nb_bounds): the group bounds, a wave per bound (bounds[g] =
// mean over up to 64 sample sketches of their g/G quantile; bounds[0] = 0,
// bounds[G] = 2^64 - 1).  The last workgroup: bstart[k] = elements of the
// blocks before k (a running scan over the sketches' sizes).
__global__ __launch_bounds__(kPT) void k_gl_prep(const uint64_t* __restrict__ data,
                                                 const uint64_t* __restrict__ starts,
                                                 const uint32_t* __restrict__ sizes, uint32_t count,
                                                 uint32_t G, uint64_t* __restrict__ bounds,
                                                 uint32_t nb_bounds, uint64_t* __restrict__ bstart) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (blockIdx.x < nb_bounds) {
    const uint32_t g = blockIdx.x * (kPT / 64) + wave;
    if (g > G) return;
    const uint32_t K = min(count, 64u);
    double x = 0.0, used = 0.0;
    if ((uint32_t)lane < K && g > 0 && g < G) {
      const uint32_t i = (uint32_t)((uint64_t)lane * count / K);
      const uint32_t sz = sizes[i];
      if (sz) {
        x = (double)data[starts[i] + (uint64_t)g * sz / G];
        used = 1.0;
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      x += __shfl_xor(x, o, 64);
      used += __shfl_xor(used, o, 64);
    }
    if (lane) return;
    if (g == 0) {
      bounds[0] = 0;
    } else if (g == G) {
      bounds[G] = ~0ull;
    } else {
      const double m = used > 0.0 ? x / used : 0.0;
      bounds[g] = m >= 18446744073709549568.0 ? ~0ull : (uint64_t)m;
    }
    return;
  }
  // block starts: thread t sums block (base + t)'s sizes, then a block scan
  __shared__ unsigned long long s_w[kPT / 64];
  const uint32_t n_blk = (count + kTile - 1) / kTile;
  unsigned long long carry = 0;
  for (uint32_t base = 0; base < n_blk; base += kPT) {
    const uint32_t k = base + tid;
    unsigned long long t = 0;
    if (k < n_blk)
      for (uint32_t i = k * kTile; i < min(count, k * kTile + kTile); ++i) t += sizes[i];
    unsigned long long incl = t;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const unsigned long long y = __shfl_up(incl, o, 64);
      if (lane >= o) incl += y;
    }
    if (lane == 63) s_w[wave] = incl;
    __syncthreads();
    unsigned long long before = carry;
    for (int w = 0; w < wave; ++w) before += s_w[w];
    if (k < n_blk) bstart[k] = before + incl - t;
    if (k == n_blk - 1) bstart[n_blk] = before + incl;
    unsigned long long tot = 0;
    for (int w = 0; w < kPT / 64; ++w) tot += s_w[w];
    __syncthreads();
    carry += tot;
  }
}

// pos[i][g] = first element of sketch i in value group g (lower bound of
// bounds[g]; pos[i][0] = 0, pos[i][G] = size).  A workgroup per sketch stages
// every kPosStride-th element in LDS with one coalesced pass, and a thread per
// bound searches that sample and then the one cache line it points at.  (A
// thread per (sketch, bound) binary-searching the sketch took 21 us for config
// 4: the threads of a sketch share the top of the search tree, so its last ~6
// levels are the dependent misses — which is also why a 64-element sample,
// leaving 6 levels to search in global memory, measured the same.)  This
// version: 19.8 us — a stride-8 sample touches every 64-B line of the sketch,
// so the launch is bound by reading the sketches once (80 MB).  A sketch
// above kPosSamples * kPosStride elements samples with a larger stride.
constexpr uint32_t kPosStride = 8, kPosSamples = 2048;
__global__ __launch_bounds__(kPT) void k_gl_pos(const uint64_t* __restrict__ data,
                                                const uint64_t* __restrict__ starts,
                                                const uint32_t* __restrict__ sizes, uint32_t count,
                                                uint32_t G, const uint64_t* __restrict__ bounds,
                                                uint32_t* __restrict__ pos) {
  __shared__ uint64_t s_smp[kPosSamples];
  const uint32_t i = blockIdx.x;
  const uint32_t sz = sizes[i];
  const uint64_t* S = data + starts[i];
  uint32_t stride = kPosStride;
  while ((uint64_t)stride * kPosSamples < sz) stride <<= 1;
  const uint32_t ns = (sz + stride - 1) / stride;  // sample k = S[k * stride]
  for (uint32_t k = threadIdx.x; k < ns; k += kPT) s_smp[k] = S[(uint64_t)k * stride];
  __syncthreads();
  uint32_t* out = pos + (uint64_t)i * (G + 1);
  for (uint32_t g = threadIdx.x; g <= G; g += kPT) {
    if (g == 0 || g == G) {
      out[g] = g == 0 ? 0 : sz;
      continue;
    }
    const uint64_t x = bounds[g];
    // lo = samples below x: the lower bound lies in ((lo - 1) * stride, lo * stride]
    uint32_t lo = 0, hi = ns;
    while (lo < hi) {
      const uint32_t mid = (lo + hi) >> 1;
      if (s_smp[mid] < x) lo = mid + 1; else hi = mid;
    }
    uint32_t a = lo ? (lo - 1) * stride + 1 : 0, e = min(sz, lo * stride);
    while (a < e) {
      const uint32_t mid = (a + e) >> 1;
      if (S[mid] < x) a = mid + 1; else e = mid;
    }
    out[g] = a;
  }
}

// One workgroup per (block, value group).  A group of at most kGCap elements
// (the normal case) is read ONCE: its elements are spread over all 256 threads
// (element i of the group -> its sketch through an owner map in LDS) and held in
// registers through the histogram, the scans and the scatter into LDS, then
// copied out with contiguous stores.  A larger group (skewed values) takes a
// wave per sketch, reads it twice and scatters straight to global memory.
// (Round 3's first version took the wave-per-sketch loops for every group:
// ~39 elements per sketch and group left a third of the lanes idle behind
// serial load -> atomic chains; config 4: 127 us, now 66 us.  Scattering
// straight to global memory instead of assembling in LDS — 10 instead of 47 KB
// of LDS, twice the workgroups per CU — measured the same, 68 us.)
__global__ __launch_bounds__(kPT) void k_gl_place(const uint64_t* __restrict__ data,
                                                  const uint64_t* __restrict__ starts,
                                                  const uint32_t* __restrict__ sizes, uint32_t count,
                                                  uint32_t log_b, const uint32_t* __restrict__ pos,
                                                  const uint64_t* __restrict__ bstart,
                                                  uint64_t* __restrict__ out_data,
                                                  uint8_t* __restrict__ out_ids,
                                                  uint32_t* __restrict__ out_boff,
                                                  uint32_t* __restrict__ stat) {
  // counts, then cursors, [slot][bucket]; the row pad puts the lanes of the
  // scans (one bucket, all slots) on distinct banks
  __shared__ uint32_t s_cnt[kTile][kGB + 1];
  __shared__ uint64_t s_out[kGCap];
  __shared__ uint8_t s_oid[kGCap];
  __shared__ uint8_t s_own[kGCap];  // group element i -> its sketch's slot
  __shared__ uint64_t s_src[kTile];  // data index of slot s's group element i: s_src[s] + i
  __shared__ uint32_t s_lo[kTile], s_hi[kTile], s_pre[kTile];
  __shared__ uint32_t s_btot[kGB];
  __shared__ uint32_t s_gstart, s_gn;
  const uint32_t B = 1u << log_b;
  const uint32_t gb_log = log_b < kGLog ? log_b : kGLog, GB = 1u << gb_log;
  const uint32_t G = B >> gb_log;
  const uint32_t blk = blockIdx.x / G, g = blockIdx.x % G;
  const uint32_t s_end = min((uint32_t)kTile, count - kTile * blk);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (uint32_t i = tid; i < kTile * (kGB + 1); i += kPT) (&s_cnt[0][0])[i] = 0;
  // each sketch's range in the group (k_gl_pos), the group's start in the
  // block (the sum of the ranges' starts) and the element prefix over sketches
  if (wave == 0) {
    uint32_t lo = 0, hi = 0;
    uint64_t st = 0;
    if ((uint32_t)lane < s_end) {
      const uint32_t* p = pos + (uint64_t)(kTile * blk + lane) * (G + 1) + g;
      lo = p[0];
      hi = max(p[1], lo);  // (non-decreasing bounds: only a guard)
      st = starts[kTile * blk + lane];
    }
    const uint32_t c = hi - lo;
    const uint32_t below = wave_scan(lo);
    const uint32_t incl = wave_scan(c);
    s_lo[lane] = lo;
    s_hi[lane] = hi;
    s_pre[lane] = incl - c;
    s_src[lane] = st + lo - (incl - c);
    if (lane == 63) {
      s_gstart = below;
      s_gn = incl;
    }
  }
  __syncthreads();
  const uint32_t g_lo = s_gstart;  // the group's first element (block-relative)
  const uint32_t g_n = s_gn;
  const bool in_lds = g_n <= kGCap;
  constexpr int kPer = kGCap / kPT;
  uint64_t v[kPer];
  // 1) (slot, bucket) histogram
  if (in_lds) {
    for (uint32_t s = wave; s < s_end; s += kPT / 64)
      for (uint32_t j = s_pre[s] + lane; j < s_pre[s] + (s_hi[s] - s_lo[s]); j += 64) s_own[j] = (uint8_t)s;
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
      const uint32_t i = tid + k * kPT;
      if (i < g_n) v[k] = data[s_src[s_own[i]] + i];
    }
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
      const uint32_t i = tid + k * kPT;
      if (i < g_n) atomicAdd(&s_cnt[s_own[i]][group_bucket(v[k], gb_log)], 1u);
    }
  } else {
    for (uint32_t s = wave; s < s_end; s += kPT / 64) {
      const uint64_t* S = data + starts[kTile * blk + s];
      for (uint32_t e = s_lo[s] + lane; e < s_hi[s]; e += 64) atomicAdd(&s_cnt[s][group_bucket(S[e], gb_log)], 1u);
    }
  }
  __syncthreads();
  // 2) per bucket: slot prefix (a wave scan) and total; lane s of wave w holds
  //    bucket w + 4i's slot-s count
  for (uint32_t b = wave; b < GB; b += kPT / 64) {
    const uint32_t c = s_cnt[lane][b];
    const uint32_t incl = wave_scan(c);
    s_cnt[lane][b] = incl - c;
    if (lane == 63) s_btot[b] = incl;
  }
  __syncthreads();
  // 3) bucket starts (relative to the block) and cursors
  if (wave == 0) {
    const uint32_t t = (uint32_t)lane < GB ? s_btot[lane] : 0;
    const uint32_t incl = wave_scan(t);
    const uint32_t start = g_lo + incl - t;
    if ((uint32_t)lane < GB) {
      out_boff[(uint64_t)blk * (B + 1) + g * GB + lane] = start;
      s_btot[lane] = start;
    }
    if (lane == 63 && g + 1 == G) out_boff[(uint64_t)blk * (B + 1) + B] = g_lo + incl;
    uint32_t mx = t;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) mx = max(mx, (uint32_t)__shfl_xor(mx, o, 64));
    // one word for all 4096 workgroups: a device-scope atomic per workgroup
    // would serialise (one word takes ~88 atomics per microsecond,
    // MI355X_MICROARCH.md "dequeue"); the stat only grows, so a workgroup whose
    // maximum is not above the value it reads skips the atomic (a stale read
    // only costs an atomic)
    if (lane == 0 && mx && mx > __hip_atomic_load(stat, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
      atomicMax(stat, mx);
  }
  __syncthreads();
  for (uint32_t i = tid; i < kTile * GB; i += kPT) s_cnt[i / GB][i % GB] += s_btot[i % GB];
  __syncthreads();
  // 4) scatter: every element to its (bucket, slot) cell of the group's own
  //    contiguous part of the block
  const uint64_t base = bstart[blk];
  if (!in_lds) {
    for (uint32_t s = wave; s < s_end; s += kPT / 64) {
      const uint64_t* S = data + starts[kTile * blk + s];
      for (uint32_t e = s_lo[s] + lane; e < s_hi[s]; e += 64) {
        const uint64_t x = S[e];
        const uint32_t d = atomicAdd(&s_cnt[s][group_bucket(x, gb_log)], 1u);
        out_data[base + d] = x;
        out_ids[base + d] = (uint8_t)s;
      }
    }
    return;
  }
#pragma unroll
  for (int k = 0; k < kPer; ++k) {
    const uint32_t i = tid + k * kPT;
    if (i < g_n) {
      const uint32_t s = s_own[i];
      const uint32_t d = atomicAdd(&s_cnt[s][group_bucket(v[k], gb_log)], 1u) - g_lo;
      s_out[d] = v[k];
      s_oid[d] = (uint8_t)s;
    }
  }
  __syncthreads();
  uint64_t* od = out_data + base + g_lo;
  uint8_t* oi = out_ids + base + g_lo;
  for (uint32_t i = tid; i < g_n; i += kPT) {
    od[i] = s_out[i];
    oi[i] = s_oid[i];
  }
}

}  // namespace

uint32_t join_layout_groups(uint32_t log_b) { return log_b > kGLog ? 1u << (log_b - kGLog) : 1u; }

hipError_t join_layout_bounds(const uint64_t* data, const uint64_t* starts, const uint32_t* sizes,
                              uint32_t count, uint32_t log_b, uint64_t* bounds, hipStream_t s) {
  if (log_b > kMaxLogB) return hipErrorInvalidValue;
  const uint32_t G = join_layout_groups(log_b);
  hipLaunchKernelGGL(k_gl_prep, dim3((G + 1 + kPT / 64 - 1) / (kPT / 64)), dim3(kPT), 0, s, data, starts,
                     sizes, count, G, bounds, (G + 1 + kPT / 64 - 1) / (kPT / 64), (uint64_t*)nullptr);
  return hipGetLastError();
}

size_t join_layout_temp_bytes(uint32_t count, uint32_t log_b) {
  const uint64_t G = join_layout_groups(log_b);
  return ((G + 1) * 8 + 255) / 256 * 256 + (uint64_t)count * (G + 1) * 4;
}

hipError_t join_layout_build(const uint64_t* data, const uint64_t* starts, const uint32_t* sizes,
                             uint32_t count, uint32_t log_b, const uint64_t* d_bounds, void* temp,
                             uint64_t* out_data, uint8_t* out_ids, uint32_t* out_boff,
                             uint64_t* out_bstart, uint32_t* d_stat, hipStream_t s) {
  if (log_b > kMaxLogB) return hipErrorInvalidValue;
  if (count == 0) return hipSuccess;
  const uint32_t G = join_layout_groups(log_b);
  const uint32_t n_blk = (count + kTile - 1) / kTile;
  uint64_t* bounds_tmp = static_cast<uint64_t*>(temp);
  uint32_t* pos = reinterpret_cast<uint32_t*>(static_cast<char*>(temp) + ((G + 1) * 8 + 255) / 256 * 256);
  // bounds (unless given) and block starts in one launch, the groups' positions
  // in every sketch, then the placement
  const uint32_t nb_bounds = d_bounds ? 0 : (G + 1 + kPT / 64 - 1) / (kPT / 64);
  hipLaunchKernelGGL(k_gl_prep, dim3(nb_bounds + 1), dim3(kPT), 0, s, data, starts, sizes, count, G,
                     bounds_tmp, nb_bounds, out_bstart);
  const uint64_t* bounds = d_bounds ? d_bounds : bounds_tmp;
  hipLaunchKernelGGL(k_gl_pos, dim3(count), dim3(kPT), 0, s, data, starts, sizes, count, G, bounds, pos);
  hipLaunchKernelGGL(k_gl_place, dim3(n_blk * G), dim3(kPT), 0, s, data, starts, sizes, count, log_b, pos,
                     out_bstart, out_data, out_ids, out_boff, d_stat);
  return hipGetLastError();
}

}  // namespace sks
