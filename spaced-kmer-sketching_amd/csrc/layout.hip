// The join layout (input of k_join, join.hip; format in join_common.hpp): for
// every block of 64 consecutive sketches, each distinct value once with the
// mask of the block's sketches holding it, bucket by bucket.
//
// Buckets are two-level.  The value range is cut into G = B / 8 groups by
// common bounds (the median of up to 64 sample sketches' quantiles), and a
// group's 8 buckets are chosen by a hash of the value.  The two levels serve
// two masters:
//   * every sketch is sorted, so its part of a value group is ONE contiguous
//     range (two binary searches): the build reads each sketch's part straight
//     from the sketch, with no counting or staging pass over the whole set;
//   * within a group the buckets are hashed, so a block's bucket populations are
//     Poisson.  Fine value-range buckets are lumpy for related sketches (a
//     bucket that is large for one member of a family is large for all 64 of
//     its block: k_join over a value-range layout ran 1.2 instead of 0.6 ms,
//     DESIGN.md §5), while a group of ~1.2k block elements averages that out.
// Counts are exact for any non-decreasing bounds; all layouts whose blocks are
// joined with each other (a multi-GPU gather) must share one bounds array.
//
// Deduplicated entries (round 4): the sketches of one block are related (a
// genome family), so a value is often held by many of them.  Storing it once
// with a 64-bit sketch mask makes the join insert and probe it once instead of
// once per holder (config 4: 10.0 M block elements -> 5.75 M entries), and a
// diagonal tile needs no table at all (an entry's hits are its own mask).
//
// Build (join_layout_build), three launches: k_gl_prep (the group bounds when
// the caller gives none, and the raw block starts), k_gl_pos (every sketch's
// group starts: a workgroup per sketch), then k_gl_place, one workgroup per
// (block, region of 8 groups): for each group its elements are read once into
// registers (the next group's loads in flight while the current one is
// placed), deduplicated in an LDS hash table whose representatives collect the
// holders' bits, counted per bucket, scanned, and written to the region's own
// part of the block.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "join_common.hpp"
#include "sks_internal.hpp"

namespace sks {

namespace {

using jc::KV;
using jc::kv_eq;
using jc::kv_group_bucket;
using jc::kv_load;
using jc::kv_lt;
using jc::kv_mix;
using jc::kv_store;

constexpr int kTile = 64;
constexpr int kPT = 256;                 // threads of the layout kernels
constexpr uint32_t kGCap = 256u << jc::kGLog;  // elements of one dedup batch (a group): 2048
constexpr int kTabLog = 9 + jc::kGLog;         // dedup table: 4096 slots (load <= 1/2)
constexpr uint32_t kTab = 1u << kTabLog;
constexpr uint32_t kIdxBits = 11;        // slot word: tag21 << 11 | element index
constexpr uint32_t kIdxMask = (1u << kIdxBits) - 1;
constexpr uint32_t kTFree = 0xFFFFFFFFu;
static_assert(kGCap <= (1u << kIdxBits), "element index must fit the slot word");

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

// dedup table slot and tag of a value: independent of the top bits of kv_mix
// (the bucket, and the slow path's slices)
template <int EW>
__device__ __forceinline__ uint32_t dd_slot(const KV& v) {
  const uint64_t f = jc::fp_fold<EW>(v);
  return (((uint32_t)f ^ (uint32_t)(f >> 32)) * 0x27D4EB2Fu) >> (32 - kTabLog);
}
template <int EW>
__device__ __forceinline__ uint32_t dd_tag(const KV& v) {  // 21 bits, never all ones
  const uint32_t t = (uint32_t)(kv_mix<EW>(v) >> 28) & 0x1FFFFFu;
  return t == 0x1FFFFFu ? 0x1FFFFEu : t;
}

template <int EW>
__device__ __forceinline__ KV key_at(const uint64_t* s_key, uint32_t i) {
  if constexpr (EW == 1) return KV{s_key[i], 0};
  else return KV{s_key[2 * i], s_key[2 * i + 1]};
}

// Inserts element i (value v) into the dedup table; returns the index of the
// element that represents v (i itself when v was new).  The table is cut into
// regions, one per hash bucket of the pass (base = the bucket's region, rmask =
// its size - 1), and a value probes only its bucket's region, so reading the
// table in slot order lists the distinct values bucket by bucket.  More
// distinct values than a region holds set *full (the caller redoes the group
// with one bucket per pass and the whole table).  The probe loop has ONE exit
// edge and evaluates its stop test without short-circuit (the element a slot
// word names is read whether or not the tag matches; a free word names element
// 2047, read and ignored): the two-exit form of this loop (free slot / same
// value, the entry assigned at each exit) was miscompiled by ROCm 7.2 for
// gfx950 in round 3 (reproducer in tools/microbench/chain_exits.hip).
template <int EW>
__device__ __forceinline__ uint32_t dd_insert(uint32_t* s_tab, const uint64_t* s_key, const KV& v, uint32_t i,
                                              uint32_t base, uint32_t rmask, bool* full) {
  const uint32_t tag = dd_tag<EW>(v);
  const uint32_t word = (tag << kIdxBits) | i;
  uint32_t h = dd_slot<EW>(v) & rmask, steps = 0;
  uint32_t x = atomicCAS(&s_tab[base + h], kTFree, word);
  for (;;) {
    const KV u = key_at<EW>(s_key, x & kIdxMask);
    if ((x == kTFree) | (((x >> kIdxBits) == tag) & kv_eq<EW>(u, v)) | (steps > rmask)) break;
    h = (h + 1) & rmask;
    ++steps;
    x = atomicCAS(&s_tab[base + h], kTFree, word);
  }
  if (steps > rmask) *full = true;
  return x == kTFree ? i : (x & kIdxMask);
}

// Workgroups [0, nb_bounds): the group bounds, a wave per bound (bounds[g] =
// the lower median over up to 64 sample sketches of their g/G quantile;
// bounds[0] = 0, bounds[G] = the largest value).  The median, not the mean: a
// spaced mask leaves gaps in the value space (the masked-out bit positions are
// zero), the sketches' ranks drift apart by more than a group's population, and
// a mean of two quantiles on either side of a gap lands inside it, so that
// group takes every sketch's values up to the gap (round 6: up to 217
// elements of one sketch against 12 expected at (23, 13), groups above the
// placement's capacity at w = 45).  The median is a sampled value, exact at
// 128 bits, and an order statistic of non-decreasing sequences, so the bounds
// are non-decreasing, which is all exactness needs.  The last workgroup:
// bstart[k] = elements of the blocks before k (a running scan over the sizes).
template <int EW>
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
    KV q{0, 0};
    bool have = false;
    if ((uint32_t)lane < K && g > 0 && g < G) {
      const uint32_t i = (uint32_t)((uint64_t)lane * count / K);
      const uint32_t sz = sizes[i];
      if (sz) {
        q = kv_load<EW>(data, starts[i] + (uint64_t)g * sz / G);
        have = true;
      }
    }
    // rank of this lane's sample among the wave's (ties by lane)
    const uint64_t valid = __ballot(have);
    uint32_t rank = 0;
    for (int j = 0; j < 64; ++j) {
      const KV o{(uint64_t)__shfl((long long)q.lo, j, 64), (uint64_t)__shfl((long long)q.hi, j, 64)};
      const bool below = kv_lt<EW>(o, q) || (kv_eq<EW>(o, q) && j < lane);
      rank += ((valid >> j) & 1ull) && below ? 1u : 0u;
    }
    const uint32_t used = (uint32_t)__popcll(valid);
    KV b{0, 0};
    if (g == G) {
      if (lane) return;
      b = KV{~0ull, EW == 1 ? 0ull : ~0ull};
    } else if (used == 0) {
      if (lane) return;
    } else {
      if (!have || rank != (used - 1) / 2) return;
      b = q;
    }
    kv_store<EW>(bounds, g, b);
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
// bound searches that sample and then the one cache line it points at (a
// stride-8 sample touches every 64-B line of a u64 sketch, so the launch is
// bound by reading the sketches once).  A sketch above kPosSamples * stride
// elements samples with a larger stride.
constexpr uint32_t kPosStride = 8, kPosSamples = 2048;
template <int EW>
__global__ __launch_bounds__(kPT) void k_gl_pos(const uint64_t* __restrict__ data,
                                                const uint64_t* __restrict__ starts,
                                                const uint32_t* __restrict__ sizes, uint32_t count,
                                                uint32_t G, const uint64_t* __restrict__ bounds,
                                                uint32_t* __restrict__ pos, const ZeroSpans z) {
  __shared__ uint64_t s_smp[kPosSamples * EW];
  const uint32_t i = blockIdx.x;
  {  // the caller's spans to clear: 16-B stores over the grid, dwords at the ends
    const uint64_t nthr = (uint64_t)gridDim.x * kPT, t0 = (uint64_t)i * kPT + threadIdx.x;
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      uint32_t* p = z.p[q];
      const uint64_t nw = z.words[q];
      if (!p || !nw) continue;
      const uint64_t head = min(nw, (uint64_t)(((16u - ((uint32_t)(uintptr_t)p & 15u)) & 15u) >> 2));
      if (t0 < head) p[t0] = 0;
      uint4* v = reinterpret_cast<uint4*>(p + head);
      const uint64_t nv = (nw - head) >> 2;
      for (uint64_t k = t0; k < nv; k += nthr) v[k] = make_uint4(0, 0, 0, 0);
      const uint64_t tail = head + nv * 4;
      if (t0 < nw - tail) p[tail + t0] = 0;
    }
  }
  const uint32_t sz = sizes[i];
  const uint64_t st = starts[i];
  uint32_t stride = kPosStride;
  while ((uint64_t)stride * kPosSamples < sz) stride <<= 1;
  const uint32_t ns = (sz + stride - 1) / stride;  // sample k = S[k * stride]
  if (ns) {  // every load of the thread's samples issued before the first LDS store
    constexpr int kPer = (kPosSamples + kPT - 1) / kPT;
    KV smp[kPer];
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
      const uint32_t k = threadIdx.x + (uint32_t)u * kPT;
      smp[u] = kv_load<EW>(data, st + (uint64_t)min(k, ns ? ns - 1 : 0u) * stride);
    }
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
      const uint32_t k = threadIdx.x + (uint32_t)u * kPT;
      if (k < ns) kv_store<EW>(s_smp, k, smp[u]);
    }
  }
  __syncthreads();
  uint32_t* out = pos + (uint64_t)i * (G + 1);
  for (uint32_t g = threadIdx.x; g <= G; g += kPT) {
    if (g == 0 || g == G) {
      out[g] = g == 0 ? 0 : sz;
      continue;
    }
    const KV x = kv_load<EW>(bounds, g);
    // lo = samples below x: the lower bound lies in ((lo - 1) * stride, lo * stride]
    uint32_t lo = 0, hi = ns;
    while (lo < hi) {
      const uint32_t mid = (lo + hi) >> 1;
      if (kv_lt<EW>(kv_load<EW>(s_smp, mid), x)) lo = mid + 1; else hi = mid;
    }
    uint32_t a = lo ? (lo - 1) * stride + 1 : 0, e = min(sz, lo * stride);
    if (stride == kPosStride || a >= e) {
      // at most stride - 1 candidates: all loaded together (clamped, no branch
      // per load), the lower bound is a + the number below x
      uint32_t c = 0;
      if (a < e) {  // (an empty range, e.g. an empty sketch, loads nothing)
#pragma unroll
        for (uint32_t q = 0; q + 1 < kPosStride; ++q) {
          const uint32_t m = a + q;
          const KV y = kv_load<EW>(data, st + min(m, e - 1));
          c += (m < e && kv_lt<EW>(y, x)) ? 1u : 0u;
        }
      }
      out[g] = a + c;
      continue;
    }
    while (a < e) {
      const uint32_t mid = (a + e) >> 1;
      if (kv_lt<EW>(kv_load<EW>(data, st + mid), x)) a = mid + 1; else e = mid;
    }
    out[g] = a;
  }
}

__device__ unsigned long long g_layout_check;  // SKS check build: dedup invariant violations

#ifdef SKS_LAYOUT_STAMPS  // diagnostic build: cycles per k_gl_place phase (thread 0 of each workgroup)
// slots 0-4: phase cycles, summed in registers and stored per workgroup at the
// end (no atomics on the timed path); slots 5-9: event counts (atomics, rare)
constexpr int kMaxStampWgs = 16384;
__device__ unsigned long long g_layout_stamps[10];
__device__ unsigned long long g_layout_stamps_wg[kMaxStampWgs * 5];
#define LSTAMP(i)                                              \
  do {                                                         \
    if (threadIdx.x == 0) {                                    \
      const uint64_t t_ = __builtin_amdgcn_s_memtime();        \
      st_acc[i] += t_ - st_last;                               \
      st_last = t_;                                            \
    }                                                          \
  } while (0)
#define LSTAMP_FLUSH()                                                                  \
  do {                                                                                  \
    if (threadIdx.x == 0 && blockIdx.x < kMaxStampWgs)                                  \
      for (int q_ = 0; q_ < 5; ++q_) g_layout_stamps_wg[blockIdx.x * 5 + q_] = st_acc[q_]; \
  } while (0)
#else
#define LSTAMP(i) do {} while (0)
#define LSTAMP_FLUSH() do {} while (0)
#endif

#ifndef SKS_PLACE_DIAG
#define SKS_PLACE_DIAG 0
#endif
constexpr int kPB = 256;                     // threads of the placement kernel
#ifndef SKS_LAYOUT_STAGED
#define SKS_LAYOUT_STAGED 1  // normal-path emit through an LDS list in place order (coalesced stores)
#endif
constexpr int kTPS = kPB / 64;               // threads per sketch in the register path (4)
#ifndef SKS_LAYOUT_REGPER
#define SKS_LAYOUT_REGPER 12
#endif
constexpr int kRegPer = SKS_LAYOUT_REGPER;   // elements of its sketch per thread held in registers
constexpr uint32_t kSkCap = kTPS * kRegPer;  // a group with a sketch holding more (48) takes the bucket passes
constexpr int kSlowPer = kGCap / kPB;        // slice path: slice elements per thread
constexpr uint32_t kSpt = kTab / kPB;        // table slots per thread in the emit scan (16)
constexpr uint32_t kMaxRG = 1u << jc::kRGLogMax;
constexpr int kPassU = 4;                    // bucket passes: 64-element chunks loaded per round
static_assert(kSpt % 4 == 0, "emit reads the slots as uint4");

__device__ __forceinline__ uint64_t readlane64(uint64_t x, uint32_t l) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)x, (int)l);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(x >> 32), (int)l);
  return ((uint64_t)hi << 32) | lo;
}

// A value group's raw elements, sketch by sketch: lane s of a wave holds
// sketch s's count gc, the inclusive prefix gend (sketch s holds elements
// [gend - gc, gend) of the group) and src (element i of sketch s is
// data[src + i]); gn = the group's element count.
struct GroupMap {
  uint32_t gc, gend, gn;
  uint64_t src;
};
__device__ __forceinline__ GroupMap group_map(const uint32_t* p0, const uint32_t* p1, bool sv, uint64_t stt,
                                              int lane) {
  GroupMap m;
  const uint32_t glo = sv ? p0[lane] : 0;
  const uint32_t ghi = sv ? max(p1[lane], glo) : 0;
  m.gc = ghi - glo;
  m.gend = wave_scan(m.gc);
  m.gn = (uint32_t)__builtin_amdgcn_readlane((int)m.gend, 63);
  m.src = stt + glo - (m.gend - m.gc);
  return m;
}

// Where element b + lane of the group lives (b wave-uniform, b < gn): the lane
// walks, wave-uniformly, the few sketches whose ranges meet [b, b + 64)
// (readlanes, no LDS).  *own = its sketch slot; returns the element's index in
// `data` (meaningless for b + lane >= gn).
__device__ __forceinline__ uint64_t elem_at(const GroupMap& m, uint32_t b, int lane, uint32_t* own) {
  const uint32_t i = b + (uint32_t)lane, lim = min(b + 64, m.gn);
  uint32_t s = (uint32_t)__popcll(__ballot(m.gend <= b));  // first sketch ending after b
  uint32_t o = 0;
  uint64_t at = 0;
  for (; s < 64; ++s) {
    const uint32_t e = (uint32_t)__builtin_amdgcn_readlane((int)m.gend, (int)s);
    const uint32_t c = (uint32_t)__builtin_amdgcn_readlane((int)m.gc, (int)s);
    if (e - c >= lim) break;
    const uint64_t a = readlane64(m.src, s);
    const bool mine = (i >= e - c) & (i < e);
    o = mine ? s : o;
    at = mine ? a : at;
  }
  *own = o;
  return at + i;
}

// Thread t's view of a value group in the register path: it serves sketch
// s = t / 4 (the block's 64 sketches, 4 threads each) and loads elements
// e = t % 4 + 4 k of the sketch's part of the group (e < gc) from
// data[src + e]; the element's LDS index is gpre + e (the group's elements,
// sketch by sketch).  fat: some sketch holds more than kSkCap elements of the
// group (the group takes the bucket passes).
struct GroupView {
  uint32_t gn, gpre, gc;
  uint64_t src;
  bool fat;
};
__device__ __forceinline__ GroupView group_view(const uint32_t* p0, const uint32_t* p1, bool sv, uint64_t stt,
                                                int lane, uint32_t s) {
  const GroupMap m = group_map(p0, p1, sv, stt, lane);  // lane = sketch
  GroupView g;
  g.gn = m.gn;
  g.gc = (uint32_t)__shfl((int)m.gc, (int)s, 64);
  g.gpre = (uint32_t)__shfl((int)m.gend, (int)s, 64) - g.gc;
  const uint64_t at = m.src + (m.gend - m.gc);  // sketch lane's first element of the group
  g.src = ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(at >> 32), (int)s, 64) << 32) |
          (uint32_t)__shfl((int)(uint32_t)at, (int)s, 64);
  g.fat = __ballot(m.gc > kSkCap) != 0;
  return g;
}

template <int EW>
__device__ __forceinline__ void group_load(const uint64_t* __restrict__ data, const GroupView& g, uint32_t sub,
                                           KV (&v)[kRegPer]) {
#pragma unroll
  for (int k = 0; k < kRegPer; ++k) {
    const uint32_t e = sub + kTPS * k;
    v[k] = KV{0, 0};
    if (!g.fat && g.gn <= kGCap && e < g.gc) {
#if SKS_PLACE_DIAG == 3  // diagnostics: no global loads (values synthesised from the index)
      v[k] = KV{(g.src + e) * 0x9E3779B97F4A7C15ull, 0};
#else
      v[k] = kv_load<EW>(data, g.src + e);
#endif
    }
  }
}

// Emits one dedup pass: the table in slot order lists the pass's distinct
// values bucket by bucket (region q of 4096 >> pl slots = bucket b0 + q).
// Thread t reads slots [kSpt t, kSpt t + kSpt) (and frees them), a block scan
// of the occupied counts gives every entry its place at the cursor; the
// entries {value, mask} are written and the masks cleared for the next pass.
// Two barriers.
template <int EW>
__device__ __forceinline__ void emit_pass(uint32_t* s_tab, const uint64_t* s_key, unsigned long long* s_msk,
                                          uint32_t* s_wsum, uint32_t* boff_b0, uint32_t nb, uint32_t pl,
                                          uint64_t base, uint64_t* __restrict__ out_vals,
                                          unsigned long long* __restrict__ out_masks, uint32_t& cur, uint32_t& maxb,
                                          int tid, int lane, int wave) {
  uint32_t wv[kSpt];
#pragma unroll
  for (int q = 0; q < (int)kSpt / 4; ++q) {
    uint4* p = reinterpret_cast<uint4*>(s_tab) + tid * (kSpt / 4) + q;
    const uint4 x = *p;
    *p = make_uint4(kTFree, kTFree, kTFree, kTFree);
    wv[4 * q] = x.x;
    wv[4 * q + 1] = x.y;
    wv[4 * q + 2] = x.z;
    wv[4 * q + 3] = x.w;
  }
  uint32_t occ = 0;
#pragma unroll
  for (int q = 0; q < (int)kSpt; ++q) occ += wv[q] != kTFree;
  const uint32_t wincl = wave_scan(occ);
  if (lane == 63) s_wsum[wave] = wincl;
  __syncthreads();
  uint32_t before = 0, total = 0;
#pragma unroll
  for (int w = 0; w < kPB / 64; ++w) {
    const uint32_t x = s_wsum[w];
    before += w < wave ? x : 0;
    total += x;
  }
  const uint32_t excl = before + wincl - occ;
  const uint32_t tpb = (uint32_t)kPB >> pl;  // threads per bucket region
  const uint32_t q = (uint32_t)tid / tpb;
  if ((uint32_t)tid % tpb == 0 && q < nb) boff_b0[q] = cur + excl;
  // the pass's entries in slot order: element indices listed in the (freed)
  // table, then written with coalesced stores and the table freed again
  uint32_t d = excl;
#pragma unroll
  for (int k = 0; k < (int)kSpt; ++k)
    if (wv[k] != kTFree) s_tab[d++] = wv[k] & kIdxMask;
  __syncthreads();
  for (uint32_t e = tid; e < total; e += kPB) {
    const uint32_t i = s_tab[e];
    s_tab[e] = kTFree;
    const uint64_t o = base + cur + e;
#if SKS_PLACE_DIAG != 4  // (diagnostics 4: no global stores)
    kv_store<EW>(out_vals, o, key_at<EW>(s_key, i));
    out_masks[o] = s_msk[i];
#endif
    s_msk[i] = 0;
  }
  // the largest bucket (entries): the occupied counts of its region's threads
  uint32_t bo = occ;
  if (tpb <= 64) {
    for (uint32_t o2 = 1; o2 < tpb; o2 <<= 1) bo += __shfl_xor(bo, o2, 64);
  } else {
    bo = 0;
    for (uint32_t w = q * (tpb / 64); w < (q + 1) * (tpb / 64); ++w) bo += s_wsum[w];
  }
  maxb = max(maxb, bo);
  cur += total;
}

// One workgroup per (block, region): the region's value groups one after the
// other, the next group's elements loading into registers while the current
// one is placed, the region's entry cursor carried in registers (no cross-
// workgroup prefix).  Per group of gn <= gcap raw elements (the normal path):
//   P1  the elements go to s_key / s_own (LDS index = element index), and the
//       next group's loads are issued into the same registers
//   P2  every element is inserted into the dedup table (a region of 4096 / 8
//       slots per bucket of the group); the representative of a value (the
//       element that claimed its slot) collects the holders' sketch bits
//   P3  the table is scanned in slot order (bucket by bucket) and freed,
//   P4  the distinct entries {value, mask} are written at the region cursor.
// Bucket passes: a group above gcap elements (a dense stretch of values held
// by a whole family), or with more distinct values in one bucket than the
// bucket's table region holds, is counted per bucket and placed in passes of
// consecutive buckets holding <= gcap elements (re-read from the sketches with
// coalesced loads, compacted into s_key; a pass whose table region overflows
// is redone one bucket per pass, with the whole table).  A bucket above gcap
// elements (adversarial values only) takes the slice path: hash slices of the
// group gathered from the sketches, each deduplicated and written in slice
// order (a slice still above gcap is split in two).  Exact for any input.
template <int EW, bool CHECK>
__global__ __launch_bounds__(kPB) void k_gl_place(const uint64_t* __restrict__ data,
                                                  const uint64_t* __restrict__ starts, uint32_t count,
                                                  uint32_t log_b, const uint32_t* __restrict__ pos,
                                                  const uint64_t* __restrict__ bstart,
                                                  uint64_t* __restrict__ out_vals,
                                                  unsigned long long* __restrict__ out_masks,
                                                  uint32_t* __restrict__ out_boff, uint32_t* __restrict__ stat,
                                                  uint32_t gcap, uint32_t rg) {
  __shared__ uint64_t s_key[kGCap * EW];
  __shared__ unsigned long long s_msk[kGCap];
  __shared__ uint32_t s_tab[kTab];
  __shared__ uint32_t s_pos[(kMaxRG + 1) * kTile];  // [j * 64 + s]: sketch s's start of the region's group j
  __shared__ uint8_t s_own[kGCap];                  // LDS element -> its sketch slot
  __shared__ uint32_t s_wsum[kPB / 64];
  __shared__ uint32_t s_bcnt[1u << jc::kGLog];
  __shared__ uint32_t s_full, s_pcnt, s_gd, s_qn, s_qd;
  __shared__ unsigned long long s_stk[2 * 72];  // slice path: (slice prefix, level) work stack (prefixes up to 64 bits)
#if SKS_LAYOUT_STAGED
  __shared__ uint16_t s_stage[kGCap];  // normal-path emit: the group's entries' element indices, in place order
#endif

  const uint32_t B = 1u << log_b, gb_log = jc::lay_gb_log(log_b), GB = 1u << gb_log;
  const uint32_t G = B >> gb_log, NR = jc::lay_regions(log_b, rg), BW = jc::lay_boff_words(log_b);
  const uint32_t RG = (1u << jc::lay_rb_log(log_b, rg)) >> gb_log;
  const uint32_t blk = blockIdx.x / NR, r = blockIdx.x % NR;
  // the wave index in an SGPR: the per-wave loop bounds stay scalar
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
#ifdef SKS_LAYOUT_STAMPS
  uint64_t st_last = __builtin_amdgcn_s_memtime();
  uint64_t st_acc[5] = {0, 0, 0, 0, 0};
#endif
  const uint32_t s_end = min((uint32_t)kTile, count - kTile * blk);
  uint32_t* boff = out_boff + (uint64_t)blk * BW;
  if (r == 0 && threadIdx.x == 0) boff[BW - 1] = jc::lay_rb_log(log_b, rg);  // the join reads the region size here
  const uint64_t base = bstart[blk];
  const bool sv = (uint32_t)lane < s_end;
  const uint64_t stt = sv ? starts[kTile * blk + lane] : 0;
  for (uint32_t q = tid; q < (RG + 1) * kTile; q += kPB) {
    const uint32_t j = q / kTile, s = q % kTile;
    s_pos[q] = s < s_end ? pos[(uint64_t)(kTile * blk + s) * (G + 1) + r * RG + j] : 0;
  }
  for (uint32_t q = tid; q < kTab / 4; q += kPB)
    reinterpret_cast<uint4*>(s_tab)[q] = make_uint4(kTFree, kTFree, kTFree, kTFree);
  for (uint32_t q = tid; q < kGCap / 2; q += kPB) reinterpret_cast<uint4*>(s_msk)[q] = make_uint4(0, 0, 0, 0);
  if (tid == 0) s_full = 0;
  __syncthreads();
  // the region's entries start at its raw offset in the block
  uint32_t cur = (uint32_t)__builtin_amdgcn_readlane((int)wave_scan(sv ? s_pos[lane] : 0u), 63);
  uint32_t maxb = 0;
  KV v[kRegPer];
  const uint32_t my_s = (uint32_t)tid / kTPS, sub = (uint32_t)tid % kTPS;  // this thread's sketch
  GroupView gv = group_view(s_pos, s_pos + kTile, sv, stt, lane, my_s);
  group_load<EW>(data, gv, sub, v);
  LSTAMP(0);

  for (uint32_t j = 0; j < RG; ++j) {
    const uint32_t g = r * RG + j;
    const GroupView gj = gv;
    const uint32_t gn_j = gj.gn;
    // the next group's elements load into v (in flight while this group is
    // placed; this group's values are in LDS by then)
    bool fetched = false;
    auto load_next = [&]() {
      if (j + 1 < RG) {
        gv = group_view(s_pos + (j + 1) * kTile, s_pos + (j + 2) * kTile, sv, stt, lane, my_s);
        group_load<EW>(data, gv, sub, v);
      }
      fetched = true;
    };
    bool done = false;
    if (gn_j == 0) {  // an empty group: its buckets start (and end) at the cursor
      if ((uint32_t)tid < GB) boff[g * GB + tid] = cur;
      done = true;
    } else if (gn_j <= gcap && !gj.fat) {
      // ---- normal path ------------------------------------------------------------------------
      __syncthreads();  // the previous pass has read s_key / s_msk / s_tab / s_bcnt
#pragma unroll
      for (int k = 0; k < kRegPer; ++k) {  // P1
        const uint32_t e = sub + kTPS * k, i = gj.gpre + e;
        if (e < gj.gc) {
          if constexpr (EW == 1) s_key[i] = v[k].lo;
          else { s_key[2 * i] = v[k].lo; s_key[2 * i + 1] = v[k].hi; }
        }
      }
      if ((uint32_t)tid < GB) s_bcnt[tid] = 0;
      load_next();
      __syncthreads();
      LSTAMP(1);
      // P2 (the values read back from LDS), every element's first probe issued
      // together: keys, first compare-swaps, the named elements' keys; then the
      // (rare) rest of each chain, one exit edge (see dd_insert).  A slot word
      // is the claiming element's index; the element that claims a slot is its
      // value's representative and takes the next place of its bucket
      // (s_bcnt: entries are contiguous per bucket, in any order within it).
      bool full = false;
      const uint32_t rlog = kTabLog - gb_log, rmask = (1u << rlog) - 1;
      uint32_t h[kRegPer], w[kRegPer], rep[kRegPer];
#pragma unroll
      for (int k = 0; k < kRegPer; ++k) {
        const uint32_t e = sub + kTPS * k, i = gj.gpre + e;
        w[k] = kTFree;
        h[k] = 0;
        if (e < gj.gc) {
          const KV x = key_at<EW>(s_key, i);
          // bucket (top gb_log bits of the mix) and slot in its region (the next rlog bits)
          h[k] = (uint32_t)(kv_mix<EW>(x) >> (64 - kTabLog));
          w[k] = atomicCAS(&s_tab[h[k]], kTFree, i);
        }
      }
#pragma unroll
      for (int k = 0; k < kRegPer; ++k) {
        const uint32_t e = sub + kTPS * k, i = gj.gpre + e;
        rep[k] = kTFree;
        if (e < gj.gc) {
          const KV x = key_at<EW>(s_key, i);
          const uint32_t rbase = h[k] & ~rmask;
          uint32_t hh = h[k] & rmask, xw = w[k], steps = 0;
          KV u = key_at<EW>(s_key, xw & kIdxMask);
          for (;;) {
            if ((xw == kTFree) | kv_eq<EW>(u, x) | (steps > rmask)) break;
            hh = (hh + 1) & rmask;
            ++steps;
            xw = atomicCAS(&s_tab[rbase + hh], kTFree, i);
            u = key_at<EW>(s_key, xw & kIdxMask);
          }
          const bool f = steps > rmask;  // (an overflowed region names a foreign entry: the group is redone)
          full |= f;
          const uint32_t ri = xw == kTFree ? i : xw;
          if (CHECK && !f && !kv_eq<EW>(key_at<EW>(s_key, ri), x)) atomicAdd(&g_layout_check, 1ull);
          atomicOr(&s_msk[ri], 1ull << my_s);
          if (xw == kTFree) {  // the representative: its slot (freed at emit) and its place in the bucket
            const uint32_t bk = h[k] >> rlog;
            rep[k] = (bk << 12) | atomicAdd(&s_bcnt[bk], 1u);
            h[k] = rbase + hh;
          }
        }
      }
      if (full) s_full = 1;
      __syncthreads();
      LSTAMP(2);
      if (s_full == 0) {
        // P3: bucket starts from the counts; P4: every representative writes its
        // entry {value, mask} and frees its slot and mask
        uint32_t pre[1u << jc::kGLog], tot = 0;
#pragma unroll
        for (uint32_t b = 0; b < (1u << jc::kGLog); ++b) {
          const uint32_t c = b < GB ? s_bcnt[b] : 0u;
          pre[b] = tot;
          tot += c;
          maxb = max(maxb, c);
        }
        if ((uint32_t)tid < GB) boff[g * GB + tid] = cur + pre[tid];
#if SKS_LAYOUT_STAGED
        // representatives list their element at its place (and free their slot);
        // the group's entries then leave with coalesced stores
#pragma unroll
        for (int k = 0; k < kRegPer; ++k) {
          if (rep[k] == kTFree) continue;
          s_stage[pre[rep[k] >> 12] + (rep[k] & 4095u)] = (uint16_t)(gj.gpre + sub + kTPS * k);
          s_tab[h[k]] = kTFree;
        }
        __syncthreads();
        for (uint32_t e = (uint32_t)tid; e < tot; e += kPB) {
          const uint32_t i = s_stage[e];
          const uint64_t o = base + cur + e;
          kv_store<EW>(out_vals, o, key_at<EW>(s_key, i));
          out_masks[o] = s_msk[i];
          s_msk[i] = 0;
        }
#else
#pragma unroll
        for (int k = 0; k < kRegPer; ++k) {
          if (rep[k] == kTFree) continue;
          const uint32_t i = gj.gpre + sub + kTPS * k;
          const uint64_t o = base + cur + pre[rep[k] >> 12] + (rep[k] & 4095u);
#if SKS_PLACE_DIAG != 4  // (diagnostics 4: no global stores)
          kv_store<EW>(out_vals, o, key_at<EW>(s_key, i));
          out_masks[o] = s_msk[i];
#endif
          s_msk[i] = 0;
          s_tab[h[k]] = kTFree;
        }
#endif
        cur += tot;
        done = true;
      } else {  // a bucket region overflowed: clean up, place the group in bucket passes
        for (uint32_t q = tid; q < kTab / 4; q += kPB)
          reinterpret_cast<uint4*>(s_tab)[q] = make_uint4(kTFree, kTFree, kTFree, kTFree);
        for (uint32_t q = tid; q < kGCap / 2; q += kPB) reinterpret_cast<uint4*>(s_msk)[q] = make_uint4(0, 0, 0, 0);
        __syncthreads();
        if (tid == 0) s_full = 0;
      }
      LSTAMP(3);
    }
    if (!fetched) load_next();
    if (!done) {
      // ---- bucket passes ------------------------------------------------------------------------
      const GroupMap m = group_map(s_pos + j * kTile, s_pos + (j + 1) * kTile, sv, stt, lane);
      // visits every element of the group (coalesced, kPassU chunks per round): f(value, slot)
      auto for_each = [&](auto&& f) {
        for (uint32_t c0 = (uint32_t)wave * 64; c0 < m.gn; c0 += kPB * kPassU) {
          KV x[kPassU];
          uint32_t o[kPassU];
#pragma unroll
          for (int u = 0; u < kPassU; ++u) {
            const uint32_t b = c0 + u * kPB;
            o[u] = 0;
            x[u] = KV{0, 0};
            if (b < m.gn) {
              const uint64_t at = elem_at(m, b, lane, &o[u]);
              if (b + (uint32_t)lane < m.gn) x[u] = kv_load<EW>(data, at);
            }
          }
#pragma unroll
          for (int u = 0; u < kPassU; ++u)
            if (c0 + u * kPB + (uint32_t)lane < m.gn) f(x[u], o[u]);
        }
      };
      __syncthreads();
      if ((uint32_t)tid < GB) s_bcnt[tid] = 0;
      __syncthreads();
      for_each([&](const KV& x, uint32_t) { atomicAdd(&s_bcnt[kv_group_bucket<EW>(x, gb_log)], 1u); });
      __syncthreads();
      bool slices = false;
      for (uint32_t b = 0; b < GB; ++b) slices |= s_bcnt[b] > gcap;
      // passes [b0, b1) of consecutive buckets with <= gcap elements; one_bucket
      // after a pass whose table region overflowed
      uint32_t b0 = 0;
      bool one_bucket = false;
      while (!slices && b0 < GB) {
        uint32_t b1 = b0 + 1, n = s_bcnt[b0];
        if (!one_bucket)
          while (b1 < GB && n + s_bcnt[b1] <= gcap) n += s_bcnt[b1++];
        if (n == 0) {  // empty buckets start (and end) at the cursor
          if ((uint32_t)tid < b1 - b0) boff[g * GB + b0 + tid] = cur;
          b0 = b1;
          continue;
        }
        uint32_t pl = 0;
        while ((1u << pl) < b1 - b0) ++pl;
        __syncthreads();  // the previous pass has read s_key / s_msk / s_own / s_pcnt
        if (tid == 0) s_pcnt = 0;
        __syncthreads();
        for_each([&](const KV& x, uint32_t o) {
          if (kv_group_bucket<EW>(x, gb_log) - b0 < b1 - b0) {
            const uint32_t idx = atomicAdd(&s_pcnt, 1u);
            if constexpr (EW == 1) s_key[idx] = x.lo;
            else { s_key[2 * idx] = x.lo; s_key[2 * idx + 1] = x.hi; }
            s_own[idx] = (uint8_t)o;
          }
        });
        __syncthreads();
        const uint32_t np = s_pcnt, rlog = kTabLog - pl;
        bool full = false;
        for (uint32_t i = tid; i < np; i += kPB) {
          const KV x = key_at<EW>(s_key, i);
          bool f = false;
          const uint32_t ri = dd_insert<EW>(s_tab, s_key, x, i, (kv_group_bucket<EW>(x, gb_log) - b0) << rlog,
                                            (1u << rlog) - 1, &f);
          full |= f;
          if (CHECK && !f && !kv_eq<EW>(key_at<EW>(s_key, ri), x)) atomicAdd(&g_layout_check, 1ull);
          atomicOr(&s_msk[ri], 1ull << s_own[i]);
        }
        if (full) s_full = 1;
        __syncthreads();
        if (s_full) {  // redo these buckets one per pass
          for (uint32_t q = tid; q < kTab / 4; q += kPB)
            reinterpret_cast<uint4*>(s_tab)[q] = make_uint4(kTFree, kTFree, kTFree, kTFree);
          for (uint32_t q = tid; q < kGCap / 2; q += kPB) reinterpret_cast<uint4*>(s_msk)[q] = make_uint4(0, 0, 0, 0);
          __syncthreads();
          if (tid == 0) s_full = 0;
          one_bucket = true;
          continue;
        }
        emit_pass<EW>(s_tab, s_key, s_msk, s_wsum, boff + g * GB + b0, b1 - b0, pl, base, out_vals, out_masks, cur,
                      maxb, tid, lane, wave);
        b0 = b1;
      }
      if (slices) {
        // ---- slice path: hash slices of the group, gathered from the sketches -----------------
        const uint32_t glo = sv ? s_pos[j * kTile + lane] : 0;
        const uint32_t ghi = sv ? max(s_pos[(j + 1) * kTile + lane], glo) : 0;
        uint32_t lvl0 = max(gb_log, 1u);
        while (lvl0 < 32 && ((uint64_t)gn_j >> (lvl0 - 1)) > gcap / 2) ++lvl0;
        uint32_t bk_cur = ~0u, bk_start = cur;
        for (uint32_t q0 = 0; q0 < (1u << lvl0); ++q0) {
          // depth-first over the slice and, when it is too large, its halves
          // (smallest slice on top, so slices come out in hash order)
          __syncthreads();
          if (tid == 0) {
            s_stk[0] = q0;
            s_stk[1] = lvl0;
            s_qd = 1;
          }
          __syncthreads();
          for (;;) {
            const uint32_t depth = s_qd;
            if (depth == 0) break;
            const uint64_t q = s_stk[2 * (depth - 1)];
            const uint32_t lvl = (uint32_t)s_stk[2 * (depth - 1) + 1];
            __syncthreads();
            if (tid == 0) {
              s_qd = depth - 1;
              s_qn = 0;
              s_gd = 0;
            }
            for (uint32_t i = tid; i < kTab / 4; i += kPB)
              reinterpret_cast<uint4*>(s_tab)[i] = make_uint4(kTFree, kTFree, kTFree, kTFree);
            __syncthreads();
            for (uint32_t s = wave; s < s_end; s += kPB / 64) {
              const uint32_t a = __shfl(glo, s), b = __shfl(ghi, s);
              const uint64_t sts = __shfl(stt, s);
              for (uint32_t e = a + lane; e < b; e += 64) {
                const KV x = kv_load<EW>(data, sts + e);
                if ((kv_mix<EW>(x) >> (64 - lvl)) == q) {
                  const uint32_t idx = atomicAdd(&s_qn, 1u);
                  if (idx < gcap) {
                    if constexpr (EW == 1) s_key[idx] = x.lo;
                    else { s_key[2 * idx] = x.lo; s_key[2 * idx + 1] = x.hi; }
                    s_own[idx] = (uint8_t)s;
                  }
                }
              }
            }
            __syncthreads();
            const uint32_t nq = s_qn;
            if (nq > gcap) {
              // split the slice: one value has at most 64 holders, so halves of
              // distinct values shrink; a 64-bit mix is a bijection for u64 values
              if (lvl < 64) {
                if (tid == 0) {
                  const uint32_t d = s_qd;
                  s_stk[2 * d] = 2 * q + 1;
                  s_stk[2 * d + 1] = lvl + 1;
                  s_stk[2 * d + 2] = 2 * q;
                  s_stk[2 * d + 3] = lvl + 1;
                  s_qd = d + 2;
                }
              } else if (tid == 0) {
                atomicAdd(stat + 1, 1u);  // > gcap 128-bit values with one 64-bit mix: layout invalid
              }
              __syncthreads();
              continue;
            }
            const uint32_t bq = (uint32_t)(q >> (lvl - gb_log));  // the slice's bucket
            if (bq != bk_cur) {  // first slice of a bucket
              if (bk_cur != ~0u) maxb = max(maxb, cur - bk_start);
              bk_cur = bq;
              bk_start = cur;
              if (tid == 0) boff[g * GB + bq] = cur;
            }
            for (uint32_t i = tid; i < nq; i += kPB) s_msk[i] = 0;
            __syncthreads();
            bool rp[kSlowPer];
#pragma unroll
            for (int k = 0; k < kSlowPer; ++k) {
              const uint32_t i = tid + k * kPB;
              rp[k] = false;
              if (i < nq) {
                const KV x = key_at<EW>(s_key, i);
                bool full_unused = false;  // one region of kTab slots for <= gcap <= kTab / 2 elements
                const uint32_t ri = dd_insert<EW>(s_tab, s_key, x, i, 0u, kTab - 1, &full_unused);
                if (CHECK && !kv_eq<EW>(key_at<EW>(s_key, ri), x)) atomicAdd(&g_layout_check, 1ull);
                atomicOr(&s_msk[ri], 1ull << s_own[i]);
                rp[k] = ri == i;
              }
            }
            __syncthreads();
#pragma unroll
            for (int k = 0; k < kSlowPer; ++k) {
              if (!rp[k]) continue;
              const uint32_t i = tid + k * kPB;
              const uint32_t d = atomicAdd(&s_gd, 1u);
              const uint64_t o = base + cur + d;
              kv_store<EW>(out_vals, o, key_at<EW>(s_key, i));
              out_masks[o] = s_msk[i];
            }
            __syncthreads();
            cur += s_gd;
          }
        }
        if (bk_cur != ~0u) maxb = max(maxb, cur - bk_start);
        // leave the table free and the masks clear for the next group
        __syncthreads();
        for (uint32_t q = tid; q < kTab / 4; q += kPB)
          reinterpret_cast<uint4*>(s_tab)[q] = make_uint4(kTFree, kTFree, kTFree, kTFree);
        for (uint32_t q = tid; q < kGCap / 2; q += kPB) reinterpret_cast<uint4*>(s_msk)[q] = make_uint4(0, 0, 0, 0);
#ifdef SKS_LAYOUT_STAMPS
        if (tid == 0) atomicAdd(&g_layout_stamps[8], 1ull);
#endif
      }
      LSTAMP(4);
    }
  }
  if (tid == 0) boff[B + r] = cur;
  LSTAMP_FLUSH();
  // the largest block-bucket: one word for every workgroup; the stat only
  // grows, so a workgroup whose maximum is not above the value it reads skips
  // the atomic (one word takes ~88 atomics per microsecond)
  if (wave == 0) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) maxb = max(maxb, (uint32_t)__shfl_xor(maxb, o, 64));
    if (lane == 0 && maxb && maxb > __hip_atomic_load(stat, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
      atomicMax(stat, maxb);
  }
}


// ---- u64 values (w <= 32): the dedup table holds the values themselves ---------------------
// k_gl_place1 is k_gl_place for u64 values with the values, not element
// indices, in a 2048-slot table of 64-bit words (one compare-swap per probe and
// no key array: 35 KB of LDS, four workgroups per CU).  The table's empty word is
// 0, so the value 0 (a poly-A k-mer) is kept apart as s_zero: its mix is 0, so
// it is the first value of bucket 0 (and of the first slice of bucket 0).
constexpr uint32_t kVLog = 8 + jc::kGLog, kVT = 1u << kVLog;  // value slots (2048)
constexpr uint32_t kVSpt = kVT / kPB;              // slots per thread in a scan emit (8)

static_assert(kGCap <= kVT, "a normal-path group fits the value table");
#ifndef SKS_LAYOUT_HALF_AT
#define SKS_LAYOUT_HALF_AT (kVT / 2)
#endif
constexpr uint32_t kHalfAt = SKS_LAYOUT_HALF_AT;   // predicted distinct values above which a group takes two halves
static_assert(kVSpt % 2 == 0, "scan emit reads slot pairs");

// Inserts v != 0 into the table region [rbase, rbase + rmask] starting at
// slot h0: one loop exit (see dd_insert).  Returns the slot holding v, or ~0u
// when the region is full; *claimed: this call stored v (v was new).
__device__ __forceinline__ uint32_t vt_insert(unsigned long long* s_vt, unsigned long long v, uint32_t rbase,
                                              uint32_t h0, uint32_t rmask, unsigned long long x, bool* claimed) {
  uint32_t hh = h0, steps = 0;
  for (;;) {
    if ((x == 0ull) | (x == v) | (steps > rmask)) break;
    hh = (hh + 1) & rmask;
    ++steps;
    x = atomicCAS(&s_vt[rbase + hh], 0ull, v);
  }
  *claimed = x == 0ull;
  return steps > rmask ? ~0u : rbase + hh;
}

// A pass of the value table: the values whose mix starts with a prefix of
// `lvl` bits in [q0, q0 + span).  span > 1 only at the bucket level (lvl =
// gb_log, span a power of two); the whole table is the pass's one region.
struct VPass {
  uint32_t lvl, span;
  uint64_t q0;
};
__device__ __forceinline__ bool vp_in(const VPass& p, uint64_t mix) {
  const uint64_t top = p.lvl ? mix >> (64 - p.lvl) : 0ull;
  return top - p.q0 < p.span;
}
template <bool CHECK>
#ifndef SKS_LAYOUT_WAVES
#define SKS_LAYOUT_WAVES 4
#endif
__global__ __launch_bounds__(kPB) __attribute__((amdgpu_waves_per_eu(SKS_LAYOUT_WAVES))) void k_gl_place1(const uint64_t* __restrict__ data,
                                                   const uint64_t* __restrict__ starts, uint32_t count,
                                                   uint32_t log_b, const uint32_t* __restrict__ pos,
                                                   const uint64_t* __restrict__ bstart,
                                                   uint64_t* __restrict__ out_vals,
                                                   unsigned long long* __restrict__ out_masks,
                                                   uint32_t* __restrict__ out_boff, uint32_t* __restrict__ stat,
                                                   uint32_t gcap, uint32_t rg) {
  __shared__ unsigned long long s_vt[kVT];  // values (0: empty)
  __shared__ unsigned long long s_vm[kVT];  // their sketch masks
  __shared__ uint32_t s_pos[(kMaxRG + 1) * kTile];
  __shared__ uint32_t s_bcnt[1u << jc::kGLog];
  __shared__ unsigned long long s_zero;       // holders of the value 0
  __shared__ uint32_t s_full, s_sd;
  __shared__ unsigned long long s_sq[72];     // pass stack: q0
  __shared__ uint32_t s_sl[72];               // pass stack: lvl << 8 | log2(span)
  __shared__ uint32_t s_w8[(1u << jc::kGLog) * (kPB / 64)];  // pass emit: per-bucket wave totals
#if SKS_LAYOUT_STAGED
  __shared__ uint16_t s_stage[kVT];  // normal-path emit: the group's entries' table slots, in place order
#endif

  const uint32_t B = 1u << log_b, gb_log = jc::lay_gb_log(log_b), GB = 1u << gb_log;
  const uint32_t G = B >> gb_log, NR = jc::lay_regions(log_b, rg), BW = jc::lay_boff_words(log_b);
  const uint32_t RG = (1u << jc::lay_rb_log(log_b, rg)) >> gb_log;
  const uint32_t blk = blockIdx.x / NR, r = blockIdx.x % NR;
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
#ifdef SKS_LAYOUT_STAMPS
  uint64_t st_last = __builtin_amdgcn_s_memtime();
  uint64_t st_acc[5] = {0, 0, 0, 0, 0};
#endif
  const uint32_t s_end = min((uint32_t)kTile, count - kTile * blk);
  uint32_t* boff = out_boff + (uint64_t)blk * BW;
  if (r == 0 && threadIdx.x == 0) boff[BW - 1] = jc::lay_rb_log(log_b, rg);  // the join reads the region size here
  const uint64_t base = bstart[blk];
  const bool sv = (uint32_t)lane < s_end;
  const uint64_t stt = sv ? starts[kTile * blk + lane] : 0;
  for (uint32_t q = tid; q < (RG + 1) * kTile; q += kPB) {
    const uint32_t j = q / kTile, s = q % kTile;
    s_pos[q] = s < s_end ? pos[(uint64_t)(kTile * blk + s) * (G + 1) + r * RG + j] : 0;
  }
  for (uint32_t q = tid; q < kVT / 2; q += kPB) {
    reinterpret_cast<uint4*>(s_vt)[q] = make_uint4(0, 0, 0, 0);
    reinterpret_cast<uint4*>(s_vm)[q] = make_uint4(0, 0, 0, 0);
  }
  if ((uint32_t)tid < (1u << jc::kGLog)) s_bcnt[tid] = 0;
  if (tid == 0) {
    s_full = 0;
    s_zero = 0;
  }
  __syncthreads();
  uint32_t cur = (uint32_t)__builtin_amdgcn_readlane((int)wave_scan(sv ? s_pos[lane] : 0u), 63);
  uint32_t maxb = 0;
  KV v[kRegPer];
  const uint32_t my_s = (uint32_t)tid / kTPS, sub = (uint32_t)tid % kTPS;
  const unsigned long long my_bit = 1ull << my_s;
  GroupView gv = group_view(s_pos, s_pos + kTile, sv, stt, lane, my_s);
  group_load<1>(data, gv, sub, v);
  uint32_t dshare = 1u << 16;  // distinct / raw of the region's last placed group (16.16)
  LSTAMP(0);

  // emit of a pass (thread t reads slots [8 t, 8 t + 8)): the pass's table holds
  // the values of buckets [q0, q0 + span) (a slice of one bucket when span = 1)
  // in one region; each thread counts its values per bucket, a wave scan per
  // bucket and the waves' totals place them bucket by bucket (any order within
  // a bucket), the value 0 first when the pass holds prefix 0
  auto emit_pass1 = [&](const VPass& p, uint32_t g, uint32_t first) {
    constexpr uint32_t NB = 1u << jc::kGLog;
    unsigned long long wv[kVSpt];
#pragma unroll
    for (int q = 0; q < (int)kVSpt / 2; ++q) {
      const ulonglong2 x = reinterpret_cast<const ulonglong2*>(s_vt)[tid * (kVSpt / 2) + q];
      wv[2 * q] = x.x;
      wv[2 * q + 1] = x.y;
    }
    uint32_t bq[kVSpt], cnt[NB];
#pragma unroll
    for (uint32_t b = 0; b < NB; ++b) cnt[b] = 0;
#pragma unroll
    for (int k = 0; k < (int)kVSpt; ++k) {
      const uint64_t mx = kv_mix<1>(KV{wv[k], 0});
      bq[k] = p.span > 1 ? (uint32_t)((mx >> (64 - gb_log)) - p.q0) : 0u;
#pragma unroll
      for (uint32_t b = 0; b < NB; ++b) cnt[b] += (wv[k] != 0ull && bq[k] == b) ? 1u : 0u;
    }
    uint32_t off[NB];
#pragma unroll
    for (uint32_t b = 0; b < NB; ++b) {
      const uint32_t incl = wave_scan(cnt[b]);
      off[b] = incl - cnt[b];
      if (lane == 63) s_w8[b * (kPB / 64) + wave] = incl;
    }
    __syncthreads();
    const uint32_t zero = (p.q0 == 0 && s_zero) ? 1u : 0u;
    uint32_t start = zero, total = zero;
#pragma unroll
    for (uint32_t b = 0; b < NB; ++b) {
      uint32_t tb = 0, before = 0;
#pragma unroll
      for (int w = 0; w < kPB / 64; ++w) {
        const uint32_t x = s_w8[b * (kPB / 64) + w];
        tb += x;
        before += w < wave ? x : 0u;
      }
      off[b] += start + before;
      if (p.span > 1 && (uint32_t)tid == b && b < p.span)
        boff[g * GB + (uint32_t)p.q0 + b] = cur + (b == 0 ? 0u : start);
      maxb = max(maxb, tb + (b == 0 ? zero : 0u));
      start += tb;
      total += tb;
    }
    if (p.span == 1 && first && tid == 0) boff[g * GB + (uint32_t)(p.q0 >> (p.lvl - gb_log))] = cur;
#pragma unroll
    for (int k = 0; k < (int)kVSpt; ++k) {
      if (wv[k] == 0ull) continue;
      uint32_t d = 0;
#pragma unroll
      for (uint32_t b = 0; b < NB; ++b)
        if (bq[k] == b) d = off[b]++;
      const uint32_t slot = tid * kVSpt + k;
      const uint64_t o = base + cur + d;
      out_vals[o] = wv[k];
      out_masks[o] = s_vm[slot];
      s_vt[slot] = 0ull;
      s_vm[slot] = 0ull;
    }
    if (tid == 0 && zero) {
      out_vals[base + cur] = 0ull;
      out_masks[base + cur] = s_zero;
    }
    cur += total;
    __syncthreads();  // every thread has read s_zero / s_w8
    if (tid == 0 && zero) s_zero = 0;
  };

  for (uint32_t j = 0; j < RG; ++j) {
    const uint32_t g = r * RG + j;
    const GroupView gj = gv;
    const uint32_t gn_j = gj.gn;
    bool done = false, fetched = false;
    if (gn_j == 0) {  // an empty group: its buckets start (and end) at the cursor
      if ((uint32_t)tid < GB) boff[g * GB + tid] = cur;
      done = true;
    } else if (gn_j <= gcap && !gj.fat) {
      // ---- normal path: the group's buckets from registers, in one or two passes ---------------
      // every element's first compare-swap issued together, then the (rare) rest of
      // the chains; a representative (the element that stored its value) takes the
      // next place of its bucket (entries contiguous per bucket, any order within).
      // The whole table is one region (placement goes by the bucket counters, not by
      // slot order); a group predicted to hold more than kHalfAt distinct values
      // (raw count x the region's running distinct share) is placed in two halves
      // of its buckets, keeping the table at most about half full (linear probing
      // at a load near 1 walks long chains: unrelated genomes' largest groups).
      const uint32_t nh = (GB > 1 && (uint64_t)gn_j * dshare > ((uint64_t)kHalfAt << 16)) ? 2u : 1u;
      const uint32_t bn = GB / nh;
      uint32_t dsum = 0;
      for (uint32_t hf = 0; hf < nh; ++hf) {
        const uint32_t blo = hf * bn;
        __syncthreads();  // the previous emit has freed its slots and reset s_bcnt / s_zero
        uint32_t h[kRegPer], bk[kRegPer];
        unsigned long long x0[kRegPer];
#pragma unroll
        for (int k = 0; k < kRegPer; ++k) {
          const uint32_t e = sub + kTPS * k;
          const uint64_t m = kv_mix<1>(v[k]);
          x0[k] = ~0ull;
          bk[k] = gb_log ? (uint32_t)(m >> (64 - gb_log)) : 0u;
          h[k] = (uint32_t)((gb_log ? m << gb_log : m) >> (64 - kVLog));  // (the bits after the bucket)
          if (e < gj.gc && v[k].lo != 0ull && bk[k] - blo < bn) x0[k] = atomicCAS(&s_vt[h[k]], 0ull, v[k].lo);
        }
        LSTAMP(1);
        bool full = false;
        uint32_t rep[kRegPer];
#pragma unroll
        for (int k = 0; k < kRegPer; ++k) {
          const uint32_t e = sub + kTPS * k;
          rep[k] = kTFree;
          if (e < gj.gc) {
            if (v[k].lo == 0ull) {  // (bucket 0: the first half)
              if (hf == 0) atomicOr(&s_zero, my_bit);
              continue;
            }
            if (bk[k] - blo >= bn) continue;
            bool claimed;
            const uint32_t slot = vt_insert(s_vt, v[k].lo, 0u, h[k], kVT - 1, x0[k], &claimed);
            if (slot == ~0u) {  // (unreachable: at most gcap <= kVT values)
              full = true;
              continue;
            }
            if (CHECK && s_vt[slot] != v[k].lo) atomicAdd(&g_layout_check, 1ull);
            atomicOr(&s_vm[slot], my_bit);
            if (claimed) {
              rep[k] = (bk[k] << 12) | atomicAdd(&s_bcnt[bk[k]], 1u);
              h[k] = slot;
            }
          }
        }
        if (full) atomicAdd(stat + 1, 1u);  // the layout is invalid (the caller retries)
        LSTAMP(2);
        if (hf + 1 == nh) {  // the next group's loads (in flight during the emit)
          if (j + 1 < RG) {
            gv = group_view(s_pos + (j + 1) * kTile, s_pos + (j + 2) * kTile, sv, stt, lane, my_s);
            group_load<1>(data, gv, sub, v);
          }
          fetched = true;
        }
        __syncthreads();
        const uint32_t zero = (hf == 0 && s_zero) ? 1u : 0u;  // the value 0: first in bucket 0
        uint32_t pre[1u << jc::kGLog], tot = zero;
#pragma unroll
        for (uint32_t b = 0; b < (1u << jc::kGLog); ++b) {
          const uint32_t c = b - blo < bn ? s_bcnt[b] : 0u;
          pre[b] = tot;
          tot += c;
          maxb = max(maxb, c + (b == 0 ? zero : 0u));
        }
        if ((uint32_t)tid < bn) boff[g * GB + blo + tid] = cur + (tid == 0 ? 0u : pre[blo + tid]);
#if SKS_LAYOUT_STAGED
        // each representative lists its table slot at its place; then the group's
        // entries leave with coalesced stores (a wave writes 512 contiguous bytes
        // of values and of masks) instead of one scattered 8-byte store each
#pragma unroll
        for (int k = 0; k < kRegPer; ++k)
          if (rep[k] != kTFree) s_stage[pre[rep[k] >> 12] + (rep[k] & 4095u)] = (uint16_t)h[k];
        if (tid == 0 && zero) s_stage[0] = 0xFFFFu;  // the value 0 (not in the table)
        __syncthreads();
        for (uint32_t e = (uint32_t)tid; e < tot; e += kPB) {
          const uint32_t slot = s_stage[e];
          const uint64_t o = base + cur + e;
          if (slot == 0xFFFFu) {
            out_vals[o] = 0ull;
            out_masks[o] = s_zero;
          } else {
            out_vals[o] = s_vt[slot];
            out_masks[o] = s_vm[slot];
            s_vt[slot] = 0ull;
            s_vm[slot] = 0ull;
          }
        }
#else
#pragma unroll
        for (int k = 0; k < kRegPer; ++k) {
          if (rep[k] == kTFree) continue;
          const uint64_t o = base + cur + pre[rep[k] >> 12] + (rep[k] & 4095u);
#if SKS_PLACE_DIAG != 4
          out_vals[o] = s_vt[h[k]];
          out_masks[o] = s_vm[h[k]];
#endif
          s_vt[h[k]] = 0ull;
          s_vm[h[k]] = 0ull;
        }
        if (tid == 0 && zero) {
          out_vals[base + cur] = 0ull;
          out_masks[base + cur] = s_zero;
        }
#endif
        cur += tot;
        dsum += tot;
        LSTAMP(3);
        __syncthreads();  // counts and s_zero read; the table is free again
        if ((uint32_t)tid < GB) s_bcnt[tid] = 0;
        if (tid == 0) s_zero = 0;
      }
      dshare = (uint32_t)(((uint64_t)dsum << 16) / gn_j);
      done = true;
    }
    if (!fetched && j + 1 < RG) {
      gv = group_view(s_pos + (j + 1) * kTile, s_pos + (j + 2) * kTile, sv, stt, lane, my_s);
      group_load<1>(data, gv, sub, v);
    }
    if (!done) {
      // ---- passes: prefixes of the values' mixes, re-read from the sketches --------------------
      // (a group above gcap raw elements, or with a sketch above kSkCap elements):
      // the buckets in parts of about 1536 elements; a pass whose table overflows
      // (more than 2048 distinct values) is split (buckets into halves, then a
      // bucket into hash slices), depth first, so entries come out in bucket and
      // slice order
      const GroupMap m = group_map(s_pos + j * kTile, s_pos + (j + 1) * kTile, sv, stt, lane);
#ifdef SKS_LAYOUT_STAMPS
      if (tid == 0) {
        atomicAdd(&g_layout_stamps[8], 1ull);
        atomicAdd(&g_layout_stamps[gj.fat ? 5 : gn_j > gcap ? 6 : 7], 1ull);
      }
#endif
      __syncthreads();
      if (tid == 0) {
        uint32_t parts = 1;  // predicted distinct values (raw x the running distinct share) per part <= 1536
        while (parts < GB && (uint64_t)gn_j * dshare > ((uint64_t)(3 * kVT / 4) << 16) * parts) parts <<= 1;
        const uint32_t sp_log = gb_log - (31 - __builtin_clz(parts));  // log2(GB / parts)
        for (uint32_t q = 0; q < parts; ++q) {  // rightmost first: the leftmost is on top
          s_sq[q] = (uint64_t)(parts - 1 - q) << sp_log;
          s_sl[q] = (gb_log << 8) | sp_log;
        }
        s_sd = parts;
      }
      __syncthreads();
      uint32_t bk_start = cur;
      const uint32_t cur0 = cur;
      for (;;) {
        const uint32_t depth = s_sd;
        if (depth == 0) break;
        VPass p;
        p.q0 = s_sq[depth - 1];
        p.lvl = s_sl[depth - 1] >> 8;
        const uint32_t sl2 = s_sl[depth - 1] & 255u;
        p.span = 1u << sl2;
        __syncthreads();
        if (tid == 0) s_sd = depth - 1;
        bool full = false;
        for (uint32_t c0 = (uint32_t)wave * 64; c0 < m.gn; c0 += kPB * kPassU) {
          KV x[kPassU];
          uint32_t o[kPassU];
#pragma unroll
          for (int u = 0; u < kPassU; ++u) {
            const uint32_t b = c0 + u * kPB;
            o[u] = 0;
            x[u] = KV{0, 0};
            if (b < m.gn) {
              const uint64_t at = elem_at(m, b, lane, &o[u]);
              if (b + (uint32_t)lane < m.gn) x[u] = kv_load<1>(data, at);
            }
          }
#pragma unroll
          for (int u = 0; u < kPassU; ++u) {
            if (c0 + u * kPB + (uint32_t)lane >= m.gn) continue;
            const uint64_t mx = kv_mix<1>(x[u]);
            if (!vp_in(p, mx)) continue;
            if (x[u].lo == 0ull) {
              atomicOr(&s_zero, 1ull << o[u]);
              continue;
            }
            const uint32_t h0 = (uint32_t)((p.lvl ? mx << p.lvl : mx) >> (64 - kVLog));
            bool claimed;
            const uint32_t slot = vt_insert(s_vt, x[u].lo, 0u, h0, kVT - 1, atomicCAS(&s_vt[h0], 0ull, x[u].lo),
                                            &claimed);
            if (slot == ~0u) {
              full = true;
              continue;
            }
            if (CHECK && s_vt[slot] != x[u].lo) atomicAdd(&g_layout_check, 1ull);
            atomicOr(&s_vm[slot], 1ull << o[u]);
          }
        }
        if (full) s_full = 1;
        __syncthreads();
        if (s_full) {  // split the pass: halves of its buckets, or two hash slices of its bucket
          for (uint32_t q = tid; q < kVT / 2; q += kPB) {
            reinterpret_cast<uint4*>(s_vt)[q] = make_uint4(0, 0, 0, 0);
            reinterpret_cast<uint4*>(s_vm)[q] = make_uint4(0, 0, 0, 0);
          }
          __syncthreads();
          if (tid == 0) {
#ifdef SKS_LAYOUT_STAMPS
            atomicAdd(&g_layout_stamps[9], 1ull);
#endif
            s_full = 0;
            s_zero = 0;
            const uint32_t d = s_sd;
            if (p.span > 1) {
              const uint32_t h2 = sl2 - 1;
              s_sq[d] = p.q0 + (p.span >> 1);
              s_sl[d] = (p.lvl << 8) | h2;
              s_sq[d + 1] = p.q0;
              s_sl[d + 1] = (p.lvl << 8) | h2;
            } else {
              s_sq[d] = 2 * p.q0 + 1;
              s_sl[d] = (p.lvl + 1) << 8;
              s_sq[d + 1] = 2 * p.q0;
              s_sl[d + 1] = (p.lvl + 1) << 8;
            }
            s_sd = d + 2;
          }
          __syncthreads();
          continue;
        }
        // the first slice of a bucket starts the bucket
        uint32_t first = 0;
        if (p.span == 1) {
          const uint32_t sh = p.lvl - gb_log;
          first = (p.q0 & ((1ull << sh) - 1)) == 0 ? 1u : 0u;
          if (first) bk_start = cur;
        }
        emit_pass1(p, g, first);
        if (p.span == 1) maxb = max(maxb, cur - bk_start);
      }
      dshare = (uint32_t)(((uint64_t)(cur - cur0) << 16) / gn_j);
      LSTAMP(4);
    }
  }
  if (tid == 0) boff[B + r] = cur;
  LSTAMP_FLUSH();
  if (wave == 0) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) maxb = max(maxb, (uint32_t)__shfl_xor(maxb, o, 64));
    if (lane == 0 && maxb && maxb > __hip_atomic_load(stat, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
      atomicMax(stat, maxb);
  }
}

}  // namespace

uint32_t join_layout_region_log(uint32_t n_blk, uint32_t log_b) {
  // region size: 8 groups when the grid fills the chip at 8 groups per
  // workgroup (1024 or more workgroups), else fewer, down to 2, so a small
  // build (a rank's own blocks, config 5's four blocks) is not one long
  // sequence of groups per workgroup on a few CUs (SKS_LAYOUT_RG forces one)
  static const char* force = getenv("SKS_LAYOUT_RG");
  if (force) return std::min<uint32_t>(jc::kRGLogMax, (uint32_t)atoi(force));
  uint32_t rg = jc::kRGLogMax;
  while (rg > 1 && (uint64_t)n_blk * jc::lay_regions(log_b, rg) < 1024) --rg;
  return rg;
}

uint32_t join_layout_groups(uint32_t log_b) { return jc::lay_groups(log_b); }
uint32_t join_layout_boff_words(uint32_t log_b) { return jc::lay_boff_words(log_b); }

hipError_t join_layout_bounds(const uint64_t* data, const uint64_t* starts, const uint32_t* sizes,
                              uint32_t count, uint32_t log_b, int ew, uint64_t* bounds, hipStream_t s) {
  if (log_b > jc::kMaxLogB || (ew != 1 && ew != 2)) return hipErrorInvalidValue;
  const uint32_t G = jc::lay_groups(log_b);
  const uint32_t nb = (G + 1 + kPT / 64 - 1) / (kPT / 64);
  if (ew == 1)
    hipLaunchKernelGGL(k_gl_prep<1>, dim3(nb), dim3(kPT), 0, s, data, starts, sizes, count, G, bounds, nb,
                       (uint64_t*)nullptr);
  else
    hipLaunchKernelGGL(k_gl_prep<2>, dim3(nb), dim3(kPT), 0, s, data, starts, sizes, count, G, bounds, nb,
                       (uint64_t*)nullptr);
  return hipGetLastError();
}

// temp = bounds | pos[count][G + 1]
size_t join_layout_temp_bytes(uint32_t count, uint32_t log_b, int ew) {
  const uint64_t G = jc::lay_groups(log_b);
  return ((G + 1) * 8 * ew + 255) / 256 * 256 + (uint64_t)count * (G + 1) * 4 + 16;
}

// SKS_LAYOUT_GROUP_CAP (diagnostics, clamped to [64, kGCap]): the largest
// group placed by the fast path and the largest slice of the slow path; tests
// lower it to drive the slow path and its slice splits with small inputs
static uint32_t group_cap() {  // read per build (tests change it within one process)
  const char* e = getenv("SKS_LAYOUT_GROUP_CAP");
  return e ? std::max<uint32_t>(64, std::min<uint32_t>(kGCap, (uint32_t)atoi(e))) : kGCap;
}

unsigned long long layout_check_take() {
  unsigned long long h = 0;
  (void)hipMemcpyFromSymbol(&h, HIP_SYMBOL(g_layout_check), sizeof h);
  const unsigned long long z = 0;
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_layout_check), &z, sizeof z);
  return h;
}

hipError_t join_layout_build(const uint64_t* data, const uint64_t* starts, const uint32_t* sizes,
                             uint32_t count, uint32_t log_b, int ew, const uint64_t* d_bounds, void* temp,
                             uint64_t* out_vals, uint64_t* out_masks, uint32_t* out_boff,
                             uint64_t* out_bstart, uint32_t* d_stat, bool check, hipStream_t s,
                             const ZeroSpans* zero, uint32_t blocks_hint) {
  if (log_b > jc::kMaxLogB || (ew != 1 && ew != 2)) return hipErrorInvalidValue;
  if (count == 0) return hipSuccess;
  const ZeroSpans zs = zero ? *zero : ZeroSpans{};
  const uint32_t G = jc::lay_groups(log_b);
  const uint32_t n_blk = (count + kTile - 1) / kTile;
  uint64_t* bounds_tmp = static_cast<uint64_t*>(temp);
  uint32_t* pos = reinterpret_cast<uint32_t*>(static_cast<char*>(temp) + ((G + 1) * 8 * ew + 255) / 256 * 256);
  // bounds (unless given) and block starts in one launch, the groups' positions
  // in every sketch, then the placement: a workgroup per (block, region)
  const uint32_t nb_bounds = d_bounds ? 0 : (G + 1 + kPT / 64 - 1) / (kPT / 64);
  const uint64_t* bounds = d_bounds ? d_bounds : bounds_tmp;
  // region size: 8 groups when the grid fills the chip at 8 groups per
  // workgroup (1024 or more workgroups), else fewer, down to 2, so a small
  // build (a rank's own blocks, config 5's four blocks) is not one long
  // sequence of groups per workgroup on a few CUs (SKS_LAYOUT_RG forces one)
  // (blocks_hint: the blocks that hold sketches, when many are empty — a rank's
  // exchange buffer — so the region size fits the work, not the row count)
  const uint32_t rg = join_layout_region_log(blocks_hint ? std::min(blocks_hint, n_blk) : n_blk, log_b);
  const dim3 grid_place(n_blk * jc::lay_regions(log_b, rg));
  auto* masks = reinterpret_cast<unsigned long long*>(out_masks);
  if (ew == 1) {
    hipLaunchKernelGGL(k_gl_prep<1>, dim3(nb_bounds + 1), dim3(kPT), 0, s, data, starts, sizes, count, G,
                       bounds_tmp, nb_bounds, out_bstart);
    hipLaunchKernelGGL(k_gl_pos<1>, dim3(count), dim3(kPT), 0, s, data, starts, sizes, count, G, bounds, pos, zs);
    if (check)
      hipLaunchKernelGGL((k_gl_place1<true>), grid_place, dim3(kPB), 0, s, data, starts, count, log_b, pos,
                         out_bstart, out_vals, masks, out_boff, d_stat, group_cap(), rg);
    else
      hipLaunchKernelGGL((k_gl_place1<false>), grid_place, dim3(kPB), 0, s, data, starts, count, log_b, pos,
                         out_bstart, out_vals, masks, out_boff, d_stat, group_cap(), rg);
  } else {
    hipLaunchKernelGGL(k_gl_prep<2>, dim3(nb_bounds + 1), dim3(kPT), 0, s, data, starts, sizes, count, G,
                       bounds_tmp, nb_bounds, out_bstart);
    hipLaunchKernelGGL(k_gl_pos<2>, dim3(count), dim3(kPT), 0, s, data, starts, sizes, count, G, bounds, pos, zs);
    if (check)
      hipLaunchKernelGGL((k_gl_place<2, true>), grid_place, dim3(kPB), 0, s, data, starts, count, log_b, pos,
                         out_bstart, out_vals, masks, out_boff, d_stat, group_cap(), rg);
    else
      hipLaunchKernelGGL((k_gl_place<2, false>), grid_place, dim3(kPB), 0, s, data, starts, count, log_b, pos,
                         out_bstart, out_vals, masks, out_boff, d_stat, group_cap(), rg);
  }
#ifdef SKS_LAYOUT_STAMPS
  {
    unsigned long long h[10] = {0};
    (void)hipStreamSynchronize(s);
    (void)hipMemcpyFromSymbol(h, HIP_SYMBOL(g_layout_stamps), sizeof h);
    const unsigned long long z[10] = {0};
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_layout_stamps), z, sizeof z);
    const uint32_t nw = std::min<uint32_t>(grid_place.x, kMaxStampWgs);
    std::vector<unsigned long long> wg((size_t)nw * 5);
    (void)hipMemcpyFromSymbol(wg.data(), HIP_SYMBOL(g_layout_stamps_wg), wg.size() * 8);
    for (uint32_t b = 0; b < nw; ++b)
      for (int q = 0; q < 5; ++q) h[q] += wg[(size_t)b * 5 + q];
    const double wgs = (double)nw;
    fprintf(stderr, "[k_gl_place stamps] cycles per workgroup: setup %.0f load wait+first CAS %.0f chains %.0f "
            "emit %.0f passes %.0f | groups in passes %llu (fat %llu, above cap %llu, full %llu), "
            "pass splits %llu (%.0f workgroups)\n",
            h[0] / wgs, h[1] / wgs, h[2] / wgs, h[3] / wgs, h[4] / wgs, h[8], h[5], h[6], h[7], h[9], wgs);
  }
#endif
  return hipGetLastError();
}

SKS_CODE_OBJECT_HOOK(layout)

}  // namespace sks
