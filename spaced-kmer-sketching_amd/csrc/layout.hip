// The join layout (input of k_join, join.hip; format in join_common.hpp): for
// every block of 64 consecutive sketches, each distinct value once with the
// mask of the block's sketches holding it, bucket by bucket.
//
// Buckets are two-level.  The value range is cut into G = B / 8 groups by
// common bounds (quantiles averaged over up to 64 sample sketches), and a
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
constexpr uint32_t kGCap = 2048;         // elements of one dedup batch (a group)
constexpr int kPer = kGCap / kPT;        // elements per thread
constexpr int kTabLog = 12;              // dedup table: 4096 slots (load <= 1/2)
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
// element that represents v (i itself when v was new: *claimed = its slot).
// The table is cut into one region of kTab >> rb slots per hash bucket of the
// group (rb = the bucket bits) and a value probes only its bucket's region, so
// reading the table in slot order lists the distinct values bucket by bucket.
// More distinct values than a region holds (never at the group sizes the
// bucket count is chosen for) set *full: the caller redoes the group on the
// slow path.  The probe loop has ONE exit edge and evaluates its stop test
// without short-circuit (the element a slot word names is read whether or not
// the tag matches; a free word names element 2047, read and ignored): the
// two-exit form of this loop (free slot / same value, the entry assigned at
// each exit) was miscompiled by ROCm 7.2 for gfx950 in round 3 (DESIGN.md §5;
// reproducer in tools/microbench/chain_exits.hip).
template <int EW>
__device__ __forceinline__ uint32_t dd_insert(uint32_t* s_tab, const uint64_t* s_key, const KV& v, uint32_t i,
                                              uint32_t rb, uint32_t* claimed, bool* full) {
  const uint32_t tag = dd_tag<EW>(v);
  const uint32_t word = (tag << kIdxBits) | i;
  const uint32_t rlog = kTabLog - rb, rmask = (1u << rlog) - 1;
  const uint32_t base = rb ? (uint32_t)(kv_mix<EW>(v) >> (64 - rb)) << rlog : 0u;
  uint32_t h = dd_slot<EW>(v) & rmask, steps = 0;
  uint32_t x = atomicCAS(&s_tab[base + h], kTFree, word);
  for (;;) {
    const KV u = key_at<EW>(s_key, x & kIdxMask);
    if ((x == kTFree) | (((x >> kIdxBits) == tag) & kv_eq<EW>(u, v)) | (steps > rmask)) break;
    h = (h + 1) & rmask;
    ++steps;
    x = atomicCAS(&s_tab[base + h], kTFree, word);
  }
  *claimed = base + h;
  if (steps > rmask) *full = true;
  return x == kTFree ? i : (x & kIdxMask);
}

// Workgroups [0, nb_bounds): the group bounds, a wave per bound (bounds[g] =
// mean over up to 64 sample sketches of their g/G quantile; bounds[0] = 0,
// bounds[G] = the largest value).  128-bit values are averaged as doubles
// (hi * 2^64 + lo) and split back: every step is monotonic, so the bounds are
// non-decreasing, which is all exactness needs.  The last workgroup:
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
    double x = 0.0, used = 0.0;
    if ((uint32_t)lane < K && g > 0 && g < G) {
      const uint32_t i = (uint32_t)((uint64_t)lane * count / K);
      const uint32_t sz = sizes[i];
      if (sz) {
        const KV q = kv_load<EW>(data, starts[i] + (uint64_t)g * sz / G);
        x = EW == 1 ? (double)q.lo : (double)q.hi * 18446744073709551616.0 + (double)q.lo;
        used = 1.0;
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      x += __shfl_xor(x, o, 64);
      used += __shfl_xor(used, o, 64);
    }
    if (lane) return;
    KV b{0, 0};
    if (g == G) {
      b = KV{~0ull, EW == 1 ? 0ull : ~0ull};
    } else if (g > 0) {
      const double m = used > 0.0 ? x / used : 0.0;
      if (EW == 1) {
        b.lo = m >= 18446744073709549568.0 ? ~0ull : (uint64_t)m;
      } else {
        const double h = floor(m * (1.0 / 18446744073709551616.0));
        b.hi = h >= 18446744073709549568.0 ? ~0ull : (uint64_t)h;
        const double r = m - h * 18446744073709551616.0;  // exact
        b.lo = r >= 18446744073709549568.0 ? ~0ull : (uint64_t)r;
      }
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
                                                uint32_t* __restrict__ pos, uint32_t* __restrict__ zero_words,
                                                uint32_t n_zero) {
  __shared__ uint64_t s_smp[kPosSamples * EW];
  const uint32_t i = blockIdx.x;
  // the placement's tickets and look-back words start at zero (grid-strided)
  for (uint32_t z = i * kPT + threadIdx.x; z < n_zero; z += gridDim.x * kPT) zero_words[z] = 0;
  const uint32_t sz = sizes[i];
  const uint64_t st = starts[i];
  uint32_t stride = kPosStride;
  while ((uint64_t)stride * kPosSamples < sz) stride <<= 1;
  const uint32_t ns = (sz + stride - 1) / stride;  // sample k = S[k * stride]
  for (uint32_t k = threadIdx.x; k < ns; k += kPT) kv_store<EW>(s_smp, k, kv_load<EW>(data, st + (uint64_t)k * stride));
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
    while (a < e) {
      const uint32_t mid = (a + e) >> 1;
      if (kv_lt<EW>(kv_load<EW>(data, st + mid), x)) a = mid + 1; else e = mid;
    }
    out[g] = a;
  }
}

__device__ unsigned long long g_layout_check;  // SKS check build: dedup invariant violations

// One workgroup per (block, value group).  A region's groups write one
// contiguous run of entries, so each workgroup needs the distinct counts of
// the region's earlier groups: it takes a ticket (its order in the region,
// which is also the group it handles — HIP promises no dispatch order, and a
// workgroup only ever waits for workgroups that took earlier tickets, so all
// of them are running), deduplicates its group, publishes the group's count
// and looks back over its predecessors' published counts (decoupled
// look-back; an 8-byte {flag, value} word per group, agent-scope atomics on
// both sides).  Phases of the normal path (a group of <= gcap elements):
//   P1  its elements (read into registers) go to s_key, masks cleared
//   P2  every element is inserted into the dedup table; the representative of
//       its value (the element that claimed a slot) collects the holders' bits
//       in s_msk; representatives are counted per (bucket, lane & 15)
//   P3  wave 0 scans the counts (cursors); the group's count is published and
//       the region prefix looked up
//   P4  bucket starts -> boff; representatives take a cursor and write
//       {value, mask} at region start + prefix + cursor
// A group above gcap elements (skewed values) takes the slow path: the prefix
// first, then hash slices of the group, each gathered from the sketches,
// deduplicated and written in slice order (a slice that still holds more than
// gcap elements is split in two); exact for any input, reading the group once
// per slice.
constexpr uint64_t kStAgg = 1ull << 62, kStInc = 1ull << 63;

#ifdef SKS_LAYOUT_STAMPS  // diagnostic build: cycles per k_gl_place phase (thread 0 of each workgroup)
__device__ unsigned long long g_layout_stamps[10];
#define LSTAMP(i)                                              \
  do {                                                         \
    if (threadIdx.x == 0) {                                    \
      const uint64_t t_ = __builtin_amdgcn_s_memtime();        \
      atomicAdd(&g_layout_stamps[i], (unsigned long long)(t_ - st_last)); \
      st_last = t_;                                            \
    }                                                          \
  } while (0)
#else
#define LSTAMP(i) do {} while (0)
#endif

__device__ __forceinline__ void status_publish(unsigned long long* st, uint64_t v) {
  __hip_atomic_store(st, (unsigned long long)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// sum of the distinct counts of groups [0, j) of the region (thread 0 only)
__device__ __forceinline__ uint32_t region_prefix(unsigned long long* st, uint32_t j) {
  uint32_t prefix = 0;
  for (int p = (int)j - 1; p >= 0; --p) {
    unsigned long long v;
    while (((v = __hip_atomic_load(st + p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) >> 62) == 0)
      __builtin_amdgcn_s_sleep(1);
    prefix += (uint32_t)v;
    if (v & kStInc) break;
  }
  return prefix;
}

template <int EW, bool CHECK>
__global__ __launch_bounds__(kPT) void k_gl_place(const uint64_t* __restrict__ data,
                                                  const uint64_t* __restrict__ starts, uint32_t count,
                                                  uint32_t log_b, const uint32_t* __restrict__ pos,
                                                  const uint64_t* __restrict__ bstart,
                                                  uint64_t* __restrict__ out_vals,
                                                  unsigned long long* __restrict__ out_masks,
                                                  uint32_t* __restrict__ out_boff, uint32_t* __restrict__ stat,
                                                  uint32_t gcap, uint32_t* __restrict__ tickets,
                                                  unsigned long long* __restrict__ status) {
  __shared__ uint64_t s_key[kGCap * EW];
  __shared__ unsigned long long s_msk[kGCap];
  __shared__ uint32_t s_tab[kTab];
  __shared__ uint8_t s_own[kGCap];   // element i of the group -> its sketch's slot
  __shared__ uint64_t s_src[kTile];  // element index in `data` of slot s's element i: s_src[s] + i
  __shared__ uint32_t s_wsum[kPT / 64];
  __shared__ uint32_t s_j, s_pre, s_gd, s_qn, s_qd, s_full;
  __shared__ uint32_t s_stk[2 * 72];  // slow path: (slice, level) work stack

  const uint32_t B = 1u << log_b, gb_log = jc::lay_gb_log(log_b), GB = 1u << gb_log;
  const uint32_t G = B >> gb_log, NR = jc::lay_regions(log_b);
  const uint32_t RG = (1u << jc::lay_rb_log(log_b)) >> gb_log;
  const uint32_t blk = blockIdx.x / G, r = (blockIdx.x % G) / RG;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
#ifdef SKS_LAYOUT_STAMPS
  uint64_t st_last = __builtin_amdgcn_s_memtime();
#endif
  if (tid == 0) s_j = RG == 1 ? 0u : atomicAdd(&tickets[blk * NR + r], 1u);
  for (uint32_t i = tid; i < kTab / 4; i += kPT)
    reinterpret_cast<uint4*>(s_tab)[i] = make_uint4(kTFree, kTFree, kTFree, kTFree);
  for (uint32_t i = tid; i < kGCap / 2; i += kPT) reinterpret_cast<uint4*>(s_msk)[i] = make_uint4(0, 0, 0, 0);
  __syncthreads();
  const uint32_t j = s_j, g = r * RG + j;
  unsigned long long* st = status + (uint64_t)(blk * NR + r) * RG;
  const uint32_t s_end = min((uint32_t)kTile, count - kTile * blk);
  uint32_t* boff = out_boff + (uint64_t)blk * (B + NR);
  const uint64_t base = bstart[blk];
  const bool sv = (uint32_t)lane < s_end;
  const uint32_t* prow = pos + (uint64_t)(kTile * blk + (sv ? lane : 0)) * (G + 1);
  const uint64_t stt = sv ? starts[kTile * blk + lane] : 0;
  // lane s: its sketch's range [glo, ghi) in the group; the region's raw offset
  const uint32_t glo = sv ? prow[g] : 0;
  const uint32_t ghi = sv ? max(prow[g + 1], glo) : 0;
  const uint32_t roff = __shfl(wave_scan(sv ? prow[r * RG] : 0), 63);
  const uint32_t gc = ghi - glo, gincl = wave_scan(gc), gpre = gincl - gc;
  const uint32_t gn = __shfl(gincl, 63);
  uint32_t maxb = 0;
  LSTAMP(0);

  bool normal = gn <= gcap;
  if (normal) {
    // ---- normal path -------------------------------------------------------------------------
    for (uint32_t s = wave; s < s_end; s += kPT / 64) {  // owner map: element i -> slot
      const uint32_t ps = __shfl(gpre, s), cs = __shfl(gc, s);
      for (uint32_t e = lane; e < cs; e += 64) s_own[ps + e] = (uint8_t)s;
    }
    if (wave == 0) s_src[lane] = stt + glo - gpre;
    if (tid == 0) s_full = 0;
    __syncthreads();
    LSTAMP(1);
    KV v[kPer];
    uint32_t sl[kPer];
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
      const uint32_t i = tid + k * kPT;
      sl[k] = 0;
      v[k] = KV{0, 0};
      if (i < gn) {
        const uint32_t s = s_own[i];
        sl[k] = s;
        v[k] = kv_load<EW>(data, s_src[s] + i);
      }
    }
    // P1
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
      const uint32_t i = tid + k * kPT;
      if (i < gn) {
        if constexpr (EW == 1) s_key[i] = v[k].lo;
        else { s_key[2 * i] = v[k].lo; s_key[2 * i + 1] = v[k].hi; }
      }
    }
    __syncthreads();
    LSTAMP(2);
    // P2: dedup; the representative's mask collects the holders' bits
    bool full = false;
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
      const uint32_t i = tid + k * kPT;
      if (i < gn) {
        uint32_t h;
        const uint32_t ri = dd_insert<EW>(s_tab, s_key, v[k], i, gb_log, &h, &full);
        if (CHECK && !kv_eq<EW>(key_at<EW>(s_key, ri), v[k])) atomicAdd(&g_layout_check, 1ull);
        atomicOr(&s_msk[ri], 1ull << sl[k]);
      }
    }
    if (full) s_full = 1;
    __syncthreads();
    LSTAMP(3);
    normal = s_full == 0;
    if (normal) {
      // P3: the table in slot order lists the distinct values bucket by bucket;
      // thread t owns slots [16 t, 16 t + 16): occupied counts, block scan
      constexpr uint32_t kSpt = kTab / kPT;
      uint32_t wv[kSpt];
#pragma unroll
      for (int q = 0; q < (int)kSpt / 4; ++q) {
        const uint4 x = reinterpret_cast<const uint4*>(s_tab)[tid * (kSpt / 4) + q];
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
      for (int w = 0; w < kPT / 64; ++w) {
        const uint32_t x = s_wsum[w];
        before += w < wave ? x : 0;
        total += x;
      }
      const uint32_t excl = before + wincl - occ;  // entries before this thread's slots
      if (tid == 0) {
        if (j == 0) {
          if (RG > 1) status_publish(st, kStInc | total);
          s_pre = 0;
        } else {
          status_publish(st + j, kStAgg | total);
          const uint32_t pre = region_prefix(st, j);
          status_publish(st + j, kStInc | (uint64_t)(pre + total));
          s_pre = pre;
        }
      }
      // bucket b's slots are threads [b * tpb, (b + 1) * tpb): its start and size
      const uint32_t tpb = kPT >> gb_log;
      const uint32_t b = tid / tpb;
      __syncthreads();
      LSTAMP(4);
      const uint32_t start = roff + s_pre;
      if (tid % tpb == 0) boff[g * GB + b] = start + excl;
      if (tid == 0 && j + 1 == RG) boff[B + r] = start + total;
      // P4: write this thread's entries in slot order
      uint32_t d = excl;
#pragma unroll
      for (int q = 0; q < (int)kSpt; ++q) {
        if (wv[q] == kTFree) continue;
        const uint32_t i = wv[q] & kIdxMask;
        const uint64_t o = base + start + d;
        ++d;
        kv_store<EW>(out_vals, o, key_at<EW>(s_key, i));
        out_masks[o] = s_msk[i];
      }
      // largest bucket: per bucket, the sum of its threads' occupied counts
      uint32_t bo = occ;
      for (uint32_t o2 = 1; o2 < tpb && o2 < 64; o2 <<= 1) bo += __shfl_xor(bo, o2, 64);
      if (tpb > 64) {  // a bucket spans waves (gb_log < 2): add the other waves' sums
        if (lane == 0) s_wsum[wave] = bo;
        __syncthreads();
        bo = 0;
        for (uint32_t w = (tid / tpb) * (tpb / 64); w < (tid / tpb + 1) * (tpb / 64); ++w) bo += s_wsum[w];
      }
      maxb = max(maxb, bo);
      LSTAMP(5);
    }
  }
  if (!normal) {
    // ---- slow path: the prefix first, then hash slices of the group ------------------------
    for (uint32_t q = tid; q < kTab / 4; q += kPT)  // (after a full table on the normal path)
      reinterpret_cast<uint4*>(s_tab)[q] = make_uint4(kTFree, kTFree, kTFree, kTFree);
    if (tid == 0) s_pre = region_prefix(st, j);
    __syncthreads();
    const uint32_t start = roff + s_pre;
    uint32_t cur = start;
    uint32_t lvl0 = max(gb_log, 1u);
    while (lvl0 < 32 && ((uint64_t)gn >> (lvl0 - 1)) > gcap / 2) ++lvl0;
    uint32_t bk_cur = ~0u, bk_start = cur;
    for (uint32_t q0 = 0; q0 < (1u << lvl0); ++q0) {
      // depth-first over the slice and, when it is too large, its halves
      // (smallest slice on top, so slices come out in hash order)
      if (tid == 0) {
        s_stk[0] = q0;
        s_stk[1] = lvl0;
        s_qd = 1;
      }
      __syncthreads();
      for (;;) {
        const uint32_t depth = s_qd;
        if (depth == 0) break;
        const uint32_t q = s_stk[2 * (depth - 1)], lvl = s_stk[2 * (depth - 1) + 1];
        __syncthreads();
        if (tid == 0) {
          s_qd = depth - 1;
          s_qn = 0;
          s_gd = 0;
        }
        for (uint32_t i = tid; i < kTab / 4; i += kPT)
          reinterpret_cast<uint4*>(s_tab)[i] = make_uint4(kTFree, kTFree, kTFree, kTFree);
        __syncthreads();
        for (uint32_t s = wave; s < s_end; s += kPT / 64) {
          const uint32_t a = __shfl(glo, s), b = __shfl(ghi, s);
          const uint64_t sts = __shfl(stt, s);
          for (uint32_t e = a + lane; e < b; e += 64) {
            const KV x = kv_load<EW>(data, sts + e);
            if ((kv_mix<EW>(x) >> (64 - lvl)) == (uint64_t)q) {
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
        const uint32_t bq = (uint32_t)((uint64_t)q >> (lvl - gb_log));  // the slice's bucket
        if (bq != bk_cur) {  // first slice of a bucket
          if (bk_cur != ~0u) maxb = max(maxb, cur - bk_start);
          bk_cur = bq;
          bk_start = cur;
          if (tid == 0) boff[g * GB + bq] = cur;
        }
        for (uint32_t i = tid; i < nq; i += kPT) s_msk[i] = 0;
        __syncthreads();
        bool rp[kPer];
#pragma unroll
        for (int k = 0; k < kPer; ++k) {
          const uint32_t i = tid + k * kPT;
          rp[k] = false;
          if (i < nq) {
            const KV x = key_at<EW>(s_key, i);
            uint32_t h;
            bool full_unused = false;  // one region of kTab slots for <= gcap <= kTab / 2 elements
            const uint32_t ri = dd_insert<EW>(s_tab, s_key, x, i, 0u, &h, &full_unused);
            if (CHECK && !kv_eq<EW>(key_at<EW>(s_key, ri), x)) atomicAdd(&g_layout_check, 1ull);
            atomicOr(&s_msk[ri], 1ull << s_own[i]);
            rp[k] = ri == i;
          }
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < kPer; ++k) {
          if (!rp[k]) continue;
          const uint32_t i = tid + k * kPT;
          const uint32_t d = atomicAdd(&s_gd, 1u);
          const uint64_t o = base + cur + d;
          kv_store<EW>(out_vals, o, key_at<EW>(s_key, i));
          out_masks[o] = s_msk[i];
        }
        __syncthreads();
        cur += s_gd;
      }
      __syncthreads();  // every thread has read the empty stack before the next slice is pushed
    }
    if (bk_cur != ~0u) maxb = max(maxb, cur - bk_start);
    LSTAMP(7);
#ifdef SKS_LAYOUT_STAMPS
    if (tid == 0) atomicAdd(&g_layout_stamps[8], 1ull);
#endif
    if (tid == 0) {
      status_publish(st + j, kStInc | (uint64_t)(cur - roff));
      if (j + 1 == RG) boff[B + r] = cur;
    }
  }
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

}  // namespace

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

// temp = bounds | pos[count][G + 1] | tickets[n_blk * NR] (even) | look-back words[n_blk * G]
size_t join_layout_temp_bytes(uint32_t count, uint32_t log_b, int ew) {
  const uint64_t G = jc::lay_groups(log_b), n_blk = (count + kTile - 1) / kTile;
  const uint64_t n_tick = n_blk * jc::lay_regions(log_b);
  return ((G + 1) * 8 * ew + 255) / 256 * 256 + (uint64_t)count * (G + 1) * 4 + ((n_tick + 1) & ~1ull) * 4 +
         n_blk * G * 8 + 16;
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
                             uint64_t* out_bstart, uint32_t* d_stat, bool check, hipStream_t s) {
  if (log_b > jc::kMaxLogB || (ew != 1 && ew != 2)) return hipErrorInvalidValue;
  if (count == 0) return hipSuccess;
  const uint32_t G = jc::lay_groups(log_b);
  const uint32_t n_blk = (count + kTile - 1) / kTile;
  uint64_t* bounds_tmp = static_cast<uint64_t*>(temp);
  uint32_t* pos = reinterpret_cast<uint32_t*>(static_cast<char*>(temp) + ((G + 1) * 8 * ew + 255) / 256 * 256);
  // placement tickets [n_blk * NR] u32, then look-back words [n_blk * G] u64
  const uint64_t n_tick = (uint64_t)n_blk * jc::lay_regions(log_b);
  uint32_t* tickets = pos + (((uint64_t)count * (G + 1) + 1) & ~(uint64_t)1);  // 8-byte aligned
  unsigned long long* status =
      reinterpret_cast<unsigned long long*>(tickets + ((n_tick + 1) & ~(uint64_t)1));
  const uint32_t n_zero = (uint32_t)(((n_tick + 1) & ~(uint64_t)1) + 2ull * n_blk * G);
  // bounds (unless given) and block starts in one launch, the groups' positions
  // in every sketch (and the zeroed look-back state), then the placement
  const uint32_t nb_bounds = d_bounds ? 0 : (G + 1 + kPT / 64 - 1) / (kPT / 64);
  const uint64_t* bounds = d_bounds ? d_bounds : bounds_tmp;
  const dim3 grid_place(n_blk * G);
  auto* masks = reinterpret_cast<unsigned long long*>(out_masks);
  if (ew == 1) {
    hipLaunchKernelGGL(k_gl_prep<1>, dim3(nb_bounds + 1), dim3(kPT), 0, s, data, starts, sizes, count, G,
                       bounds_tmp, nb_bounds, out_bstart);
    hipLaunchKernelGGL(k_gl_pos<1>, dim3(count), dim3(kPT), 0, s, data, starts, sizes, count, G, bounds, pos,
                       tickets, n_zero);
    if (check)
      hipLaunchKernelGGL((k_gl_place<1, true>), grid_place, dim3(kPT), 0, s, data, starts, count, log_b, pos,
                         out_bstart, out_vals, masks, out_boff, d_stat, group_cap(), tickets, status);
    else
      hipLaunchKernelGGL((k_gl_place<1, false>), grid_place, dim3(kPT), 0, s, data, starts, count, log_b, pos,
                         out_bstart, out_vals, masks, out_boff, d_stat, group_cap(), tickets, status);
  } else {
    hipLaunchKernelGGL(k_gl_prep<2>, dim3(nb_bounds + 1), dim3(kPT), 0, s, data, starts, sizes, count, G,
                       bounds_tmp, nb_bounds, out_bstart);
    hipLaunchKernelGGL(k_gl_pos<2>, dim3(count), dim3(kPT), 0, s, data, starts, sizes, count, G, bounds, pos,
                       tickets, n_zero);
    if (check)
      hipLaunchKernelGGL((k_gl_place<2, true>), grid_place, dim3(kPT), 0, s, data, starts, count, log_b, pos,
                         out_bstart, out_vals, masks, out_boff, d_stat, group_cap(), tickets, status);
    else
      hipLaunchKernelGGL((k_gl_place<2, false>), grid_place, dim3(kPT), 0, s, data, starts, count, log_b, pos,
                         out_bstart, out_vals, masks, out_boff, d_stat, group_cap(), tickets, status);
  }
#ifdef SKS_LAYOUT_STAMPS
  {
    unsigned long long h[10] = {0};
    (void)hipStreamSynchronize(s);
    (void)hipMemcpyFromSymbol(h, HIP_SYMBOL(g_layout_stamps), sizeof h);
    const unsigned long long z[10] = {0};
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_layout_stamps), z, sizeof z);
    const double wgs = (double)grid_place.x;
    fprintf(stderr, "[k_gl_place stamps] cycles per workgroup: ticket+meta %.0f own %.0f load+P1 %.0f P2 %.0f "
            "P3+lookback %.0f P4 %.0f | slow groups %llu, cycles each %.0f (%.0f workgroups)\n", h[0] / wgs,
            h[1] / wgs, h[2] / wgs, h[3] / wgs, h[4] / wgs, h[5] / wgs, h[8], h[8] ? h[7] / (double)h[8] : 0.0, wgs);
  }
#endif
  return hipGetLastError();
}

}  // namespace sks
