// Post-scan stages of the sketch build: survivor compaction, per-genome radix
// sort, unique, bottom-s selection, export to a fixed-stride layout, and the
// synthetic-genome generator used by the bench and tests.
//
// The reference collapses duplicate selected k-mers by inserting them into an
// std::unordered_map (kmer.hpp:170-178).  Here a genome's survivors are
// radix-sorted (rocPRIM) and run-length uniqued, which yields the same set and
// leaves it sorted for the merge-based intersection kernel.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <rocprim/rocprim.hpp>
#include <rocprim/block/block_radix_sort.hpp>

#include "sks_hash.hpp"
#include "sks_internal.hpp"

namespace sks {

hipError_t Scratch::reserve(size_t n) {
  if (n <= bytes) return hipSuccess;
  // grow by at least half: a caller whose need creeps up (the reference sweep's
  // sketches grow with k over its first configurations) reallocates a few
  // times, not once per call (a reallocation costs 0.1-1 ms of hipMalloc)
  const size_t grown = bytes + bytes / 2;
  // queued work may still read the old buffer (metadata uploads do not wait
  // for their stream): it is reused only after the owner stream's queued work;
  // an ownerless buffer waits for the device (growth is rare)
  if (ptr) {
    if (owner) {
      cache_release_after(ptr, bytes, *owner);
    } else {
      (void)hipDeviceSynchronize();
      (void)hipFree(ptr);
    }
  }
  ptr = nullptr;
  bytes = 0;
  size_t want = std::max<size_t>(std::max<size_t>(n, grown), 1 << 20);
  hipError_t e = owner ? cache_alloc(&ptr, want) : hipMalloc(&ptr, want);
  if (e == hipSuccess) bytes = want;
  return e;
}

void Scratch::release() {
  if (ptr) (void)hipFree(ptr);
  ptr = nullptr;
  bytes = 0;
}

namespace {

constexpr int kB = 256;
constexpr uint64_t kBigSegment = 1ull << 21;  // device-wide sort per segment above this
constexpr uint32_t kSelCap = 18432;  // distinct candidates per genome k_bottom_select holds in LDS

template <bool PAIRS>
hipError_t sort_impl(const uint64_t* keys_in, uint64_t* keys_out, const uint64_t* vals_in,
                     uint64_t* vals_out, uint64_t total, const std::vector<uint64_t>& host_off,
                     const uint64_t* d_off, int end_bit, Scratch& tmp, hipStream_t s) {
  const size_t n_seg = host_off.size() - 1;
  if (total == 0) return hipSuccess;
  uint64_t max_len = 0;
  for (size_t g = 0; g < n_seg; ++g) max_len = std::max(max_len, host_off[g + 1] - host_off[g]);
  if (end_bit < 1) end_bit = 1;
  if (n_seg == 1 || max_len > kBigSegment || total >= (1ull << 32)) {
    for (size_t g = 0; g < n_seg; ++g) {
      uint64_t b = host_off[g], len = host_off[g + 1] - b;
      if (len == 0) continue;
      size_t need = 0;
      hipError_t e;
      if constexpr (PAIRS)
        e = rocprim::radix_sort_pairs(nullptr, need, keys_in + b, keys_out + b, vals_in + b,
                                      vals_out + b, len, 0, end_bit, s);
      else
        e = rocprim::radix_sort_keys(nullptr, need, keys_in + b, keys_out + b, len, 0, end_bit, s);
      if (e != hipSuccess) return e;
      if ((e = tmp.reserve(need)) != hipSuccess) return e;
      need = tmp.bytes;
      if constexpr (PAIRS)
        e = rocprim::radix_sort_pairs(tmp.ptr, need, keys_in + b, keys_out + b, vals_in + b,
                                      vals_out + b, len, 0, end_bit, s);
      else
        e = rocprim::radix_sort_keys(tmp.ptr, need, keys_in + b, keys_out + b, len, 0, end_bit, s);
      if (e != hipSuccess) return e;
    }
    return hipSuccess;
  }
  size_t need = 0;
  hipError_t e;
  if constexpr (PAIRS)
    e = rocprim::segmented_radix_sort_pairs(nullptr, need, keys_in, keys_out, vals_in, vals_out,
                                            (unsigned)total, (unsigned)n_seg, d_off, d_off + 1, 0,
                                            end_bit, s);
  else
    e = rocprim::segmented_radix_sort_keys(nullptr, need, keys_in, keys_out, (unsigned)total,
                                           (unsigned)n_seg, d_off, d_off + 1, 0, end_bit, s);
  if (e != hipSuccess) return e;
  if ((e = tmp.reserve(need)) != hipSuccess) return e;
  need = tmp.bytes;
  if constexpr (PAIRS)
    return rocprim::segmented_radix_sort_pairs(tmp.ptr, need, keys_in, keys_out, vals_in, vals_out,
                                               (unsigned)total, (unsigned)n_seg, d_off, d_off + 1,
                                               0, end_bit, s);
  else
    return rocprim::segmented_radix_sort_keys(tmp.ptr, need, keys_in, keys_out, (unsigned)total,
                                              (unsigned)n_seg, d_off, d_off + 1, 0, end_bit, s);
}

// pext / pdep of the mask's bits (BitRuns): the masks are kernel arguments
// (SGPRs), a zero step is skipped by a uniform branch
__device__ __forceinline__ uint64_t runs_pack(uint64_t x, const BitRuns& r) {
  x &= r.mask;
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    const uint64_t mv = r.mv[i];
    if (mv) {
      const uint64_t t = x & mv;
      x = (x ^ t) | (t >> (1 << i));
    }
  }
  return x;
}

__device__ __forceinline__ uint64_t runs_expand(uint64_t x, const BitRuns& r) {
  // a packed key holds popcount(mask) bits; anything above them (a segment tag,
  // compact_regions) is not part of the k-mer
  const int width = __popcll(r.mask);
  if (width < 64) x &= (1ull << width) - 1;
#pragma unroll
  for (int i = 5; i >= 0; --i) {
    const uint64_t mv = r.mv[i];
    if (mv) x = (x & ~mv) | ((x << (1 << i)) & mv);
  }
  return x & r.mask;
}

template <bool PACK>
__global__ void k_compact(const uint64_t* __restrict__ src, uint64_t* __restrict__ dst,
                          const uint64_t* __restrict__ src_off, const uint64_t* __restrict__ dst_off,
                          const BitRuns runs, int tag_shift) {
  const uint32_t g = blockIdx.y;
  const uint64_t len = dst_off[g + 1] - dst_off[g];
  const uint64_t so = src_off[g], d0 = dst_off[g];
  const uint64_t tag = tag_shift >= 0 ? (uint64_t)g << tag_shift : 0;  // the segment above the key bits
  for (uint64_t i = (uint64_t)blockIdx.x * kB + threadIdx.x; i < len; i += (uint64_t)gridDim.x * kB)
    dst[d0 + i] = (PACK ? runs_pack(src[so + i], runs) : src[so + i]) | tag;
}

__global__ void k_bits_expand(uint64_t* __restrict__ keys, uint64_t n, const BitRuns runs) {
  for (uint64_t i = (uint64_t)blockIdx.x * kB + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kB)
    keys[i] = runs_expand(keys[i], runs);
}

__global__ void k_flags(const uint64_t* __restrict__ keys, const uint64_t* __restrict__ keys2,
                        const uint64_t* __restrict__ off, uint32_t* __restrict__ flag) {
  const uint32_t g = blockIdx.y;
  const uint64_t b = off[g], e = off[g + 1];
  for (uint64_t i = b + (uint64_t)blockIdx.x * kB + threadIdx.x; i < e; i += (uint64_t)gridDim.x * kB) {
    bool first = (i == b) || keys[i] != keys[i - 1] || (keys2 && keys2[i] != keys2[i - 1]);
    flag[i] = first ? 1u : 0u;
  }
}

__global__ void k_uniq_counts(const uint64_t* __restrict__ pos, const uint64_t* __restrict__ off,
                              uint32_t n_seg, uint64_t* __restrict__ uniq) {
  uint32_t g = blockIdx.x * kB + threadIdx.x;
  if (g < n_seg) uniq[g] = pos[off[g + 1]] - pos[off[g]];
}

template <bool EXPAND>
__global__ void k_scatter(const uint64_t* __restrict__ vals, const uint64_t* __restrict__ vals2,
                          const uint64_t* __restrict__ off, const uint32_t* __restrict__ flag,
                          const uint64_t* __restrict__ pos, const uint64_t* __restrict__ limit,
                          const uint64_t* __restrict__ dst_off, uint64_t* __restrict__ out,
                          uint64_t* __restrict__ out2, const BitRuns runs, uint64_t keep, uint64_t keep2) {
  const uint32_t g = blockIdx.y;
  const uint64_t b = off[g], e = off[g + 1];
  const uint64_t p0 = pos[b], lim = limit ? limit[g] : ~0ull, d0 = dst_off ? dst_off[g] : p0;
  for (uint64_t i = b + (uint64_t)blockIdx.x * kB + threadIdx.x; i < e; i += (uint64_t)gridDim.x * kB) {
    if (!flag[i]) continue;
    uint64_t r = pos[i] - p0;
    if (r < lim) {  // keep / keep2 drop a segment tag (compact_regions)
      out[d0 + r] = EXPAND ? runs_expand(vals[i], runs) : vals[i] & keep;
      if (out2) out2[d0 + r] = vals2[i] & keep2;
    }
  }
}

__global__ void k_synth(uint8_t* __restrict__ out, uint64_t n, uint64_t seed, uint64_t mut_seed,
                        uint64_t mut_thresh, uint64_t pos_offset) {
  // 16 bytes per thread, one 16-B store
  const uint64_t i0 = ((uint64_t)blockIdx.x * kB + threadIdx.x) * 16;
  if (i0 >= n) return;
  uint32_t w[4] = {0, 0, 0, 0};
  const uint32_t lut = 0x54474341u;  // "ACGT"
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    uint64_t p = pos_offset + i0 + k;
    uint32_t b = (uint32_t)(splitmix64_at(seed, p) >> 62);
    if (mut_thresh) {
      uint64_t u = splitmix64_at(mut_seed, p);
      if (u < mut_thresh) b = (b + 1 + (uint32_t)((u >> 32) % 3)) & 3;
    }
    w[k >> 2] |= ((lut >> (8 * b)) & 0xFFu) << (8 * (k & 3));
  }
  if (i0 + 16 <= n) {
    *reinterpret_cast<uint4*>(out + i0) = make_uint4(w[0], w[1], w[2], w[3]);
  } else {
    for (int k = 0; i0 + k < n; ++k) out[i0 + k] = (uint8_t)(w[k >> 2] >> (8 * (k & 3)));
  }
}

__global__ void k_export(const uint64_t* __restrict__ data, const uint64_t* __restrict__ starts,
                         const uint32_t* __restrict__ sizes, int ew, uint64_t* __restrict__ dst,
                         uint64_t stride, uint32_t* __restrict__ dst_sizes) {
  const uint32_t g = blockIdx.y;
  const uint64_t n = (uint64_t)sizes[g] * ew, src = starts[g] * ew, d = (uint64_t)g * stride * ew;
  const uint64_t cap = stride * ew;
  for (uint64_t i = (uint64_t)blockIdx.x * kB + threadIdx.x; i < cap; i += (uint64_t)gridDim.x * kB)
    dst[d + i] = i < n ? data[src + i] : ~0ull;
  if (blockIdx.x == 0 && threadIdx.x == 0) dst_sizes[g] = sizes[g];
}

__global__ void k_interleave(const uint64_t* __restrict__ lo, const uint64_t* __restrict__ hi,
                             uint64_t n, uint64_t* __restrict__ out) {
  for (uint64_t i = (uint64_t)blockIdx.x * kB + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kB) {
    out[2 * i] = lo[i];
    out[2 * i + 1] = hi[i];
  }
}

__global__ void k_seg_ids(uint64_t* __restrict__ out, const uint64_t* __restrict__ off) {
  const uint32_t g = blockIdx.y;
  const uint64_t b = off[g], len = off[g + 1] - b;
  for (uint64_t i = (uint64_t)blockIdx.x * kB + threadIdx.x; i < len; i += (uint64_t)gridDim.x * kB)
    out[b + i] = g;
}

__global__ void k_iota(uint64_t* __restrict__ out, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * kB + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kB)
    out[i] = i;
}

__global__ void k_gather(const uint64_t* __restrict__ src, const uint64_t* __restrict__ idx,
                         uint64_t n, uint64_t* __restrict__ out) {
  for (uint64_t i = (uint64_t)blockIdx.x * kB + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kB)
    out[i] = src[idx[i]];
}

// ACGT (either case) -> 0..3, anything else -> 4 (fasta_processing.cpp:35-69)
__device__ __forceinline__ uint32_t base_code(uint8_t c) {
  const uint32_t low = c | 0x20u;
  const uint32_t code = ((low >> 1) ^ (low >> 2)) & 3u;
  return ("acgt"[code] == (char)low) ? code : 4u;
}

__global__ void k_materialise(const uint8_t* __restrict__ seq, const uint64_t* __restrict__ seg_begin,
                              uint32_t n_seg, const uint64_t* __restrict__ pos, uint64_t n, int w,
                              uint64_t mask_lo, uint64_t mask_hi, uint64_t* __restrict__ out) {
  for (uint64_t i = (uint64_t)blockIdx.x * kB + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kB) {
    const uint64_t p = pos[i];
    uint32_t lo = 0, hi = n_seg;  // last segment with seg_begin <= p
    while (lo + 1 < hi) {
      const uint32_t mid = (lo + hi) >> 1;
      if (seg_begin[mid] <= p) lo = mid; else hi = mid;
    }
    const uint64_t sb = n_seg ? seg_begin[lo] : 0;
    // run history before the window: at most 64 - w bases, stopping at a
    // non-ACGT byte or the segment start (the reference starts each run
    // with an empty window, kmer_sliding.cpp:129)
    uint64_t h = 0;
    while (h + w < 64 && p > sb + h && base_code(seq[p - h - 1]) < 4) ++h;
    uint64_t fl = 0, fh = 0, rl = 0, rh = 0;
    for (uint64_t b = p - h; b < p + w; ++b) {  // F <<= 2, F[0..1] = base
      const uint64_t c = base_code(seq[b]) & 3u;
      fh = (fh << 2) | (fl >> 62);
      fl = (fl << 2) | c;
    }
    for (int k = 0; k < w; ++k) {  // R = sum comp(b_k) << 2k
      const uint64_t c = (base_code(seq[p + k]) & 3u) ^ 3u;
      if (k < 32) rl |= c << (2 * k);
      else rh |= c << (2 * (k - 32));
    }
    const uint64_t fml = fl & mask_lo, fmh = fh & mask_hi, rml = rl & mask_lo, rmh = rh & mask_hi;
    const bool f_lt = fmh < rmh || (fmh == rmh && fml < rml);  // kmer_sliding.cpp:165
    out[4 * i + 0] = f_lt ? fl : rl;
    out[4 * i + 1] = f_lt ? fh : rh;
    out[4 * i + 2] = f_lt ? fml : rml;
    out[4 * i + 3] = f_lt ? fmh : rmh;
  }
}

inline unsigned grid_for(uint64_t n) {
  uint64_t g = (n + kB - 1) / kB;
  return (unsigned)std::min<uint64_t>(std::max<uint64_t>(g, 1), 65535);
}

// ---- bottom-s selection over C-sorted unique candidates ---------------------------------
// One workgroup per genome.  The genome's distinct candidate k-mers arrive sorted
// by value; their fmh values are computed into LDS, the s-th smallest fmh F* is
// found by an 8-bit-digit radix select, and the kept k-mers — fmh < F*, plus the
// first (in k-mer order) of those with fmh == F* up to s — are written in
// k-mer order: exactly the s distinct k-mers with the smallest (fmh, k-mer).
constexpr int kSelB = 1024;
constexpr int kSelWaves = kSelB / 64;

// exclusive block scan of a predicate; returns this thread's rank, *total = count
__device__ __forceinline__ uint32_t block_rank(bool p, uint32_t* wsum, uint32_t* total) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint64_t bal = __ballot(p);
  const uint32_t in_wave = (uint32_t)__popcll(bal & ((1ull << lane) - 1));
  if (lane == 0) wsum[wave] = (uint32_t)__popcll(bal);
  __syncthreads();
  uint32_t before = 0, all = 0;
#pragma unroll
  for (int w = 0; w < kSelWaves; ++w) {
    const uint32_t c = wsum[w];
    before += w < wave ? c : 0u;
    all += c;
  }
  __syncthreads();
  *total = all;
  return before + in_wave;
}

// exclusive block scan of one count per thread (wsum: kSelWaves words)
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* wsum) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t inc = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t t = __shfl_up(inc, o, 64);
    if (lane >= o) inc += t;
  }
  if (lane == 63) wsum[wave] = inc;
  __syncthreads();
  uint32_t before = inc - v;
#pragma unroll
  for (int w = 0; w < kSelWaves; ++w) before += w < wave ? wsum[w] : 0u;
  __syncthreads();
  return before;
}

// Block-wide maximum of one value per thread (wsum64: kSelWaves words).
__device__ __forceinline__ uint64_t block_max(uint64_t v, uint64_t* wsum64) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const uint64_t t = __shfl_xor(v, o, 64);
    v = t > v ? t : v;
  }
  if ((threadIdx.x & 63) == 0) wsum64[threadIdx.x >> 6] = v;
  __syncthreads();
  uint64_t m = 0;
#pragma unroll
  for (int w = 0; w < kSelWaves; ++w) m = wsum64[w] > m ? wsum64[w] : m;
  __syncthreads();
  return m;
}

// Radix select (8-bit digits, most significant first) of the kk-th smallest
// (1-based) of the values f[i], i < n, with valid(i).  Starts at the digit of
// vmax's top bit (the candidates' fmh are below the scan's threshold, so the
// digits above it are zero) and stops as soon as the chosen digit's bucket is
// kept whole (kk equals its population) — with 64-bit hashes two or three
// digits instead of eight.  The kept values are those with
// (v & pmask) < prefix, plus, with (v & pmask) == prefix, all of them (whole)
// or the first kk in index order.
struct RadixSel {
  uint64_t prefix, pmask;
  uint32_t kk;
  bool whole;
};
// count(shift, prefix, pmask) adds this thread's values v with (v & pmask) ==
// prefix to hist[(v >> shift) & 255].
template <class Count>
__device__ __forceinline__ RadixSel radix_select_by(Count count, uint32_t kk, uint64_t vmax,
                                                    uint32_t* hist, uint32_t* s_sel) {
  const int tid = threadIdx.x;
  RadixSel r{0, 0, kk, false};
  const int top = vmax ? 63 - __builtin_clzll(vmax) : 0;
  for (int shift = (top / 8) * 8; shift >= 0; shift -= 8) {
    for (int i = tid; i < 256; i += kSelB) hist[i] = 0;
    __syncthreads();
    count(shift, r.prefix, r.pmask);
    __syncthreads();
    if (tid < 64) {  // wave 0: the digit where the running count reaches kk
      uint32_t h4[4], sum = 0;
#pragma unroll
      for (int q = 0; q < 4; ++q) { h4[q] = hist[4 * tid + q]; sum += h4[q]; }
      uint32_t incl = sum;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t t = __shfl_up(incl, o, 64);
        if (tid >= o) incl += t;
      }
      const uint64_t bal = __ballot(incl >= r.kk);
      const int L = __builtin_ctzll(bal);
      if (tid == L) {
        uint32_t c = incl - sum;
        int q = 0;
        while (c + h4[q] < r.kk) c += h4[q++];
        s_sel[0] = 4 * L + q;  // digit
        s_sel[1] = c;          // valid values below it
        s_sel[2] = h4[q];      // its population
      }
    }
    __syncthreads();
    r.prefix |= (uint64_t)s_sel[0] << shift;
    r.pmask |= 255ull << shift;
    r.kk -= s_sel[1];
    const bool whole = r.kk == s_sel[2];
    __syncthreads();
    if (whole) {
      r.whole = true;
      break;
    }
  }
  return r;
}

// The same over values f[i], i < n, with valid(i), in LDS (striped).
template <class Valid>
__device__ __forceinline__ RadixSel radix_select(const uint64_t* f, uint32_t n, uint32_t kk,
                                                 uint64_t vmax, Valid valid, uint32_t* hist,
                                                 uint32_t* s_sel) {
  return radix_select_by(
      [&](int shift, uint64_t prefix, uint64_t pmask) {
        for (uint32_t i = threadIdx.x; i < n; i += kSelB) {
          const uint64_t v = f[i];
          if (valid(i) && (v & pmask) == prefix) atomicAdd(&hist[(v >> shift) & 255u], 1u);
        }
      },
      kk, vmax, hist, s_sel);
}

template <int FLAVOUR>
__global__ __launch_bounds__(kSelB) void k_bottom_select(const uint64_t* __restrict__ uk,
                                                         const uint64_t* __restrict__ uoff,
                                                         const uint64_t* __restrict__ dst_off,
                                                         const uint64_t* __restrict__ limit,
                                                         uint64_t kconst,
                                                         uint64_t* __restrict__ out) {
  extern __shared__ uint64_t f[];
  __shared__ uint32_t hist[256];
  __shared__ uint32_t wsum[kSelWaves];
  __shared__ uint64_t wsum64[kSelWaves];
  __shared__ uint32_t s_sel[3];
  const uint32_t g = blockIdx.x;
  const uint64_t b = uoff[g], n = uoff[g + 1] - b;
  const uint64_t lim = limit[g];
  const int tid = threadIdx.x;
  if (lim == 0) return;
  uint64_t* dst = out + dst_off[g];
  if (n <= lim) {  // every distinct candidate is kept
    for (uint64_t i = tid; i < n; i += kSelB) dst[i] = uk[b + i];
    return;
  }
  uint64_t mx = 0;
  for (uint64_t i = tid; i < n; i += kSelB) {
    const uint64_t v = hash_bitset128<FLAVOUR>(uk[b + i], 0) ^ kconst;
    f[i] = v;
    mx = v > mx ? v : mx;
  }
  mx = block_max(mx, wsum64);  // its barriers also publish f[]
  const RadixSel sel = radix_select(f, (uint32_t)n, (uint32_t)lim, mx, [](uint32_t) { return true; },
                                    hist, s_sel);
  // keep the selected values in k-mer order
  uint32_t eq_base = 0, out_base = 0;
  for (uint64_t base = 0; base < n; base += kSelB) {
    const uint64_t i = base + tid;
    const uint64_t v = i < n ? f[i] & sel.pmask : ~0ull;
    const bool eq = i < n && !sel.whole && v == sel.prefix;
    uint32_t eq_tot, keep_tot;
    const uint32_t eq_rank = eq_base + block_rank(eq, wsum, &eq_tot);
    const bool keep = i < n && (v < sel.prefix || (v == sel.prefix && (sel.whole || eq_rank < sel.kk)));
    const uint32_t pos = out_base + block_rank(keep, wsum, &keep_tot);
    if (keep) dst[pos] = uk[b + i];
    eq_base += eq_tot;
    out_base += keep_tot;
  }
}

// Bottom-s post-processing of one genome in one workgroup, straight from the
// scan's record region: candidates packed to their mask bits, sorted in the
// block (rocPRIM block radix sort, keys in registers), duplicates flagged, fmh
// of the distinct ones into LDS, then k_bottom_select's radix select and an
// in-order compaction. Replaces compaction + segmented sort + unique + scatter
// + select (five kernels and a host sync) for genomes of <= kFuseCap candidates.
// res[g] = sketch size, or ~0 when the genome has fewer than s distinct
// candidates under a finite threshold (the build retries it).
// ITEMS keys per thread (8, 12 or 16): the smallest that holds the pass's
// largest genome, so that padding is not sorted (pads cost as much as keys).
constexpr uint32_t kFuseMaxItems = 16;
constexpr uint32_t kFuseCap = kSelB * kFuseMaxItems;  // 16384 candidates
#ifndef SKS_FUSE_RADIX_BITS
#define SKS_FUSE_RADIX_BITS 0
#endif
#ifndef SKS_FUSE_RANK
#define SKS_FUSE_RANK default_for_radix_sort
#endif
template <int ITEMS>
using FuseSort = rocprim::block_radix_sort<unsigned long long, kSelB, ITEMS, rocprim::empty_type, 1, 1,
                                           SKS_FUSE_RADIX_BITS,
                                           rocprim::block_radix_rank_algorithm::SKS_FUSE_RANK>;
// The sort is a counting sort on the top kBkLog bits of the packed keys (4096
// buckets, four per thread) followed by an insertion sort of each thread's
// buckets in LDS; rocPRIM's block radix sort — whose LDS exchange is 74% bank
// conflicts and 0.24 of the kernel's 0.54 ms on config 4 — remains the
// fallback when a bucket holds more than kBkMax keys (keys crowding a few top
// bit patterns, e.g. low-complexity sequence).
constexpr int kBkLog = 12;
constexpr uint32_t kBk = 1u << kBkLog;
constexpr uint32_t kBkPer = kBk / kSelB;
constexpr uint32_t kBkMax = 64;
template <int ITEMS>
constexpr size_t fuse_lds() {
  constexpr size_t rp = sizeof(typename FuseSort<ITEMS>::storage_type);
  constexpr size_t cs = kSelB * ITEMS * sizeof(uint64_t) + kBk * sizeof(uint32_t);  // keys + buckets
  return rp > cs ? rp : cs;
}

// Sorting networks (odd-even merge sort, checked over all 0-1 inputs) for one
// bucket of c <= N keys in LDS: loaded into registers padded with ~0 (the
// largest key), sorted branch-free, the first c written back.
constexpr uint8_t kNet8[19][2] = {{0, 2}, {1, 3}, {4, 6}, {5, 7}, {0, 4}, {1, 5}, {2, 6}, {3, 7}, {0, 1}, {2, 3},
                                  {4, 5}, {6, 7}, {2, 4}, {3, 5}, {1, 4}, {3, 6}, {1, 2}, {3, 4}, {5, 6}};
constexpr uint8_t kNet16[63][2] = {
    {0, 1},  {2, 3},   {0, 2},   {1, 3},  {1, 2},   {4, 5},   {6, 7},   {4, 6},   {5, 7},   {5, 6},  {0, 4},
    {2, 6},  {2, 4},   {1, 5},   {3, 7},  {3, 5},   {1, 2},   {3, 4},   {5, 6},   {8, 9},   {10, 11}, {8, 10},
    {9, 11}, {9, 10},  {12, 13}, {14, 15}, {12, 14}, {13, 15}, {13, 14}, {8, 12},  {10, 14}, {10, 12}, {9, 13},
    {11, 15}, {11, 13}, {9, 10}, {11, 12}, {13, 14}, {0, 8},   {4, 12},  {4, 8},   {2, 10},  {6, 14},  {6, 10},
    {2, 4},  {6, 8},   {10, 12}, {1, 9},  {5, 13},  {5, 9},   {3, 11},  {7, 15},  {7, 11},  {3, 5},   {7, 9},
    {11, 13}, {1, 2},  {3, 4},   {5, 6},  {7, 8},   {9, 10},  {11, 12}, {13, 14}};
template <int N>
__device__ __forceinline__ void bucket_sort(uint64_t* b, uint32_t c) {
  if (c > (uint32_t)N) {  // beyond the network: insertion sort in LDS (c <= kBkMax)
    for (uint32_t i = 1; i < c; ++i) {
      const uint64_t key = b[i];
      uint32_t j = i;
      while (j > 0 && b[j - 1] > key) {
        b[j] = b[j - 1];
        --j;
      }
      b[j] = key;
    }
    return;
  }
  uint64_t r[N];
#pragma unroll
  for (int i = 0; i < N; ++i) r[i] = (uint32_t)i < c ? b[i] : ~0ull;
  constexpr int E = N == 8 ? 19 : 63;
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int x = N == 8 ? kNet8[e][0] : kNet16[e][0], y = N == 8 ? kNet8[e][1] : kNet16[e][1];
    const uint64_t lo = r[x] < r[y] ? r[x] : r[y], hi = r[x] < r[y] ? r[y] : r[x];
    r[x] = lo;
    r[y] = hi;
  }
#pragma unroll
  for (int i = 0; i < N; ++i)
    if ((uint32_t)i < c) b[i] = r[i];
}

#ifdef SKS_FUSE_STAMPS  // diagnostic build: cycles from start to the end of each phase (workgroup 0)
__device__ unsigned long long g_fuse_stamps[10];
#define FSTAMP(i)                                                                   \
  do {                                                                              \
    if (threadIdx.x == 0 && blockIdx.x == 0) g_fuse_stamps[i] = __builtin_amdgcn_s_memtime() - f_t0; \
  } while (0)
#else
#define FSTAMP(i) do {} while (0)
#endif
template <int FLAVOUR, int ITEMS>
__global__ __launch_bounds__(kSelB) void k_bottom_fused(uint64_t* __restrict__ rec,
                                                        const uint64_t* __restrict__ src_off,
                                                        const uint64_t* __restrict__ cnt,
                                                        const uint64_t* __restrict__ retry_ok,
                                                        const uint64_t* __restrict__ dst_off,
                                                        uint64_t s_param, int key_bits,
                                                        const BitRuns runs, uint64_t kconst,
                                                        uint64_t* __restrict__ out,
                                                        uint64_t* __restrict__ res,
                                                        const uint64_t* __restrict__ cap,
                                                        uint32_t* __restrict__ set_sizes,
                                                        uint64_t* __restrict__ set_starts) {
  constexpr uint32_t kCap = kSelB * ITEMS;
  extern __shared__ unsigned char smem[];
  auto& sort_storage = *reinterpret_cast<typename FuseSort<ITEMS>::storage_type*>(smem);
  __shared__ unsigned long long s_last[kSelB];
  __shared__ uint32_t hist[256];
  __shared__ uint32_t wsum[kSelWaves];
  __shared__ uint64_t wsum64[kSelWaves];
  __shared__ uint32_t s_sel[3];
  const uint32_t g = blockIdx.x;
  const int tid = threadIdx.x;
  const uint64_t base = src_off[g];
  const uint64_t n64 = cnt[g];
  if (cap && n64 > cap[g]) {  // the scan counted more than its region kept
    if (tid == 0) {
      res[g] = kBottomOverflow;
      if (set_sizes) set_sizes[g] = 0;
    }
    return;
  }
  const uint32_t n = (uint32_t)n64;  // <= kCap (host-checked: max_cnt or the caps)
#ifdef SKS_FUSE_STAMPS
  const uint64_t f_t0 = __builtin_amdgcn_s_memtime();
#endif

  // striped (coalesced) loads: the counting sort takes the keys in any order;
  // blocked order (thread t: positions t * ITEMS ..) starts after the sort
  unsigned long long k[ITEMS];
#pragma unroll
  for (uint32_t j = 0; j < ITEMS; ++j) {
    const uint32_t i = j * kSelB + tid;
    k[j] = i < n ? runs_pack(rec[base + i], runs) : ~0ull;  // pads sort after equal keys
  }
  {
    uint64_t* skeys = reinterpret_cast<uint64_t*>(smem);
    uint32_t* sbin = reinterpret_cast<uint32_t*>(smem + kCap * sizeof(uint64_t));
    const int shift = key_bits > kBkLog ? key_bits - kBkLog : 0;
    // bucket = top kBkLog bits of the packed key; packed keys fit key_bits, the
    // clamp only keeps a key that did not (a future packing change) inside sbin,
    // in the last bucket, which keeps the order (larger keys, larger buckets)
    auto bk_of = [&](uint64_t key) { return (uint32_t)min(key >> shift, (uint64_t)(kBk - 1)); };
#pragma unroll
    for (uint32_t q = 0; q < kBkPer; ++q) sbin[tid * kBkPer + q] = 0;
    __syncthreads();
    FSTAMP(0);
#pragma unroll
    for (uint32_t j = 0; j < ITEMS; ++j)
      if (j * kSelB + tid < n) atomicAdd(&sbin[bk_of(k[j])], 1u);
    __syncthreads();
    FSTAMP(1);
    uint32_t cb[kBkPer], sum = 0, mx = 0;
#pragma unroll
    for (uint32_t q = 0; q < kBkPer; ++q) {
      cb[q] = sbin[tid * kBkPer + q];
      sum += cb[q];
      mx = cb[q] > mx ? cb[q] : mx;
    }
    // exclusive scan of the per-thread sums and the largest bucket, block-wide
    const int lane = tid & 63, wave = tid >> 6;
    uint32_t inc = sum;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t t = __shfl_up(inc, o, 64);
      if (lane >= o) inc += t;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) mx = max(mx, (uint32_t)__shfl_xor(mx, o, 64));
    if (lane == 63) wsum[wave] = inc;
    if (lane == 0) hist[wave] = mx;  // hist[] is free until the select
    __syncthreads();
    uint32_t excl = inc - sum, bmax = 0;
#pragma unroll
    for (int w = 0; w < kSelWaves; ++w) {
      excl += w < wave ? wsum[w] : 0u;
      bmax = hist[w] > bmax ? hist[w] : bmax;
    }
    __syncthreads();
    if (bmax > kBkMax) {  // uniform: the keys are still in registers
      // the block sort takes blocked input: pads (~0) are the largest keys, so
      // the striped arrangement sorts to the same result
      FuseSort<ITEMS>().sort(k, sort_storage, 0, key_bits);
    } else {
      uint32_t run = excl;
#pragma unroll
      for (uint32_t q = 0; q < kBkPer; ++q) {  // bucket cursors
        sbin[tid * kBkPer + q] = run;
        run += cb[q];
      }
      __syncthreads();
#pragma unroll
      for (uint32_t j = 0; j < ITEMS; ++j)
        if (j * kSelB + tid < n) skeys[atomicAdd(&sbin[bk_of(k[j])], 1u)] = k[j];
      __syncthreads();
      FSTAMP(2);
      // this thread's buckets are the contiguous range [excl, excl + sum), ~2.7
      // keys per bucket: each bucket is sorted in registers by a sorting network
      // (8 keys, or 16 for the ~0.3% of buckets above 8; kBkMax bounds them)
      uint32_t packed_cnt = 0;
#pragma unroll
      for (uint32_t q = 0; q < kBkPer; ++q) packed_cnt |= cb[q] << (8 * q);
      uint32_t st = excl;
#pragma unroll 1
      for (uint32_t q = 0; q < kBkPer; ++q) {
        const uint32_t c = (packed_cnt >> (8 * q)) & 255u;
        if (c > 8) bucket_sort<16>(skeys + st, c);
        else if (c > 1) bucket_sort<8>(skeys + st, c);
        st += c;
      }
      __syncthreads();
      FSTAMP(3);
#pragma unroll
      for (uint32_t j = 0; j < ITEMS; ++j) {
        const uint32_t i = tid * ITEMS + j;
        k[j] = i < n ? skeys[i] : ~0ull;
      }
    }
  }
  s_last[tid] = k[ITEMS - 1];
  __syncthreads();
  const unsigned long long before = tid ? s_last[tid - 1] : 0ull;
  uint64_t fv[ITEMS];
  uint32_t mine = 0, dmask = 0;
#pragma unroll
  for (uint32_t j = 0; j < ITEMS; ++j) {
    const uint32_t i = tid * ITEMS + j;
    const bool is_dup = i > 0 && k[j] == (j ? k[j - 1] : before);
    const bool valid = i < n && !is_dup;
    fv[j] = valid ? hash_bitset128<FLAVOUR>(runs_expand(k[j], runs), 0) ^ kconst : 0ull;
    mine += valid ? 1u : 0u;
    dmask |= (valid ? 0u : 1u) << j;
  }
  FSTAMP(4);
  uint32_t distinct;
  {
    uint32_t v = mine;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if ((tid & 63) == 0) wsum[tid >> 6] = v;
    __syncthreads();
    distinct = 0;
#pragma unroll
    for (int w = 0; w < kSelWaves; ++w) distinct += wsum[w];
    __syncthreads();
  }
  FSTAMP(5);
  if (distinct < s_param && retry_ok[g]) {
    if (tid == 0) {
      res[g] = ~0ull;
      if (set_sizes) set_sizes[g] = 0;
    }
    return;
  }
  const uint64_t lim = distinct < s_param ? distinct : s_param;
  if (tid == 0) {
    res[g] = lim;
    if (set_sizes) set_sizes[g] = (uint32_t)lim;
    if (set_starts) set_starts[g] = dst_off[g];
  }
  uint64_t* dst = out + dst_off[g];
  const bool all = distinct <= lim;
  RadixSel sel{0, 0, 0, true};
  if (!all) {
    uint64_t mx = 0;
#pragma unroll
    for (uint32_t j = 0; j < ITEMS; ++j) mx = fv[j] > mx ? fv[j] : mx;  // 0 for non-distinct
    mx = block_max(mx, wsum64);
    // the distinct candidates' fmh are in registers (fv, 0 where dmask is set)
    sel = radix_select_by(
        [&](int shift, uint64_t prefix, uint64_t pmask) {
#pragma unroll
          for (uint32_t j = 0; j < ITEMS; ++j)
            if (!((dmask >> j) & 1u) && (fv[j] & pmask) == prefix)
              atomicAdd(&hist[(fv[j] >> shift) & 255u], 1u);
        },
        (uint32_t)lim, mx, hist, s_sel);
  }
  FSTAMP(6);
  // keep (all distinct) or the selected ones, in k-mer order: the sorted keys,
  // their fmh and validity are in registers in blocked order (thread t holds
  // positions t * ITEMS ..), so two block scans place them — the ties at the
  // selected digit (the first kk in k-mer order) and the kept ones
  uint32_t lt_m = 0, eq_m = 0;
#pragma unroll
  for (uint32_t j = 0; j < ITEMS; ++j) {
    const bool ok = !((dmask >> j) & 1u);
    const uint64_t v = fv[j] & sel.pmask;
    const bool eq = ok && !all && !sel.whole && v == sel.prefix;
    const bool lt = ok && (all || v < sel.prefix || (v == sel.prefix && sel.whole));
    lt_m |= (lt ? 1u : 0u) << j;
    eq_m |= (eq ? 1u : 0u) << j;
  }
  uint32_t eq_rank = block_excl_scan((uint32_t)__builtin_popcount(eq_m), wsum);
  uint32_t keep_m = lt_m;
#pragma unroll
  for (uint32_t j = 0; j < ITEMS; ++j)
    if ((eq_m >> j) & 1u) keep_m |= (eq_rank++ < sel.kk ? 1u : 0u) << j;
  uint32_t pos = block_excl_scan((uint32_t)__builtin_popcount(keep_m), wsum);
  // the kept keys go through LDS (the sorted keys' array is free again) so the
  // global writes are coalesced and each expansion runs once per kept key
  uint64_t* skept = reinterpret_cast<uint64_t*>(smem);
#pragma unroll
  for (uint32_t j = 0; j < ITEMS; ++j)
    if ((keep_m >> j) & 1u) skept[pos++] = k[j];
  __syncthreads();
  for (uint32_t i = tid; i < (uint32_t)lim; i += kSelB) dst[i] = runs_expand(skept[i], runs);
  FSTAMP(7);
}

template <int FLAVOUR>
__global__ void k_fmh_narrow(uint64_t* __restrict__ keys, uint64_t n, uint64_t kconst) {
  const uint64_t i = (uint64_t)blockIdx.x * kB + threadIdx.x;
  if (i < n) keys[i] = hash_bitset128<FLAVOUR>(keys[i], 0) ^ kconst;
}

}  // namespace

hipError_t seg_sort_keys(const uint64_t* keys_in, uint64_t* keys_out, uint64_t total,
                         const std::vector<uint64_t>& host_off, const uint64_t* d_off, int end_bit,
                         Scratch& tmp, hipStream_t s) {
  return sort_impl<false>(keys_in, keys_out, nullptr, nullptr, total, host_off, d_off, end_bit,
                          tmp, s);
}

hipError_t seg_sort_pairs(const uint64_t* keys_in, uint64_t* keys_out, const uint64_t* vals_in,
                          uint64_t* vals_out, uint64_t total, const std::vector<uint64_t>& host_off,
                          const uint64_t* d_off, int end_bit, Scratch& tmp, hipStream_t s) {
  return sort_impl<true>(keys_in, keys_out, vals_in, vals_out, total, host_off, d_off, end_bit,
                         tmp, s);
}

hipError_t compact_regions(const uint64_t* src, uint64_t* dst, const uint64_t* d_src_off,
                           const uint64_t* d_dst_off, uint32_t n_seg, uint64_t max_len,
                           hipStream_t s, const BitRuns* pack, int tag_shift) {
  if (n_seg == 0 || max_len == 0) return hipSuccess;
  if (pack && pack->n)
    hipLaunchKernelGGL(k_compact<true>, dim3(grid_for(max_len), n_seg), dim3(kB), 0, s, src, dst,
                       d_src_off, d_dst_off, *pack, tag_shift);
  else
    hipLaunchKernelGGL(k_compact<false>, dim3(grid_for(max_len), n_seg), dim3(kB), 0, s, src, dst,
                       d_src_off, d_dst_off, BitRuns{}, tag_shift);
  return hipGetLastError();
}

hipError_t launch_seg_ids(uint64_t* out, const uint64_t* d_off, uint32_t n_seg, uint64_t max_len, hipStream_t s) {
  if (n_seg == 0 || max_len == 0) return hipSuccess;
  hipLaunchKernelGGL(k_seg_ids, dim3(grid_for(max_len), n_seg), dim3(kB), 0, s, out, d_off);
  return hipGetLastError();
}

int seg_tag_bits(uint32_t n_seg) {
  int b = 0;
  while (b < 32 && (1ull << b) < n_seg) ++b;
  return b;
}

BitRuns bit_runs(uint64_t mask) {
  BitRuns r;
  for (int b = 0; b < 64; ++b)  // runs = set bits whose lower neighbour is clear
    if (((mask >> b) & 1) && (b == 0 || !((mask >> (b - 1)) & 1))) ++r.n;
  r.mask = mask;
  uint64_t m = mask, mk = ~m << 1;  // Hacker's Delight 7-4: bits to move by 2^i
  for (int i = 0; i < 6; ++i) {
    uint64_t mp = mk ^ (mk << 1);
    for (int sh = 2; sh < 64; sh <<= 1) mp ^= mp << sh;  // parallel prefix (zeros to the right)
    const uint64_t mv = mp & m;
    r.mv[i] = mv;
    m = (m ^ mv) | (mv >> (1 << i));
    mk &= ~mp;
  }
  return r;
}

hipError_t launch_bits_expand(uint64_t* keys, uint64_t n, const BitRuns& runs, hipStream_t s) {
  if (n == 0 || runs.n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_bits_expand, dim3(grid_for(n)), dim3(kB), 0, s, keys, n, runs);
  return hipGetLastError();
}

hipError_t seg_unique_scan(const uint64_t* keys, const uint64_t* keys2, uint64_t total,
                           uint64_t max_len, const uint64_t* d_off, uint32_t n_seg, uint32_t* d_flag,
                           uint64_t* d_pos, uint64_t* d_uniq, Scratch& tmp, hipStream_t s) {
  if (n_seg == 0) return hipSuccess;
  hipError_t e;
  if (total) {
    // max segment length bound: total (grid-stride loop covers any length)
    hipLaunchKernelGGL(k_flags, dim3(grid_for(std::min<uint64_t>(max_len, 1ull << 24)), n_seg),
                       dim3(kB), 0, s, keys, keys2, d_off, d_flag);
    if ((e = hipGetLastError()) != hipSuccess) return e;
  }
  if ((e = hipMemsetAsync(d_flag + total, 0, sizeof(uint32_t), s)) != hipSuccess) return e;
  size_t need = 0;
  e = rocprim::exclusive_scan(nullptr, need, d_flag, d_pos, (uint64_t)0, (size_t)(total + 1),
                              rocprim::plus<uint64_t>(), s);
  if (e != hipSuccess) return e;
  if ((e = tmp.reserve(need)) != hipSuccess) return e;
  need = tmp.bytes;
  e = rocprim::exclusive_scan(tmp.ptr, need, d_flag, d_pos, (uint64_t)0, (size_t)(total + 1),
                              rocprim::plus<uint64_t>(), s);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_uniq_counts, dim3((n_seg + kB - 1) / kB), dim3(kB), 0, s, d_pos, d_off,
                     n_seg, d_uniq);
  return hipGetLastError();
}

hipError_t seg_unique_scatter(const uint64_t* vals, const uint64_t* vals2, uint64_t total,
                              uint64_t max_len, const uint64_t* d_off, uint32_t n_seg,
                              const uint32_t* d_flag,
                              const uint64_t* d_pos, const uint64_t* d_limit,
                              const uint64_t* d_dst_off, uint64_t* out, uint64_t* out2,
                              hipStream_t s, const BitRuns* expand, uint64_t keep, uint64_t keep2) {
  if (n_seg == 0 || total == 0) return hipSuccess;
  const dim3 grid(grid_for(std::min<uint64_t>(max_len, 1ull << 24)), n_seg);
  if (expand && expand->n)
    hipLaunchKernelGGL(k_scatter<true>, grid, dim3(kB), 0, s, vals, vals2, d_off, d_flag, d_pos,
                       d_limit, d_dst_off, out, out2, *expand, keep, keep2);
  else
    hipLaunchKernelGGL(k_scatter<false>, grid, dim3(kB), 0, s, vals, vals2, d_off, d_flag, d_pos,
                       d_limit, d_dst_off, out, out2, BitRuns{}, keep, keep2);
  return hipGetLastError();
}

// Sorted unique union of n u64 values (any order, duplicates allowed) into out;
// *n_out = number of distinct values (host, after a stream sync).  The sort runs
// on a scratch copy; `tmp` holds it and the rocPRIM temporaries.
hipError_t sort_unique_u64(const uint64_t* in, uint64_t n, uint64_t* out, uint64_t* n_out,
                           Scratch& tmp, hipStream_t s) {
  *n_out = 0;
  if (n == 0) return hipSuccess;
  if (n >= (1ull << 32)) return hipErrorInvalidValue;
  size_t sort_bytes = 0, uniq_bytes = 0;
  hipError_t e;
  if ((e = rocprim::radix_sort_keys(nullptr, sort_bytes, in, out, (size_t)n, 0, 64, s)) != hipSuccess)
    return e;
  if ((e = rocprim::unique(nullptr, uniq_bytes, out, out, (uint64_t*)nullptr, (size_t)n,
                           rocprim::equal_to<uint64_t>(), s)) != hipSuccess)
    return e;
  const size_t o_sorted = 0, o_cnt = (n * 8 + 15) & ~(size_t)15, o_tmp = o_cnt + 16;
  if ((e = tmp.reserve(o_tmp + std::max(sort_bytes, uniq_bytes))) != hipSuccess) return e;
  char* w = static_cast<char*>(tmp.ptr);
  uint64_t* sorted = reinterpret_cast<uint64_t*>(w + o_sorted);
  uint64_t* d_cnt = reinterpret_cast<uint64_t*>(w + o_cnt);
  void* t = w + o_tmp;
  size_t tb = tmp.bytes - o_tmp;
  if ((e = rocprim::radix_sort_keys(t, tb, in, sorted, (size_t)n, 0, 64, s)) != hipSuccess) return e;
  tb = tmp.bytes - o_tmp;
  if ((e = rocprim::unique(t, tb, sorted, out, d_cnt, (size_t)n, rocprim::equal_to<uint64_t>(), s)) !=
      hipSuccess)
    return e;
  return pinned_d2h(n_out, d_cnt, 8, s);
}

// The same for 128-bit k-mers (w > 32) stored as (lo, hi) word pairs: on a
// little-endian device the pair IS the __uint128_t hi * 2^64 + lo, so one radix
// sort over 128 bits orders them like the reference's operator< on 128-bit
// dynamic_bitsets (most significant block first).  in/out 16-byte aligned.
hipError_t sort_unique_u128(const uint64_t* in, uint64_t n, uint64_t* out, uint64_t* n_out,
                            Scratch& tmp, hipStream_t s) {
  using u128 = rocprim::uint128_t;
  *n_out = 0;
  if (n == 0) return hipSuccess;
  if (n >= (1ull << 32)) return hipErrorInvalidValue;
  if ((reinterpret_cast<uintptr_t>(in) | reinterpret_cast<uintptr_t>(out)) & 15) return hipErrorInvalidValue;
  const u128* kin = reinterpret_cast<const u128*>(in);
  u128* kout = reinterpret_cast<u128*>(out);
  size_t sort_bytes = 0, uniq_bytes = 0;
  hipError_t e;
  if ((e = rocprim::radix_sort_keys(nullptr, sort_bytes, kin, kout, (size_t)n, 0, 128, s)) != hipSuccess)
    return e;
  if ((e = rocprim::unique(nullptr, uniq_bytes, kout, kout, (uint64_t*)nullptr, (size_t)n,
                           rocprim::equal_to<u128>(), s)) != hipSuccess)
    return e;
  const size_t o_sorted = 0, o_cnt = (n * 16 + 15) & ~(size_t)15, o_tmp = o_cnt + 16;
  if ((e = tmp.reserve(o_tmp + std::max(sort_bytes, uniq_bytes))) != hipSuccess) return e;
  char* w = static_cast<char*>(tmp.ptr);
  u128* sorted = reinterpret_cast<u128*>(w + o_sorted);
  uint64_t* d_cnt = reinterpret_cast<uint64_t*>(w + o_cnt);
  void* t = w + o_tmp;
  size_t tb = tmp.bytes - o_tmp;
  if ((e = rocprim::radix_sort_keys(t, tb, kin, sorted, (size_t)n, 0, 128, s)) != hipSuccess) return e;
  tb = tmp.bytes - o_tmp;
  if ((e = rocprim::unique(t, tb, sorted, kout, d_cnt, (size_t)n, rocprim::equal_to<u128>(), s)) !=
      hipSuccess)
    return e;
  return pinned_d2h(n_out, d_cnt, 8, s);
}

hipError_t launch_synth(uint8_t* out, uint64_t n, uint64_t seed, uint64_t mut_seed,
                        uint64_t mut_thresh, uint64_t pos_offset, hipStream_t s) {
  if (n == 0) return hipSuccess;
  uint64_t threads = (n + 15) / 16;
  uint64_t blocks = (threads + kB - 1) / kB;
  hipLaunchKernelGGL(k_synth, dim3((unsigned)blocks), dim3(kB), 0, s, out, n, seed, mut_seed,
                     mut_thresh, pos_offset);
  return hipGetLastError();
}

hipError_t launch_export(const uint64_t* data, const uint64_t* starts, const uint32_t* sizes,
                         uint32_t n, int elem_words, uint64_t* dst, uint64_t stride,
                         uint32_t* dst_sizes, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_export, dim3(grid_for(stride * elem_words), n), dim3(kB), 0, s, data, starts,
                     sizes, elem_words, dst, stride, dst_sizes);
  return hipGetLastError();
}

hipError_t launch_materialise(const uint8_t* seq, const uint64_t* seg_begin, uint32_t n_seg,
                              const uint64_t* pos, uint64_t n, int w, uint64_t mask_lo,
                              uint64_t mask_hi, uint64_t* out, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_materialise, dim3(grid_for(n)), dim3(kB), 0, s, seq, seg_begin, n_seg, pos, n,
                     w, mask_lo, mask_hi, out);
  return hipGetLastError();
}

hipError_t launch_fmh_narrow(uint64_t* keys, uint64_t n, uint64_t kconst, int flavour,
                             hipStream_t s) {
  if (n == 0) return hipSuccess;
  const uint64_t blocks = (n + kB - 1) / kB;
  if (flavour == 0)
    hipLaunchKernelGGL(k_fmh_narrow<0>, dim3((unsigned)blocks), dim3(kB), 0, s, keys, n, kconst);
  else
    hipLaunchKernelGGL(k_fmh_narrow<1>, dim3((unsigned)blocks), dim3(kB), 0, s, keys, n, kconst);
  return hipGetLastError();
}

uint32_t bottom_select_capacity() { return kSelCap; }

hipError_t launch_bottom_select(const uint64_t* uk, const uint64_t* d_uoff, const uint64_t* d_dst,
                                const uint64_t* d_lim, uint32_t n_seg, uint64_t kconst,
                                int flavour, uint64_t* out, hipStream_t s) {
  if (n_seg == 0) return hipSuccess;
  const size_t lds = (size_t)kSelCap * sizeof(uint64_t);
  static const hipError_t a0 = hipFuncSetAttribute(
      reinterpret_cast<const void*>(k_bottom_select<0>), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  static const hipError_t a1 = hipFuncSetAttribute(
      reinterpret_cast<const void*>(k_bottom_select<1>), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (a0 != hipSuccess) return a0;
  if (a1 != hipSuccess) return a1;
  if (flavour == 0)
    hipLaunchKernelGGL(k_bottom_select<0>, dim3(n_seg), dim3(kSelB), lds, s, uk, d_uoff, d_dst, d_lim,
                       kconst, out);
  else
    hipLaunchKernelGGL(k_bottom_select<1>, dim3(n_seg), dim3(kSelB), lds, s, uk, d_uoff, d_dst, d_lim,
                       kconst, out);
  return hipGetLastError();
}

uint32_t bottom_fused_capacity() { return kFuseCap; }

hipError_t launch_bottom_fused(uint64_t* rec, const uint64_t* d_src_off, const uint64_t* d_cnt,
                               const uint64_t* d_retry_ok, const uint64_t* d_dst_off,
                               uint32_t n_seg, uint64_t max_cnt, uint64_t s_param, int key_bits,
                               const BitRuns& runs, uint64_t kconst, int flavour, uint64_t* out,
                               uint64_t* d_res, hipStream_t s, const uint64_t* d_cap, uint32_t* set_sizes,
                               uint64_t* set_starts) {
  if (n_seg == 0) return hipSuccess;
  if (max_cnt > kFuseCap) return hipErrorInvalidValue;
  auto go = [&](auto kernel, size_t lds) -> hipError_t {
    const hipError_t a = hipFuncSetAttribute(reinterpret_cast<const void*>(kernel),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (a != hipSuccess) return a;
    hipLaunchKernelGGL(kernel, dim3(n_seg), dim3(kSelB), lds, s, rec, d_src_off, d_cnt, d_retry_ok,
                       d_dst_off, s_param, key_bits, runs, kconst, out, d_res, d_cap, set_sizes, set_starts);
#ifdef SKS_FUSE_STAMPS
    {
      unsigned long long h[10] = {0};
      (void)hipStreamSynchronize(s);
      (void)hipMemcpyFromSymbol(h, HIP_SYMBOL(g_fuse_stamps), sizeof h);
      fprintf(stderr, "[k_bottom_fused stamps] n_seg %u max_cnt %llu: zero %llu count %llu scatter %llu isort %llu "
              "hash %llu distinct %llu select %llu write %llu\n", n_seg, (unsigned long long)max_cnt, h[0], h[1],
              h[2], h[3], h[4], h[5], h[6], h[7]);
    }
#endif
    return hipGetLastError();
  };
  if (max_cnt <= kSelB * 8)
    return flavour == 0 ? go(k_bottom_fused<0, 8>, fuse_lds<8>()) : go(k_bottom_fused<1, 8>, fuse_lds<8>());
  if (max_cnt <= kSelB * 12)
    return flavour == 0 ? go(k_bottom_fused<0, 12>, fuse_lds<12>())
                        : go(k_bottom_fused<1, 12>, fuse_lds<12>());
  return flavour == 0 ? go(k_bottom_fused<0, 16>, fuse_lds<16>()) : go(k_bottom_fused<1, 16>, fuse_lds<16>());
}

hipError_t launch_iota(uint64_t* out, uint64_t n, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_iota, dim3(grid_for(n)), dim3(kB), 0, s, out, n);
  return hipGetLastError();
}

hipError_t launch_gather(const uint64_t* src, const uint64_t* idx, uint64_t n, uint64_t* out,
                         hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_gather, dim3(grid_for(n)), dim3(kB), 0, s, src, idx, n, out);
  return hipGetLastError();
}

hipError_t launch_interleave(const uint64_t* lo, const uint64_t* hi, uint64_t n, uint64_t* out,
                             hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_interleave, dim3(grid_for(n)), dim3(kB), 0, s, lo, hi, n, out);
  return hipGetLastError();
}

SKS_CODE_OBJECT_HOOK(post)

}  // namespace sks
