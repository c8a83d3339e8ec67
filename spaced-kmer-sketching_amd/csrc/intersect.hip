// Kernel 2 — pairwise sketch intersection counts.
//
// The reference counts |A ∩ B| by iterating the smaller kmer_set and probing
// the larger hash map (kmer_set.cpp:23-41), one pair per cilk_for iteration
// (kmer_set.cpp:167-184).  Sketches here are sorted unique arrays, so a pair
// is a sorted-merge count.  One 64-lane wavefront owns one pair: the smaller
// sketch is split evenly over the lanes, each lane lower_bounds its first
// element in the larger sketch and merges forward; a wave reduction gives the
// count.  The result is the same integer the reference computes.
#include <hip/hip_runtime.h>

#include <cstdint>

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

hipError_t launch_intersect_all(const uint64_t* data, const uint64_t* starts, const uint32_t* sizes,
                                int elem_words, uint32_t n, uint32_t row_begin, uint32_t row_end,
                                int32_t* out, hipStream_t s) {
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
