// Containment and ANI on the device, from exact intersection counts.
//
// The reference turns every ordered pair's count into containment and ANI on
// the host after the comparison (kmer-sketching.cpp:195-200):
//   containment(inter, |A|) = inter == 0 ? 0 : inter / |A|     (ani_estimation.cpp:24-28)
//   binomial_estimator(c, k) = c <= 0 ? 0 : pow(c, 1.0 / k)    (ani_estimation.cpp:38-42)
// with A the FIRST set of the pair and k = popcount(mask) / 2.  Here the same
// double arithmetic runs next to the counts (one thread per ordered pair), so
// an all-vs-all call ends with the ANI matrix in HBM instead of 10^6 host pow()
// calls.  The device pow is the ROCm math library's (within 1 ulp); the GPU
// tests compare every config-4 pair with the host's sks_ani_from_counts.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "sks_ani.hpp"
#include "sks_internal.hpp"

namespace sks {

namespace {

constexpr int kAB = 256;
constexpr int kTile = 64;

// ani[i * n + j] for rows [row_begin, row_end) of the dense n x n count
// matrix; |S_i| = counts[i][i]
__global__ __launch_bounds__(kAB) void k_ani_matrix(const int32_t* __restrict__ counts, uint32_t n,
                                                    uint32_t row_begin, uint32_t row_end, double inv_k,
                                                    double* __restrict__ cont, double* __restrict__ ani) {
  const uint64_t idx = (uint64_t)row_begin * n + (uint64_t)blockIdx.x * kAB + threadIdx.x;
  if (idx >= (uint64_t)row_end * n) return;
  const uint32_t i = (uint32_t)(idx / n);
  double c;
  const double a = ani_of(counts[idx], counts[(uint64_t)i * n + i], inv_k, &c);
  if (cont) cont[idx] = c;
  ani[idx] = a;
}

// Packed symmetric tiles: out[t][0][r][c] = ANI(i, j) and out[t][1][c][r] =
// ANI(j, i) for i = 64 I + r, j = 64 J + c (a diagonal tile's [0] already holds
// every ordered pair of its block; [1] repeats them transposed).
__global__ __launch_bounds__(kAB) void k_ani_tiles(const int32_t* __restrict__ packed,
                                                   const uint32_t* __restrict__ tiles, uint64_t n_tiles,
                                                   uint32_t n, const int32_t* __restrict__ sizes, double inv_k,
                                                   double* __restrict__ out) {
  const uint64_t idx = (uint64_t)blockIdx.x * kAB + threadIdx.x;
  if (idx >= n_tiles * kTile * kTile) return;
  const uint64_t t = idx / (kTile * kTile);
  const uint32_t rc = (uint32_t)(idx % (kTile * kTile)), r = rc / kTile, c = rc % kTile;
  const uint32_t i = tiles[2 * t] * kTile + r, j = tiles[2 * t + 1] * kTile + c;
  const int32_t x = packed[idx];
  double* o = out + t * 2 * kTile * kTile;
  o[rc] = i < n && j < n ? ani_of(x, sizes[i], inv_k, nullptr) : 0.0;
  o[kTile * kTile + c * kTile + r] = i < n && j < n ? ani_of(x, sizes[j], inv_k, nullptr) : 0.0;
}

__global__ __launch_bounds__(kAB) void k_ani_root(double* __restrict__ out, uint32_t size, double inv_k) {
  const uint32_t i = blockIdx.x * kAB + threadIdx.x;
  if (i <= size) out[i] = ani_of((int32_t)i, (int32_t)size, inv_k, nullptr);
}

}  // namespace

hipError_t launch_ani_root(double* out, uint32_t size, int kmer_num_ones, hipStream_t s) {
  const double inv_k = ((double)1.0) / ((double)kmer_num_ones);
  hipLaunchKernelGGL(k_ani_root, dim3(size / kAB + 1), dim3(kAB), 0, s, out, size, inv_k);
  return hipGetLastError();
}

hipError_t launch_ani_matrix(const int32_t* counts, uint32_t n, int kmer_num_ones, double* cont, double* ani,
                             hipStream_t s) {
  return launch_ani_rows(counts, n, 0, n, kmer_num_ones, cont, ani, s);
}

hipError_t launch_ani_rows(const int32_t* counts, uint32_t n, uint32_t row_begin, uint32_t row_end,
                           int kmer_num_ones, double* cont, double* ani, hipStream_t s) {
  if (row_end > n || row_begin >= row_end) return hipSuccess;
  const uint64_t cells = (uint64_t)(row_end - row_begin) * n;
  const double inv_k = ((double)1.0) / ((double)kmer_num_ones);
  hipLaunchKernelGGL(k_ani_matrix, dim3((unsigned)((cells + kAB - 1) / kAB)), dim3(kAB), 0, s, counts, n, row_begin,
                     row_end, inv_k, cont, ani);
  return hipGetLastError();
}

hipError_t launch_ani_tiles(const int32_t* packed, const uint32_t* tiles, uint64_t n_tiles, uint32_t n,
                            const int32_t* sizes, int kmer_num_ones, double* out, hipStream_t s) {
  const uint64_t cells = n_tiles * kTile * kTile;
  if (!cells) return hipSuccess;
  const double inv_k = ((double)1.0) / ((double)kmer_num_ones);
  hipLaunchKernelGGL(k_ani_tiles, dim3((unsigned)((cells + kAB - 1) / kAB)), dim3(kAB), 0, s, packed, tiles,
                     n_tiles, n, sizes, inv_k, out);
  return hipGetLastError();
}

SKS_CODE_OBJECT_HOOK(ani)

}  // namespace sks
