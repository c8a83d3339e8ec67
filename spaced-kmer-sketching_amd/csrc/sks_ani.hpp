// Containment / ANI of one ordered pair on the device, shared by the ANI
// kernels (ani.hip) and the join's fused tile conversion (join.hip):
//   containment(inter, |A|) = inter == 0 ? 0 : inter / |A|     (ani_estimation.cpp:24-28)
//   binomial_estimator(c, k) = c <= 0 ? 0 : pow(c, 1.0 / k)    (ani_estimation.cpp:38-42)
// with A the FIRST set of the pair (kmer-sketching.cpp:195-200).  Also the row
// ranges of the dense kernel: rows [row_begin, row_end) of ani[i * n + j] from
// the n x n count matrix, so a caller can convert the rows an all-pairs call
// has finished (sks_ani_rows).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace sks {

__device__ __forceinline__ double ani_of(int32_t inter, int32_t size_first, double inv_k, double* cont) {
  const double c = inter == 0 ? 0.0 : (double)inter / (double)size_first;
  if (cont) *cont = c;
  return c <= 0.0 ? 0.0 : pow(c, inv_k);
}

// out[i] = ani_of(i, size) for i in [0, size]: the fused ANI of a row whose set
// holds `size` elements reads its value here instead of evaluating pow (the
// same function, so the same doubles)
hipError_t launch_ani_root(double* out, uint32_t size, int kmer_num_ones, hipStream_t s);
hipError_t launch_ani_rows(const int32_t* counts, uint32_t n, uint32_t row_begin, uint32_t row_end,
                           int kmer_num_ones, double* cont, double* ani, hipStream_t s);
}  // namespace sks
