// Row ranges of the dense containment / ANI kernel (ani.hip): rows
// [row_begin, row_end) of ani[i * n + j] from the n x n count matrix, so a caller
// can convert the rows an all-pairs call has finished (sks_ani_rows).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace sks {
hipError_t launch_ani_rows(const int32_t* counts, uint32_t n, uint32_t row_begin, uint32_t row_end,
                           int kmer_num_ones, double* cont, double* ani, hipStream_t s);
}  // namespace sks
