// Which lane/byte holds which A[row][k] / B[k][col] element of
// v_mfma_i32_32x32x32_i8 on gfx950?  (The programming guide gives the bf16
// maps and says to check other dtypes with exact integer data.)  Candidate
// maps are tried with random 0/1 operands against a host product; the ones
// that match are printed.  C/D: col = lane & 31, row = (reg & 3) + 8 * (reg >> 2)
// + 4 * (lane >> 5) (dtype-independent on gfx950).
//   hipcc --offload-arch=gfx950 -O2 tools/microbench/mfma_i8_layout.hip -o /tmp/mfma_i8 && /tmp/mfma_i8
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

// candidate k index of byte j (0..15) held by lane l
__host__ __device__ inline int k_of(int map, int l, int j) {
  const int h = l >> 5;
  switch (map) {
    case 0: return 16 * h + j;                              // contiguous 16 per half
    case 1: return (j < 8) ? 8 * h + j : 16 + 8 * h + (j - 8);  // two K=16 steps
    default: return 2 * j + h;                              // interleaved
  }
}

__global__ void k_probe(const signed char* A, const signed char* B, int* D, int map) {
  const int l = threadIdx.x;
  v4i a, b;
  signed char* pa = reinterpret_cast<signed char*>(&a);
  signed char* pb = reinterpret_cast<signed char*>(&b);
  for (int j = 0; j < 16; ++j) {
    const int k = k_of(map, l, j);
    pa[j] = A[(l & 31) * 32 + k];  // A[row][k]
    pb[j] = B[k * 32 + (l & 31)];  // B[k][col]
  }
  v16i acc = {};
  acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, acc, 0, 0, 0);
  for (int r = 0; r < 16; ++r) {
    const int row = (r & 3) + 8 * (r >> 2) + 4 * (l >> 5), col = l & 31;
    D[row * 32 + col] = acc[r];
  }
}

int main() {
  std::vector<signed char> A(32 * 32), B(32 * 32);
  srand(7);
  for (auto& x : A) x = rand() & 1;
  for (auto& x : B) x = rand() & 1;
  std::vector<int> want(32 * 32, 0);
  for (int r = 0; r < 32; ++r)
    for (int c = 0; c < 32; ++c)
      for (int k = 0; k < 32; ++k) want[r * 32 + c] += A[r * 32 + k] * B[k * 32 + c];
  signed char *dA, *dB;
  int* dD;
  hipMalloc(&dA, 1024);
  hipMalloc(&dB, 1024);
  hipMalloc(&dD, 4096);
  hipMemcpy(dA, A.data(), 1024, hipMemcpyHostToDevice);
  hipMemcpy(dB, B.data(), 1024, hipMemcpyHostToDevice);
  int found = 0;
  for (int map = 0; map < 3; ++map) {
    hipLaunchKernelGGL(k_probe, dim3(1), dim3(64), 0, 0, dA, dB, dD, map);
    std::vector<int> got(1024);
    hipMemcpy(got.data(), dD, 4096, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < 1024; ++i) bad += got[i] != want[i];
    printf("map %d: %d of 1024 wrong\n", map, bad);
    if (!bad) found = 1;
  }
  return found ? 0 : 1;
}
