// LDS atomic / read throughput on gfx950: 256-thread workgroups, 3 per CU,
// each lane hits pseudo-random 8-B-aligned slots of a 32 KB table.
//   hipcc --offload-arch=gfx950 -O3 lds_atomics.hip -o lds_atomics && ./lds_atomics
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int kSlots = 4096;
constexpr int kIters = 4096;

template <int OP>
__global__ __launch_bounds__(256) void k(unsigned long long* out) {
  __shared__ unsigned long long tab[kSlots];
  for (int i = threadIdx.x; i < kSlots; i += 256) tab[i] = i;
  __syncthreads();
  uint32_t x = threadIdx.x * 2654435761u + blockIdx.x;
  unsigned long long acc = 0;
  for (int it = 0; it < kIters; ++it) {
    x = x * 1664525u + 1013904223u;
    const uint32_t h = x >> 20;  // 0..4095
    if constexpr (OP == 0) acc += atomicCAS(&tab[h], (unsigned long long)it, (unsigned long long)x);
    else if constexpr (OP == 1) atomicOr(&tab[h], 1ull << (x & 63));
    else if constexpr (OP == 2) atomicOr(reinterpret_cast<unsigned*>(tab) + h, 1u << (x & 31));
    else if constexpr (OP == 3) atomicAdd(reinterpret_cast<unsigned*>(tab) + h, 1u);
    else if constexpr (OP == 4) acc += tab[h];
    else if constexpr (OP == 5) { ulonglong2 v = reinterpret_cast<ulonglong2*>(tab)[h >> 1]; acc += v.x ^ v.y; }
    else if constexpr (OP == 6) acc += atomicCAS(reinterpret_cast<unsigned*>(tab) + h, (unsigned)it, x);
    else if constexpr (OP == 7) atomicAdd(reinterpret_cast<unsigned*>(tab) + (threadIdx.x * 65 + (x & 63)) % (2 * kSlots), 1u);
  }
  __syncthreads();
  if (acc == 42) out[0] = tab[threadIdx.x];
}

int main() {
  unsigned long long* out;
  hipMalloc(&out, 64);
  const char* names[] = {"ds_cmpst_rtn_b64", "ds_or_b64", "ds_or_b32", "ds_add_u32 random",
                         "ds_read_b64", "ds_read_b128", "ds_cmpst_rtn_b32", "ds_add_u32 row-stride-65"};
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const int grid = 256 * 3;
  for (int op = 0; op < 8; ++op) {
    for (int rep = 0; rep < 2; ++rep) {
      hipEventRecord(a);
      switch (op) {
        case 0: k<0><<<grid, 256>>>(out); break;
        case 1: k<1><<<grid, 256>>>(out); break;
        case 2: k<2><<<grid, 256>>>(out); break;
        case 3: k<3><<<grid, 256>>>(out); break;
        case 4: k<4><<<grid, 256>>>(out); break;
        case 5: k<5><<<grid, 256>>>(out); break;
        case 6: k<6><<<grid, 256>>>(out); break;
        case 7: k<7><<<grid, 256>>>(out); break;
      }
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      const double lane_ops = (double)grid * 256 * kIters;
      if (rep) printf("%-26s %8.3f ms  %.3e lane-ops/s  %.2f lane-ops/clk/CU @2.4GHz\n", names[op], ms,
                      lane_ops / (ms * 1e-3), lane_ops / (ms * 1e-3) / 256 / 2.4e9);
    }
  }
  return 0;
}
