// Integer-op throughput probe for gfx950 (design input for the sketch kernel's hash).
// Each kernel runs ITERS x UNROLL independent ops per lane over 4 chains; the host
// prints lane-ops/s and the ratio to a v_add_u32 baseline.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); return 1; } } while (0)

constexpr int ITERS = 4096;
constexpr uint64_t M64 = 0x0e9846af9b1a615dull;

__device__ __forceinline__ uint64_t mix_b(uint64_t x) {
  x ^= x >> 32; x *= M64; x ^= x >> 32; x *= M64; x ^= x >> 28; return x;
}

template <int OP>
__global__ __launch_bounds__(256) void k_rate(uint64_t* out, uint64_t seed) {
  uint64_t a = seed + threadIdx.x * 0x9e3779b97f4a7c15ull + blockIdx.x;
  uint64_t b = a ^ 0x1234567887654321ull, c = a * 3 + 1, d = a ^ (a >> 7);
  uint32_t a32 = (uint32_t)a, b32 = (uint32_t)b, c32 = (uint32_t)c, d32 = (uint32_t)d;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      if constexpr (OP == 0) {  // v_add_u32 baseline
        a32 += 0x9e3779b9u; b32 += a32; c32 += b32; d32 += c32;
      } else if constexpr (OP == 1) {  // v_mul_lo_u32
        a32 *= 0x9b1a615du; b32 *= 0x9b1a615du; c32 *= 0x9b1a615du; d32 *= 0x9b1a615du;
      } else if constexpr (OP == 2) {  // v_mul_hi_u32
        a32 = __umulhi(a32, 0x9b1a615du) + 1; b32 = __umulhi(b32, 0x9b1a615du) + 1;
        c32 = __umulhi(c32, 0x9b1a615du) + 1; d32 = __umulhi(d32, 0x9b1a615du) + 1;
      } else if constexpr (OP == 3) {  // 64x64->64 multiply by constant
        a = (a ^ (a >> 29)) * M64; b = (b ^ (b >> 29)) * M64; c = (c ^ (c >> 29)) * M64; d = (d ^ (d >> 29)) * M64;
      } else if constexpr (OP == 4) {  // v_mul_u32_u24
        a32 = __umul24(a32, 0x9e3779u) + 7; b32 = __umul24(b32, 0x9e3779u) + 7;
        c32 = __umul24(c32, 0x9e3779u) + 7; d32 = __umul24(d32, 0x9e3779u) + 7;
      } else if constexpr (OP == 5) {  // 64-bit shifts (variable)
        a = (a << (b32 & 31)) ^ (a >> 3); b = (b >> (a32 & 31)) ^ (b << 5);
        c = (c << (d32 & 31)) ^ (c >> 3); d = (d >> (c32 & 31)) ^ (d << 5);
        a32 = (uint32_t)a; b32 = (uint32_t)b; c32 = (uint32_t)c; d32 = (uint32_t)d;
      } else if constexpr (OP == 6) {  // full boost-B mix (counted as one "op")
        a = mix_b(a + 0x9e3779b9u); b = mix_b(b + 0x9e3779b9u);
        c = mix_b(c + 0x9e3779b9u); d = mix_b(d + 0x9e3779b9u);
      } else if constexpr (OP == 7) {  // u32 x u32 -> u64 (v_mad_u64_u32)
        a = (uint64_t)(uint32_t)a * 0x9b1a615du + (a >> 32); b = (uint64_t)(uint32_t)b * 0x9b1a615du + (b >> 32);
        c = (uint64_t)(uint32_t)c * 0x9b1a615du + (c >> 32); d = (uint64_t)(uint32_t)d * 0x9b1a615du + (d >> 32);
      }
    }
  }
  uint64_t r = a ^ b ^ c ^ d ^ a32 ^ b32 ^ c32 ^ d32;
  if (r == 0x123) out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

template <int OP>
int run(const char* name, uint64_t* d_out, double base_rate, double* rate_out) {
  int dev; CHECK(hipGetDevice(&dev));
  hipDeviceProp_t p; CHECK(hipGetDeviceProperties(&p, dev));
  int blocks = p.multiProcessorCount * 8;
  hipEvent_t e0, e1; CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
  k_rate<OP><<<blocks, 256>>>(d_out, 1);
  CHECK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int r = 0; r < 5; ++r) {
    CHECK(hipEventRecord(e0));
    k_rate<OP><<<blocks, 256>>>(d_out, 1 + r);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms; CHECK(hipEventElapsedTime(&ms, e0, e1));
    if (ms < best) best = ms;
  }
  double ops = (double)blocks * 256 * ITERS * 8 * 4;
  double rate = ops / (best * 1e-3);
  *rate_out = rate;
  printf("%-28s %9.3f ms  %10.3e lane-ops/s  rel_to_add=%.3f\n", name, best, rate,
         base_rate > 0 ? rate / base_rate : 1.0);
  return 0;
}

int main() {
  uint64_t* d_out; CHECK(hipMalloc(&d_out, 1 << 24));
  double base = 0, r;
  if (run<0>("v_add_u32 (chain)", d_out, 0, &base)) return 1;
  if (run<1>("v_mul_lo_u32", d_out, base, &r)) return 1;
  if (run<2>("v_mul_hi_u32(+add)", d_out, base, &r)) return 1;
  if (run<3>("u64*const (+xorshift)", d_out, base, &r)) return 1;
  if (run<4>("v_mul_u32_u24(+add)", d_out, base, &r)) return 1;
  if (run<5>("u64 var shifts (4 ops)", d_out, base, &r)) return 1;
  if (run<6>("boost-B mix", d_out, base, &r)) return 1;
  if (run<7>("u32*u32->u64 (+add)", d_out, base, &r)) return 1;
  hipDeviceProp_t p; CHECK(hipGetDeviceProperties(&p, 0));
  printf("device %s CUs=%d clock=%d kHz\n", p.gcnArchName, p.multiProcessorCount, p.clockRate);
  return 0;
}
