// Per-instruction VALU throughput on gfx950 with inline asm (no constant
// folding).  Each kernel issues ITERS x 16 x 8 independent instances of one
// instruction per lane; the host prints time relative to v_xor_b32.
// Also times two 64x64->64 multiply-by-constant lowerings and two hash_mix
// variants (design input for scan.hip).
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); return 1; } } while (0)

constexpr int ITERS = 2048;
constexpr uint32_t MLO = 0x9b1a615du, MHI = 0x0e9846afu;

#define REP8(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)

template <int OP>
__global__ __launch_bounds__(256) void k(uint32_t* out, uint32_t seed) {
  uint32_t r[8], h[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) { r[i] = seed * (threadIdx.x + 1) + i * 77; h[i] = r[i] ^ 0x5555u; }
  const uint32_t s = seed | 1;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int u = 0; u < 16; ++u) {
#define B(i)                                                                                      \
  if constexpr (OP == 0) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(r[i]) : "v"(s));            \
  if constexpr (OP == 1) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(r[i]) : "v"(s));         \
  if constexpr (OP == 2) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(r[i]) : "v"(s));         \
  if constexpr (OP == 3) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(*(uint64_t*)&h[i & ~1]) : "v"(r[i]), "v"(s) : "vcc"); \
  if constexpr (OP == 4) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(r[i]) : "v"(s));        \
  if constexpr (OP == 5) asm volatile("v_mul_hi_u32_u24 %0, %0, %1" : "+v"(r[i]) : "v"(s));     \
  if constexpr (OP == 6) asm volatile("v_add3_u32 %0, %0, %1, %1" : "+v"(r[i]) : "v"(s));       \
  if constexpr (OP == 7) asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(*(uint64_t*)&r[i & ~1]) : "v"(*(uint64_t*)&h[i & ~1])); \
  if constexpr (OP == 8) asm volatile("v_lshrrev_b64 %0, 28, %0" : "+v"(*(uint64_t*)&r[i & ~1])); \
  if constexpr (OP == 9) asm volatile("v_alignbit_b32 %0, %0, %1, 7" : "+v"(r[i]) : "v"(h[i]));  \
  if constexpr (OP == 10) asm volatile("v_mad_u32_u24 %0, %0, %1, %1" : "+v"(r[i]) : "v"(s));   \
  if constexpr (OP == 11) asm volatile("v_and_b32 %0, %0, %1" : "+v"(r[i]) : "v"(s));            \
  if constexpr (OP == 12) asm volatile("v_add_u32 %0, %0, %1" : "+v"(r[i]) : "v"(s));            \
  if constexpr (OP == 13) asm volatile("v_lshlrev_b32 %0, 3, %0" : "+v"(r[i]));                  \
  if constexpr (OP == 14) asm volatile("v_mov_b32 %0, %1" : "=v"(r[i]) : "v"(h[i]));             \
  if constexpr (OP == 15) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(r[i]) : "v"(s) : "vcc"); \
  if constexpr (OP == 16) asm volatile("v_cmp_lt_u64 vcc, %0, %1" :: "v"(*(uint64_t*)&r[i & ~1]), "v"(*(uint64_t*)&h[i & ~1]) : "vcc"); \
  if constexpr (OP == 17) asm volatile("v_xor_b32_e64 %0, %0, %1" : "+v"(r[i]) : "v"(s));        \
  if constexpr (OP == 18) asm volatile("v_perm_b32 %0, %0, %1, %1" : "+v"(r[i]) : "v"(s));       \
  if constexpr (OP == 19) asm volatile("v_bfe_u32 %0, %0, 3, 9" : "+v"(r[i]));                   \
  if constexpr (OP == 20) asm volatile("v_or3_b32 %0, %0, %1, %1" : "+v"(r[i]) : "v"(s));       \
  if constexpr (OP == 21) asm volatile("v_lshl_or_b32 %0, %0, 3, %1" : "+v"(r[i]) : "v"(s));
      REP8(B)
#undef B
    }
  }
  uint32_t x = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) x ^= r[i];
  if (x == 0x12345) out[threadIdx.x] = x;
}

// 64-bit multiply by constant, lowered two ways; 8 independent chains.
__device__ __forceinline__ uint64_t mulA(uint64_t x) {  // compiler's: mul_lo, mad_u64, mul_lo, add3
  return x * ((uint64_t)MHI << 32 | MLO);
}
__device__ __forceinline__ uint64_t mulB(uint64_t x) {  // mul_lo + 2 x mad_u64 (asm)
  uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  uint32_t t;
  asm volatile("v_mul_lo_u32 %0, %1, %2" : "=v"(t) : "v"(lo), "s"(MHI));
  uint64_t acc = t;  // (t, 0)
  uint64_t t2;
  asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %3" : "=&v"(t2) : "v"(hi), "s"(MLO), "v"(acc) : "vcc");
  uint64_t acc2 = (uint64_t)(uint32_t)t2 << 32;  // (0, t2)
  uint64_t r;
  asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %3" : "=&v"(r) : "v"(lo), "s"(MLO), "v"(acc2) : "vcc");
  return r;
}

template <int V>
__global__ __launch_bounds__(256) void kmul(uint64_t* out, uint64_t seed) {
  uint64_t r[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) r[i] = seed * (threadIdx.x + 1) + i * 0x9e3779b97f4a7c15ull;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        uint64_t x = r[i] ^ (r[i] >> 32);
        r[i] = V == 0 ? mulA(x) : mulB(x);
      }
    }
  }
  uint64_t x = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) x ^= r[i];
  if (x == 0x12345) out[threadIdx.x] = x;
}

template <class K, class... A>
float time_kernel(K kern, int blocks, A... args) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, args...);
  (void)hipDeviceSynchronize();
  float best = 1e30f;
  for (int r = 0; r < 5; ++r) {
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, args...);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    if (ms < best) best = ms;
  }
  return best;
}

int main() {
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, 0));
  const int blocks = p.multiProcessorCount * 8;  // 8 waves per SIMD
  uint32_t* out;
  CHECK(hipMalloc(&out, 1 << 20));
  const double insts = (double)blocks * 4 * ITERS * 16 * 8;  // wave-instructions
  const char* names[] = {"v_xor_b32", "v_mul_lo_u32", "v_mul_hi_u32", "v_mad_u64_u32",
                         "v_mul_u32_u24", "v_mul_hi_u32_u24", "v_add3_u32", "v_lshl_add_u64",
                         "v_lshrrev_b64", "v_alignbit_b32", "v_mad_u32_u24", "v_and_b32",
                         "v_add_u32", "v_lshlrev_b32", "v_mov_b32", "v_cndmask_b32",
                         "v_cmp_lt_u64", "v_xor_b32_e64", "v_perm_b32", "v_bfe_u32", "v_or3_b32",
                         "v_lshl_or_b32"};
  constexpr int NOPS = 22;
  float t[NOPS];
  t[0] = time_kernel(k<0>, blocks, out, 3u);
  t[1] = time_kernel(k<1>, blocks, out, 3u);
  t[2] = time_kernel(k<2>, blocks, out, 3u);
  t[3] = time_kernel(k<3>, blocks, out, 3u);
  t[4] = time_kernel(k<4>, blocks, out, 3u);
  t[5] = time_kernel(k<5>, blocks, out, 3u);
  t[6] = time_kernel(k<6>, blocks, out, 3u);
  t[7] = time_kernel(k<7>, blocks, out, 3u);
  t[8] = time_kernel(k<8>, blocks, out, 3u);
  t[9] = time_kernel(k<9>, blocks, out, 3u);
  t[10] = time_kernel(k<10>, blocks, out, 3u);
  t[11] = time_kernel(k<11>, blocks, out, 3u);
  t[12] = time_kernel(k<12>, blocks, out, 3u);
  t[13] = time_kernel(k<13>, blocks, out, 3u);
  t[14] = time_kernel(k<14>, blocks, out, 3u);
  t[15] = time_kernel(k<15>, blocks, out, 3u);
  t[16] = time_kernel(k<16>, blocks, out, 3u);
  t[17] = time_kernel(k<17>, blocks, out, 3u);
  t[18] = time_kernel(k<18>, blocks, out, 3u);
  t[19] = time_kernel(k<19>, blocks, out, 3u);
  t[20] = time_kernel(k<20>, blocks, out, 3u);
  t[21] = time_kernel(k<21>, blocks, out, 3u);
  const double simds = p.multiProcessorCount * 4.0;
  for (int i = 0; i < NOPS; ++i) {
    double per_simd = insts / simds;  // wave-instructions per SIMD
    double ns_per = t[i] * 1e6 / per_simd;
    printf("%-18s %8.3f ms  rel=%5.2f  ns/wave-inst/SIMD=%.3f (cycles@2.4GHz=%.2f)\n", names[i], t[i],
           t[i] / t[0], ns_per, ns_per * 2.4);
  }
  uint64_t* o64 = (uint64_t*)out;
  float ma = time_kernel(kmul<0>, blocks, o64, (uint64_t)3);
  float mb = time_kernel(kmul<1>, blocks, o64, (uint64_t)3);
  double muls = (double)blocks * 256 * ITERS * 4 * 8;
  printf("u64 mul (mul_lo,mad,mul_lo,add3) %8.3f ms  %.3e mul/s\n", ma, muls / (ma * 1e-3));
  printf("u64 mul (mul_lo,mad,mad)         %8.3f ms  %.3e mul/s\n", mb, muls / (mb * 1e-3));
  printf("device %s CUs=%d\n", p.gcnArchName, p.multiProcessorCount);
  return 0;
}
