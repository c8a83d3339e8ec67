// Hash arithmetic shared by the host API and the gfx950 kernels.
//
// frac_min_hash (reference kmer.hpp:135-149) = H(masked) ^ H(mask) ^ w ^ nonce
// with H = boost::hash_value(dynamic_bitset<unsigned long>) on a 128-bit set:
//   res = hash_value(num_bits = 128); hash_combine(res, m_bits)
//   hash_value(m_bits) = hash_range(blocks) = combine(combine(0, lo), hi)
// The Boost version is unpinned by the reference (compile.sh:8); both
// plausible flavours are provided (DESIGN.md "hash parity").
#pragma once
#include <cstdint>

#if defined(__HIPCC__)
#define SKS_HD __host__ __device__ __forceinline__
#else
#define SKS_HD inline
#endif

namespace sks {

constexpr uint64_t kGolden32 = 0x9e3779b9ULL;         // boost hash_combine constant
constexpr uint64_t kMixMul = 0x0e9846af9b1a615dULL;   // boost hash_mix<64> multiplier
constexpr uint64_t kMurmurMul = 0xc6a4a7935bd1e995ULL;
constexpr uint64_t kMurmurAdd = 0xe6546b64ULL;

// x * M (mod 2^64) for a compile-time constant M.  On gfx950 every 32-bit
// integer multiply issues at the rate of any other VOP3 op, so the cost is the
// instruction count: this lowering uses 1 v_mul_lo_u32 + 2 v_mad_u64_u32
// (the compiler's default is 2 v_mul_lo_u32 + 1 v_mad_u64_u32 + 1 v_add3_u32);
// measured 15% faster in tools/microbench/isa_rates.hip.
template <uint64_t M>
SKS_HD uint64_t mul_const(uint64_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
  // written so that hipcc emits v_mul_lo_u32 + 2 x v_mad_u64_u32 (the low
  // word of hi*mlo + lo*mhi is formed by the first mad's 32-bit add)
  const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  const uint32_t cross = hi * (uint32_t)M + lo * (uint32_t)(M >> 32);
  return (uint64_t)lo * (uint32_t)M + ((uint64_t)cross << 32);
#else
  return x * M;
#endif
}

// Flavour B (Boost >= 1.81): boost::hash_detail::hash_mix_impl<64>::fn
SKS_HD uint64_t hash_mix(uint64_t x) {
  x ^= x >> 32;
  x = mul_const<kMixMul>(x);
  x ^= x >> 32;
  x = mul_const<kMixMul>(x);
  x ^= x >> 28;
  return x;
}
SKS_HD uint64_t combine_mix(uint64_t seed, uint64_t v) { return hash_mix(seed + kGolden32 + v); }

// Flavour A (Boost 1.71-1.80): boost::hash_detail::hash_combine_impl (64-bit)
SKS_HD uint64_t combine_legacy(uint64_t h, uint64_t k) {
  k = mul_const<kMurmurMul>(k);
  k ^= k >> 47;
  k = mul_const<kMurmurMul>(k);
  h ^= k;
  h = mul_const<kMurmurMul>(h);
  h += kMurmurAdd;
  return h;
}

template <int FLAVOUR>
SKS_HD uint64_t combine(uint64_t seed, uint64_t v) {
  if constexpr (FLAVOUR == 0) return combine_mix(seed, v);
  else return combine_legacy(seed, v);
}

// H of a 128-bit dynamic_bitset with blocks (lo, hi).
template <int FLAVOUR>
SKS_HD uint64_t hash_bitset128(uint64_t lo, uint64_t hi) {
  return combine<FLAVOUR>(128, combine<FLAVOUR>(combine<FLAVOUR>(0, lo), hi));
}

SKS_HD uint64_t hash_bitset128_rt(uint64_t lo, uint64_t hi, int flavour) {
  return flavour == 0 ? hash_bitset128<0>(lo, hi) : hash_bitset128<1>(lo, hi);
}

// The per-run constant part of frac_min_hash: H(mask) ^ hash<int>(w) ^ nonce.
// boost::hash<int> is the identity; `nonce` is stored as int (kmer.hpp:139-141)
// and widened to size_t by sign extension.
SKS_HD uint64_t fmh_const(uint64_t mask_lo, uint64_t mask_hi, int w, int64_t nonce, int flavour) {
  return hash_bitset128_rt(mask_lo, mask_hi, flavour) ^ (uint64_t)(int64_t)w ^
         (uint64_t)(int64_t)(int32_t)nonce;
}

// Exact divisibility test for x % c == 0 without a 64-bit division
// (Granlund-Montgomery): with c = 2^s * d, d odd,
//   x % c == 0  <=>  (x mod 2^s == 0)  and  (x * d^-1 mod 2^64 <= floor((2^64 - 1) / d))
// (d | x  <=>  x * d^-1 = x / d <= (2^64 - 1) / d;  2^s | x is independent).
struct DivTest {
  uint32_t low_mask;  // low s bits (s <= 63; bits above 31 checked via dlim below)
  uint64_t dinv;
  uint64_t lim;
  uint32_t rot;       // s
};

inline DivTest make_div_test(uint64_t c) {
  DivTest t{};
  uint32_t s = 0;
  while (((c >> s) & 1) == 0) ++s;  // c > 0
  uint64_t d = c >> s;
  uint64_t inv = d;  // Newton iteration: inverse of odd d modulo 2^64
  for (int i = 0; i < 6; ++i) inv *= 2 - d * inv;
  t.rot = s;
  t.dinv = inv;
  t.lim = ~0ull / d;
  t.low_mask = s >= 32 ? 0xFFFFFFFFu : ((1u << s) - 1);
  return t;
}

// x * m (mod 2^64) for a wave-uniform runtime m (same lowering as mul_const).
SKS_HD uint64_t mul_uniform(uint64_t x, uint64_t m) {
  const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  const uint32_t cross = hi * (uint32_t)m + lo * (uint32_t)(m >> 32);
  return (uint64_t)lo * (uint32_t)m + ((uint64_t)cross << 32);
}

// s >= 32 needs the high word too: rare (c a multiple of 2^32) and handled by
// the caller passing high_mask.
SKS_HD bool div_test(uint64_t x, uint32_t low_mask, uint32_t high_mask, uint64_t dinv,
                     uint64_t lim) {
  return ((((uint32_t)x & low_mask) | ((uint32_t)(x >> 32) & high_mask)) == 0) &
         (mul_uniform(x, dinv) <= lim);
}

// splitmix64 output p of a stream seeded with `seed` (synthetic genomes).
SKS_HD uint64_t splitmix64_at(uint64_t seed, uint64_t p) {
  uint64_t z = seed + (p + 1) * 0x9e3779b97f4a7c15ULL;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}

}  // namespace sks
