// Pieces shared by the join layout build (layout.hip) and the LDS hash join
// (join.hip): the layout geometry, the value mixes, the join table's slot /
// tag functions and the upper-triangle tile order.
//
// Join layout (round 4, "entry layout").  For every block of 64 consecutive
// sketches, each DISTINCT value of the block once, with a 64-bit mask of the
// block's sketches holding it (bit s = sketch 64 * blk + s).  The value range is
// cut into G value groups by common bounds; a group's values are hashed into
// kGB buckets; kRG consecutive groups form a region.  A region's entries are
// contiguous, bucket by bucket, and start at the region's RAW offset in the
// block (the number of sketch elements of the block in earlier regions), so
// every region can be written by its own workgroup without knowing how many
// distinct values the others hold: a region's tail up to the next region's raw
// offset is unused.  Arrays (n sketches, nb = ceil(n / 64) blocks, T = sum of
// sizes):
//   vals   u64[T * EW]  entry values (EW = 1: u64 k-mers, w <= 32; EW = 2:
//                       (lo, hi) 128-bit k-mers, 32 < w <= 64)
//   masks  u64[T]       sketch mask of each entry
//   boff   u32[nb * BW]  per block (BW = lay_boff_words): B bucket starts,
//                       then the NR region ends, relative to bstart[blk], and
//                       in the row's last word the region bucket log
//   bstart u64[nb + 1]  raw block starts (prefix of the sizes); bstart[nb] = T
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

// 4096 table slots for <= 1024 column entries per chunk (load <= 1/4; 2048
// slots at load <= 1/2 measured slower: longer probe chains)
#ifndef SKS_JOIN_LOG_SLOTS
#define SKS_JOIN_LOG_SLOTS 12
#endif

namespace sks {
namespace jc {

// ---- layout geometry ----------------------------------------------------------------------
#ifndef SKS_LAYOUT_GLOG
#define SKS_LAYOUT_GLOG 3
#endif
constexpr uint32_t kGLog = SKS_LAYOUT_GLOG;   // hash buckets per value group: 8
// value groups per region: 2^rg, rg in [0, kRGLogMax], chosen per build (a
// large build takes 8-group regions, a small one smaller regions so its grid
// fills the chip; layout.hip join_layout_build); the region bucket log is
// stored in the last word of every block's boff row, so each layout tells the
// join its own region size
constexpr uint32_t kRGLogMax = 6 - kGLog;  // regions of at most 64 buckets
constexpr uint32_t kMaxLogB = 14;

__host__ __device__ inline uint32_t lay_gb_log(uint32_t log_b) { return log_b < kGLog ? log_b : kGLog; }
__host__ __device__ inline uint32_t lay_groups(uint32_t log_b) { return 1u << (log_b - lay_gb_log(log_b)); }
// log2 of the buckets of one region of 2^rg groups
__host__ __device__ inline uint32_t lay_rb_log(uint32_t log_b, uint32_t rg) {
  return log_b < kGLog + rg ? log_b : kGLog + rg;
}
__host__ __device__ inline uint32_t lay_regions(uint32_t log_b, uint32_t rg) {
  return 1u << (log_b - lay_rb_log(log_b, rg));
}
// one block's boff row: B bucket starts, room for the region ends of the
// finest regions (one group each), then the region bucket log
__host__ __device__ inline uint32_t lay_boff_words(uint32_t log_b) { return (1u << log_b) + lay_regions(log_b, 0) + 1; }

// ---- values -------------------------------------------------------------------------------
// A k-mer of EW 64-bit words (hi = 0 when EW == 1).
struct KV {
  uint64_t lo, hi;
};

template <int EW>
__device__ __forceinline__ KV kv_load(const uint64_t* __restrict__ p, uint64_t i) {
  if constexpr (EW == 1) return KV{p[i], 0};
  else return KV{p[2 * i], p[2 * i + 1]};
}
template <int EW>
__device__ __forceinline__ void kv_store(uint64_t* p, uint64_t i, const KV& v) {
  p[EW * i] = v.lo;
  if constexpr (EW == 2) p[2 * i + 1] = v.hi;
}
template <int EW>
__device__ __forceinline__ bool kv_eq(const KV& a, const KV& b) {
  if constexpr (EW == 1) return a.lo == b.lo;
  else return (a.lo == b.lo) & (a.hi == b.hi);
}
template <int EW>
__device__ __forceinline__ bool kv_lt(const KV& a, const KV& b) {
  if constexpr (EW == 1) return a.lo < b.lo;
  else return a.hi < b.hi || (a.hi == b.hi && a.lo < b.lo);
}
// 64-bit mix of a value: the layout's bucket (top bits) and its dedup table
// slot (the bits below) come from it
template <int EW>
__device__ __forceinline__ uint64_t kv_mix(const KV& v) {
  if constexpr (EW == 1) return v.lo * 0x9E3779B97F4A7C15ull;
  else return (v.lo ^ (v.hi * 0xC2B2AE3D27D4EB4Full + 0x165667B19E3779F9ull)) * 0x9E3779B97F4A7C15ull;
}
// the value's hash bucket within its value group
template <int EW>
__device__ __forceinline__ uint32_t kv_group_bucket(const KV& v, uint32_t gb_log) {
  return gb_log ? (uint32_t)(kv_mix<EW>(v) >> (64 - gb_log)) : 0u;
}

// ---- the join's LDS fingerprint table ------------------------------------------------------
constexpr int kFLog = SKS_JOIN_LOG_SLOTS;
constexpr int kFSlots = 1 << kFLog;      // 32-bit table slots: fingerprint << 10 | entry
constexpr uint32_t kFFree = 0xFFFFFFFFu;  // empty slot (a tag is never all ones)

template <int EW>
__device__ __forceinline__ uint64_t fp_fold(const KV& v) {
  if constexpr (EW == 1) return v.lo;
  else return v.lo ^ (v.hi * 0x9FB21C651E98DF25ull);
}
template <int EW>
__device__ __forceinline__ uint32_t fp_slot(const KV& kv) {
  const uint64_t v = fp_fold<EW>(kv);
  return (((uint32_t)v ^ (uint32_t)(v >> 32)) * 0x85EBCA77u) >> (32 - kFLog);
}
template <int EW>
__device__ __forceinline__ uint32_t fp_tag(const KV& kv) {  // 22 bits, never all ones
  const uint32_t t = (uint32_t)((fp_fold<EW>(kv) * 0xD6E8FEB86659FD93ull) >> 42);
  return t == 0x3FFFFFu ? 0x3FFFFEu : t;
}

// (I, J) of upper-triangle tile t of nb x nb blocks, row-major, I <= J
__device__ __forceinline__ void sym_tile(uint64_t t, uint32_t nb, uint32_t& I, uint32_t& J) {
  uint32_t i = 0;
  uint64_t rem = t;
  while (rem >= nb - i) {  // row i of the upper triangle holds nb - i tiles
    rem -= nb - i;
    ++i;
  }
  I = i;
  J = i + (uint32_t)rem;
}

}  // namespace jc
}  // namespace sks
