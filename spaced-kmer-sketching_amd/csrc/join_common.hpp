// Pieces shared by the two LDS hash-join kernels (intersect.hip k_join over a
// hash-bucketed block layout, rjoin.hip k_rjoin straight from the sorted
// sketches): the fingerprint table's slot / tag functions and the
// upper-triangle tile order.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

// 4096 table slots for <= 1024 column elements per chunk (load <= 1/4; 2048
// slots at load <= 1/2 measured slower: longer probe chains)
#ifndef SKS_JOIN_LOG_SLOTS
#define SKS_JOIN_LOG_SLOTS 12
#endif

namespace sks {
namespace jc {

constexpr int kFLog = SKS_JOIN_LOG_SLOTS;
constexpr int kFSlots = 1 << kFLog;      // 32-bit table slots: fingerprint << 10 | entry
constexpr uint32_t kFFree = 0xFFFFFFFFu;  // empty slot (a tag is never all ones)

__device__ __forceinline__ uint32_t fp_slot(uint64_t v) {
  return (((uint32_t)v ^ (uint32_t)(v >> 32)) * 0x85EBCA77u) >> (32 - kFLog);
}
__device__ __forceinline__ uint32_t fp_tag(uint64_t v) {  // 22 bits, never all ones
  const uint32_t t = (uint32_t)((v * 0xD6E8FEB86659FD93ull) >> 42);
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
