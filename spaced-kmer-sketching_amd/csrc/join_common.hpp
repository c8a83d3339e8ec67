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

// Walks a table's probe chain from the occupied slot word x at index h to the
// first free slot or the slot naming value v's entry, and returns that word
// (kFFree: v is absent; with insert, the walk claimed the free slot at h for
// `word`).  Callers take the entry from the returned word.
//
// The loop has ONE exit, its stop test evaluated without short-circuit (the
// entry x names is read whether or not the tag matches; for a free word that is
// entry 1023, read and ignored).  Written with two exits (free / match) and the
// entry index assigned at the match exit, the compiler (ROCm 7.2, gfx950)
// merged the exits and kept the joined entry in the register of the element's
// own entry index, updated on every tag match: an element whose chain passed a
// slot with its tag but another value, and then claimed a free slot, came out
// naming the other value's entry.  k_join then counted that column element
// with a foreign mask (about one insert in 10^7; a diagonal count one short,
// one stray +1; tools/layout_verify.py and tools/join_repeat.py found it).
__device__ __forceinline__ uint32_t join_chain(uint32_t x, uint32_t& h, uint32_t tag, uint64_t v, uint32_t word,
                                               uint32_t* s_slot, const ulonglong2* s_ent, bool insert) {
  for (;;) {
    const uint64_t ev = s_ent[x & 1023u].x;
    if ((x == kFFree) | (((x >> 10) == tag) & (ev == v))) return x;
    h = (h + 1) & (kFSlots - 1);
    x = insert ? atomicCAS(&s_slot[h], kFFree, word) : s_slot[h];
  }
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
