// Minimal reproducer of the round-3 probe-loop miscompile.
//
// Round 3's k_join inserted each column element into an LDS table of 32-bit
// slots (tag << 10 | entry) with a probe loop that had TWO exits: a free slot
// (claim it: the element's entry is its own index) and a slot naming the same
// value (the element joins that entry).  ROCm 7.2 for gfx950 compiled it so
// that, for the second element of a thread, the joined entry lived in the
// register of the element's own entry index and was updated on every TAG match
// before the value compare: an element whose chain passed a slot with its tag
// but another value, and then claimed a free slot, came out naming the other
// value's entry.  The fix (join.hip chain, layout.hip dd_insert) is a loop with
// ONE exit edge whose stop test is evaluated without short-circuit.
//
// This program runs both loop forms on the same inputs and checks, for every
// element, that the entry it names holds its value.  A weak tag (runtime
// tag_bits, default 3) makes tag matches between different values frequent,
// so a miscompiled form fails on the first run from its own invariant.
//   hipcc --offload-arch=gfx950 -O3 -o chain_exits chain_exits.hip && ./chain_exits
// Exit status 1 when the ONE-exit form violates the invariant (the product's
// form); the two-exit form's count is reported (non-zero = the miscompile
// reproduces on this toolchain).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

constexpr int kB = 512, kCap = 1024, kMade = kCap / kB, kSlots = 4096;
constexpr uint32_t kFree = 0xFFFFFFFFu;

__device__ __forceinline__ uint32_t slot_of(uint64_t v) {
  return (((uint32_t)v ^ (uint32_t)(v >> 32)) * 0x85EBCA77u) >> 20;
}
__device__ __forceinline__ uint32_t tag_of(uint64_t v, uint32_t tag_bits) {
  const uint32_t t = (uint32_t)((v * 0xD6E8FEB86659FD93ull) >> (64 - tag_bits));
  return t == (1u << tag_bits) - 1 ? t - 1 : t;
}

// ONE_EXIT = false: round 3's form (two exits, entry assigned at each)
template <bool ONE_EXIT>
__global__ __launch_bounds__(kB) void k_insert(const uint64_t* __restrict__ vals, uint32_t tag_bits,
                                               uint32_t* __restrict__ out_ent) {
  __shared__ uint32_t s_slot[kSlots];
  __shared__ ulonglong2 s_ent[kCap];
  const int tid = threadIdx.x;
  const uint64_t* v_in = vals + (uint64_t)blockIdx.x * kCap;
  for (int i = tid; i < kSlots; i += kB) s_slot[i] = kFree;
  uint64_t cv[kMade];
#pragma unroll
  for (int u = 0; u < kMade; ++u) {
    cv[u] = v_in[tid + kB * u];
    s_ent[tid + kB * u] = make_ulonglong2(cv[u], 1ull << (u + 1));
  }
  __syncthreads();
  uint32_t hs[kMade], prev[kMade], tags[kMade], ent[kMade];
#pragma unroll
  for (int u = 0; u < kMade; ++u) {
    const uint32_t e = tid + kB * u;
    hs[u] = slot_of(cv[u]);
    tags[u] = tag_of(cv[u], tag_bits);
    prev[u] = atomicCAS(&s_slot[hs[u]], kFree, (tags[u] << 10) | e);
    ent[u] = 0;
  }
#pragma unroll
  for (int u = 0; u < kMade; ++u) {
    const uint64_t v = cv[u];
    const uint32_t e = tid + kB * u;
    uint32_t h = hs[u], x = prev[u];
    if (ONE_EXIT) {
      for (;;) {
        const uint64_t ev = s_ent[x & 1023u].x;
        if ((x == kFree) | (((x >> 10) == tags[u]) & (ev == v))) break;
        h = (h + 1) & (kSlots - 1);
        x = atomicCAS(&s_slot[h], kFree, (tags[u] << 10) | e);
      }
      if (x == kFree) {
        ent[u] = e;
      } else {
        ent[u] = x & 1023u;
        atomicOr(&s_ent[ent[u]].y, 1ull << (u + 1));
      }
    } else {
      for (;;) {
        if (x == kFree) {
          ent[u] = e;
          break;
        }
        if ((x >> 10) == tags[u] && s_ent[x & 1023u].x == v) {
          atomicOr(&s_ent[x & 1023u].y, 1ull << (u + 1));
          ent[u] = x & 1023u;
          break;
        }
        h = (h + 1) & (kSlots - 1);
        x = atomicCAS(&s_slot[h], kFree, (tags[u] << 10) | e);
      }
    }
  }
#pragma unroll
  for (int u = 0; u < kMade; ++u) out_ent[(uint64_t)blockIdx.x * kCap + tid + kB * u] = ent[u];
}

int main(int argc, char** argv) {
  const uint32_t tag_bits = argc > 1 ? (uint32_t)atoi(argv[1]) : 3;
  const uint32_t chunks = argc > 2 ? (uint32_t)atoi(argv[2]) : 8192;
  // values: a pool of 600 per chunk, so a chunk of 1024 holds duplicates
  std::vector<uint64_t> h((size_t)chunks * kCap);
  uint64_t x = 0x9E3779B97F4A7C15ull;
  for (uint32_t c = 0; c < chunks; ++c) {
    std::vector<uint64_t> pool(600);
    for (auto& p : pool) {
      x ^= x << 13; x ^= x >> 7; x ^= x << 17;
      p = x;
    }
    for (int i = 0; i < kCap; ++i) {
      x ^= x << 13; x ^= x >> 7; x ^= x << 17;
      h[(size_t)c * kCap + i] = pool[x % pool.size()];
    }
  }
  uint64_t* d_v;
  uint32_t* d_e;
  if (hipMalloc(&d_v, h.size() * 8) != hipSuccess || hipMalloc(&d_e, h.size() * 4) != hipSuccess) return 2;
  (void)hipMemcpy(d_v, h.data(), h.size() * 8, hipMemcpyHostToDevice);
  std::vector<uint32_t> ent(h.size());
  long bad[2] = {0, 0};
  for (int form = 0; form < 2; ++form) {
    if (form == 0)
      hipLaunchKernelGGL(k_insert<false>, dim3(chunks), dim3(kB), 0, 0, d_v, tag_bits, d_e);
    else
      hipLaunchKernelGGL(k_insert<true>, dim3(chunks), dim3(kB), 0, 0, d_v, tag_bits, d_e);
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    (void)hipMemcpy(ent.data(), d_e, ent.size() * 4, hipMemcpyDeviceToHost);
    for (uint32_t c = 0; c < chunks; ++c)
      for (int i = 0; i < kCap; ++i) {
        const uint32_t e = ent[(size_t)c * kCap + i];
        if (e >= (uint32_t)kCap || h[(size_t)c * kCap + e] != h[(size_t)c * kCap + i]) ++bad[form];
      }
  }
  printf("tag_bits %u, %u chunks x %d inserts: two-exit form %ld elements naming a foreign entry, "
         "one-exit form %ld\n", tag_bits, chunks, kCap, bad[0], bad[1]);
  (void)hipFree(d_v);
  (void)hipFree(d_e);
  return bad[1] ? 1 : 0;
}
