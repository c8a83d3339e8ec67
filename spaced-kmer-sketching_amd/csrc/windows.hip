// Every window of a record-stream piece, dense by start position, for a HOST
// predicate (the reference's std::function<bool(const kmer)> plug-in point,
// kmer.hpp:93-103, called once per window at kmer_sliding.cpp:183).
//
// An arbitrary host callback cannot run in a kernel, so the facade's
// std::function builders (cpp/facade.cpp for_each_window) have the GPU extract
// each window's canonical kmer (kmer_bits and masked_bits, kmer_sliding.cpp:
// 144-181) and hand it to the predicate on the host.  Unlike the list build
// (sks_kmer_list_build: scan, compaction, a position sort, re-materialisation)
// nothing here is selected, so nothing is sorted: window p of the piece lands
// at output row p - first, with one validity bit per row.
//
// One thread per 64 consecutive starts (one validity word): it slides the
// reference's two windows over the bytes from 64 - w before its first start,
// exactly as nucleotide_string_to_kmers does over a run (a non-ACGT byte ends
// the run and the next run starts from empty windows, kmer_sliding.cpp:129):
//   F = (F << 2) | code            128 bits: up to 64 bases of history
//                                  (update_kmer_window, :26-31)
//   R = (R >> 2) | (code^3) << 2(w-1)   w bases (update_complement_kmer_window, :42-47)
//   canonical = F & M < R & M ? F : R   (:159-175)
// Output row: {kmer_bits lo, hi, masked lo} for w <= 32 (the masked bits of a
// <= 64-bit mask fit one word), {kmer lo, hi, masked lo, hi} for w > 32.
// The piece's bytes before `first` are history only: a caller cutting a long
// stream into pieces passes up to 64 - w bytes in front of each, so F holds
// the same history as over the whole stream.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "sks_internal.hpp"

namespace sks {

namespace {

constexpr int kWB = 256;

// ACGT (either case) -> 0..3, anything else -> 4 (fasta_processing.cpp:35-69)
__device__ __forceinline__ uint32_t win_code(uint8_t c) {
  const uint32_t low = c | 0x20u;
  const uint32_t code = ((low >> 1) ^ (low >> 2)) & 3u;
  return ("acgt"[code] == (char)low) ? code : 4u;
}

template <int WORDS>
__global__ __launch_bounds__(kWB) void k_windows_dense(const uint8_t* __restrict__ seq, uint64_t n_bytes,
                                                       uint64_t first, uint64_t n_win, int w, uint64_t m_lo,
                                                       uint64_t m_hi, uint64_t* __restrict__ rows,
                                                       uint64_t* __restrict__ valid) {
  const uint64_t t = (uint64_t)blockIdx.x * kWB + threadIdx.x;
  const uint64_t i0 = t * 64;  // this thread's first output row
  if (i0 >= n_win) return;
  const uint64_t p0 = first + i0;
  const uint64_t s = p0 + w >= 64 ? p0 + w - 64 : 0;  // F's oldest base for window p0
  const uint64_t end = min(n_bytes, p0 + 64 + (uint64_t)w - 1);
  const uint64_t last_row = min(n_win, i0 + 64);
  const int top = 2 * (w - 1);  // R's newest base
  uint64_t fl = 0, fh = 0, rl = 0, rh = 0, vbits = 0;
  int run = 0;
  for (uint64_t b = s; b < end; ++b) {
    const uint32_t c = win_code(seq[b]);
    if (c == 4u) {
      fl = fh = rl = rh = 0;
      run = 0;
    } else {
      fh = (fh << 2) | (fl >> 62);
      fl = (fl << 2) | c;
      rl = (rl >> 2) | (rh << 62);
      rh >>= 2;
      const uint64_t cc = (uint64_t)(c ^ 3u);
      if (top < 64) rl |= cc << top;
      else rh |= cc << (top - 64);
      run = min(run + 1, 64);
    }
    if (b + 1 < p0 + (uint64_t)w) continue;
    const uint64_t i = b + 1 - (uint64_t)w - first;  // window starting at b - w + 1
    if (i >= last_row) break;
    if (run < w) continue;
    vbits |= 1ull << (i - i0);
    const uint64_t fml = fl & m_lo, fmh = fh & m_hi, rml = rl & m_lo, rmh = rh & m_hi;
    const bool f_lt = fmh < rmh || (fmh == rmh && fml < rml);  // kmer_sliding.cpp:165
    uint64_t* o = rows + i * WORDS;
    o[0] = f_lt ? fl : rl;
    o[1] = f_lt ? fh : rh;
    o[2] = f_lt ? fml : rml;
    if (WORDS == 4) o[3] = f_lt ? fmh : rmh;
  }
  valid[t] = vbits;
}

}  // namespace

hipError_t launch_windows_dense(const uint8_t* seq, uint64_t n_bytes, uint64_t first, uint64_t n_win, int w,
                                uint64_t m_lo, uint64_t m_hi, uint64_t* rows, uint64_t* valid, hipStream_t s) {
  if (n_win == 0) return hipSuccess;
  const uint64_t threads = (n_win + 63) / 64;
  const dim3 grid((unsigned)((threads + kWB - 1) / kWB));
  if (w <= 32)
    hipLaunchKernelGGL(k_windows_dense<3>, grid, dim3(kWB), 0, s, seq, n_bytes, first, n_win, w, m_lo, m_hi, rows,
                       valid);
  else
    hipLaunchKernelGGL(k_windows_dense<4>, grid, dim3(kWB), 0, s, seq, n_bytes, first, n_win, w, m_lo, m_hi, rows,
                       valid);
  return hipGetLastError();
}

SKS_CODE_OBJECT_HOOK(windows)

}  // namespace sks
