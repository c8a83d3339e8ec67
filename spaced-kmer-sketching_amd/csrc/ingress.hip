// Device-side FASTA ingress: strings_from_fasta (reference
// fasta_processing.cpp:79-133) on the GPU, producing the same "record stream"
// as the host parser (fasta.cpp parse_fasta_bytes): each record's content
// followed by one '\n' separator.
//
// The host parser is a sequential state machine over lines.  Its state is one
// bit (have_name) plus the pending content, and both are determined by a few
// per-line facts, so the machine becomes line-parallel:
//
//   line class  H = starts with '>', E = empty, S = anything else,
//               Ssp = S containing ' '
//   have_name after line l  = value set by the last "setter" at or before l
//                             (H sets len > 1, Ssp sets false; others keep)
//                             -> an inclusive scan with "last non-zero wins"
//   a push (record end) happens at every H / E line with have_name set
//   before it, and at EOF when have_name is set at the end
//   an S line is part of a pushed record  <=>  have_name before it and the
//   next H / E / Ssp event after it is not Ssp (EOF counts as a push)
//                             -> the same scan over the reversed event list
//
// Passes (n = file bytes, L = lines; byte passes work on aligned 4 KiB spans):
//   1. newlines per span + exclusive scan           (reads n bytes)
//   2. newline positions, lines holding a ' '       (reads n bytes, writes 8 B/line)
//   3. per-line class / setter / event              (per line)
//   4. two last-non-zero scans                      (per line, u8)
//   5. per-line output length + push flag, scans    (per line)
//   6. stream bytes per span, assembled in LDS      (reads n, writes <= n)
//   7. record ends, EOF separator                   (per line)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <rocprim/rocprim.hpp>

#include "sks_internal.hpp"

namespace sks {

namespace {

constexpr int kB = 256;
constexpr int kSpan = kB * 16;            // input bytes per work-group (16 per thread)
constexpr int kSpanLines = kSpan + 1;     // lines a span can touch

// line class bits
constexpr uint8_t kH = 1, kE = 2, kSsp = 4, kNamed = 8;

struct LastNonZero {
  __host__ __device__ uint8_t operator()(uint8_t a, uint8_t b) const { return b ? b : a; }
};

// High bit of every zero byte of t, exactly (no borrow between bytes).
__device__ __forceinline__ uint32_t zero_bytes(uint32_t t) {
  const uint32_t y = (t & 0x7F7F7F7Fu) + 0x7F7F7F7Fu;
  return ~(y | t | 0x7F7F7F7Fu);
}

// 16-bit mask of the bytes of q equal to the byte replicated in c4.
__device__ __forceinline__ uint32_t byte_eq_mask(const uint4& q, uint32_t c4) {
  const uint32_t w[4] = {q.x, q.y, q.z, q.w};
  uint32_t m = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint32_t z = zero_bytes(w[i] ^ c4);
    m |= (((z >> 7) & 1u) | ((z >> 14) & 2u) | ((z >> 21) & 4u) | ((z >> 28) & 8u)) << (4 * i);
  }
  return m;
}

// Spans are aligned in absolute address terms: virtual offset v = i + align,
// span s = [s * kSpan, (s + 1) * kSpan), thread t holds v0 = s * kSpan + 16 t,
// so every load is one aligned uint4 (an aligned 16-byte block holding a
// valid byte never crosses a page).  Bytes outside [0, n) are masked off.
struct SpanThread {
  uint64_t v0;
  uint32_t valid;  // 16-bit mask of bytes inside [0, n)
  uint4 q;
};

__device__ __forceinline__ SpanThread span_load(const uint8_t* raw, uint64_t n, uint32_t align) {
  SpanThread t;
  t.v0 = (uint64_t)blockIdx.x * kSpan + threadIdx.x * 16u;
  const uint64_t end = n + align;
  uint32_t valid = 0xFFFFu;
  if (t.v0 < align) valid = align - t.v0 >= 16 ? 0u : (valid << (align - t.v0)) & 0xFFFFu;
  if (t.v0 + 16 > end) valid &= t.v0 >= end ? 0u : (0xFFFFu >> (t.v0 + 16 - end));
  t.valid = valid;
  t.q = valid ? *reinterpret_cast<const uint4*>(raw - align + t.v0) : make_uint4(0, 0, 0, 0);
  return t;
}

// Exclusive prefix sum over the work-group (s_tmp: one word per wave).
__device__ __forceinline__ uint32_t block_exclusive_sum(uint32_t v, uint32_t* s_tmp,
                                                        uint32_t* total) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t x = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(x, d, 64);
    if (lane >= d) x += y;
  }
  if (lane == 63) s_tmp[wave] = x;
  __syncthreads();
  uint32_t base = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < kB / 64; ++w) {
    const uint32_t t = s_tmp[w];
    base += w < wave ? t : 0u;
    tot += t;
  }
  *total = tot;
  return base + x - v;
}

__device__ __forceinline__ uint64_t line_start(const uint64_t* nl, uint64_t l) {
  return l ? nl[l - 1] + 1 : 0;
}
__device__ __forceinline__ uint64_t line_end(const uint64_t* nl, uint64_t n_nl, uint64_t n,
                                             uint64_t l) {
  return l < n_nl ? nl[l] : n;
}

// Pass 1: newlines per span.
__global__ __launch_bounds__(kB) void k_span_count(const uint8_t* raw, uint64_t n, uint32_t align,
                                                   uint32_t* span_nl) {
  __shared__ uint32_t s_tmp[kB / 64];
  const SpanThread t = span_load(raw, n, align);
  uint32_t total;
  (void)block_exclusive_sum(__popc(byte_eq_mask(t.q, 0x0A0A0A0Au) & t.valid), s_tmp, &total);
  if (threadIdx.x == 0) span_nl[blockIdx.x] = total;
}

// Pass 2: newline positions (in order), the lines holding a ' ', and the
// first byte of every line (fb[l]; '\n' for an empty line, 0 past EOF) so
// that pass 3 reads per-line bytes sequentially.  The line of a byte is the
// number of newlines before it: the span offset plus the block scan.
__global__ __launch_bounds__(kB) void k_span_lines(const uint8_t* raw, uint64_t n, uint32_t align,
                                                   const uint64_t* span_off, uint64_t* nl,
                                                   uint8_t* has_space, uint8_t* fb) {
  __shared__ uint32_t s_tmp[kB / 64];
  __shared__ uint4 s_bytes[kB + 1];
  const SpanThread t = span_load(raw, n, align);
  s_bytes[threadIdx.x] = t.q;
  if (threadIdx.x == 0) {
    // the 16 bytes after the span (for the first byte of a line starting there)
    const uint64_t v = (uint64_t)(blockIdx.x + 1) * kSpan;
    s_bytes[kB] = v < n + align ? *reinterpret_cast<const uint4*>(raw - align + v)
                                : make_uint4(0, 0, 0, 0);
  }
  uint32_t nlm = byte_eq_mask(t.q, 0x0A0A0A0Au) & t.valid;
  uint32_t spm = byte_eq_mask(t.q, 0x20202020u) & t.valid;
  uint32_t total;
  const uint64_t base = span_off[blockIdx.x] + block_exclusive_sum(__popc(nlm), s_tmp, &total);
  const uint64_t i0 = t.v0 - align;  // input index of byte 0 (when valid)
  if (blockIdx.x == 0 && threadIdx.x == 0) fb[0] = raw[0];
  while (spm) {
    const int b = __ffs(spm) - 1;
    spm &= spm - 1;
    has_space[base + __popc(nlm & ((1u << b) - 1))] = 1;
  }
  const uint8_t* sb = reinterpret_cast<const uint8_t*>(s_bytes);
  uint64_t r = base;
  while (nlm) {
    const int b = __ffs(nlm) - 1;
    nlm &= nlm - 1;
    const uint64_t p = i0 + b;
    nl[r] = p;
    fb[r + 1] = p + 1 < n ? sb[threadIdx.x * 16 + b + 1] : 0;
    ++r;
  }
}

// Pass 3
__global__ __launch_bounds__(kB) void k_classify(const uint8_t* fb, uint64_t n, const uint64_t* nl,
                                                 uint64_t n_nl, uint64_t L, const uint8_t* has_space,
                                                 uint8_t* cls, uint8_t* setter, uint8_t* ev_rev) {
  const uint64_t l = (uint64_t)blockIdx.x * kB + threadIdx.x;
  if (l >= L) return;
  const uint64_t st = line_start(nl, l), en = line_end(nl, n_nl, n, l);
  const uint64_t len = en - st;
  uint8_t c;
  if (len == 0) c = kE;
  else if (fb[l] == '>') c = kH | (len > 1 ? kNamed : 0);
  else c = has_space[l] ? kSsp : 0;
  cls[l] = c;
  setter[l] = (c & kH) ? ((c & kNamed) ? 2 : 1) : ((c & kSsp) ? 1 : 0);
  ev_rev[L - 1 - l] = (c & (kH | kE)) ? 1 : ((c & kSsp) ? 2 : 0);
}

// Pass 5: out_len = bytes line l contributes to the stream.
__global__ __launch_bounds__(kB) void k_out_len(const uint64_t* nl, uint64_t n_nl, uint64_t n,
                                                uint64_t L, const uint8_t* cls,
                                                const uint8_t* have_after, const uint8_t* nxt_rev,
                                                uint64_t* out_len, uint32_t* push_cnt, uint8_t* kept) {
  const uint64_t l = (uint64_t)blockIdx.x * kB + threadIdx.x;
  if (l >= L) return;
  const uint8_t c = cls[l];
  const bool before = l ? have_after[l - 1] == 2 : false;
  const uint8_t next = l + 1 < L ? nxt_rev[L - 2 - l] : 0;  // 0: only plain S lines up to EOF
  const bool is_s = (c & (kH | kE | kSsp)) == 0;
  const bool keep = is_s && before && next != 2;
  const bool push = (c & (kH | kE)) && before;
  const uint64_t len = line_end(nl, n_nl, n, l) - line_start(nl, l);
  out_len[l] = keep ? len : (uint64_t)push;
  push_cnt[l] = push;
  kept[l] = keep ? 1 : (push ? 2 : 0);
}

struct Summary {
  uint64_t total;      // stream bytes
  uint64_t n_records;
  uint64_t eof_push;
};

__global__ void k_summary(uint64_t L, const uint64_t* out_off, const uint64_t* out_len,
                          const uint32_t* push_rank, const uint32_t* push_cnt,
                          const uint8_t* have_after, Summary* s) {
  if (L == 0) {
    s->total = s->n_records = s->eof_push = 0;
    return;
  }
  const uint64_t eof = have_after[L - 1] == 2;
  s->eof_push = eof;
  s->total = out_off[L - 1] + out_len[L - 1] + eof;
  s->n_records = (uint64_t)push_rank[L - 1] + push_cnt[L - 1] + eof;
}

// Pass 6a (per line, after the scans): dst[l] maps line l's input bytes to
// stream positions (kept line: stream = dst + i) or holds the separator's
// stream position (push line).  Also record ends and the EOF separator.
__global__ __launch_bounds__(kB) void k_line_dst(uint64_t L, const uint64_t* nl, const uint8_t* kept,
                                                 const uint64_t* out_off, const uint32_t* push_rank,
                                                 const Summary* sum, uint64_t* dst, uint8_t* out,
                                                 uint64_t* rec_end) {
  const uint64_t l = (uint64_t)blockIdx.x * kB + threadIdx.x;
  if (l >= L) return;
  const uint8_t ty = kept[l];
  dst[l] = ty == 1 ? out_off[l] - line_start(nl, l) : out_off[l];
  if (rec_end && ty == 2) rec_end[push_rank[l]] = out_off[l];
  if (l == L - 1 && sum->eof_push) {
    out[sum->total - 1] = '\n';
    if (rec_end) rec_end[sum->n_records - 1] = sum->total - 1;
  }
}

// Pass 6b (per span): span_out[s] = stream bytes produced by the input before
// span s (a push line's separator counts at its first byte);
// span_out[spans] = the stream without the EOF separator.
__global__ __launch_bounds__(kB) void k_span_out(uint64_t spans, uint64_t n, uint32_t align,
                                                 const uint64_t* span_off, const uint64_t* nl,
                                                 const uint8_t* kept, const uint64_t* out_off,
                                                 const uint64_t* out_len, const Summary* sum,
                                                 uint64_t* span_out) {
  const uint64_t sp = (uint64_t)blockIdx.x * kB + threadIdx.x;
  if (sp > spans) return;
  if (sp == spans) {
    span_out[sp] = sum->total - sum->eof_push;
    return;
  }
  const uint64_t v = sp * kSpan;
  const uint64_t i = v > align ? v - align : 0;
  const uint64_t l = span_off[sp];  // line of byte i
  const uint64_t st = line_start(nl, l);
  span_out[sp] = out_off[l] + (kept[l] == 1 ? i - st : (st < i ? out_len[l] : 0));
}

// Pass 6c: the stream bytes of one 4 KiB input span, [span_out[s],
// span_out[s + 1]), are assembled in LDS — kept bytes by position, separators
// whose stream position falls in the range — and written with aligned 16-byte
// stores (byte stores only at the two ends).  All per-line inputs are
// precomputed so a work-group waits on one round of loads.
__global__ __launch_bounds__(kB) void k_copy(const uint8_t* raw, uint64_t n, uint32_t align,
                                             const uint64_t* span_off, const uint64_t* span_out,
                                             uint64_t L, const uint8_t* kept, const uint64_t* dst,
                                             uint8_t* out) {
  __shared__ int32_t s_rel[kSpanLines];
  __shared__ uint32_t s_out[kSpan / 4 + 8];
  __shared__ uint32_t s_tmp[kB / 64];
  const SpanThread t = span_load(raw, n, align);
  const uint64_t l0 = span_off[blockIdx.x];  // line of the span's first byte
  const uint64_t o0 = span_out[blockIdx.x], o1 = span_out[blockIdx.x + 1];
  const uint64_t vbeg = (uint64_t)blockIdx.x * kSpan;
  const uint64_t ibeg = vbeg > align ? vbeg - align : 0;
  const uint32_t nlm = byte_eq_mask(t.q, 0x0A0A0A0Au) & t.valid;
  uint32_t total;
  uint32_t j = block_exclusive_sum(__popc(nlm), s_tmp, &total);
  uint8_t* so = reinterpret_cast<uint8_t*>(s_out);
  for (uint32_t q = threadIdx.x; q <= total; q += kB) {
    const uint64_t l = l0 + q;
    int32_t rel = INT32_MIN;
    if (l < L) {
      const uint8_t ty = kept[l];
      const uint64_t d = dst[l];
      if (ty == 1) rel = (int32_t)(int64_t)(d + ibeg - o0);
      else if (ty == 2 && d >= o0 && d < o1) so[d - o0] = '\n';
    }
    s_rel[q] = rel;
  }
  __syncthreads();
  if (t.valid) {
    const uint32_t w[4] = {t.q.x, t.q.y, t.q.z, t.q.w};
    const int32_t r0 = (int32_t)(int64_t)(t.v0 - align - ibeg);  // byte 0 relative to ibeg
    int32_t rel = s_rel[j];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      if (!((t.valid >> k) & 1u)) continue;
      const uint8_t ch = (uint8_t)(w[k >> 2] >> ((k & 3) * 8));
      if (ch == '\n') rel = s_rel[++j];
      else if (rel != INT32_MIN) so[rel + r0 + k] = ch;
    }
  }
  __syncthreads();
  if (o1 <= o0) return;
  const uintptr_t a0 = reinterpret_cast<uintptr_t>(out + o0);
  const uintptr_t a1 = reinterpret_cast<uintptr_t>(out + o1);
  const uintptr_t blk0 = a0 & ~uintptr_t(15);
  const uint32_t n_blk = (uint32_t)((((a1 + 15) & ~uintptr_t(15)) - blk0) / 16);
  for (uint32_t bi = threadIdx.x; bi < n_blk; bi += kB) {
    const uintptr_t ba = blk0 + (uintptr_t)bi * 16;
    const int64_t r = (int64_t)ba - (int64_t)a0;  // LDS offset of the block's first byte
    if (ba >= a0 && ba + 16 <= a1) {
      const uint32_t wi = (uint32_t)r >> 2, sh = (uint32_t)r & 3;
      uint32_t x[5];
#pragma unroll
      for (int k = 0; k < 5; ++k) x[k] = s_out[wi + k];
      uint4 v;
      v.x = __builtin_amdgcn_alignbyte(x[1], x[0], sh);
      v.y = __builtin_amdgcn_alignbyte(x[2], x[1], sh);
      v.z = __builtin_amdgcn_alignbyte(x[3], x[2], sh);
      v.w = __builtin_amdgcn_alignbyte(x[4], x[3], sh);
      *reinterpret_cast<uint4*>(ba) = v;
    } else {
      for (int k = 0; k < 16; ++k) {
        const uintptr_t a = ba + k;
        if (a >= a0 && a < a1) *reinterpret_cast<uint8_t*>(a) = so[r + k];
      }
    }
  }
}

unsigned grid_for(uint64_t n) { return (unsigned)std::max<uint64_t>(1, (n + kB - 1) / kB); }

size_t align_up(size_t x) { return (x + 255) & ~size_t(255); }

}  // namespace

hipError_t fasta_parse_device(const uint8_t* raw, uint64_t n, uint8_t* out, uint64_t out_cap,
                              uint64_t* rec_end, uint64_t rec_cap, Scratch& work, Scratch& tmp,
                              hipStream_t s, uint64_t* out_bytes, uint64_t* n_records,
                              bool* too_small) {
  *too_small = false;
  *out_bytes = *n_records = 0;
  if (n == 0) return hipSuccess;
  hipError_t e;
#define SKS_CK(x)                          \
  do {                                     \
    if ((e = (x)) != hipSuccess) return e; \
  } while (0)

  const uint32_t align = (uint32_t)(reinterpret_cast<uintptr_t>(raw) & 15);
  const uint64_t spans = (n + align + kSpan - 1) / kSpan;
  if (spans >= (1ull << 31)) return hipErrorInvalidValue;

  // pass 1: newlines per span and their exclusive scan (sizes every per-line array)
  const size_t o_snl = 0;
  const size_t o_soff = o_snl + align_up((spans + 1) * 4);
  const size_t o_sum = o_soff + align_up((spans + 1) * 8);
  const size_t o_lines = o_sum + align_up(sizeof(Summary));
  SKS_CK(work.reserve(o_lines));
  uint32_t* span_nl = reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(work.ptr) + o_snl);
  uint64_t* span_off = reinterpret_cast<uint64_t*>(reinterpret_cast<char*>(work.ptr) + o_soff);
  SKS_CK(hipMemsetAsync(span_nl + spans, 0, 4, s));  // the scan's extra element: total
  hipLaunchKernelGGL(k_span_count, dim3((unsigned)spans), dim3(kB), 0, s, raw, n, align, span_nl);
  size_t need = 0;
  SKS_CK(rocprim::exclusive_scan(nullptr, need, span_nl, span_off, uint64_t(0), spans + 1,
                                 rocprim::plus<uint64_t>(), s));
  SKS_CK(tmp.reserve(need));
  SKS_CK(rocprim::exclusive_scan(tmp.ptr, need, span_nl, span_off, uint64_t(0), spans + 1,
                                 rocprim::plus<uint64_t>(), s));
  uint64_t n_nl = 0;
  uint8_t last = 0;
  SKS_CK(pinned_d2h(&n_nl, span_off + spans, sizeof n_nl, s));
  SKS_CK(pinned_d2h(&last, raw + n - 1, 1, s));
  const uint64_t L = n_nl + (last != '\n');  // a trailing partial line is a line
  if (L >= (1ull << 32)) return hipErrorInvalidValue;  // push ranks are u32

  // per-line arrays after the span arrays, one allocation (grown in place:
  // Scratch::reserve reallocates, so take pointers afterwards)
  size_t o = o_lines;
  const size_t o_nl = o;   o += align_up(n_nl * 8);
  const size_t o_sp = o;   o += align_up(L);
  const size_t o_fb = o;   o += align_up(L + 1);
  const size_t o_cls = o;  o += align_up(L);
  const size_t o_set = o;  o += align_up(L);
  const size_t o_hav = o;  o += align_up(L);
  const size_t o_evr = o;  o += align_up(L);
  const size_t o_nxr = o;  o += align_up(L);
  const size_t o_kep = o;  o += align_up(L);
  const size_t o_len = o;  o += align_up(L * 8);
  const size_t o_off = o;  o += align_up(L * 8);
  const size_t o_pc = o;   o += align_up(L * 4);
  const size_t o_pr = o;   o += align_up(L * 4);
  const size_t o_dst = o;  o += align_up(L * 8);
  const size_t o_spo = o;  o += align_up((spans + 1) * 8);
  if (o > work.bytes) {
    // keep the span offsets across the reallocation
    Scratch grown;
    grown.owner = work.owner;
    SKS_CK(grown.reserve(o));
    SKS_CK(hipMemcpyAsync(grown.ptr, work.ptr, o_lines, hipMemcpyDeviceToDevice, s));
    SKS_CK(hipStreamSynchronize(s));
    work.release();
    work = grown;
  }
  char* base = reinterpret_cast<char*>(work.ptr);
  span_off = reinterpret_cast<uint64_t*>(base + o_soff);
  Summary* d_sum = reinterpret_cast<Summary*>(base + o_sum);
  uint64_t* nl = reinterpret_cast<uint64_t*>(base + o_nl);
  uint8_t* has_space = reinterpret_cast<uint8_t*>(base + o_sp);
  uint8_t* fb = reinterpret_cast<uint8_t*>(base + o_fb);
  uint8_t* cls = reinterpret_cast<uint8_t*>(base + o_cls);
  uint8_t* setter = reinterpret_cast<uint8_t*>(base + o_set);
  uint8_t* have_after = reinterpret_cast<uint8_t*>(base + o_hav);
  uint8_t* ev_rev = reinterpret_cast<uint8_t*>(base + o_evr);
  uint8_t* nxt_rev = reinterpret_cast<uint8_t*>(base + o_nxr);
  uint8_t* kept = reinterpret_cast<uint8_t*>(base + o_kep);
  uint64_t* out_len = reinterpret_cast<uint64_t*>(base + o_len);
  uint64_t* out_off = reinterpret_cast<uint64_t*>(base + o_off);
  uint32_t* push_cnt = reinterpret_cast<uint32_t*>(base + o_pc);
  uint32_t* push_rank = reinterpret_cast<uint32_t*>(base + o_pr);
  uint64_t* dst = reinterpret_cast<uint64_t*>(base + o_dst);
  uint64_t* span_out = reinterpret_cast<uint64_t*>(base + o_spo);

  // pass 2, 3
  SKS_CK(hipMemsetAsync(has_space, 0, L, s));
  hipLaunchKernelGGL(k_span_lines, dim3((unsigned)spans), dim3(kB), 0, s, raw, n, align, span_off,
                     nl, has_space, fb);
  hipLaunchKernelGGL(k_classify, dim3(grid_for(L)), dim3(kB), 0, s, fb, n, nl, n_nl, L, has_space,
                     cls, setter, ev_rev);
  // pass 4
  need = 0;
  SKS_CK(rocprim::inclusive_scan(nullptr, need, setter, have_after, L, LastNonZero{}, s));
  SKS_CK(tmp.reserve(need));
  SKS_CK(rocprim::inclusive_scan(tmp.ptr, need, setter, have_after, L, LastNonZero{}, s));
  SKS_CK(rocprim::inclusive_scan(tmp.ptr, need, ev_rev, nxt_rev, L, LastNonZero{}, s));
  // pass 5
  hipLaunchKernelGGL(k_out_len, dim3(grid_for(L)), dim3(kB), 0, s, nl, n_nl, n, L, cls, have_after,
                     nxt_rev, out_len, push_cnt, kept);
  need = 0;
  size_t need2 = 0;
  SKS_CK(rocprim::exclusive_scan(nullptr, need, out_len, out_off, uint64_t(0), L,
                                 rocprim::plus<uint64_t>(), s));
  SKS_CK(rocprim::exclusive_scan(nullptr, need2, push_cnt, push_rank, uint32_t(0), L,
                                 rocprim::plus<uint32_t>(), s));
  SKS_CK(tmp.reserve(std::max(need, need2)));
  SKS_CK(rocprim::exclusive_scan(tmp.ptr, need, out_len, out_off, uint64_t(0), L,
                                 rocprim::plus<uint64_t>(), s));
  SKS_CK(rocprim::exclusive_scan(tmp.ptr, need2, push_cnt, push_rank, uint32_t(0), L,
                                 rocprim::plus<uint32_t>(), s));
  hipLaunchKernelGGL(k_summary, dim3(1), dim3(1), 0, s, L, out_off, out_len, push_rank, push_cnt,
                     have_after, d_sum);
  Summary h{};
  SKS_CK(pinned_d2h(&h, d_sum, sizeof h, s));
  *out_bytes = h.total;
  *n_records = h.n_records;
  if (!out) return hipSuccess;  // size query
  if (h.total > out_cap || (rec_end && h.n_records > rec_cap)) {
    *too_small = true;
    return hipSuccess;
  }
  // pass 6: per-line stream mapping, per-span stream offsets, span copy
  hipLaunchKernelGGL(k_line_dst, dim3(grid_for(L)), dim3(kB), 0, s, L, nl, kept, out_off, push_rank,
                     d_sum, dst, out, rec_end);
  hipLaunchKernelGGL(k_span_out, dim3(grid_for(spans + 1)), dim3(kB), 0, s, spans, n, align, span_off,
                     nl, kept, out_off, out_len, d_sum, span_out);
  hipLaunchKernelGGL(k_copy, dim3((unsigned)spans), dim3(kB), 0, s, raw, n, align, span_off, span_out,
                     L, kept, dst, out);
  return hipGetLastError();
#undef SKS_CK
}

SKS_CODE_OBJECT_HOOK(ingress)

}  // namespace sks
