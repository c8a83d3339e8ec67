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
// Passes (n = file bytes, L = lines):
//   1. count '\n'                                   (reduce, reads n bytes)
//   2. positions of '\n'                            (select, reads n bytes)
//   3. mark lines that contain ' '                  (reads n bytes)
//   4. per-line class / setter / event              (per line)
//   5. two last-non-zero scans                      (per line, u8)
//   6. per-line output length + push flag, scans    (per line)
//   7. copy kept bytes, 4 KiB input spans per group (reads n, writes <= n)
//   8. '\n' separators and record ends              (per line)
// Everything except pass 7 touches O(L) words; pass 7 is a streaming copy.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <rocprim/rocprim.hpp>

#include "sks_internal.hpp"

namespace sks {

namespace {

constexpr int kB = 256;
constexpr int kSpan = 4096;               // input bytes per copy work-group
constexpr int kSpanLines = kSpan + 1;     // lines a span can touch

// line class bits
constexpr uint8_t kH = 1, kE = 2, kSsp = 4, kNamed = 8;

struct IsNewline {
  __device__ bool operator()(uint8_t b) const { return b == '\n'; }
};
struct NewlineCount {
  __device__ uint64_t operator()(uint8_t b) const { return b == '\n'; }
};
struct LastNonZero {
  __host__ __device__ uint8_t operator()(uint8_t a, uint8_t b) const { return b ? b : a; }
};

// number of newline positions < i  (= index of the line holding byte i)
__device__ __forceinline__ uint64_t line_of(const uint64_t* nl, uint64_t n_nl, uint64_t i) {
  uint64_t lo = 0, hi = n_nl;
  while (lo < hi) {
    uint64_t mid = (lo + hi) >> 1;
    if (nl[mid] < i) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

__device__ __forceinline__ uint64_t line_start(const uint64_t* nl, uint64_t l) {
  return l ? nl[l - 1] + 1 : 0;
}
__device__ __forceinline__ uint64_t line_end(const uint64_t* nl, uint64_t n_nl, uint64_t n,
                                             uint64_t l) {
  return l < n_nl ? nl[l] : n;
}

// Pass 3: a ' ' byte marks its line (benign same-value races).
__global__ __launch_bounds__(kB) void k_spaces(const uint8_t* raw, uint64_t n, const uint64_t* nl,
                                               uint64_t n_nl, uint8_t* has_space) {
  const uint64_t stride = (uint64_t)gridDim.x * kB * 16;
  for (uint64_t b = ((uint64_t)blockIdx.x * kB + threadIdx.x) * 16; b < n; b += stride) {
    const uint64_t e = b + 16 < n ? b + 16 : n;
    for (uint64_t i = b; i < e; ++i)
      if (raw[i] == ' ') has_space[line_of(nl, n_nl, i)] = 1;
  }
}

// Pass 4
__global__ __launch_bounds__(kB) void k_classify(const uint8_t* raw, uint64_t n, const uint64_t* nl,
                                                 uint64_t n_nl, uint64_t L, const uint8_t* has_space,
                                                 uint8_t* cls, uint8_t* setter, uint8_t* ev_rev) {
  const uint64_t l = (uint64_t)blockIdx.x * kB + threadIdx.x;
  if (l >= L) return;
  const uint64_t st = line_start(nl, l), en = line_end(nl, n_nl, n, l);
  const uint64_t len = en - st;
  uint8_t c;
  if (len == 0) c = kE;
  else if (raw[st] == '>') c = kH | (len > 1 ? kNamed : 0);
  else c = has_space[l] ? kSsp : 0;
  cls[l] = c;
  setter[l] = (c & kH) ? ((c & kNamed) ? 2 : 1) : ((c & kSsp) ? 1 : 0);
  ev_rev[L - 1 - l] = (c & (kH | kE)) ? 1 : ((c & kSsp) ? 2 : 0);
}

// Pass 6: out_len = bytes line l contributes to the stream.
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
  kept[l] = keep;
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

// Pass 7: work-group per 4 KiB span of the input (spans are aligned in
// absolute address terms so every 16-byte load is aligned); the lines the span
// touches are staged in LDS, each thread moves 16 input bytes.
__global__ __launch_bounds__(kB) void k_copy(const uint8_t* raw, uint64_t n, uint32_t align,
                                             const uint64_t* nl, uint64_t n_nl,
                                             const uint8_t* kept, const uint64_t* out_off,
                                             uint8_t* out) {
  __shared__ int32_t s_start[kSpanLines];
  __shared__ uint64_t s_dst[kSpanLines];
  __shared__ uint64_t s_l[2];
  const uint64_t vbeg = (uint64_t)blockIdx.x * kSpan;
  const uint64_t ibeg = vbeg > align ? vbeg - align : 0;
  const uint64_t iend = std::min<uint64_t>(n, vbeg + kSpan - align);
  if (threadIdx.x < 2) s_l[threadIdx.x] = line_of(nl, n_nl, threadIdx.x ? iend - 1 : ibeg);
  __syncthreads();
  const uint64_t l0 = s_l[0];
  const int m = (int)(s_l[1] - l0 + 1);
  for (int j = threadIdx.x; j < m; j += kB) {
    const uint64_t l = l0 + j;
    const uint64_t st = line_start(nl, l);
    s_start[j] = st <= ibeg ? 0 : (int32_t)(st - ibeg);
    s_dst[j] = kept[l] ? out_off[l] - st : ~0ull;
  }
  __syncthreads();
  const uint64_t v0 = vbeg + (uint64_t)threadIdx.x * 16;  // virtual offset of this thread's block
  if (v0 + 16 <= align || v0 >= n + align) return;
  const uint4 q = *reinterpret_cast<const uint4*>(raw - align + v0);
  const uint32_t w[4] = {q.x, q.y, q.z, q.w};
  const uint64_t i0 = v0 > align ? v0 - align : 0;  // first valid byte
  const int32_t r0 = (int32_t)(i0 - ibeg);
  int lo = 0, hi = m - 1;  // last j with s_start[j] <= r0
  while (lo < hi) {
    int mid = (lo + hi + 1) >> 1;
    if (s_start[mid] <= r0) lo = mid;
    else hi = mid - 1;
  }
  int j = lo;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const uint64_t v = v0 + k;
    if (v < align || v >= n + align) continue;
    const uint64_t i = v - align;
    const int32_t r = (int32_t)(i - ibeg);
    while (j + 1 < m && s_start[j + 1] <= r) ++j;
    const uint8_t b = (uint8_t)(w[k >> 2] >> ((k & 3) * 8));
    const uint64_t d = s_dst[j];
    if (b != '\n' && d != ~0ull) out[d + i] = b;
  }
}

// Pass 8: separators and record ends.
__global__ __launch_bounds__(kB) void k_push(uint64_t L, const uint8_t* cls, const uint8_t* have_after,
                                             const uint64_t* out_off, const uint32_t* push_rank,
                                             const Summary* sum, uint8_t* out, uint64_t* rec_end) {
  const uint64_t l = (uint64_t)blockIdx.x * kB + threadIdx.x;
  if (l >= L) return;
  const bool before = l ? have_after[l - 1] == 2 : false;
  if ((cls[l] & (kH | kE)) && before) {
    out[out_off[l]] = '\n';
    if (rec_end) rec_end[push_rank[l]] = out_off[l];
  }
  if (l == L - 1 && sum->eof_push) {
    out[sum->total - 1] = '\n';
    if (rec_end) rec_end[sum->n_records - 1] = sum->total - 1;
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
#define SKS_CK(x)                     \
  do {                                \
    if ((e = (x)) != hipSuccess) return e; \
  } while (0)

  // pass 1: count newlines (the count sizes every per-line array)
  auto nl_count_it = rocprim::make_transform_iterator(raw, NewlineCount{});
  SKS_CK(work.reserve(256));
  uint64_t* d_cnt = reinterpret_cast<uint64_t*>(work.ptr);
  size_t need = 0;
  SKS_CK(rocprim::reduce(nullptr, need, nl_count_it, d_cnt, uint64_t(0), n, rocprim::plus<uint64_t>(), s));
  SKS_CK(tmp.reserve(need));
  SKS_CK(rocprim::reduce(tmp.ptr, need, nl_count_it, d_cnt, uint64_t(0), n, rocprim::plus<uint64_t>(), s));
  uint64_t n_nl = 0;
  uint8_t last = 0;
  SKS_CK(hipMemcpyAsync(&n_nl, d_cnt, sizeof n_nl, hipMemcpyDeviceToHost, s));
  SKS_CK(hipMemcpyAsync(&last, raw + n - 1, 1, hipMemcpyDeviceToHost, s));
  SKS_CK(hipStreamSynchronize(s));
  const uint64_t L = n_nl + (last != '\n');  // a trailing partial line is a line

  // per-line arrays, one allocation
  size_t o = 0;
  const size_t o_cnt = o;  o += align_up(sizeof(uint64_t));
  const size_t o_sum = o;  o += align_up(sizeof(Summary));
  const size_t o_nl = o;   o += align_up(n_nl * 8);
  const size_t o_sp = o;   o += align_up(L);
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
  SKS_CK(work.reserve(o));
  char* base = reinterpret_cast<char*>(work.ptr);
  d_cnt = reinterpret_cast<uint64_t*>(base + o_cnt);
  Summary* d_sum = reinterpret_cast<Summary*>(base + o_sum);
  uint64_t* nl = reinterpret_cast<uint64_t*>(base + o_nl);
  uint8_t* has_space = reinterpret_cast<uint8_t*>(base + o_sp);
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

  // pass 2: newline positions
  if (n_nl) {
    rocprim::counting_iterator<uint64_t> idx(0);
    need = 0;
    SKS_CK(rocprim::select(nullptr, need, idx, raw, nl, d_cnt, n, IsNewline{}, s));
    SKS_CK(tmp.reserve(need));
    SKS_CK(rocprim::select(tmp.ptr, need, idx, raw, nl, d_cnt, n, IsNewline{}, s));
  }
  // pass 3, 4
  SKS_CK(hipMemsetAsync(has_space, 0, L, s));
  {
    const uint64_t blocks = std::min<uint64_t>((n + kB * 16 - 1) / (kB * 16), 1u << 20);
    hipLaunchKernelGGL(k_spaces, dim3((unsigned)blocks), dim3(kB), 0, s, raw, n, nl, n_nl, has_space);
  }
  hipLaunchKernelGGL(k_classify, dim3(grid_for(L)), dim3(kB), 0, s, raw, n, nl, n_nl, L, has_space,
                     cls, setter, ev_rev);
  // pass 5
  need = 0;
  SKS_CK(rocprim::inclusive_scan(nullptr, need, setter, have_after, L, LastNonZero{}, s));
  SKS_CK(tmp.reserve(need));
  SKS_CK(rocprim::inclusive_scan(tmp.ptr, need, setter, have_after, L, LastNonZero{}, s));
  SKS_CK(rocprim::inclusive_scan(tmp.ptr, need, ev_rev, nxt_rev, L, LastNonZero{}, s));
  // pass 6
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
  SKS_CK(hipMemcpyAsync(&h, d_sum, sizeof h, hipMemcpyDeviceToHost, s));
  SKS_CK(hipStreamSynchronize(s));
  *out_bytes = h.total;
  *n_records = h.n_records;
  if (!out) return hipSuccess;  // size query
  if (h.total > out_cap || (rec_end && h.n_records > rec_cap)) {
    *too_small = true;
    return hipSuccess;
  }
  // pass 7, 8
  const uint32_t align = (uint32_t)(reinterpret_cast<uintptr_t>(raw) & 15);
  const uint64_t spans = (n + align + kSpan - 1) / kSpan;
  hipLaunchKernelGGL(k_copy, dim3((unsigned)spans), dim3(kB), 0, s, raw, n, align, nl, n_nl, kept,
                     out_off, out);
  hipLaunchKernelGGL(k_push, dim3(grid_for(L)), dim3(kB), 0, s, L, cls, have_after, out_off,
                     push_rank, d_sum, out, rec_end);
  return hipGetLastError();
#undef SKS_CK
}

}  // namespace sks
