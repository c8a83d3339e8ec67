// Kernel 2 (default from round 3) — all-pairs intersection straight from the
// sorted sketches ("range join").
//
// The reference counts |A ∩ B| by probing the larger hash map for every
// element of the smaller set (kmer_set.cpp:23-41), one pair per cilk_for
// iteration (kmer_set.cpp:167-184).  As in k_join (intersect.hip), the n x n
// matrix is cut into 64 x 64 tiles of (row block, column block) and a
// workgroup joins the two blocks in an LDS hash table: the column elements of
// a chunk go into a fingerprint table (value -> 64-bit mask of the columns
// holding it), every row element probes once, and a hit with mask m adds m to
// the row's bit-sliced counters (a carry chain of LDS atomic XORs).
//
// What differs is the input.  k_join reads a hash-bucketed, block-major copy
// of the sketches that six launches build per call (counts, column sums, scan,
// offsets, staging, placement: ~0.2 ms for config 4).  Here the sketches are
// read where they lie: the value range is cut into B buckets by common bounds,
// and since every sketch is sorted, sketch i's part of bucket b is the
// contiguous range [pos[i][b], pos[i][b + 1]).  A chunk (whole buckets [bs, be)
// of the column block holding <= cap elements, or a slice of one larger bucket)
// is 64 contiguous ranges, one per column sketch, concatenated in sketch order;
// the row elements of [bs, be) are 64 contiguous ranges too, and a row
// element's row is the range it came from (no id array).  The whole "layout"
// is bounds (B + 1 u64), pos (n x (B + 1) u32) and each column block's bucket
// starts pre[blk][b] = sum over its sketches of pos[i][b]: three small launches.
//
// Thread map for the ranges: thread t serves sketch s = t / 8 of the block,
// lane k = t % 8 takes elements k, k + 8, ... of its range, so each wave reads
// 8 sketches' ranges as 64-byte runs.  Loads run ahead of their use: waves
// 0-1 read the bucket positions of the chunk after the next one into
// registers, and every thread its first two column and row elements of the
// next chunk, while the current chunk is inserted and probed; the ranges are
// double-buffered in LDS.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>

#include "join_common.hpp"
#include "sks_internal.hpp"

namespace sks {

namespace {

using jc::fp_slot;
using jc::fp_tag;
using jc::join_chain;
using jc::kFFree;
using jc::kFSlots;
using jc::sym_tile;

constexpr int kRB = 512;              // threads per workgroup (8 waves)
constexpr int kTile = 64;
constexpr int kRCap = 1024;           // column elements per chunk (entry index: 10 bits)
constexpr int kRWin = 256;            // bucket starts staged per window
constexpr int kPlanes = 32;           // bit-sliced counter planes (any int32 count)
constexpr uint32_t kNoSlot = 0xFFFFFFFFu;
constexpr int kPB = 256;              // threads of the prefix kernel
constexpr uint64_t kMaxGrid = 1ull << 22;
static_assert(kRCap == 1024, "entry index: 10 bits; join_chain reads entry x & 1023 of any slot word");

// pre[blk * (B + 1) + b] = sum of pos[i * (B + 1) + b] over the block's sketches
__global__ __launch_bounds__(kPB) void k_rj_prefix(const uint32_t* __restrict__ pos, uint32_t n,
                                                    uint32_t B, uint32_t* __restrict__ pre) {
  const uint64_t B1 = B + 1;
  const uint64_t idx = (uint64_t)blockIdx.x * kPB + threadIdx.x;
  const uint32_t n_blk = (n + kTile - 1) / kTile;
  if (idx >= (uint64_t)n_blk * B1) return;
  const uint32_t blk = (uint32_t)(idx / B1), b = (uint32_t)(idx % B1);
  const uint32_t i0 = blk * kTile, i1 = min(n, i0 + kTile);
  uint32_t t = 0;
  for (uint32_t i = i0; i < i1; ++i) t += pos[i * B1 + b];
  pre[idx] = t;
}

// Common bucket bounds: bounds[b] = mean over up to 64 sample sketches (spread
// over the set) of each one's b/B quantile (intersect.hip k_bounds' rule),
// one wave per bound so the samples are read in parallel.  Any non-decreasing
// bounds give exact counts: each sample's quantiles are non-decreasing in b,
// and the same reduction tree for every b keeps the rounded means so.
__global__ __launch_bounds__(kPB) void k_rj_bounds(const uint64_t* __restrict__ data,
                                                    const uint64_t* __restrict__ starts,
                                                    const uint32_t* __restrict__ sizes, uint32_t n,
                                                    uint32_t B, uint64_t* __restrict__ bounds) {
  const uint32_t b = blockIdx.x * (kPB / 64) + (threadIdx.x >> 6);
  const uint32_t lane = threadIdx.x & 63;
  if (b > B) return;
  const uint32_t K = min(n, 64u);
  double x = 0.0, used = 0.0;
  if (lane < K && b > 0 && b < B) {
    const uint32_t i = (uint32_t)((uint64_t)lane * n / K);
    const uint32_t sz = sizes[i];
    if (sz) {
      x = (double)data[starts[i] + (uint64_t)b * sz / B];
      used = 1.0;
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    x += __shfl_xor(x, o, 64);
    used += __shfl_xor(used, o, 64);
  }
  if (lane) return;
  if (b == 0) { bounds[0] = 0; return; }
  if (b == B) { bounds[B] = ~0ull; return; }
  const double m = used > 0.0 ? x / used : 0.0;
  bounds[b] = m >= 18446744073709549568.0 ? ~0ull : (uint64_t)m;
}

// pos[i][b] = first element of sketch i >= bounds[b] (pos[i][B] = size): one
// workgroup per sketch, rounds of kPB x kPosItems consecutive elements (thread
// t takes elements kPosItems t .. of the round, all loaded before any is
// used).  An element's bucket is the largest b < B with bounds[b] <= v: a
// binary search over the bounds (LDS when they fit) for the thread's first
// element, then a forward walk (the sketch is sorted).  Element e fills
// pos[b] = e for the buckets after its predecessor's, up to its own.
// O(size + B) per sketch instead of (B + 1) binary searches of it.
constexpr int kPosItems = 8;
template <bool LDS_BOUNDS>
__global__ __launch_bounds__(kPB) void k_rj_pos(const uint64_t* __restrict__ data,
                                                 const uint64_t* __restrict__ starts,
                                                 const uint32_t* __restrict__ sizes, uint32_t B,
                                                 const uint64_t* __restrict__ g_bounds,
                                                 uint32_t* __restrict__ pos) {
  extern __shared__ uint64_t s_bnd[];
  __shared__ uint32_t s_last[kPB];  // bucket of each thread's last element this round
  __shared__ uint32_t s_carry;
  const uint32_t i = blockIdx.x, tid = threadIdx.x;
  const uint32_t sz = sizes[i];
  const uint64_t* S = data + starts[i];
  uint32_t* P = pos + (uint64_t)i * (B + 1);
  const uint64_t* bnd = g_bounds;
  if constexpr (LDS_BOUNDS) {
    for (uint32_t b = tid; b <= B; b += kPB) s_bnd[b] = g_bounds[b];
    bnd = s_bnd;
  }
  if (tid == 0) s_carry = 0xFFFFFFFFu;  // bucket of the element before the round (~0: none)
  __syncthreads();
  constexpr uint32_t kRound = kPB * kPosItems;
  for (uint32_t e0 = 0; e0 < sz; e0 += kRound) {
    const uint32_t eb = e0 + tid * kPosItems;
    const uint32_t n_mine = eb < sz ? min((uint32_t)kPosItems, sz - eb) : 0;
    uint64_t v[kPosItems];
#pragma unroll
    for (int u = 0; u < kPosItems; ++u) v[u] = (uint32_t)u < n_mine ? S[eb + u] : 0;
    uint32_t bk[kPosItems];
    uint32_t cur = 0;
    if (n_mine) {
      uint32_t lo = 0, hi = B - 1;
      while (lo < hi) {
        const uint32_t mid = (lo + hi + 1) >> 1;
        if (bnd[mid] <= v[0]) lo = mid; else hi = mid - 1;
      }
      cur = lo;
    }
#pragma unroll
    for (int u = 0; u < kPosItems; ++u) {
      if ((uint32_t)u < n_mine)
        while (cur + 1 < B && bnd[cur + 1] <= v[u]) ++cur;
      bk[u] = cur;
    }
    s_last[tid] = n_mine ? bk[n_mine - 1] : 0xFFFFFFFFu;
    __syncthreads();
    if (n_mine) {
      uint32_t prev = tid ? s_last[tid - 1] : s_carry;
#pragma unroll
      for (int u = 0; u < kPosItems; ++u) {
        if ((uint32_t)u >= n_mine) break;
        for (uint32_t b = prev + 1; b <= bk[u]; ++b) P[b] = eb + u;  // prev = ~0: from bucket 0
        prev = bk[u];
      }
    }
    __syncthreads();
    if (tid == 0) s_carry = s_last[(min(kRound, sz - e0) - 1) / kPosItems];
    __syncthreads();
  }
  const uint32_t last = s_carry;  // bucket of the last element (~0: empty sketch)
  for (uint32_t b = tid; b <= B; b += kPB)
    if (last == 0xFFFFFFFFu || b > last) P[b] = sz;
}

// One thread's share of a chunk, read from the LDS ranges once: column
// elements at chunk-order positions x = clo, clo + 8, ... < chi, element x at
// data[csrc + x]; row elements at data[j], j = rlo, rlo + 8, ... < rhi; and the
// first two of each, loaded ahead.
struct ChunkRegs {
  uint32_t clo, chi, csrc, rlo, rhi;
  uint64_t c[2], r[2];
};

// inclusive prefix sum over the 64 lanes of a wave (DPP row shifts, then the
// row broadcasts of lanes 15 and 31; no LDS)
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false);  // row_shr:1
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false);  // row_shr:2
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false);  // row_shr:4
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false);  // row_shr:8
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);  // row_bcast:15
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);  // row_bcast:31
  return v;
}

struct RJoinArgs {
  const uint64_t* data;
  const uint64_t* starts;
  const uint32_t* pos;   // [n][B + 1]
  const uint32_t* cpre;  // [n_cb][B + 1] column block bucket starts
  uint32_t B, n, n_col_blocks, n_groups, buckets_per_group;
  int sym;
  uint32_t row_begin, row_end;
  uint64_t tile_begin;
  const uint32_t* tiles;  // optional (I, J) list, global block indices, sym semantics
  int32_t* out;
  uint64_t ld;
  uint32_t cap;  // column elements per chunk (<= kRCap)
  int packed;    // out = [tile - tile_begin][64][64]
};

// 6 waves per SIMD: three workgroups per CU, as the LDS allows (<= 80 VGPRs)
__global__ __launch_bounds__(kRB, 6) void k_rjoin(RJoinArgs a) {
  __shared__ uint32_t s_slot[kFSlots];
  __shared__ ulonglong2 s_ent[kRCap];                    // {value, mask of the columns holding it}
  __shared__ unsigned long long s_pl[kPlanes * kTile];  // plane b of row r at [b * 64 + r]
  __shared__ uint32_t s_coff[kRWin + 1];
  __shared__ uint16_t s_next[kRWin];
  // chunk ranges, double-buffered: column sketch s starts at element s_cb, its
  // elements are [s_cp[s], s_cp[s + 1]) of the chunk's concatenated order; row
  // sketch s is [s_rb, s_re)
  __shared__ uint32_t s_cb[2][kTile], s_cp[2][kTile + 1], s_rb[2][kTile], s_re[2][kTile];
  __shared__ uint32_t s_self[kTile];
  __shared__ uint32_t s_top;

  const uint64_t t = a.tile_begin + blockIdx.x / a.n_groups;
  const uint32_t grp = blockIdx.x % a.n_groups;
  uint32_t I, J;
  if (a.tiles) {
    I = a.tiles[2 * t];
    J = a.tiles[2 * t + 1];
  } else if (a.sym) {
    sym_tile(t, a.n_col_blocks, I, J);
  } else {
    I = (uint32_t)(t / a.n_col_blocks);
    J = (uint32_t)(t % a.n_col_blocks);
  }
  const bool rows_mode = !a.sym && !a.tiles;
  const uint32_t row0 = (rows_mode ? a.row_begin : 0) + I * kTile;
  const uint32_t row_lim = rows_mode ? a.row_end : a.n;
  const uint32_t col0 = J * kTile;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint32_t r_valid = min<uint32_t>(kTile, row_lim - row0);
  const uint32_t c_valid = min<uint32_t>(kTile, a.n - col0);
  const uint64_t B1 = a.B + 1;
  const uint32_t* coff = a.cpre + (uint64_t)J * B1;
  // a tile on the diagonal: its rows are its columns
  const bool self_tile = row0 == col0;

  // waves 0 / 1: lane s holds column / row sketch s's start and positions row
  bool my_ok = false;
  uint32_t my_st = 0;
  const uint32_t* my_pos = a.pos;
  if (wave < 2) {
    const uint32_t i = wave == 0 ? col0 + lane : row0 + lane;
    my_ok = (uint32_t)lane < (wave == 0 ? c_valid : r_valid);
    if (my_ok) {
      my_st = (uint32_t)a.starts[i];
      my_pos = a.pos + (uint64_t)i * B1;
    }
  }
  // a chunk's ranges: waves 0-1 read pos[bs], pos[be] of their sketch into
  // registers (pos_load) one chunk before they store them (store_ranges)
  auto pos_load = [&](uint32_t bs, uint32_t be, uint32_t& pb, uint32_t& pe) {
    pb = pe = 0;
    if (my_ok) {
      pb = my_pos[bs];
      pe = my_pos[be];
    }
  };
  auto store_ranges = [&](int buf, uint32_t pb, uint32_t pe) {  // waves 0-1, all lanes
    if (wave == 0) {
      const uint32_t c = pe - pb;
      const uint32_t incl = wave_incl_scan(c);
      s_cb[buf][lane] = my_st + pb;
      s_cp[buf][lane] = incl - c;
      if (lane == 63) s_cp[buf][kTile] = incl;
    } else {
      s_rb[buf][lane] = my_st + pb;
      s_re[buf][lane] = my_st + pe;
    }
  };

  for (int i = tid; i < kFSlots / 4; i += kRB)
    reinterpret_cast<uint4*>(s_slot)[i] = make_uint4(kFFree, kFFree, kFFree, kFFree);
  for (int i = tid; i < kPlanes * kTile / 2; i += kRB) reinterpret_cast<uint4*>(s_pl)[i] = make_uint4(0, 0, 0, 0);
  if (tid < kTile) s_self[tid] = 0;
  if (tid == 0) s_top = 0;
  uint32_t top = 0;
  auto add_hits = [&](uint32_t r, unsigned long long m) {
    if (self_tile && ((m >> r) & 1ull)) {  // (a slice of a large bucket may not hold it)
      atomicAdd(&s_self[r], 1u);
      m &= ~(1ull << r);
    }
    unsigned long long* p = &s_pl[r];
    uint32_t b = 0;
    for (; m && b < kPlanes; ++b) m &= atomicXor(p + b * kTile, m);
    top = max(top, b);
  };
  auto lookup = [&](uint64_t v, uint32_t h, uint32_t x) -> unsigned long long {
    if (x != kFFree) x = join_chain(x, h, fp_tag(v), v, 0u, s_slot, s_ent, false);
    return x == kFFree ? 0ull : s_ent[x & 1023u].y;
  };

  const int rs_s = tid >> 3, rs_k = tid & 7;  // range map: sketch, lane within it
  // this thread's share of a chunk (chunk order [c0, c1)) from the ranges in
  // buffer `rb`, with its first two column and row elements
  auto fetch_first = [&](int rb, uint32_t c0, uint32_t c1, bool rows, ChunkRegs& o) {
    o.clo = o.chi = o.rlo = o.rhi = 0;
    o.csrc = 0;
    o.c[0] = o.c[1] = o.r[0] = o.r[1] = 0;
    if ((uint32_t)rs_s < c_valid) {
      const uint32_t p0 = s_cp[rb][rs_s], p1 = s_cp[rb][rs_s + 1];
      o.clo = max(p0, c0) + rs_k;
      o.chi = min(p1, c1);
      o.csrc = s_cb[rb][rs_s] - p0;
      if (o.clo < o.chi) o.c[0] = a.data[o.csrc + o.clo];
      if (o.clo + 8 < o.chi) o.c[1] = a.data[o.csrc + o.clo + 8];
      o.clo -= c0;  // chunk-relative: the entry index of the first element
      o.chi = o.chi > c0 ? o.chi - c0 : 0;
      o.csrc += c0;
    }
    if (rows && (uint32_t)rs_s < r_valid) {
      o.rlo = s_rb[rb][rs_s] + rs_k;
      o.rhi = s_re[rb][rs_s];
      if (o.rlo < o.rhi) o.r[0] = a.data[o.rlo];
      if (o.rlo + 8 < o.rhi) o.r[1] = a.data[o.rlo + 8];
    }
  };
  // insert value v as entry e of column rs_s: one 32-bit compare-swap; a value
  // already present adds the column bit to the entry its slot names.  The entry
  // is written before its slot can name it (a wave's LDS operations complete
  // in order), so no barrier separates staging from inserting.  Returns the
  // entry now holding v.
  // resolve an insert whose first compare-swap at slot h returned x
  auto insert_chain = [&](uint64_t v, uint32_t e, uint32_t tag, uint32_t h, uint32_t x) -> uint32_t {
    if (x != kFFree) x = join_chain(x, h, tag, v, (tag << 10) | e, s_slot, s_ent, true);  // (join_common.hpp)
    if (x == kFFree) return e;
    atomicOr(&s_ent[x & 1023u].y, 1ull << rs_s);
    return x & 1023u;
  };
  int buf = 0;

  const uint32_t b0 = grp * a.buckets_per_group;
  const uint32_t b1 = min(a.B, b0 + a.buckets_per_group);
  for (uint32_t wb = b0; wb < b1; wb += kRWin) {
    const uint32_t we = min(b1, wb + kRWin);
    __syncthreads();  // previous window fully consumed
    for (uint32_t i = tid; i <= we - wb; i += kRB) s_coff[i] = coff[wb + i];
    __syncthreads();
    for (uint32_t i = tid; i < we - wb; i += kRB) {
      const uint32_t cs = s_coff[i];
      uint32_t lo = i + 1, hi = we - wb;
      while (lo < hi) {
        const uint32_t mid = (lo + hi + 1) >> 1;
        if (s_coff[mid] - cs <= a.cap) lo = mid; else hi = mid - 1;
      }
      s_next[i] = (uint16_t)lo;
    }
    __syncthreads();
    auto chunk_end = [&](uint32_t bs) { return wb + (uint32_t)s_next[bs - wb]; };
    // the chunk after (bs, be, cs, ce): the next slice of an oversized bucket,
    // or the next whole buckets (bs == we: none)
    auto advance = [&](uint32_t bs, uint32_t be, uint32_t ce, uint32_t& nbs, uint32_t& nbe, uint32_t& ncs,
                       uint32_t& nce) {
      if (ce < s_coff[be - wb]) {
        nbs = bs;
        nbe = be;
        ncs = ce;
      } else {
        nbs = be;
        nbe = nbs < we ? chunk_end(nbs) : nbs;
        ncs = s_coff[nbs - wb];
      }
      nce = min(s_coff[nbe - wb], ncs + a.cap);
    };
    uint32_t bs = wb, be = chunk_end(wb);
    uint32_t cs = s_coff[0], ce = min(s_coff[be - wb], cs + a.cap);
    uint32_t qb = 0, qe = 0;  // waves 0-1: pos of the chunk after the current one
    if (wave < 2) {
      uint32_t pb, pe;
      pos_load(bs, be, pb, pe);
      store_ranges(buf, pb, pe);
      uint32_t x0, x1, x2, x3;
      advance(bs, be, ce, x0, x1, x2, x3);
      if (x0 < we) pos_load(x0, x1, qb, qe);
    }
    __syncthreads();
    ChunkRegs cur, nxt;
    fetch_first(buf, 0, ce - cs, !(self_tile && ce == s_coff[be - wb]), cur);
    while (bs < we) {
      uint32_t nbs, nbe, ncs, nce;
      advance(bs, be, ce, nbs, nbe, ncs, nce);
      const bool has_next = nbs < we;
      const uint32_t cbase = s_coff[bs - wb];  // chunk order: [cs - cbase, ce - cbase)
      const bool whole = cs == cbase && ce == s_coff[be - wb];
      // the next chunk's ranges, from registers (its buffer was last read
      // before the barrier that ended the previous chunk); the previous
      // chunk's table entries all go (cheaper than tracking who made which)
      if (has_next && wave < 2) store_ranges(buf ^ 1, qb, qe);
      for (int i = tid; i < kFSlots / 4; i += kRB)
        reinterpret_cast<uint4*>(s_slot)[i] = make_uint4(kFFree, kFFree, kFFree, kFFree);
      __syncthreads();
      // in flight during the inserts and probes: the positions of the chunk
      // after the next (waves 0-1) and the next chunk's first elements
      if (has_next && wave < 2) {
        uint32_t x0, x1, x2, x3;
        advance(nbs, nbe, nce, x0, x1, x2, x3);
        if (x0 < we) pos_load(x0, x1, qb, qe);
      }
      if (has_next)
        fetch_first(buf ^ 1, ncs - s_coff[nbs - wb], nce - s_coff[nbs - wb],
                    !(self_tile && ncs == s_coff[nbs - wb] && nce == s_coff[nbe - wb]), nxt);
      // 1) stage + insert this thread's column elements
      uint32_t ent0 = kNoSlot, ent1 = kNoSlot;
      {
        // the two register elements: both entries written and both first
        // compare-swaps issued before either chain is resolved
        const bool in0 = cur.clo < cur.chi, in1 = cur.clo + 8 < cur.chi;
        const unsigned long long bit = 1ull << rs_s;
        const uint32_t t0 = fp_tag(cur.c[0]), t1 = fp_tag(cur.c[1]);
        const uint32_t h0 = fp_slot(cur.c[0]), h1 = fp_slot(cur.c[1]);
        uint32_t x0 = kFFree, x1 = kFFree;
        if (in0) s_ent[cur.clo] = make_ulonglong2(cur.c[0], bit);
        if (in1) s_ent[cur.clo + 8] = make_ulonglong2(cur.c[1], bit);
        if (in0) x0 = atomicCAS(&s_slot[h0], kFFree, (t0 << 10) | cur.clo);
        if (in1) x1 = atomicCAS(&s_slot[h1], kFFree, (t1 << 10) | (cur.clo + 8));
        if (in0) ent0 = insert_chain(cur.c[0], cur.clo, t0, h0, x0);
        if (in1) ent1 = insert_chain(cur.c[1], cur.clo + 8, t1, h1, x1);
        for (uint32_t x = cur.clo + 16; x < cur.chi; x += 8) {
          const uint64_t v = a.data[cur.csrc + x];
          s_ent[x] = make_ulonglong2(v, bit);
          const uint32_t tg = fp_tag(v), hh = fp_slot(v);
          insert_chain(v, x, tg, hh, atomicCAS(&s_slot[hh], kFFree, (tg << 10) | x));
        }
      }
      __syncthreads();
      // 2) probe.  A diagonal tile's chunk of whole buckets has its column
      //    elements as its row elements: each one's hits are the final mask of
      //    the entry it created or joined (the first two in registers; any
      //    further ones look their value up like a row element)
      if (self_tile && whole) {
        if ((uint32_t)rs_s < r_valid) {
          if (ent0 != kNoSlot) add_hits(rs_s, s_ent[ent0].y);
          if (ent1 != kNoSlot) add_hits(rs_s, s_ent[ent1].y);
          for (uint32_t x = cur.clo + 16; x < cur.chi; x += 8) {
            const uint64_t v = a.data[cur.csrc + x];
            const uint32_t h = fp_slot(v);
            add_hits(rs_s, lookup(v, h, s_slot[h]));
          }
        }
      } else if ((uint32_t)rs_s < r_valid) {
        const bool ok0 = cur.rlo < cur.rhi, ok1 = cur.rlo + 8 < cur.rhi;
        const uint32_t h0 = fp_slot(cur.r[0]), h1 = fp_slot(cur.r[1]);
        const uint32_t x0 = ok0 ? s_slot[h0] : kFFree, x1 = ok1 ? s_slot[h1] : kFFree;
        const unsigned long long m0 = lookup(cur.r[0], h0, x0);
        if (m0) add_hits(rs_s, m0);
        const unsigned long long m1 = lookup(cur.r[1], h1, x1);
        if (m1) add_hits(rs_s, m1);
        for (uint32_t j = cur.rlo + 16; j < cur.rhi; j += 8) {
          const uint64_t v = a.data[j];
          const uint32_t h = fp_slot(v);
          const unsigned long long m = lookup(v, h, s_slot[h]);
          if (m) add_hits(rs_s, m);
        }
      }
      __syncthreads();
      buf ^= 1;
      cur = nxt;
      bs = nbs;
      be = nbe;
      cs = ncs;
      ce = nce;
    }
  }
  __syncthreads();
  // planes the carry chains reached (unrelated tiles: none or one)
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) top = max(top, (uint32_t)__shfl_xor(top, o, 64));
  if (lane == 0 && top) atomicMax(&s_top, top);
  __syncthreads();
  const int np = (int)s_top;
  for (uint32_t r = tid >> 6; r < kTile; r += kRB / 64) {  // a wave per row, a lane per column
    const uint32_t c = lane;
    uint32_t cnt = 0;
    for (int b = 0; b < np; ++b) cnt |= (uint32_t)((s_pl[b * kTile + r] >> c) & 1ull) << b;
    if (self_tile && c == r) cnt += s_self[r];
    if (!cnt) continue;
    const uint32_t gr = row0 + r, gc = col0 + c;
    if (gr >= row_lim || gc >= a.n) continue;
    if (a.packed) {
      atomicAdd(&a.out[(t - a.tile_begin) * (kTile * kTile) + r * kTile + c], (int32_t)cnt);
      continue;
    }
    const uint64_t orow = rows_mode ? gr - a.row_begin : gr;
    atomicAdd(&a.out[orow * a.ld + gc], (int32_t)cnt);
  }
  // the mirror of an off-diagonal symmetric tile: a wave per column, a lane per
  // row, so each wave's atomics fall on one output row (k_join's flush)
  if (!a.packed && !rows_mode && I != J) {
    for (uint32_t c = tid >> 6; c < kTile; c += kRB / 64) {
      const uint32_t r = lane;
      uint32_t cnt = 0;
      for (int b = 0; b < np; ++b) cnt |= (uint32_t)((s_pl[b * kTile + r] >> c) & 1ull) << b;
      const uint32_t gr = row0 + r, gc = col0 + c;
      if (!cnt || gr >= row_lim || gc >= a.n) continue;
      atomicAdd(&a.out[(uint64_t)gc * a.ld + gr], (int32_t)cnt);
    }
  }
}

}  // namespace

hipError_t rjoin_bounds(const uint64_t* data, const uint64_t* starts, const uint32_t* sizes, uint32_t n,
                        uint32_t B, uint64_t* bounds, hipStream_t s) {
  hipLaunchKernelGGL(k_rj_bounds, dim3((B + 1 + kPB / 64 - 1) / (kPB / 64)), dim3(kPB), 0, s, data, starts,
                     sizes, n, B, bounds);
  return hipGetLastError();
}

hipError_t rjoin_pos(const uint64_t* data, const uint64_t* starts, const uint32_t* sizes, uint32_t n,
                     uint32_t B, const uint64_t* bounds, uint32_t* pos, hipStream_t s) {
  if (!n) return hipSuccess;
  const size_t lds = (size_t)(B + 1) * 8;
  if (lds <= 32 * 1024 + 8) {
    hipLaunchKernelGGL(k_rj_pos<true>, dim3(n), dim3(kPB), lds, s, data, starts, sizes, B, bounds, pos);
  } else {
    hipLaunchKernelGGL(k_rj_pos<false>, dim3(n), dim3(kPB), 0, s, data, starts, sizes, B, bounds, pos);
  }
  return hipGetLastError();
}

hipError_t rjoin_block_prefix(const uint32_t* pos, uint32_t n, uint32_t B, uint32_t* pre, hipStream_t s) {
  const uint64_t cells = (uint64_t)((n + kTile - 1) / kTile) * (B + 1);
  if (!cells) return hipSuccess;
  hipLaunchKernelGGL(k_rj_prefix, dim3((unsigned)((cells + kPB - 1) / kPB)), dim3(kPB), 0, s, pos, n, B, pre);
  return hipGetLastError();
}

hipError_t rjoin_launch(const uint64_t* data, const uint64_t* starts, const uint32_t* pos,
                        const uint32_t* pre, uint32_t n, uint32_t B, bool sym, uint32_t row_begin,
                        uint32_t row_end, uint64_t tile_begin, uint64_t tile_end, const uint32_t* d_tiles,
                        bool packed, int32_t* out, hipStream_t s) {
  const uint32_t n_cb = (n + kTile - 1) / kTile;
  const uint32_t n_rb = sym ? n_cb : (row_end - row_begin + kTile - 1) / kTile;
  if (!d_tiles) {
    const uint64_t all = sym ? (uint64_t)n_cb * (n_cb + 1) / 2 : (uint64_t)n_rb * n_cb;
    if (!sym) {
      tile_begin = 0;
      tile_end = all;
    }
    tile_end = std::min(tile_end, all);
  }
  if (tile_begin >= tile_end) return hipSuccess;
  const uint64_t tiles = tile_end - tile_begin;
  RJoinArgs ra{};
  ra.data = data;
  ra.starts = starts;
  ra.pos = pos;
  ra.cpre = pre;
  ra.B = B;
  ra.n = n;
  ra.n_col_blocks = n_cb;
  ra.sym = (sym || d_tiles) ? 1 : 0;
  ra.row_begin = row_begin;
  ra.row_end = row_end;
  ra.tiles = d_tiles;
  ra.out = out;
  ra.ld = n;
  ra.cap = join_cap();
  ra.packed = packed ? 1 : 0;
  // bucket groups per tile as for k_join: ~64 buckets per workgroup while the
  // grid is small, >= ~1024 workgroups in all, >= 16 buckets each
  // (SKS_RJOIN_WGS, diagnostics: the total)
  static const uint64_t wgs_env = getenv("SKS_RJOIN_WGS") ? strtoull(getenv("SKS_RJOIN_WGS"), 0, 10) : 0;
  uint64_t want = wgs_env ? (wgs_env + tiles - 1) / tiles
                          : std::max<uint64_t>(std::min<uint64_t>((B + 63) / 64, (65536 + tiles - 1) / tiles),
                                               (1024 + tiles - 1) / tiles);
  if (!wgs_env) want = std::min<uint64_t>(want, std::max<uint32_t>(1, B / 16));
  const uint32_t groups = (uint32_t)std::min<uint64_t>(B, std::max<uint64_t>(1, want));
  ra.buckets_per_group = (B + groups - 1) / groups;
  ra.n_groups = (B + ra.buckets_per_group - 1) / ra.buckets_per_group;
  const uint64_t per = std::max<uint64_t>(1, kMaxGrid / ra.n_groups);
  for (uint64_t t0 = tile_begin; t0 < tile_end; t0 += per) {
    const uint64_t nt = std::min(per, tile_end - t0);
    ra.tile_begin = t0;
    if (packed) ra.out = out + (t0 - tile_begin) * (uint64_t)(kTile * kTile);
    hipLaunchKernelGGL(k_rjoin, dim3((unsigned)(nt * ra.n_groups)), dim3(kRB), 0, s, ra);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

}  // namespace sks
