// Kernel 2 — k_join: |S_i ∩ S_j| for all pairs of a 64 x 64 tile of (row,
// column) sketches, as one LDS hash join of the two 64-sketch blocks instead of
// 4096 pairwise merges.
//
// The reference counts one pair at a time: iterate the smaller kmer_set, probe
// the larger hash map (kmer_set.cpp:23-41), one pair per cilk_for iteration of
// the all-pairs list (kmer_set.cpp:167-184, generators.hpp:44-58).  Here the
// input is the join layout (layout.hip; format in join_common.hpp): per block,
// each distinct value once with the mask of the block's sketches holding it.
//   * Off-diagonal tile (I != J): per chunk of the column block's entries, every
//     entry {value, column mask C} is staged in LDS and inserted into a
//     fingerprint table (one 32-bit compare-swap: the entries of a block are
//     distinct, so an insert only looks for a free slot); every row entry
//     {value, row mask R} probes it once, and a hit adds C to each row r of R.
//   * Diagonal tile (I == J): no table.  An entry held by the sketches M is in
//     the intersection of every pair (r, c) of M: for each r of M it adds M to
//     row r (the (r, r) bit as a plain per-row count).
// Counts are bit-sliced: plane b of tile row r is the 64-bit word of bit b of
// the row's 64 column counts, and adding a column mask m is a carry chain of
// LDS atomic XORs (m &= old after each plane), about log2(|m|) + 2 atomics.
// The result equals the reference's count for every pair: a value shared by
// sketches i and j is one entry in each block (or one entry holding both bits
// in a diagonal tile), and it meets its partner exactly once.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <vector>

#include "join_common.hpp"
#include "sks_ani.hpp"
#include "sks_internal.hpp"

namespace sks {

namespace {

using jc::fp_slot;
using jc::fp_tag;
using jc::kFFree;
using jc::kFSlots;
using jc::KV;
using jc::kv_eq;
using jc::kv_load;
using jc::sym_tile;

constexpr int kTile = 64;
// workgroups per launch at most (HIP caps a grid at 2^32 - 1 work-items);
// larger grids are cut into slices
constexpr uint64_t kMaxGrid = 1ull << 22;
// 512 threads (8 waves): four workgroups per CU for u64 values (32 waves),
// three for 128-bit values, hide the LDS round trips of the insert and probe chains
constexpr int kJB = 512;
constexpr int kJCap = 1024;             // column entries per chunk (10-bit entry index)
#ifndef SKS_JOIN_CAP2
#define SKS_JOIN_CAP2 1024
#endif
// column entries per chunk by value width (128-bit values: a smaller chunk
// can buy LDS for another workgroup per CU), and per thread
template <int EW>
constexpr int jcap() { return EW == 1 ? kJCap : SKS_JOIN_CAP2; }
template <int EW>
constexpr int jmade() { return jcap<EW>() / kJB; }
static_assert(SKS_JOIN_CAP2 % kJB == 0 && SKS_JOIN_CAP2 <= kJCap, "128-bit chunk capacity");
#ifndef SKS_JOIN_ROWPF
#define SKS_JOIN_ROWPF 1
#endif
constexpr int kJRowPf = SKS_JOIN_ROWPF;   // row entries per thread held in registers per chunk
// buckets per window: a workgroup stages the bucket offsets of 64 buckets at a
// time; a window may hold several layout regions (each region's entries are
// contiguous, with a gap before the next region: chunks map their entries
// piecewise, at most kJPieces regions per chunk)
#ifndef SKS_JOIN_WINLOG
#define SKS_JOIN_WINLOG 6
#endif
constexpr int kJWinLog = SKS_JOIN_WINLOG, kJWin = 1 << kJWinLog;
static_assert(kJWinLog <= 6, "a window's buckets are scanned by one wave");
constexpr uint32_t kJPieces = 4;
// 12 planes hold counts below 2^12 per workgroup; a carry out of the top plane
// (a pair sharing >= 4096 values in one workgroup's buckets) is added to the
// output directly (16 planes cost the LDS of the fourth workgroup per CU)
#ifndef SKS_JOIN_PLANES
#define SKS_JOIN_PLANES 12
#endif
constexpr int kPlanes = SKS_JOIN_PLANES;
constexpr uint32_t kNoSlot = 0xFFFFFFFFu;
// hit items with more rows than this are spread over the wave's lanes (rows_add)
#ifndef SKS_JOIN_LIGHT
#define SKS_JOIN_LIGHT 2
#endif
constexpr uint32_t kLight = SKS_JOIN_LIGHT;
static_assert(kJCap == 1024, "entry index: 10 bits of the slot word");
static_assert(kFSlots >= kTile * kTile, "the fused ANI stages a tile's counts in the slot table");

// s_waitcnt immediate for gfx9 "vmcnt(0)" with expcnt / lgkmcnt left at their
// maxima: vmcnt = imm[3:0] | imm[15:14] << 4, expcnt = imm[6:4], lgkmcnt = imm[11:8].
// The fused ANI's fence-free hand-off (a wave drains its count atomics with this
// wait, then the workgroup bumps the tile counter) relies on gfx9 counting
// no-return atomics in vmcnt; gfx10+ counts them in vscnt, where this wait would
// not cover them.  This file is built for gfx950 only: refuse anything else.
constexpr int kWaitVmcnt0 = 0x0F70;
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__)
#error "join.hip: the fused ANI hand-off (kWaitVmcnt0) is written for gfx950 (gfx9 vmcnt semantics)"
#endif

struct JoinArgs {
  JoinLayout r, c;          // row blocks (tile row I = block r_blk0 + I) and column blocks
  uint32_t r_blk0, c_blk0;  // (tile column J = block c_blk0 + J; uint32 arithmetic, -blk0 works)
  uint32_t log_b, B, BW, n, n_col_blocks, n_groups, buckets_per_group;
  int sym;
  uint32_t row_begin, row_end;
  uint64_t tile_begin;
  const uint32_t* tiles;  // optional (I, J) list (global block indices), sym semantics
  int32_t* out;
  uint64_t ld;
  uint32_t cap;  // column entries per chunk (<= kJCap): table load <= cap / kFSlots
  int packed;    // out = [tile - tile_begin][64][64]
  // fused containment / ANI (JoinAni): null ani = counts only
  double* ani;
  const int32_t* sizes;
  double inv_k;
  uint32_t* tile_done;  // [tile - tile_begin]
  int diag_last;        // dispatch the off-diagonal tiles first, the diagonal ones last (all sym tiles, one launch)
  const double* root;   // root[x] = ani_of(x, root_size) (JoinAni::root), or null
  uint32_t root_size;
};

template <int EW>
struct JoinChunk {
  KV cv[jmade<EW>()];
  unsigned long long cm[jmade<EW>()];  // 0: no entry
  KV rv[kJRowPf];
  unsigned long long rm[kJRowPf];
};

// A chunk's entries in a window's "virtual" index space (the window's buckets
// back to back, without the gaps between layout regions), mapped to block
// positions piecewise: one piece per region the chunk touches (wave-uniform).
struct Pieces {
  uint32_t v1, v2, v3;      // virtual start of pieces 1..3 (~0u: no such piece)
  uint32_t d0, d1, d2, d3;  // block position - virtual index, per piece
};
__device__ __forceinline__ uint32_t phys(const Pieces p, uint32_t k) {
  return k + (k < p.v1 ? p.d0 : k < p.v2 ? p.d1 : k < p.v3 ? p.d2 : p.d3);
}

template <int EW, bool PIECES>
__device__ __forceinline__ void join_fetch(const uint64_t* __restrict__ cvals,
                                           const unsigned long long* __restrict__ cmasks,
                                           const uint64_t* __restrict__ rvals,
                                           const unsigned long long* __restrict__ rmasks, uint32_t cs,
                                           uint32_t ce, const Pieces cp, uint32_t rs, uint32_t re,
                                           const Pieces rp, int tid, JoinChunk<EW>& c) {
  // a chunk inside one region (the common case; a wave-uniform branch): the
  // entries are contiguous, no per-element piece compares
  if (!PIECES || cp.v1 == ~0u) {
    const unsigned long long* cm = cmasks + cp.d0;
    const uint64_t* cv = cvals + (uint64_t)cp.d0 * EW;
#pragma unroll
    for (int u = 0; u < jmade<EW>(); ++u) {
      const uint32_t k = cs + tid + kJB * u;
      c.cv[u] = k < ce ? kv_load<EW>(cv, k) : KV{0, 0};
      c.cm[u] = k < ce ? cm[k] : 0ull;
    }
  } else {
#pragma unroll
    for (int u = 0; u < jmade<EW>(); ++u) {
      const uint32_t k = cs + tid + kJB * u, q = phys(cp, k);
      c.cv[u] = k < ce ? kv_load<EW>(cvals, q) : KV{0, 0};
      c.cm[u] = k < ce ? cmasks[q] : 0ull;
    }
  }
  if (!PIECES || rp.v1 == ~0u) {
    const unsigned long long* rm = rmasks + rp.d0;
    const uint64_t* rv = rvals + (uint64_t)rp.d0 * EW;
#pragma unroll
    for (int u = 0; u < kJRowPf; ++u) {
      const uint32_t k = rs + tid + kJB * u;
      c.rv[u] = k < re ? kv_load<EW>(rv, k) : KV{0, 0};
      c.rm[u] = k < re ? rm[k] : 0ull;
    }
  } else {
#pragma unroll
    for (int u = 0; u < kJRowPf; ++u) {
      const uint32_t k = rs + tid + kJB * u, q = phys(rp, k);
      c.rv[u] = k < re ? kv_load<EW>(rvals, q) : KV{0, 0};
      c.rm[u] = k < re ? rmasks[q] : 0ull;
    }
  }
}

__device__ unsigned long long g_join_check;  // SKS check build: table invariant violations

// inclusive prefix sum over the 64 lanes of a wave (DPP; no LDS)
__device__ __forceinline__ uint32_t wave_scan(uint32_t v) {
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false);  // row_shr:1
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false);  // row_shr:2
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false);  // row_shr:4
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false);  // row_shr:8
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);  // row_bcast:15
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);  // row_bcast:31
  return v;
}

__device__ __forceinline__ unsigned long long readlane64(unsigned long long x, uint32_t l) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)x, (int)l);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(x >> 32), (int)l);
  return ((unsigned long long)hi << 32) | lo;
}

// index of the k-th set bit (k < popcount(x)) of x
__device__ __forceinline__ uint32_t nth_bit(unsigned long long x, uint32_t k) {
  uint32_t r = 0;
#pragma unroll
  for (int w = 32; w >= 1; w >>= 1) {
    const uint32_t c = (uint32_t)__popcll(x & ((1ull << w) - 1));
    if (k >= c) {
      k -= c;
      x >>= w;
      r += w;
    }
  }
  return r;
}

// end of window [.., we) in a block's boff row: the next bucket's start, or the
// region's end when we closes a region
__device__ __forceinline__ uint32_t window_end(const uint32_t* off, uint32_t we, uint32_t B, uint32_t rb_log) {
  return (we & ((1u << rb_log) - 1)) == 0 ? off[B + ((we - 1) >> rb_log)] : off[we];
}

#ifdef SKS_JOIN_STAMPS  // diagnostic build: cycles per k_join phase, summed by thread 0 of each workgroup
// slots: 0 setup, 1 window bookkeeping, 2 stage (incl. waiting for the chunk's
// loads), 3 insert, 4 probe + hit adds, 5 flush, 6 fused ANI, 7 diagonal tile
constexpr int kMaxJoinStampWgs = 65536;
__device__ unsigned long long g_join_stamps_wg[kMaxJoinStampWgs * 8];
#define JSTAMP(i)                                    \
  do {                                               \
    if (threadIdx.x == 0) {                          \
      const uint64_t t_ = __builtin_amdgcn_s_memtime(); \
      js_acc[i] += t_ - js_last;                     \
      js_last = t_;                                  \
    }                                                \
  } while (0)
#define JSTAMP_FLUSH()                                                                          \
  do {                                                                                          \
    if (threadIdx.x == 0 && blockIdx.x < kMaxJoinStampWgs)                                      \
      for (int q_ = 0; q_ < 8; ++q_) g_join_stamps_wg[(uint64_t)blockIdx.x * 8 + q_] = js_acc[q_]; \
  } while (0)
#else
#define JSTAMP(i) do {} while (0)
#define JSTAMP_FLUSH() do {} while (0)
#endif

// PIECES = false: windows also end at every region end of either layout, so a
// chunk is always contiguous (the kernel for layouts of 64-bucket regions,
// where the piece code, never taken, still cost 8% of the join); true: windows
// of 64 buckets across small regions, chunks mapped piecewise
// u64 values: four workgroups per CU — 39.4 KB of LDS (12 planes) and 64
// VGPRs (one prefetched row entry per thread; 8 registers spill outside the
// chunk loop), 8% faster than three with 80; 128-bit values: three (76 VGPRs,
// 47.4 KB; four per CU with 512-entry chunks measured equal)
template <int EW, bool CHECK, bool PIECES>
#ifndef SKS_JOIN_WPE1
#define SKS_JOIN_WPE1 8
#endif
#ifndef SKS_JOIN_WPE2
#define SKS_JOIN_WPE2 2
#endif
__global__ __launch_bounds__(kJB, EW == 1 ? SKS_JOIN_WPE1 : SKS_JOIN_WPE2) void k_join(JoinArgs a) {
  __shared__ uint32_t s_slot[kFSlots];
  __shared__ uint64_t s_ev[jcap<EW>() * EW];          // staged column entries: values
  __shared__ unsigned long long s_em[jcap<EW>()];     // ... and column masks
  __shared__ unsigned long long s_pl[kPlanes * kTile];  // plane b of row r at [b * 64 + r]
  __shared__ uint32_t s_roff[kJWin + 1], s_coff[kJWin + 1];  // block positions of the window's buckets
  __shared__ uint32_t s_rv[kJWin + 1], s_cv[kJWin + 1];      // ... and their virtual starts
  __shared__ uint8_t s_next[kJWin];
  __shared__ uint32_t s_self[kTile];
  __shared__ uint32_t s_top;  // planes used (the highest carry chain)
#ifdef SKS_JOIN_STAMPS
  uint64_t js_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  uint64_t js_last = __builtin_amdgcn_s_memtime();
#endif

  // tile of this workgroup: dispatch slot u, in tile order, or (diag_last) the
  // off-diagonal tiles in tile order and then the diagonal ones.  A tile's ANI
  // is written to host memory by its last workgroup, so the tiles finishing in
  // the launch's last round of workgroups write theirs after every count is
  // done; diagonal tiles are the cheapest (no table) and write one 64 x 64
  // block (no mirror), so they take that round.
  const uint64_t u = blockIdx.x / a.n_groups;
  uint64_t t = a.tile_begin + u;
  if (a.diag_last) {
    const uint64_t nb = a.n_col_blocks, n_off = nb * (nb - 1) / 2;
    const auto row_start = [nb](uint64_t i) { return i * nb - i * (i - 1) / 2; };  // tile (i, i)
    if (u < n_off) {  // row i of the upper triangle holds nb - 1 - i off-diagonal tiles
      uint64_t i = 0, rem = u;
      while (rem >= nb - 1 - i) {
        rem -= nb - 1 - i;
        ++i;
      }
      t = row_start(i) + 1 + rem;
    } else {
      t = row_start(u - n_off);
    }
  }
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
  const int tid = threadIdx.x, lane = tid & 63;
  const uint32_t rblk = a.r_blk0 + I, cblk = a.c_blk0 + J;
  const uint64_t rb = a.r.bstart[rblk], cb = a.c.bstart[cblk];
  const uint64_t* rvals = a.r.vals + rb * EW;
  const unsigned long long* rmasks = reinterpret_cast<const unsigned long long*>(a.r.masks) + rb;
  const uint64_t* cvals = a.c.vals + cb * EW;
  const unsigned long long* cmasks = reinterpret_cast<const unsigned long long*>(a.c.masks) + cb;
  const uint32_t* roff = a.r.boff + (uint64_t)rblk * a.BW;
  const uint32_t* coff = a.c.boff + (uint64_t)cblk * a.BW;
  // each layout's region bucket log (the last word of its boff rows): the
  // regions of the row and the column block may differ in size
  const uint32_t r_rb = roff[a.BW - 1], c_rb = coff[a.BW - 1];
  const uint32_t r_valid = min<uint32_t>(kTile, row_lim - row0);
  const unsigned long long rvm = r_valid >= 64 ? ~0ull : ((1ull << r_valid) - 1);
  // a tile on the diagonal: row block = column block of the same layout (rows
  // taken from a separate layout start off a block boundary, so never match)
  const bool self_tile = row0 == col0 && rblk == cblk && a.r.vals == a.c.vals;

  for (int i = tid; i < kFSlots / 4; i += kJB)
    reinterpret_cast<uint4*>(s_slot)[i] = make_uint4(kFFree, kFFree, kFFree, kFFree);
  for (int i = tid; i < kPlanes * kTile / 2; i += kJB) reinterpret_cast<uint4*>(s_pl)[i] = make_uint4(0, 0, 0, 0);
  if (tid < kTile) s_self[tid] = 0;
  if (tid == 0) s_top = 0;
  uint32_t top = 0;
  __syncthreads();  // table, planes and self counts cleared before any chain (the diagonal path has no other barrier)
  JSTAMP(0);

  // output of count `cnt` for tile cell (r, c) (both halves of a symmetric
  // off-diagonal tile): the carry-out path of add_hits
  auto emit = [&](uint32_t r, uint32_t c, uint32_t cnt) {
    const uint32_t gr = row0 + r, gc = col0 + c;
    if (gr >= row_lim || gc >= a.n) return;
    if (a.packed) {
      atomicAdd(&a.out[(t - a.tile_begin) * (kTile * kTile) + r * kTile + c], (int32_t)cnt);
      return;
    }
    atomicAdd(&a.out[(uint64_t)(rows_mode ? gr - a.row_begin : gr) * a.ld + gc], (int32_t)cnt);
    if (!rows_mode && I != J) atomicAdd(&a.out[(uint64_t)gc * a.ld + gr], (int32_t)cnt);
  };
  auto add_hits = [&](uint32_t r, unsigned long long m) {
    unsigned long long* p = &s_pl[r];
    uint32_t b = 0;
    for (; m && b < kPlanes; ++b) m &= atomicXor(p + b * kTile, m);
    top = max(top, b);
    while (m) {  // carried out of the top plane: 2^kPlanes per column
      const uint32_t c = __builtin_ctzll(m);
      m &= m - 1;
      emit(r, c, 1u << kPlanes);
    }
  };
  // Wave-uniform: for every lane l with an item (row mask R_l, column mask
  // C_l), add C_l to each row of R_l.  An item of at most kLight rows runs them
  // in its own lane; the rows of heavier items (an entry held by many sketches
  // of a related block) are spread over the lanes, one (item, row) per lane:
  // the wave walks its heavy items in lane order (readlanes, no LDS), giving
  // each window of 64 (item, row) pairs to its 64 lanes, instead of one lane
  // running up to 64 rows one after another.  diag: the (r, r) bit is counted
  // in s_self[r] instead (a diagonal tile's entry is in its own row).
  auto row_add = [&](uint32_t r, unsigned long long C, bool diag) {
    if (diag) {
      atomicAdd(&s_self[r], 1u);
      const unsigned long long m = C & ~(1ull << r);
      if (m) add_hits(r, m);
    } else {
      add_hits(r, C);
    }
  };
  auto rows_add = [&](unsigned long long R, unsigned long long C, bool diag) {
    const uint32_t cnt = (uint32_t)__popcll(R);
    // light items (<= kLight rows) run their rows in their own lane
    const bool heavy = cnt > kLight;
    if (!heavy) {
      while (R) {
        const uint32_t r = (uint32_t)__builtin_ctzll(R);
        R &= R - 1;
        row_add(r, C, diag);
      }
    }
    unsigned long long pend = __ballot(heavy);
    if (!pend) return;
    const uint32_t hc = heavy ? cnt : 0;
    const uint32_t incl = wave_scan(hc), excl = incl - hc;
    for (uint32_t t = 0; pend; t += 64) {
      unsigned long long myR = 0, myC = 0;
      uint32_t myk = 0;
      const uint32_t g = t + lane;
      while (pend) {
        const uint32_t o = (uint32_t)__builtin_ctzll(pend);
        const uint32_t eo = (uint32_t)__builtin_amdgcn_readlane((int)excl, (int)o);
        if (eo >= t + 64) break;
        const uint32_t co = (uint32_t)__builtin_amdgcn_readlane((int)hc, (int)o);
        const unsigned long long Ro = readlane64(R, o), Co = readlane64(C, o);
        if (g >= eo && g < eo + co) {
          myR = Ro;
          myC = Co;
          myk = g - eo;
        }
        if (eo + co > t + 64) break;  // continues in the next window
        pend &= pend - 1;
      }
      if (myR) row_add(nth_bit(myR, myk), myC, diag);
    }
  };
  auto ent_val = [&](uint32_t e) -> KV {
    if constexpr (EW == 1) return KV{s_ev[e], 0};
    else return KV{s_ev[2 * e], s_ev[2 * e + 1]};
  };
  // slot word naming v's entry, or kFFree (one exit edge; the stop test reads
  // the named entry whether or not the tag matches: see layout.hip dd_insert)
  auto chain = [&](const KV& v, uint32_t h, uint32_t x) -> uint32_t {
    const uint32_t tag = fp_tag<EW>(v);
    for (;;) {
      const KV u = ent_val(x & 1023u);
      if ((x == kFFree) | (((x >> 10) == tag) & kv_eq<EW>(u, v))) return x;
      h = (h + 1) & (kFSlots - 1);
      x = s_slot[h];
    }
  };

  const uint32_t b0 = grp * a.buckets_per_group;
  const uint32_t b1 = min(a.B, b0 + a.buckets_per_group);
  if (self_tile) {
    // ---- diagonal tile: every entry's hits are its own mask ----------------------------------
    for (uint32_t wb = b0; wb < b1;) {  // one region (contiguous entries) at a time
      const uint32_t we = min(b1, ((wb >> c_rb) + 1) << c_rb);
      const uint32_t es = coff[wb], ee = window_end(coff, we, a.B, c_rb);
      for (uint32_t k0 = es; k0 < ee; k0 += 4 * kJB) {
        unsigned long long m[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const uint32_t k = k0 + tid + u * kJB;
          m[u] = k < ee ? cmasks[k] : 0ull;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) rows_add(m[u] & rvm, m[u], true);
      }
      wb = we;
    }
    JSTAMP(7);
  } else {
    // ---- off-diagonal tile: chunks of the column block's entries -----------------------------
    uint32_t made[jmade<EW>()];  // slots this thread created in the current chunk
#pragma unroll
    for (int u = 0; u < jmade<EW>(); ++u) made[u] = kNoSlot;
    for (uint32_t wb = b0; wb < b1;) {
      uint32_t we = min(b1, ((wb >> kJWinLog) + 1) << kJWinLog);
      if constexpr (!PIECES) we = min(we, min(((wb >> c_rb) + 1) << c_rb, ((wb >> r_rb) + 1) << r_rb));
      const uint32_t nw = we - wb;
      __syncthreads();  // previous window fully consumed
      // the window's bucket positions and, by a wave scan of the bucket sizes,
      // their virtual starts (wave 0: columns, wave 1: rows; nw <= 64)
      if (tid < 128) {
        const bool col = tid < 64;
        const uint32_t i = (uint32_t)lane;
        const uint32_t* off = col ? coff : roff;
        const uint32_t rb = col ? c_rb : r_rb;
        const uint32_t st = i < nw ? off[wb + i] : 0u;
        const uint32_t len = i < nw ? window_end(off, wb + i + 1, a.B, rb) - st : 0u;
        const uint32_t v0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)st);
        const uint32_t incl = wave_scan(len);
        uint32_t* sp = col ? s_coff : s_roff;
        uint32_t* sv = col ? s_cv : s_rv;
        if (i < nw) {
          sp[i] = st;
          sv[i + 1] = v0 + incl;
        }
        if (i == 0) sv[0] = v0;
      }
      __syncthreads();
      // chunk ends: the most whole buckets from bucket i on that fit cap, within
      // kJPieces regions
      for (uint32_t i = tid; i < nw; i += kJB) {
        const uint32_t cs = s_cv[i];
        const uint32_t lim = min(nw, min((((wb + i) >> c_rb) + kJPieces) << c_rb,
                                         (((wb + i) >> r_rb) + kJPieces) << r_rb) - wb);
        uint32_t lo = i + 1, hi = lim;
        while (lo < hi) {
          const uint32_t mid = (lo + hi + 1) >> 1;
          if (s_cv[mid] - cs <= a.cap) lo = mid; else hi = mid - 1;
        }
        s_next[i] = (uint8_t)lo;
      }
      __syncthreads();
      // the pieces of buckets [bs, be) (window-relative) of a layout with
      // regions of 2^rl buckets, wave-uniform, straight line (a loop filling the
      // struct put it in scratch); a window inside one region of the layout
      // (one_region: every large layout) maps virtual = block position
      const bool c_one = (wb >> c_rb) == ((we - 1) >> c_rb), r_one = (wb >> r_rb) == ((we - 1) >> r_rb);
      auto pieces = [&](const uint32_t* sp, const uint32_t* sv, uint32_t bs, uint32_t be, uint32_t rl, bool one) {
        if (!PIECES || one) return Pieces{~0u, ~0u, ~0u, 0u, 0u, 0u, 0u};
        const uint32_t f1 = min(nw, ((((wb + bs) >> rl) + 1) << rl) - wb);
        Pieces p{~0u, ~0u, ~0u, sp[bs] - sv[bs], 0u, 0u, 0u};
        if (f1 >= be) {  // inside one region
          p.d0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)p.d0);
          return p;
        }
        const uint32_t f2 = min(nw, ((((wb + bs) >> rl) + 2) << rl) - wb);
        const uint32_t f3 = min(nw, ((((wb + bs) >> rl) + 3) << rl) - wb);
        p.v1 = f1 < be ? sv[f1] : ~0u;
        p.d1 = f1 < be ? sp[f1] - sv[f1] : 0u;
        p.v2 = f2 < be ? sv[f2] : ~0u;
        p.d2 = f2 < be ? sp[f2] - sv[f2] : 0u;
        p.v3 = f3 < be ? sv[f3] : ~0u;
        p.d3 = f3 < be ? sp[f3] - sv[f3] : 0u;
        p.v1 = (uint32_t)__builtin_amdgcn_readfirstlane((int)p.v1);
        p.v2 = (uint32_t)__builtin_amdgcn_readfirstlane((int)p.v2);
        p.v3 = (uint32_t)__builtin_amdgcn_readfirstlane((int)p.v3);
        p.d0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)p.d0);
        p.d1 = (uint32_t)__builtin_amdgcn_readfirstlane((int)p.d1);
        p.d2 = (uint32_t)__builtin_amdgcn_readfirstlane((int)p.d2);
        p.d3 = (uint32_t)__builtin_amdgcn_readfirstlane((int)p.d3);
        return p;
      };
      // chunks of whole buckets; a bucket above cap is cut into sub-chunks of
      // cap column entries, each joined with all of the bucket's row entries
      // (its column entries are distinct, so each hit is counted once)
      JSTAMP(1);
      auto chunk_end = [&](uint32_t bs) { return wb + (uint32_t)s_next[bs - wb]; };
      uint32_t bs = wb, be = chunk_end(wb);
      uint32_t cs = s_cv[0], ce = min(s_cv[be - wb], cs + a.cap);
      Pieces cp = pieces(s_coff, s_cv, 0, be - wb, c_rb, c_one), rp = pieces(s_roff, s_rv, 0, be - wb, r_rb, r_one);
      JoinChunk<EW> cur;
      join_fetch<EW, PIECES>(cvals, cmasks, rvals, rmasks, cs, ce, cp, s_rv[0], s_rv[be - wb], rp, tid, cur);
      while (bs < we) {
        const uint32_t rs = s_rv[bs - wb], re = s_rv[be - wb];
        const Pieces crp = rp;  // this chunk's row pieces (the rows beyond the prefetch)
        __builtin_amdgcn_s_waitcnt(kWaitVmcnt0);  // this chunk's entries have landed
        uint32_t nbs, nbe, ncs, nce;
        if (ce < s_cv[be - wb]) {
          nbs = bs;
          nbe = be;
          ncs = ce;
        } else {
          nbs = be;
          nbe = nbs < we ? chunk_end(nbs) : nbs;
          ncs = s_cv[nbs - wb];
        }
        nce = min(s_cv[nbe - wb], ncs + a.cap);
        JoinChunk<EW> nxt;
        if (nbs < we) {
          cp = pieces(s_coff, s_cv, nbs - wb, nbe - wb, c_rb, c_one);
          rp = pieces(s_roff, s_rv, nbs - wb, nbe - wb, r_rb, r_one);
          join_fetch<EW, PIECES>(cvals, cmasks, rvals, rmasks, ncs, nce, cp, s_rv[nbs - wb], s_rv[nbe - wb], rp, tid, nxt);
        }
        JSTAMP(1);

        // 0) free the previous chunk's slots (its probes are done: barrier below
        //    the probe loop) and stage this chunk's entries
#pragma unroll
        for (int u = 0; u < jmade<EW>(); ++u) {
          if (made[u] != kNoSlot) s_slot[made[u]] = kFFree;
          made[u] = kNoSlot;
          const uint32_t e = tid + kJB * u;
          if (cur.cm[u]) {
            if constexpr (EW == 1) s_ev[e] = cur.cv[u].lo;
            else { s_ev[2 * e] = cur.cv[u].lo; s_ev[2 * e + 1] = cur.cv[u].hi; }
            s_em[e] = cur.cm[u];
          }
        }
        __syncthreads();
        JSTAMP(2);
        // 1) insert: the chunk's values are distinct, so a compare-swap walk to
        //    the first free slot
#pragma unroll
        for (int u = 0; u < jmade<EW>(); ++u) {
          if (!cur.cm[u]) continue;
          const uint32_t e = tid + kJB * u;
          const uint32_t word = (fp_tag<EW>(cur.cv[u]) << 10) | e;
          uint32_t h = fp_slot<EW>(cur.cv[u]);
          uint32_t x = atomicCAS(&s_slot[h], kFFree, word);
          while (x != kFFree) {
            h = (h + 1) & (kFSlots - 1);
            x = atomicCAS(&s_slot[h], kFFree, word);
          }
          made[u] = h;
        }
        __syncthreads();
        JSTAMP(3);
        if (CHECK) {  // every inserted value is found, naming its own entry
#pragma unroll
          for (int u = 0; u < jmade<EW>(); ++u) {
            if (!cur.cm[u]) continue;
            const uint32_t h = fp_slot<EW>(cur.cv[u]);
            const uint32_t x = chain(cur.cv[u], h, s_slot[h]);
            if (x == kFFree || (x & 1023u) != tid + kJB * u) atomicAdd(&g_join_check, 1ull);
          }
        }
        // 2) probe with the row entries: first slots read together; a hit with
        //    column mask C adds C to each row of the entry's row mask
        uint32_t sl[kJRowPf], sh[kJRowPf];
#pragma unroll
        for (int u = 0; u < kJRowPf; ++u) {
          sl[u] = kFFree;
          sh[u] = 0;
          if (cur.rm[u] & rvm) {
            sh[u] = fp_slot<EW>(cur.rv[u]);
            sl[u] = s_slot[sh[u]];
          }
        }
#pragma unroll
        for (int u = 0; u < kJRowPf; ++u) {
          const unsigned long long rows = cur.rm[u] & rvm;
          unsigned long long m = 0;
          if (rows && sl[u] != kFFree) {
            const uint32_t x = chain(cur.rv[u], sh[u], sl[u]);
            if (x != kFFree) m = s_em[x & 1023u];
          }
          rows_add(m ? rows : 0ull, m, false);
        }
        for (uint32_t k0 = rs + kJB * kJRowPf; k0 < re; k0 += kJB) {  // (rare) rows beyond the prefetch
          const uint32_t k = k0 + tid, q = PIECES ? phys(crp, k) : k;
          const unsigned long long rows = k < re ? rmasks[q] & rvm : 0ull;
          unsigned long long m = 0;
          if (rows) {
            const KV v = kv_load<EW>(rvals, q);
            const uint32_t h = fp_slot<EW>(v);
            const uint32_t x0 = s_slot[h];
            if (x0 != kFFree) {
              const uint32_t x = chain(v, h, x0);
              if (x != kFFree) m = s_em[x & 1023u];
            }
          }
          rows_add(m ? rows : 0ull, m, false);
        }
        __syncthreads();
        JSTAMP(4);
        cur = nxt;
        bs = nbs;
        be = nbe;
        cs = ncs;
        ce = nce;
      }
      wb = we;
    }
  }
  __syncthreads();
  // planes the carry chains reached (unrelated tiles: none or one)
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) top = max(top, (uint32_t)__shfl_xor(top, o, 64));
  if (lane == 0 && top) atomicMax(&s_top, top);
  __syncthreads();
  const int np = (int)s_top;
  for (uint32_t r = tid >> 6; r < kTile; r += kJB / 64) {  // a wave per row, a lane per column
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
    const uint64_t orow = rows_mode ? (gr - a.row_begin) : gr;
    atomicAdd(&a.out[orow * a.ld + gc], (int32_t)cnt);
  }
  // the mirror (j, i) of an off-diagonal symmetric tile: a wave per column, a lane
  // per row, so each wave's atomics fall on one output row (contiguous), as above.
  // (Round 2 added it in the loop above, lanes over columns: 64 rows, 64 lines
  // per wave instruction.  Config 5, 200 related genomes, every tile dense: whole
  // call 0.180 -> 0.125 ms; config 4 unchanged, most tiles sparse.)
  if (!a.packed && !rows_mode && I != J) {
    for (uint32_t c = tid >> 6; c < kTile; c += kJB / 64) {
      const uint32_t r = lane;
      uint32_t cnt = 0;
      for (int b = 0; b < np; ++b) cnt |= (uint32_t)((s_pl[b * kTile + r] >> c) & 1ull) << b;
      const uint32_t gr = row0 + r, gc = col0 + c;
      if (!cnt || gr >= row_lim || gc >= a.n) continue;
      atomicAdd(&a.out[(uint64_t)gc * a.ld + gr], (int32_t)cnt);
    }
  }
  JSTAMP(5);
  if (!a.ani) {
    JSTAMP_FLUSH();
    return;
  }
  // ---- fused containment / ANI: the tile's last workgroup converts it --------------------------
  // The counts are only ever written by device-scope atomics, which every
  // workgroup's result reaches at the device's coherence point (that is what
  // makes the cross-XCD sums right).  So the hand-off needs no release / acquire
  // fence — on gfx950 those write back and invalidate the whole XCD L2
  // (buffer_wbl2 / buffer_inv sc1), and 4352 of them per call cost ~1 ms: every
  // wave drains its atomics (s_waitcnt vmcnt(0)), the workgroup meets at a
  // barrier, one lane counts the workgroup done, and the workgroup that completes
  // the tile reads the counts back with sc1 loads (agent-scope atomic loads, past
  // the non-coherent L2s).  It writes both orientations of the tile's ANI: (r, c)
  // with lanes over columns and (c, r) with lanes over rows, so every wave's
  // stores are one contiguous 512-byte row segment of the n x n matrix (ani may
  // be pinned host memory: PCIe writes).
#if SKS_ANI_DIAG != 2  // (diagnostics 2: no drain; the counts the finisher reads may be short)
  __builtin_amdgcn_s_waitcnt(kWaitVmcnt0);
#endif
  __syncthreads();
  if (tid == 0)
    s_top = __hip_atomic_fetch_add(a.tile_done + (t - a.tile_begin), 1u, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT) + 1 == a.n_groups;
  __syncthreads();
#if SKS_ANI_DIAG == 1  // (diagnostics 1: the hand-off only, no conversion)
  if (s_top) return;
#endif
  if (!s_top) {
    JSTAMP(6);
    JSTAMP_FLUSH();
    return;
  }
  int32_t* s_cnt = reinterpret_cast<int32_t*>(s_slot);  // the table is free: 4096 counts
  for (uint32_t q = tid; q < (uint32_t)(kTile * kTile); q += kJB) {
    const uint32_t r = q / kTile, c = q % kTile, gr = row0 + r, gc = col0 + c;
    int32_t x = 0;
    if (gr < row_lim && gc < a.n) {
      const int32_t* p = a.packed ? a.out + (t - a.tile_begin) * (kTile * kTile) + q : a.out + (uint64_t)gr * a.ld + gc;
      x = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    s_cnt[q] = x;
  }
  __syncthreads();
  // a row whose set size has the root table (bottom-s sets: every row) reads
  // its value there; fp64 pow (~230 instructions) for 8192 cells per tile was
  // ~70 us of the call
  auto conv = [&](int32_t x, int32_t size) {
    return (a.root && (uint32_t)size == a.root_size && (uint32_t)x <= a.root_size) ? a.root[x]
                                                                                    : ani_of(x, size, a.inv_k, nullptr);
  };
  for (uint32_t r = tid >> 6; r < kTile; r += kJB / 64) {
    const uint32_t gr = row0 + r, gc = col0 + lane;
    if (gr < row_lim && gc < a.n) a.ani[(uint64_t)gr * a.n + gc] = conv(s_cnt[r * kTile + lane], a.sizes[gr]);
  }
  if (I != J) {
    for (uint32_t c = tid >> 6; c < kTile; c += kJB / 64) {
      const uint32_t gr = row0 + lane, gc = col0 + c;
      if (gr < row_lim && gc < a.n) a.ani[(uint64_t)gc * a.n + gr] = conv(s_cnt[lane * kTile + c], a.sizes[gc]);
    }
  }
  JSTAMP(6);
  JSTAMP_FLUSH();
}

template <int EW, bool CHECK, bool PIECES>
hipError_t launch_join_slices(JoinArgs ja, uint64_t tile_begin, uint64_t tile_end, bool packed, int32_t* out,
                              uint32_t* tile_done, hipStream_t s) {
  const uint64_t tiles_per_launch = std::max<uint64_t>(1, kMaxGrid / ja.n_groups);
  // diagonal tiles last: a symmetric launch of every tile (no tile list, one slice)
  const uint64_t all_sym = (uint64_t)ja.n_col_blocks * (ja.n_col_blocks + 1) / 2;
  ja.diag_last = ja.sym && !ja.tiles && tile_begin == 0 && tile_end == all_sym &&
                         tile_end <= tiles_per_launch && getenv("SKS_JOIN_TILE_ORDER") == nullptr
                     ? 1
                     : 0;
  for (uint64_t t0 = tile_begin; t0 < tile_end; t0 += tiles_per_launch) {
    const uint64_t nt = std::min(tiles_per_launch, tile_end - t0);
    ja.tile_begin = t0;
    if (packed) ja.out = out + (t0 - tile_begin) * (uint64_t)(kTile * kTile);
    if (ja.ani) ja.tile_done = tile_done + (t0 - tile_begin);
    hipLaunchKernelGGL((k_join<EW, CHECK, PIECES>), dim3((unsigned)(nt * ja.n_groups)), dim3(kJB), 0, s, ja);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
#ifdef SKS_JOIN_STAMPS
    {
      (void)hipStreamSynchronize(s);
      const uint64_t nw = std::min<uint64_t>(nt * ja.n_groups, kMaxJoinStampWgs);
      std::vector<unsigned long long> h(nw * 8);
      (void)hipMemcpyFromSymbol(h.data(), HIP_SYMBOL(g_join_stamps_wg), h.size() * 8);
      double sum[8] = {0};
      for (uint64_t b = 0; b < nw; ++b)
        for (int q = 0; q < 8; ++q) sum[q] += (double)h[b * 8 + q];
      fprintf(stderr, "[k_join stamps] %llu workgroups, cycles per workgroup: setup %.0f window %.0f stage %.0f "
              "insert %.0f probe+hits %.0f flush %.0f ani %.0f diagonal %.0f\n", (unsigned long long)nw,
              sum[0] / nw, sum[1] / nw, sum[2] / nw, sum[3] / nw, sum[4] / nw, sum[5] / nw, sum[6] / nw, sum[7] / nw);
    }
#endif
  }
  return hipSuccess;
}

}  // namespace

uint32_t join_cap() {  // SKS_JOIN_CAP (diagnostics) is clamped to [64, kJCap]
  static const uint32_t cap = std::max<uint32_t>(
      64, std::min<uint32_t>(kJCap, getenv("SKS_JOIN_CAP") ? (uint32_t)atoi(getenv("SKS_JOIN_CAP"))
                                                           : kJCap));
  return cap;
}

// Bucket count for the join: mean raw block-bucket population ~ cap / 6, so a
// chunk holds several whole buckets (fewer after deduplication).
uint32_t join_log_b(uint32_t max_size) {
  uint32_t log_b = 0;
  while ((1ull << log_b) * (join_cap() / 6) < 64ull * max_size && log_b < jc::kMaxLogB) ++log_b;
  return log_b;
}

unsigned long long join_check_take() {
  unsigned long long h = 0;
  (void)hipMemcpyFromSymbol(&h, HIP_SYMBOL(g_join_check), sizeof h);
  const unsigned long long z = 0;
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_join_check), &z, sizeof z);
  return h;
}

hipError_t join_launch(const JoinLayout& rows, uint32_t r_blk0, const JoinLayout& cols, uint32_t c_blk0,
                       uint32_t n, uint32_t log_b, int ew, bool sym, uint32_t row_begin, uint32_t row_end,
                       uint64_t tile_begin, uint64_t tile_end, const uint32_t* d_tiles, bool packed,
                       int32_t* out, bool check, hipStream_t s, const JoinAni* ani, int layout_rg) {
  if (log_b > jc::kMaxLogB || (ew != 1 && ew != 2)) return hipErrorInvalidValue;
  if (ani && !sym && !d_tiles) return hipErrorInvalidValue;  // ANI of whole tiles only
  const uint32_t n_cb = (n + kTile - 1) / kTile;
  const uint32_t n_rb = sym ? n_cb : (row_end - row_begin + kTile - 1) / kTile;
  if (!d_tiles) {
    const uint64_t all_tiles = sym ? (uint64_t)n_cb * (n_cb + 1) / 2 : (uint64_t)n_rb * n_cb;
    if (!sym) { tile_begin = 0; tile_end = all_tiles; }
    tile_end = std::min(tile_end, all_tiles);
  }
  if (tile_begin >= tile_end) return hipSuccess;
  const uint64_t tiles = tile_end - tile_begin;
  const uint32_t B = 1u << log_b;
  JoinArgs ja{};
  ja.r = rows;
  ja.c = cols;
  ja.r_blk0 = r_blk0;
  ja.c_blk0 = c_blk0;
  ja.tiles = d_tiles;
  ja.packed = packed ? 1 : 0;
  ja.log_b = log_b;
  ja.B = B;
  ja.BW = jc::lay_boff_words(log_b);
  ja.n = n;
  ja.n_col_blocks = n_cb;
  ja.sym = (sym || d_tiles) ? 1 : 0;
  ja.row_begin = row_begin;
  ja.row_end = row_end;
  ja.out = out;
  ja.ld = n;
  ja.cap = std::min<uint32_t>(join_cap(), ew == 2 ? (uint32_t)jcap<2>() : (uint32_t)jcap<1>());
  if (ani) {
    ja.ani = ani->ani;
    ja.sizes = ani->sizes;
    ja.inv_k = ((double)1.0) / ((double)ani->kmer_num_ones);
    ja.root = ani->root;
    ja.root_size = ani->root_size;
  }
  uint32_t* tile_done = ani ? ani->tile_done : nullptr;
  // bucket groups per tile: ~128 buckets per workgroup (a workgroup's start-up —
  // clearing its table and count planes — and its count flush, up to 4096 global
  // atomics on a tile of related genomes, are then small beside its chunks), at
  // least ~1024 workgroups in all, at least 16 buckets each (round 3 sweep,
  // config 4: 4352 workgroups 0.681 ms against 2176: 0.705, 8704: 0.742).
  // SKS_JOIN_WGS (diagnostics) sets the total instead.  The ~128-buckets floor
  // only applies while the grid is small (<= 64K workgroups); with very many
  // tiles a tile gets fewer, larger groups (down to one).
  static const uint64_t wgs_env = getenv("SKS_JOIN_WGS") ? strtoull(getenv("SKS_JOIN_WGS"), 0, 10) : 0;
  uint64_t want = wgs_env ? (wgs_env + tiles - 1) / tiles
                          : std::max<uint64_t>(std::min<uint64_t>((B + 127) / 128, (65536 + tiles - 1) / tiles),
                                               (1024 + tiles - 1) / tiles);
  if (!wgs_env) want = std::min<uint64_t>(want, std::max<uint32_t>(1, B / 16));
  const uint32_t groups = (uint32_t)std::min<uint64_t>(B, std::max<uint64_t>(1, want));
  ja.buckets_per_group = (B + groups - 1) / groups;
  ja.n_groups = (B + ja.buckets_per_group - 1) / ja.buckets_per_group;
  // windows across regions (PIECES) unless both layouts have 64-bucket regions:
  // known only for one layout covering all n sketches (the build picks its
  // region size from its block count, join_layout_region_log); a tile list
  // joins per-rank layouts, small ones
  const bool one_layout = rows.vals == cols.vals && rows.boff == cols.boff;
  const bool big = (!d_tiles && r_blk0 == 0 && c_blk0 == 0 && one_layout &&
                    jc::lay_rb_log(log_b, join_layout_region_log(n_cb, log_b)) >= (uint32_t)kJWinLog) ||
                   (layout_rg >= 0 && one_layout && jc::lay_rb_log(log_b, (uint32_t)layout_rg) >= (uint32_t)kJWinLog);
  const bool pieces = !big;
#define SKS_JOIN_LAUNCH(E, C, P) launch_join_slices<E, C, P>(ja, tile_begin, tile_end, packed, out, tile_done, s)
  if (ew == 1) {
    if (pieces) return check ? SKS_JOIN_LAUNCH(1, true, true) : SKS_JOIN_LAUNCH(1, false, true);
    return check ? SKS_JOIN_LAUNCH(1, true, false) : SKS_JOIN_LAUNCH(1, false, false);
  }
  if (pieces) return check ? SKS_JOIN_LAUNCH(2, true, true) : SKS_JOIN_LAUNCH(2, false, true);
  return check ? SKS_JOIN_LAUNCH(2, true, false) : SKS_JOIN_LAUNCH(2, false, false);
#undef SKS_JOIN_LAUNCH
}

SKS_CODE_OBJECT_HOOK(join)

}  // namespace sks
