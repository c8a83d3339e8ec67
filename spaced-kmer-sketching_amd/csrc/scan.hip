// Kernel 1 — fused spaced-seed sketch scan for gfx950.
//
// One pass over the sequence bytes computes, for every window start, exactly
// what the reference's hot loop computes (kmer_sliding.cpp:112-186):
//   forward window F  (kmer_sliding.cpp:26-31:  F <<= 2; F[0..1] = base)
//   reverse-complement window R (:42-47: R >>= 2; R[2w-2..2w-1] = base ^ 3)
//   canonical C = min(F & M, R & M), ties -> R & M (same value)   (:159-175)
//   fmh = H(C) ^ H(M) ^ w ^ nonce   (kmer.hpp:141-148, boost hash flavour)
// and applies the selection policy (FracMinHash `fmh % c == 0`, or the
// bottom-s pre-filter `fmh <= threshold`) in the same kernel.  List mode
// (nucleotide_string_list_to_kmers) applies the FracMinHash test and emits the
// window's start position instead of the k-mer (materialised later in order).  Bytes that are
// not A/C/G/T (either case) split runs exactly like
// fasta_processing.cpp:144-179; a window is valid iff all its w bytes are
// ACGT and lie inside its segment, so k-mers never span runs or genomes.
//
// Structure (MI355X): persistent grid, each workgroup streams a contiguous
// range of 4096-window tiles.  A tile's bytes arrive with 16-B coalesced
// loads (prefetched one tile ahead into registers), are packed once into
// 2-bit words in LDS (a big-endian stream for F, a complemented little-endian
// stream for R, a 1-bit invalid map), and every lane then owns 16 consecutive
// window starts, extracting F and R with funnel shifts (v_alignbit_b32).
// Survivors (~1/c of windows) go to an LDS queue flushed with one global
// atomic per flush, so the global counters see a few thousand atomics per
// launch instead of one per survivor.
#include <hip/hip_runtime.h>

#include <cstdlib>

#include <cstdint>
#include <type_traits>

#include "sks_hash.hpp"
#include "sks_internal.hpp"

namespace sks {

namespace {

constexpr int kBlock = 256;
constexpr int kWPT = 16;                  // windows per lane
constexpr int kTile = kBlock * kWPT;      // 4096 window starts per tile
constexpr int kHaloWords = 4;             // 64 extra bases (>= w - 1 for w <= 64)
constexpr int kWords = kBlock + kHaloWords;            // 2-bit words per tile (16 bases each)
constexpr int kLoadVecs = (kWords * 16 + 16) / 16;      // 16-B loads per tile (+1 for alignment)
constexpr int kQCap = 2048;               // LDS survivor queue entries (list mode, wide path)
#ifndef SKS_SCAN_QCAP
#define SKS_SCAN_QCAP 512
#endif
// FracMinHash keeps ~1/c of the windows and bottom-s ~s/L (a few per tile), so a
// small queue suffices there and leaves LDS for more workgroups per CU; list
// mode (every selected window, c = 1 keeps all) keeps the large one.
template <int MODE>
constexpr int qcap() { return MODE == kModeList ? kQCap : SKS_SCAN_QCAP; }
constexpr unsigned char kSep = '\n';      // any non-ACGT byte

struct Geom {
  uint64_t win0;    // byte index of the tile's first window start
  uint64_t seg_end; // end byte of the segment
  uint32_t seg;
};

// Scalar (wave-uniform) segment cursor: advance `seg` until tile is inside it.
__device__ __forceinline__ Geom tile_geom(const ScanParams& p, uint64_t tile, uint32_t& seg) {
  while (seg + 1 < p.n_seg && tile >= p.tile_prefix[seg + 1]) ++seg;
  Geom g;
  g.seg = seg;
  g.win0 = p.seg_begin[seg] + (tile - p.tile_prefix[seg]) * (uint64_t)kTile;
  g.seg_end = p.seg_end[seg];
  return g;
}

// Load the 16-B vector #k of a tile: bytes [base + 16k, base + 16k + 16) where
// `base` (relative to seq, possibly negative) is 16-B aligned in absolute
// address terms, so every vector load is aligned even when the caller's
// sequence pointer is not.  Bytes at or past seg_end read as a separator.
__device__ __forceinline__ uint4 load_vec(const uint8_t* __restrict__ seq, int64_t base, int k,
                                          int64_t seg_end) {
  int64_t a = base + 16 * (int64_t)k;
  if (a + 16 <= seg_end) return *reinterpret_cast<const uint4*>(seq + a);
  uint32_t wv[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    uint32_t v = 0;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      int64_t pos = a + 4 * q + b;
      uint32_t ch = pos < seg_end ? seq[pos] : kSep;
      v |= ch << (8 * b);
    }
    wv[q] = v;
  }
  return make_uint4(wv[0], wv[1], wv[2], wv[3]);
}

// Offset of win0 inside its absolutely aligned 16-B chunk.
__device__ __forceinline__ uint32_t align_shift(const uint8_t* seq, uint64_t win0) {
  return (uint32_t)(((uintptr_t)seq + win0) & 15u);
}

// 4 ASCII bytes -> 8 bits of little-endian 2-bit codes + 4 invalid bits.
// code = ((c >> 1) ^ (c >> 2)) & 3 maps A/a C/c G/g T/t to 0 1 2 3
// (fasta_processing.cpp:35-69); a byte is valid iff it equals "acgt"[code]
// after lower-casing.
__device__ __forceinline__ void encode4(uint32_t x, uint32_t& le8, uint32_t& inv4) {
  uint32_t low = x | 0x20202020u;
  uint32_t code = ((low >> 1) ^ (low >> 2)) & 0x03030303u;
  uint32_t expect = __builtin_amdgcn_perm(0u, 0x74676361u, code);  // bytes 'a','c','g','t'
  uint32_t eq = expect ^ low;
  uint32_t t = (eq & 0x7F7F7F7Fu) + 0x7F7F7F7Fu;
  t = ~(t | eq | 0x7F7F7F7Fu);             // 0x80 in every byte where eq == 0
  uint32_t bad = (~t) & 0x80808080u;       // 0x80 in every invalid byte
  inv4 = (bad * 0x00204081u) >> 28;        // gather bits 7,15,23,31 -> 0..3
  uint32_t y = code | (code >> 6);
  le8 = (y | (y >> 12)) & 0xFFu;
}

__device__ __forceinline__ uint32_t funnel(uint32_t hi, uint32_t lo, uint32_t s) {
  return __builtin_amdgcn_alignbit(hi, lo, s);
}

// 16 ASCII bytes (x[0..4] funnel-shifted by sb bits) -> 32 bits of
// little-endian 2-bit codes (base k at bits 2k) and a 16-bit invalid map.
// Fast path: per dword, the 4 codes are gathered into bits 24..31 by one
// multiply (c0 + c1<<2 + c2<<4 + c3<<6: the cross products land below bit 24
// without overlapping), and validity of all 4 bytes is one v_sad_u8 against
// the expected lower-case letters.  Only a 16-base word holding a non-ACGT
// byte pays for the exact per-byte invalid bits (encode4).
// ALIGNED: the tile's bytes start on a dword boundary (sb == 0, wave-uniform;
// a genome starting at a 4-byte multiple, e.g. config 3), so the dwords are
// used as they are and the four alignbits go.
template <bool ALIGNED>
__device__ __forceinline__ void pack16(const uint32_t (&x)[5], uint32_t sb, uint32_t& le,
                                       uint32_t& inv) {
  uint32_t w[4], g[4], sad = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    w[k] = ALIGNED ? x[k] : funnel(x[k + 1], x[k], sb);
    const uint32_t low = w[k] | 0x20202020u;
    const uint32_t code = ((low >> 1) ^ (low >> 2)) & 0x03030303u;
    const uint32_t expect = __builtin_amdgcn_perm(0u, 0x74676361u, code);
    sad = __builtin_amdgcn_sad_u8(low, expect, sad);
    g[k] = code * 0x01041040u;  // gathered codes in bits 24..31
  }
  // bytes 3 of g[0..3] -> bytes 0..3 of le
  const uint32_t g01 = __builtin_amdgcn_perm(g[1], g[0], 0x0c0c0703u);
  const uint32_t g23 = __builtin_amdgcn_perm(g[3], g[2], 0x0c0c0703u);
  le = __builtin_amdgcn_perm(g23, g01, 0x05040100u);
  inv = 0;
  if (sad) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      uint32_t le8, inv4;
      encode4(w[k], le8, inv4);
      inv |= inv4 << (4 * k);
    }
  }
}

__device__ __forceinline__ uint32_t rev_pairs(uint32_t x) {
  uint32_t r = __builtin_bitreverse32(x);
  return ((r >> 1) & 0x55555555u) | ((r & 0x55555555u) << 1);
}


template <int MODE>
struct Queue {
  uint64_t key[qcap<MODE>()];
  uint64_t val[MODE == kModeBottom ? qcap<MODE>() : 1];
  uint32_t n;
  unsigned long long base;
  unsigned long long wins;  // windows of the current segment not yet published
};

template <int MODE>
__device__ __forceinline__ void emit(const ScanParams& p, Queue<MODE>& q, uint32_t seg,
                                     uint64_t key, uint64_t val) {
  uint32_t slot = atomicAdd(&q.n, 1u);
  if (slot < (uint32_t)qcap<MODE>()) {
    q.key[slot] = key;
    if constexpr (MODE == kModeBottom) q.val[slot] = val;
  } else {  // queue full: rare direct path
    unsigned long long g = atomicAdd(&p.seg_count[seg], 1ull);
    if (g < p.seg_out_cap[seg]) {
      uint64_t o = p.seg_out_off[seg] + g;
      p.out_key[o] = key;
      if constexpr (MODE == kModeBottom) p.out_val[o] = val;
    }
  }
}

// Block-wide flush of the LDS queue to segment `seg` (call from all threads).
template <int MODE>
__device__ __forceinline__ void flush(const ScanParams& p, Queue<MODE>& q, uint32_t seg) {
  __syncthreads();
  // the workgroup's window count: one global atomic per flush, not one per
  // wave — when a small input gives every workgroup one tile, all of them
  // finish together and the segment's counter word serialises the atomics
  // (one word takes ~88 per microsecond, MI355X_MICROARCH.md "dequeue")
  if (threadIdx.x == 0 && q.wins) atomicAdd(&p.seg_windows[seg], q.wins);
  constexpr uint32_t cap = qcap<MODE>();
  uint32_t n = q.n < cap ? q.n : cap;
  if (n) {
    if (threadIdx.x == 0) q.base = atomicAdd(&p.seg_count[seg], (unsigned long long)n);
    __syncthreads();
    uint64_t base = q.base;
    uint64_t cap = p.seg_out_cap[seg];
    uint64_t off = p.seg_out_off[seg];
    for (uint32_t i = threadIdx.x; i < n; i += kBlock) {
      if (base + i < cap) {
        p.out_key[off + base + i] = q.key[i];
        if constexpr (MODE == kModeBottom) p.out_val[off + base + i] = q.val[i];
      }
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    q.n = 0;
    q.wins = 0;
  }
  __syncthreads();
}

// Windows hashed by this thread for the current segment -> the workgroup's
// LDS total (published by the next flush of that segment).
__device__ __forceinline__ void add_windows(unsigned long long& wins, uint32_t cnt) {
  uint32_t v = cnt;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  if ((threadIdx.x & 63) == 0 && v) atomicAdd(&wins, (unsigned long long)v);
}

// frac_min_hash of a canonical k-mer (w <= 32, so the high block is 0).
template <int FLAVOUR>
__device__ __forceinline__ uint64_t fmh_narrow(const ScanParams& p, uint64_t c) {
  uint64_t h;
  if constexpr (FLAVOUR == 0) {
    h = hash_mix(c + kGolden32);                // combine(0, lo)
    h = hash_mix(h + kGolden32);                // combine(h, hi = 0)
    h = hash_mix(h + (128 + kGolden32));        // combine(num_bits = 128, h)
  } else {
    h = hash_bitset128<1>(c, 0);
  }
  return h ^ p.kconst;
}

// Flavour B up to the third hash_mix's second multiply: h = mix(mix(c+K)+K);
// x = h + 128 + K; x ^= x >> 32; x *= M; x ^= x >> 32. The rest of the hash
// is H = y ^ (y >> 28) with y = x * M, and fmh = H ^ kconst. The low 4 bits
// of H need only the low 32 bits of y, i.e. one v_mul_lo_u32 (low-bits
// pre-filter of the FracMinHash test, scan_kernel<..., PRE = 1>).
__device__ __forceinline__ uint64_t mix3_head(uint64_t c) {
  uint64_t h = hash_mix(c + kGolden32);
  h = hash_mix(h + kGolden32);
  uint64_t x = h + (128 + kGolden32);
  x ^= x >> 32;
  x = mul_const<kMixMul>(x);
  return x ^ (x >> 32);
}

template <int MODE>
__device__ __forceinline__ bool keep_fmh(const ScanParams& p, uint64_t f, uint64_t thresh) {
  if constexpr (MODE != kModeBottom) return div_test(f, p.low_mask, p.high_mask, p.dinv, p.dlim);
  else return f <= thresh;
}

constexpr int kBeOff = 2;  // s_be[kBeOff + i] = word i; two zero words in front

#ifndef SKS_SCAN_MIN_WAVES
#define SKS_SCAN_MIN_WAVES 1
#endif

constexpr uint32_t kCandCap = 128;  // pre-filter candidates per wave (< 64 + 64)

template <int MODE, int FLAVOUR, int PRE = 0>
__global__ __launch_bounds__(kBlock, SKS_SCAN_MIN_WAVES) void scan_kernel(ScanParams p) {
  __shared__ uint32_t s_raw[kLoadVecs * 4];
  __shared__ uint32_t s_be[kWords + 2 + kBeOff];
  __shared__ uint32_t s_lc[kWords + 2];
  __shared__ uint32_t s_inv[kWords + 2];
  __shared__ Queue<MODE> q;
  // (z, c) of windows past the low-bits pre-filter, per wave (PRE only)
  __shared__ ulonglong2 s_cand[PRE ? (kBlock / 64) * kCandCap : 1];

  __shared__ unsigned long long s_next;  // dynamic tiles: the next chunk's first tile

  const int tid = threadIdx.x;
  // Tiles: static — workgroup b streams the contiguous range b·T/grid ..; or
  // dynamic (p.tile_queue) — a persistent grid whose workgroups take chunks of
  // p.chunk consecutive tiles, the first one b·chunk, the rest from one global
  // counter, so no workgroup is left with a range when the others are done
  // (a static range's tail is up to one range: ~1/16 of the kernel).  A chunk's
  // grab is issued by thread 0 at its first tile and published through LDS at
  // its last, so the atomic's latency hides behind the chunk's tiles.
  const bool dyn = p.tile_queue != nullptr;
  uint64_t t_begin, t_end;
  if (dyn) {
    t_begin = (uint64_t)blockIdx.x * p.chunk;
    t_end = min(t_begin + p.chunk, p.n_tiles);
  } else {
    t_begin = (uint64_t)blockIdx.x * p.n_tiles / gridDim.x;
    t_end = (uint64_t)(blockIdx.x + 1) * p.n_tiles / gridDim.x;
  }
  if (tid == 0) {
    q.n = 0;
    q.wins = 0;
  }
  if (t_begin >= t_end) return;
  unsigned long long grab = 0;  // thread 0: the pending chunk grab

  const int w = p.w;
  // F of the window at base b is read as the 64 big-endian bits starting at
  // base b - (32 - w): its low 2w bits are F, the bits above are older bases
  // that the mask (bits < 2w) removes, so no per-window shift is needed.
  const uint32_t dshift = 2 * (32 - w);          // 0..62 bits
  const bool dword = dshift >= 32;
  const uint32_t dbits = dshift & 31;
  const uint64_t wmask_bits = (w >= 64) ? ~0ull : ((1ull << w) - 1);
  const uint64_t region_bits = (kWPT - 1 + w >= 64) ? ~0ull : ((1ull << (kWPT - 1 + w)) - 1);
  if (tid < kBeOff) s_be[tid] = 0;

  // segment cursors (wave-uniform) for the current tile and the prefetch
  uint32_t seg_lo = 0, seg_hi = p.n_seg;
  while (seg_lo + 1 < seg_hi) {  // last segment with tile_prefix[seg] <= t_begin
    uint32_t mid = (seg_lo + seg_hi) >> 1;
    if (p.tile_prefix[mid] <= t_begin) seg_lo = mid; else seg_hi = mid;
  }
  uint32_t cur_seg = seg_lo, pf_seg = seg_lo;

  // prefetch the first tile
  Geom pg = tile_geom(p, t_begin, pf_seg);
  int64_t pf_base = (int64_t)pg.win0 - align_shift(p.seq, pg.win0);
  uint4 v0 = load_vec(p.seq, pf_base, tid, (int64_t)pg.seg_end);
  uint4 v1 = make_uint4(0, 0, 0, 0);
  if (tid < kLoadVecs - kBlock) v1 = load_vec(p.seq, pf_base, kBlock + tid, (int64_t)pg.seg_end);

  uint32_t win_count = 0;
  uint32_t count_seg = cur_seg;

  for (uint64_t tile = t_begin; tile < t_end;) {
    Geom g = tile_geom(p, tile, cur_seg);
    if (g.seg != count_seg) {  // segment change: publish the previous segment
      add_windows(q.wins, win_count);
      win_count = 0;
      flush<MODE>(p, q, count_seg);
      count_seg = g.seg;
    }
    const uint32_t shift = align_shift(p.seq, g.win0);
    const uint64_t thresh = (MODE == kModeBottom) ? p.seg_thresh[g.seg] : 0;
    const bool last_of_chunk = tile + 1 == t_end;
    if (dyn && tid == 0) {
      if (tile == t_begin)
        grab = (unsigned long long)gridDim.x * p.chunk + atomicAdd(p.tile_queue, (unsigned long long)p.chunk);
      if (last_of_chunk) s_next = grab;
    }

    // 1) raw bytes -> LDS
    reinterpret_cast<uint4*>(s_raw)[tid] = v0;
    if (tid < kLoadVecs - kBlock) reinterpret_cast<uint4*>(s_raw)[kBlock + tid] = v1;
    __syncthreads();
    // the next tile: the chunk's next, else the next chunk's first (read here,
    // after the barrier; s_next is rewritten only at the next chunk's last tile)
    const uint64_t next_tile = !last_of_chunk ? tile + 1 : dyn ? (uint64_t)s_next : p.n_tiles;

    // 2) pack: word i covers bases [16 i, 16 i + 16) of the tile
    {
      const uint32_t sb = (shift & 3) * 8;  // wave-uniform
      auto pack_words = [&](auto aligned) {
        for (int i = tid; i < kWords; i += kBlock) {
          const uint32_t wi = (16 * i + shift) >> 2;  // dword offset in s_raw
          uint32_t x[5];
#pragma unroll
          for (int k = 0; k < 5; ++k) x[k] = (decltype(aligned)::value && k == 4) ? 0u : s_raw[wi + k];
          uint32_t le, inv;
          pack16<decltype(aligned)::value>(x, sb, le, inv);
          s_be[kBeOff + i] = rev_pairs(le);
          s_lc[i] = ~le;
          s_inv[i] = inv;
        }
      };
      if (sb == 0) pack_words(std::true_type{});
      else pack_words(std::false_type{});
    }
    __syncthreads();

    // 3) prefetch the next tile while this one is hashed
    if (next_tile < (dyn ? p.n_tiles : t_end)) {
      Geom ng = tile_geom(p, next_tile, pf_seg);
      pf_base = (int64_t)ng.win0 - align_shift(p.seq, ng.win0);
      v0 = load_vec(p.seq, pf_base, tid, (int64_t)ng.seg_end);
      if (tid < kLoadVecs - kBlock) v1 = load_vec(p.seq, pf_base, kBlock + tid, (int64_t)ng.seg_end);
    }

    // 4) 16 windows per lane: starts 16*tid + j
    uint32_t be[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) be[k] = s_be[kBeOff + tid - 2 + k];  // words tid-2 .. tid+2
    uint32_t bs[3];  // BE words shifted back by (32 - w) bases
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const uint32_t hi = dword ? be[k] : be[k + 1];
      const uint32_t lo = dword ? be[k + 1] : be[k + 2];
      bs[k] = funnel(hi, lo, dbits);
    }
    const uint32_t lc0 = s_lc[tid], lc1 = s_lc[tid + 1], lc2 = s_lc[tid + 2];
    const uint64_t inv64 = (uint64_t)s_inv[tid] | ((uint64_t)s_inv[tid + 1] << 16) |
                           ((uint64_t)s_inv[tid + 2] << 32) | ((uint64_t)s_inv[tid + 3] << 48);
    const bool lane_clean = (inv64 & region_bits) == 0;
    // canonical masked k-mer of window j (runtime j allowed)
    auto canon = [&](uint32_t j) -> uint64_t {
      const uint32_t fh = j ? funnel(bs[0], bs[1], 32 - 2 * j) : bs[0];
      const uint32_t fl = j ? funnel(bs[1], bs[2], 32 - 2 * j) : bs[1];
      const uint64_t F = (((uint64_t)fh) << 32) | fl;
      const uint32_t rl = j ? funnel(lc1, lc0, 2 * j) : lc0;
      const uint32_t rh = j ? funnel(lc2, lc1, 2 * j) : lc1;
      const uint64_t R = (((uint64_t)rh) << 32) | rl;
      const uint64_t fm = F & p.mask_lo, rm = R & p.mask_lo;
      return fm < rm ? fm : rm;
    };
    // Hot loop: no branches — one keep bit per window, so the compiler can
    // interleave the 16 independent hash chains.  Survivors (~1/c) are
    // re-derived and emitted afterwards.
    if constexpr (PRE) {
      // FracMinHash with an even c: a window survives only if the low
      // min(s, 4) bits of its fmh are zero, and those follow from the low 32
      // bits of the last multiply. Windows passing that test (1/8 for c = 1000)
      // are queued per wave in LDS and finished 64 at a time, all lanes busy.
      const int lane = tid & 63;
      // the wave's candidate buffer, wave-uniform: readfirstlane keeps it in an
      // SGPR so a candidate's LDS address is one v_lshl_add_u32 of its rank
      ulonglong2* cb = s_cand + __builtin_amdgcn_readfirstlane(tid >> 6) * kCandCap;
      const uint32_t pmask = p.low_mask & 0xFu;
      const uint32_t kbits = (uint32_t)p.kconst & pmask;
      // low bits of c = 2^s * d the pre-filter has not tested (none when s <= 4):
      // a finished candidate needs only d | fmh then
      const uint32_t rest_lo = p.low_mask & ~0xFu, rest_hi = p.high_mask;
      uint32_t cnt = 0;  // wave-uniform
      auto finish = [&](uint32_t n) {  // candidates [0, n), n <= 64
        __builtin_amdgcn_wave_barrier();
        if ((uint32_t)lane < n) {
          const ulonglong2 e = cb[lane];
          uint64_t y = mul_const<kMixMul>(e.x);
          y ^= y >> 28;
          const uint64_t f = y ^ p.kconst;
          bool keep = mul_uniform(f, p.dinv) <= p.dlim;
          if (rest_lo | rest_hi)  // wave-uniform
            keep = keep && ((((uint32_t)f & rest_lo) | ((uint32_t)(f >> 32) & rest_hi)) == 0);
          if (keep) emit<MODE>(p, q, g.seg, e.y, 0);
        }
        __builtin_amdgcn_wave_barrier();
      };
      auto window_pre = [&](auto checked, int j) {
          const uint64_t c = canon(j);
          const uint64_t z = mix3_head(c);
          const uint32_t ylo = (uint32_t)z * (uint32_t)kMixMul;
          bool pass = ((ylo ^ (ylo >> 28)) & pmask) == kbits;
          if constexpr (decltype(checked)::value) {
            const bool valid = ((inv64 >> j) & wmask_bits) == 0;
            win_count += valid ? 1u : 0u;
            pass = pass && valid;
          }
          const uint64_t bal = __ballot(pass);
          const uint32_t below = __builtin_amdgcn_mbcnt_hi(
              (uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
          if (pass) cb[cnt + below] = make_ulonglong2(z, c);
          cnt += (uint32_t)__popcll(bal);
          if (cnt >= 64) {
            finish(64);
            const uint32_t rest = cnt - 64;  // < 64: move them to the front
            ulonglong2 t = make_ulonglong2(0, 0);
            if ((uint32_t)lane < rest) t = cb[64 + lane];
            __builtin_amdgcn_wave_barrier();
            if ((uint32_t)lane < rest) cb[lane] = t;
            cnt = rest;
          }
      };
      if (__all(lane_clean)) {
#pragma unroll
        for (int j = 0; j < kWPT; ++j) window_pre(std::false_type{}, j);
        win_count += kWPT;
      } else {  // waves holding an invalid base: rare, kept out of the unrolled code
#pragma unroll 1
        for (int j = 0; j < kWPT; ++j) window_pre(std::true_type{}, j);
      }
      if (cnt) finish(cnt);
    } else {
    uint32_t keepmask = 0;
    // bottom-s, flavour B: the candidate test only needs fmh's top 28 bits, which
    // are the top bits of the last product y (H = y ^ (y >> 28) changes only
    // bits < 36), so the xor-shift, the constant and the 64-bit compare go; a
    // window whose top 28 bits equal the threshold's passes even if fmh > T (a
    // superset of candidates: the post-processing selects exactly)
    const uint32_t thr_top = (uint32_t)(thresh >> 36);
    const uint32_t k_top = (uint32_t)(p.kconst >> 32);
    auto keep_window = [&](uint64_t c) -> bool {
      if constexpr (MODE == kModeBottom && FLAVOUR == 0) {
        const uint64_t y = mul_const<kMixMul>(mix3_head(c));
        return (((uint32_t)(y >> 32) ^ k_top) >> 4) <= thr_top;
      } else {
        return keep_fmh<MODE>(p, fmh_narrow<FLAVOUR>(p, c), thresh);
      }
    };
    if (__all(lane_clean)) {
#pragma unroll
      for (int j = 0; j < kWPT; ++j) keepmask |= (keep_window(canon(j)) ? 1u : 0u) << j;
      win_count += kWPT;
    } else {  // waves holding an invalid base: rare, kept out of the unrolled code
#pragma unroll 1
      for (int j = 0; j < kWPT; ++j) {
        const bool valid = ((inv64 >> j) & wmask_bits) == 0;
        win_count += valid ? 1u : 0u;
        keepmask |= (keep_window(canon(j)) && valid ? 1u : 0u) << j;
      }
    }
    while (keepmask) {
      const uint32_t j = __builtin_ctz(keepmask);
      keepmask &= keepmask - 1;
      if constexpr (MODE == kModeList) {
        emit<MODE>(p, q, g.seg, g.win0 + (uint64_t)(kWPT * tid) + j, 0);  // window start byte
      } else {
        const uint64_t c = canon(j);
        // bottom-s: the candidate's fmh is recomputed after compaction
        // (launch_fmh_narrow) instead of here, where the whole wave would wait
        // on the ~45-VALU hash for the ~5% of lanes holding a candidate
        if constexpr (MODE == kModeFrac) emit<MODE>(p, q, g.seg, c, 0);
        else emit<MODE>(p, q, g.seg, c, c);
      }
    }
    }  // !PRE

    // 5) flush the queue once it is half full
    __syncthreads();
    if (q.n >= (uint32_t)qcap<MODE>() / 2) {
      add_windows(q.wins, win_count);
      win_count = 0;
      flush<MODE>(p, q, g.seg);
    }
    if (!last_of_chunk) {
      ++tile;
    } else if (dyn) {  // next chunk (every thread holds the same next_tile): exits past n_tiles
      t_begin = tile = next_tile;
      t_end = min(next_tile + p.chunk, p.n_tiles);
    } else {
      break;
    }
  }
  add_windows(q.wins, win_count);
  flush<MODE>(p, q, count_seg);
}

// ---- wide path: 32 < w <= 64 (128-bit windows) -------------------------------------
// Same structure; F and R are 128-bit.  Survivors carry (lo, hi) in (key, val)
// for FracMinHash and (fmh, lo) + hi in a side array for bottom-s.
template <int MODE, int FLAVOUR>
__global__ __launch_bounds__(kBlock) void scan_kernel_wide(ScanParams p) {
  __shared__ uint32_t s_raw[kLoadVecs * 4];
  __shared__ uint32_t s_be[kWords + 2];
  __shared__ uint32_t s_lc[kWords + 2];
  __shared__ uint32_t s_inv[kWords + 2];
  __shared__ uint64_t q_a[kQCap / 2], q_b[kQCap / 2], q_c[kQCap / 2];
  __shared__ uint32_t q_n;
  __shared__ unsigned long long q_base, q_wins;

  const int tid = threadIdx.x;
  const uint64_t t_begin = (uint64_t)blockIdx.x * p.n_tiles / gridDim.x;
  const uint64_t t_end = (uint64_t)(blockIdx.x + 1) * p.n_tiles / gridDim.x;
  if (tid == 0) {
    q_n = 0;
    q_wins = 0;
  }
  if (t_begin >= t_end) return;
  constexpr uint32_t cap = kQCap / 2;

  const int w = p.w;
  const uint32_t fshift = 128 - 2 * w;  // 0..62
  const uint64_t wmask_bits = (w >= 64) ? ~0ull : ((1ull << w) - 1);

  uint32_t seg_lo = 0, seg_hi = p.n_seg;
  while (seg_lo + 1 < seg_hi) {
    uint32_t mid = (seg_lo + seg_hi) >> 1;
    if (p.tile_prefix[mid] <= t_begin) seg_lo = mid; else seg_hi = mid;
  }
  uint32_t cur_seg = seg_lo, pf_seg = seg_lo;
  Geom pg = tile_geom(p, t_begin, pf_seg);
  int64_t pf_base = (int64_t)pg.win0 - align_shift(p.seq, pg.win0);
  uint4 v0 = load_vec(p.seq, pf_base, tid, (int64_t)pg.seg_end);
  uint4 v1 = make_uint4(0, 0, 0, 0);
  if (tid < kLoadVecs - kBlock) v1 = load_vec(p.seq, pf_base, kBlock + tid, (int64_t)pg.seg_end);
  uint32_t win_count = 0;
  uint32_t count_seg = cur_seg;

  auto wflush = [&](uint32_t seg) {
    __syncthreads();
    if (tid == 0 && q_wins) atomicAdd(&p.seg_windows[seg], q_wins);
    uint32_t n = q_n < cap ? q_n : cap;
    if (n) {
      if (tid == 0) q_base = atomicAdd(&p.seg_count[seg], (unsigned long long)n);
      __syncthreads();
      uint64_t base = q_base, c = p.seg_out_cap[seg], off = p.seg_out_off[seg];
      for (uint32_t i = tid; i < n; i += kBlock)
        if (base + i < c) {
          p.out_key[off + base + i] = q_a[i];
          if (MODE != kModeList) p.out_val[off + base + i] = q_b[i];
          if (MODE == kModeBottom) p.out_hi[off + base + i] = q_c[i];
        }
    }
    __syncthreads();
    if (tid == 0) {
      q_n = 0;
      q_wins = 0;
    }
    __syncthreads();
  };

  for (uint64_t tile = t_begin; tile < t_end; ++tile) {
    Geom g = tile_geom(p, tile, cur_seg);
    if (g.seg != count_seg) {
      add_windows(q_wins, win_count);
      win_count = 0;
      wflush(count_seg);
      count_seg = g.seg;
    }
    const uint32_t shift = align_shift(p.seq, g.win0);
    const uint64_t thresh = (MODE == kModeBottom) ? p.seg_thresh[g.seg] : 0;
    reinterpret_cast<uint4*>(s_raw)[tid] = v0;
    if (tid < kLoadVecs - kBlock) reinterpret_cast<uint4*>(s_raw)[kBlock + tid] = v1;
    __syncthreads();
    for (int i = tid; i < kWords; i += kBlock) {
      const uint32_t b0 = 16 * i + shift;
      const uint32_t wi = b0 >> 2, sb = (b0 & 3) * 8;
      uint32_t x[5];
#pragma unroll
      for (int k = 0; k < 5; ++k) x[k] = s_raw[wi + k];
      uint32_t le, inv;
      pack16<false>(x, sb, le, inv);
      s_be[i] = rev_pairs(le);
      s_lc[i] = ~le;
      s_inv[i] = inv;
    }
    __syncthreads();
    if (tile + 1 < t_end) {
      Geom ng = tile_geom(p, tile + 1, pf_seg);
      pf_base = (int64_t)ng.win0 - align_shift(p.seq, ng.win0);
      v0 = load_vec(p.seq, pf_base, tid, (int64_t)ng.seg_end);
      if (tid < kLoadVecs - kBlock) v1 = load_vec(p.seq, pf_base, kBlock + tid, (int64_t)ng.seg_end);
    }
    uint32_t be[5], lc[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) { be[k] = s_be[tid + k]; lc[k] = s_lc[tid + k]; }
    // 80 invalid bits: bases [16 tid, 16 tid + 80)
    const uint64_t inv_lo = (uint64_t)s_inv[tid] | ((uint64_t)s_inv[tid + 1] << 16) |
                            ((uint64_t)s_inv[tid + 2] << 32) | ((uint64_t)s_inv[tid + 3] << 48);
    const uint64_t inv_hi = (uint64_t)s_inv[tid + 4];
#pragma unroll
    for (int j = 0; j < kWPT; ++j) {
      // 128 BE bits of bases [16 tid + j, 16 tid + j + 64)
      uint32_t f3 = j ? funnel(be[0], be[1], 32 - 2 * j) : be[0];
      uint32_t f2 = j ? funnel(be[1], be[2], 32 - 2 * j) : be[1];
      uint32_t f1 = j ? funnel(be[2], be[3], 32 - 2 * j) : be[2];
      uint32_t f0 = j ? funnel(be[3], be[4], 32 - 2 * j) : be[3];
      uint64_t Fh = ((uint64_t)f3 << 32) | f2, Fl = ((uint64_t)f1 << 32) | f0;
      // >> fshift (0..62)
      if (fshift) { Fl = (Fl >> fshift) | (Fh << (64 - fshift)); Fh >>= fshift; }
      uint32_t r0 = j ? funnel(lc[1], lc[0], 2 * j) : lc[0];
      uint32_t r1 = j ? funnel(lc[2], lc[1], 2 * j) : lc[1];
      uint32_t r2 = j ? funnel(lc[3], lc[2], 2 * j) : lc[2];
      uint32_t r3 = j ? funnel(lc[4], lc[3], 2 * j) : lc[3];
      uint64_t Rl = ((uint64_t)r1 << 32) | r0, Rh = ((uint64_t)r3 << 32) | r2;
      uint64_t fml = Fl & p.mask_lo, fmh = Fh & p.mask_hi;
      uint64_t rml = Rl & p.mask_lo, rmh = Rh & p.mask_hi;
      bool f_lt = (fmh < rmh) || (fmh == rmh && fml < rml);
      uint64_t cl = f_lt ? fml : rml, ch = f_lt ? fmh : rmh;
      // window bits [j, j + w) of the 80-bit invalid map
      uint64_t iv = (inv_lo >> j) | (j ? (inv_hi << (64 - j)) : 0);
      bool valid = (iv & wmask_bits) == 0;
      win_count += valid ? 1u : 0u;
      uint64_t h;
      if constexpr (FLAVOUR == 0) {
        h = hash_mix(cl + kGolden32);
        h = hash_mix(h + kGolden32 + ch);
        h = hash_mix(h + (128 + kGolden32));
      } else {
        h = hash_bitset128<1>(cl, ch);
      }
      uint64_t f = h ^ p.kconst;
      bool keep = (MODE != kModeBottom) ? div_test(f, p.low_mask, p.high_mask, p.dinv, p.dlim)
                                        : (f <= thresh);
      if (valid && keep) {
        uint32_t slot = atomicAdd(&q_n, 1u);
        uint64_t a = (MODE == kModeList) ? g.win0 + (uint64_t)(kWPT * tid) + j
                                         : (MODE == kModeFrac) ? cl : f;
        uint64_t b = (MODE == kModeFrac) ? ch : cl;
        if (slot < cap) {
          q_a[slot] = a; q_b[slot] = b; q_c[slot] = ch;
        } else {
          unsigned long long gi = atomicAdd(&p.seg_count[g.seg], 1ull);
          if (gi < p.seg_out_cap[g.seg]) {
            uint64_t o = p.seg_out_off[g.seg] + gi;
            p.out_key[o] = a;
            if (MODE != kModeList) p.out_val[o] = b;
            if (MODE == kModeBottom) p.out_hi[o] = ch;
          }
        }
      }
    }
    __syncthreads();
    if (q_n >= cap / 2) {
      add_windows(q_wins, win_count);
      win_count = 0;
      wflush(g.seg);
    }
  }
  add_windows(q_wins, win_count);
  wflush(count_seg);
}

constexpr int kGridOversubscribe = 16;
constexpr int kDynOversubscribe = 2;

template <class K>
int occupancy_grid(K kernel, int device) {
  int per_cu = 0;
  (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, kBlock, 0);
  int cus = 0;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device);
  if (per_cu < 1) per_cu = 1;
  if (cus < 1) cus = 1;
  return per_cu * cus;
}

}  // namespace

uint64_t scan_tiles_for(uint64_t seg_bytes) { return (seg_bytes + kTile - 1) / kTile; }

hipError_t launch_scan(const ScanParams& p, int mode, int flavour, bool wide, int device,
                       hipStream_t stream, int grid_override) {
  if (p.n_tiles == 0) return hipSuccess;
  auto pick = [&](auto kernel) -> hipError_t {
    // Oversubscribe the resident slots 16x (config 3, pre-filter kernel: 20480
    // workgroups of ~36 tiles): the workgroup dispatcher then refills CUs as
    // ranges finish, which evens out per-CU speed differences and keeps every
    // SIMD at its wave limit. Measured on config 3 (tools/scan_grid_sweep.py):
    // 5.95 ms at 1x, 5.19 ms at 8x-16x before the pre-filter; with it 4.7 ms at
    // 8x and 16x (equal within noise in full benches), 5.6 ms at 32x and 9.2 at
    // 64x (per-workgroup start-up and flush costs).
    ScanParams q = p;
    q.tile_queue = nullptr;  // static tile ranges
    int grid = grid_override > 0 ? grid_override : kGridOversubscribe * occupancy_grid(kernel, device);
    if ((uint64_t)grid > p.n_tiles) grid = (int)p.n_tiles;
    hipLaunchKernelGGL(kernel, dim3(grid), dim3(kBlock), 0, stream, q);
    return hipGetLastError();
  };
  // dynamic tiles (narrow kernels, p.tile_queue set): twice the resident
  // workgroups (every slot filled even if the occupancy query is conservative),
  // chunks of ~T / (16 grid) tiles, 2..16: the tail is at most one chunk, and
  // the counter takes <= ~1 grab per 16 tiles (config 3: ~21 per microsecond,
  // below the ~88 one word serves, MI355X_MICROARCH.md)
  auto pick_dyn = [&](auto kernel) -> hipError_t {
    ScanParams q = p;
    int grid = grid_override > 0 ? grid_override : kDynOversubscribe * occupancy_grid(kernel, device);
    const uint64_t per = p.n_tiles / ((uint64_t)grid * 16);
    // smallest chunk 3 (SKS_SCAN_MIN_CHUNK overrides): config 2's one 5 Mb genome
    // (1221 tiles) scans in 27.4 us in chunks of 3 against 32.2 in chunks of 2
    // (1: 43, 4: 30, 6: 29); 128 config-4 genomes are the same at 2 and 3
    static const uint64_t min_chunk = getenv("SKS_SCAN_MIN_CHUNK") ? std::max(1, atoi(getenv("SKS_SCAN_MIN_CHUNK"))) : 3;
    q.chunk = (uint32_t)std::min<uint64_t>(16, std::max<uint64_t>(min_chunk, per));
    const uint64_t need = (p.n_tiles + q.chunk - 1) / q.chunk;
    if ((uint64_t)grid > need) grid = (int)need;
    hipLaunchKernelGGL(kernel, dim3(grid), dim3(kBlock), 0, stream, q);
    return hipGetLastError();
  };
  if (!wide && p.tile_queue) {
    if (mode == kModeFrac) {
      static const bool no_pre = getenv("SKS_NO_PREFILTER") != nullptr;
      if (flavour == 0 && (p.low_mask & 0xFu) && !no_pre) return pick_dyn(scan_kernel<kModeFrac, 0, 1>);
      return flavour == 0 ? pick_dyn(scan_kernel<kModeFrac, 0>) : pick_dyn(scan_kernel<kModeFrac, 1>);
    }
    if (mode == kModeBottom)
      return flavour == 0 ? pick_dyn(scan_kernel<kModeBottom, 0>) : pick_dyn(scan_kernel<kModeBottom, 1>);
  }
  if (!wide) {
    if (mode == kModeFrac) {
      static const bool no_pre = getenv("SKS_NO_PREFILTER") != nullptr;
      if (flavour == 0 && (p.low_mask & 0xFu) && !no_pre) return pick(scan_kernel<kModeFrac, 0, 1>);
      return flavour == 0 ? pick(scan_kernel<kModeFrac, 0>) : pick(scan_kernel<kModeFrac, 1>);
    }
    if (mode == kModeList) return flavour == 0 ? pick(scan_kernel<kModeList, 0>) : pick(scan_kernel<kModeList, 1>);
    return flavour == 0 ? pick(scan_kernel<kModeBottom, 0>) : pick(scan_kernel<kModeBottom, 1>);
  }
  if (mode == kModeFrac) return flavour == 0 ? pick(scan_kernel_wide<kModeFrac, 0>) : pick(scan_kernel_wide<kModeFrac, 1>);
  if (mode == kModeList) return flavour == 0 ? pick(scan_kernel_wide<kModeList, 0>) : pick(scan_kernel_wide<kModeList, 1>);
  return flavour == 0 ? pick(scan_kernel_wide<kModeBottom, 0>) : pick(scan_kernel_wide<kModeBottom, 1>);
}

SKS_CODE_OBJECT_HOOK(scan)

}  // namespace sks
