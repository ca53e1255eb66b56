// sbam_check.hip — record-boundary checker, FindRecordStart scan and record-chain walk (gfx950).
//
//  * full.Checker / eager.Checker at every uncompressed offset
//      (check/.../check/full/Checker.scala:22-184, eager/Checker.scala:24-126, PosChecker.scala:43-63)
//  * full-check Counts reduction (check/.../full/error/Counts.scala; cli/.../full/FullCheck.scala:141-191)
//  * FindRecordStart.withDelta (check/.../bam/spark/FindRecordStart.scala:30-63)
//  * RecordStream / PosStream chain (check/.../bam/iterator/RecordStream.scala:27-41)
//
// Layout: a workgroup stages a tile of the uncompressed stream (8 KiB of positions + a
// 768-B halo) in LDS and, while staging, builds an LDS bitmap of "CIGAR op invalid at this byte"
// ((b & 0xf) > 8 — an op's validity depends only on its first byte).  Each lane then evaluates FOUR
// consecutive positions from ten shared LDS dwords (v_alignbyte per offset).  The first record of a
// position is checked against the window; a CIGAR scan is a masked ctz over the bitmap (16 ops per 64-bit
// word) instead of a per-lane loop whose wave cost is the slowest lane; read names are checked 4 bytes at a
// time (SWAR).  Positions whose first record passes (true starts and rare near-misses) continue the
// 10-record chain from global memory.  The full check's Counts pass over interior tiles (k_check_bits) is
// bit-sliced: each per-position predicate is a bit of a per-lane 32-position plane, the reference-index
// predicates are evaluated once per byte offset and shared by the four positions that read that int32, and flags,
// keys and PASS0 bits are counted / formed on whole planes.
#include <algorithm>
#include <atomic>
#include <type_traits>

#include "sbam_internal.h"

namespace sbam {

#define SB_DEV __device__ __forceinline__

constexpr uint32_t W_SUCC = 0x80000000u, W_HALO = 0x00800000u;
constexpr uint32_t W_PASS0 = 0x40000000u;  // internal: first record passed, chain pending
constexpr uint32_t W_NONE = 0xffffffffu;   // internal: position outside [x0, x1)
constexpr int kCheckThreads = 256;
constexpr int kTile = 8192;                 // positions per tile (64-aligned tile bases)
constexpr int kHalo = 768;                  // staged bytes past the tile (fixed fields + 255-B name + ops)
constexpr int kWin = kTile + kHalo;         // staged window (multiple of 16)
constexpr int kOpcWords = kWin / 128 + 4;   // per residue class: one bit per 4 window bytes (+ pad)
constexpr int kNameWords = kWin / 32 + 4;   // one bit per window byte (+ pad)
constexpr int kLdsLens = 4096;              // contig lengths kept in LDS when n_ref fits
// workgroups per CU the register budget is sized for (launch bounds): k_check over boundary tiles / interior tiles,
// k_check_bits (6: a few constants spill, +7 GB scratch traffic, same time; round 4 with the LDS trimmed to 26.8 KB
// so that 6 workgroups fit: 41.5 vs 41.2 ms — not latency-bound)
constexpr int kCheckWgs = 4, kCheckWgsInt = 5, kCheckWgsBits = 5;
constexpr int kFlushTiles = 7;              // 7 tiles x 32 positions per lane < 255 (8-bit planes / counters)
static_assert(kWin % 16 == 0, "window");
static_assert((kTile / (4 * kCheckThreads)) % 2 == 0, "groups pair up within a tile (add4_paired)");

SB_DEV int lane_id() { return __lane_id(); }

SB_DEV uint64_t shfl_xor64(uint64_t v, int m) {
  const uint32_t lo = __shfl_xor((int)(uint32_t)v, m, 64), hi = __shfl_xor((int)(uint32_t)(v >> 32), m, 64);
  return ((uint64_t)hi << 32) | lo;
}
SB_DEV uint32_t wave_sum(uint32_t v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor((int)v, o, 64);
  return v;
}
SB_DEV uint32_t wave_incl_scan_u32(uint32_t v) {
  const int lane = __lane_id();
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = (uint32_t)__shfl_up((int)v, d, 64);
    if (lane >= d) v += y;
  }
  return v;
}
SB_DEV uint32_t wave_or(uint32_t v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v |= __shfl_xor((int)v, o, 64);
  return v;
}

// ---- byte-class SWAR ---------------------------------------------------------------------------
// (op validity, Checker.MAX_CIGAR_OP = 8, check/.../check/Checker.scala:21: (b & 0xf) + 7 carries into bit 4 iff
// (b & 0xf) > 8 — stage_tile)
// bytes outside allowedReadNameChars = ('!' to '?') ++ ('A' to '~') (Checker.scala:12-17), bit 7 of each byte
SB_DEV uint32_t name_bad_bytes(uint32_t w) {
  const uint32_t hi = w & 0x80808080u, lo7 = w & 0x7f7f7f7fu;
  const uint32_t lt33 = ~(lo7 + 0x5f5f5f5fu) & 0x80808080u;
  const uint32_t eq127 = (lo7 + 0x01010101u) & 0x80808080u;
  const uint32_t z = lo7 ^ 0x40404040u;
  const uint32_t eq64 = ~((z + 0x7f7f7f7fu) | z) & 0x80808080u;
  return hi | lt33 | eq127 | eq64;
}

SB_DEV int32_t g_i32(const uint8_t *u, int64_t x) {
  return (int32_t)((uint32_t)u[x] | ((uint32_t)u[x + 1] << 8) | ((uint32_t)u[x + 2] << 16) | ((uint32_t)u[x + 3] << 24));
}

// PosChecker.getRefPosError as bits {negIdx, bigIdx, negPos, bigPos}.  negPos = refPos < -1 in every branch;
// bigPos only when 0 <= refIdx < n_ref and refPos > len[refIdx] (note '>': refPos == len passes).
SB_DEV uint32_t ref_err(int32_t ri, int32_t rp, const int32_t *lensL, const int64_t *lensG, int32_t nref) {
  uint32_t f = (ri < -1) ? 1u : 0u;
  f |= (ri >= nref) ? 2u : 0u;
  f |= (rp < -1) ? 4u : 0u;
  if ((uint32_t)ri < (uint32_t)nref && rp > 0) {
    const int64_t len = lensL ? (int64_t)lensL[ri] : lensG[ri];
    f |= ((int64_t)rp > len) ? 8u : 0u;
  }
  return f;
}

// (l_seq + 1) / 2 + l_seq and 32 + l_read_name + 4 n_cigar + that, in Java Int (wrap, '/' toward zero)
SB_DEV bool too_few_remaining(int32_t bs, int32_t lrn, int32_t nc, int32_t ls) {
  // (ls + 1) / 2 truncated toward zero (Int division) = (ls + 1 + [ls < -1]) >> 1, arithmetic, also across the
  // int32 wrap at ls = INT_MAX: a compare and a carry-in add instead of a sign extract, an add and a shift
  const int32_t half = (int32_t)((uint32_t)ls + 1u + (ls < -1 ? 1u : 0u)) >> 1;
  const int32_t nsq = (int32_t)((uint32_t)half + (uint32_t)ls);
  const int32_t implied = (int32_t)(32u + (uint32_t)lrn + 4u * (uint32_t)nc + (uint32_t)nsq);
  return bs < implied;
}

// ---- generic chain (global memory): records k, k+1, ... from logical start s, read cursor a -----------------
// full/Checker.scala:22-184 line by line; EAGER stops at the first failing group (boolean identical).
struct GlobalBytes {
  const uint8_t *u;
  SB_DEV uint32_t operator()(int64_t x) const { return u[x]; }
};

template <bool EAGER, class Bytes>
SB_DEV uint32_t check_chain(const StreamView &sv, const Bytes &u, int64_t s, int64_t a, int k, int R) {
  auto g_i32 = [&](const Bytes &b, int64_t x) -> int32_t {
    return (int32_t)(b(x) | (b(x + 1) << 8) | (b(x + 2) << 16) | (b(x + 3) << 24));
  };
  for (;;) {
    if (k == R) return W_SUCC | ((uint32_t)k << 24);
    if (a + 36 > sv.L) {
      if (!sv.eof_real) return W_HALO;
      if (k > 0 && s == sv.L) return W_SUCC | ((uint32_t)k << 24);
      return 1u | ((uint32_t)k << 24);
    }
    const int32_t bs = g_i32(u, a), ri = g_i32(u, a + 4), rp = g_i32(u, a + 8), bmn = g_i32(u, a + 12);
    const int32_t fnc = g_i32(u, a + 16), ls = g_i32(u, a + 20), nri = g_i32(u, a + 24), nrp = g_i32(u, a + 28);
    const uint32_t K = (uint32_t)k << 24;
    uint32_t F = ref_err(ri, rp, nullptr, sv.lens, sv.nref) << 1;
    const int32_t lrn = bmn & 0xff;
    const uint32_t flag = ((uint32_t)fnc) >> 16;
    const int32_t nc = fnc & 0xffff;
    F |= too_few_remaining(bs, lrn, nc, ls) ? (1u << 18) : 0u;
    F |= ref_err(nri, nrp, nullptr, sv.lens, sv.nref) << 5;
    if (EAGER && (F || lrn < 2 || ((flag & 4u) == 0 && (ls == 0 || nc == 0)))) return K | (F ? F : (1u << 12));
    int64_t c = a + 36;
    if (lrn == 0) {
      F |= 1u << 12;
    } else if (lrn == 1) {
      F |= 1u << 13;
    } else {
      if (c + lrn > sv.L) {
        if (!sv.eof_real) return W_HALO;
        return K | F | (1u << 9);
      }
      if (u(c + lrn - 1) != 0) {
        F |= 1u << 10;
      } else {
        for (int32_t i = 0; i < lrn - 1; i++) {
          const uint32_t b = u(c + i);
          if (!((b - 33u <= 30u) || (b - 65u <= 61u))) { F |= 1u << 11; break; }
        }
      }
      c += lrn;
      if (EAGER && F) return K | F;
    }
    bool cig_err = false;
    for (int32_t i = 0; i < nc; i++) {
      if (c + 4 > sv.L) {
        if (!sv.eof_real) return W_HALO;
        F |= 1u << 14;
        cig_err = true;
        break;
      }
      const uint32_t op = u(c);
      c += 4;
      if ((op & 0xfu) > 8u) { F |= 1u << 15; cig_err = true; break; }
    }
    if (!cig_err && (flag & 4u) == 0 && (ls == 0 || nc == 0)) {
      F |= (ls == 0) ? (1u << 16) : 0u;  // EmptyMapped(emptySeq, emptyCigar) → (emptyMappedCigar, emptyMappedSeq)
      F |= (nc == 0) ? (1u << 17) : 0u;
    }
    if (F) return K | F;
    const int64_t nxt = s + 4 + (int64_t)bs;
    if (nxt > c) {
      if (nxt > sv.L && !sv.eof_real) return W_HALO;
      a = nxt > sv.L ? sv.L : nxt;  // skip past EOF clamps (parity unpinned: SURVEY §8(c))
    } else {
      a = c;
    }
    s = nxt;
    k++;
  }
}

// ---- chain pass ----------------------------------------------------------------------------------------------
// k_check leaves, for every position of [x0, x1), a bit meaning "the record read at this position passes every
// check" (PASS0).  A position's call is Success iff the first R records of its chain pass, so k_chains walks
// the chain of each PASS0 position: a record whose start is itself a PASS0 position is already known to pass
// (one bit read + 12 bytes to find the next record); any other record is checked in full from global memory.
// A failing chain clears its bit, so the bitmap becomes the success bitmap; bits are only a shortcut (a
// cleared bit is re-checked in full), so concurrent clears never change a result.
SB_DEV uint32_t walk_chain(const StreamView &sv, const unsigned long long *bitmap, int64_t x0a, int64_t x1, int64_t p,
                           int R) {
  int64_t s = p, a = p;
  int k = 0;
  for (;;) {
    if (k == R) return W_SUCC | ((uint32_t)k << 24);
    if (a + 36 > sv.L) {
      if (!sv.eof_real) return W_HALO;
      if (k > 0 && s == sv.L) return W_SUCC | ((uint32_t)k << 24);
      return 1u | ((uint32_t)k << 24);
    }
    const int32_t bs = g_i32(sv.u, a);
    int64_t c_end;
    const int64_t r = a - x0a;
    const bool fast = a == s && a < x1 && r >= 0 && ((bitmap[r >> 6] >> (r & 63)) & 1ull);
    if (fast) {
      const int32_t lrn = sv.u[a + 12];
      const int32_t nc = (int32_t)((uint32_t)sv.u[a + 16] | ((uint32_t)sv.u[a + 17] << 8));
      c_end = a + 36 + (lrn >= 2 ? lrn : 0) + 4 * (int64_t)nc;
    } else {
      // full check of this record: the generic chain restricted to one record (k fixed, R = k + 1)
      const uint32_t w = check_chain<false>(sv, GlobalBytes{sv.u}, s, a, k, k + 1);
      if (w == W_HALO || !(w & W_SUCC)) return w;
      const int32_t lrn = sv.u[a + 12];
      const int32_t nc = (int32_t)((uint32_t)sv.u[a + 16] | ((uint32_t)sv.u[a + 17] << 8));
      c_end = a + 36 + (lrn >= 2 ? lrn : 0) + 4 * (int64_t)nc;
    }
    const int64_t nxt = s + 4 + (int64_t)bs;
    if (nxt > c_end) {
      if (nxt > sv.L && !sv.eof_real) return W_HALO;
      a = nxt > sv.L ? sv.L : nxt;
    } else {
      a = c_end;
    }
    s = nxt;
    k++;
  }
}

SB_DEV void count_chain_result(const CountsDev &cd, uint32_t w, bool bykey) {
  if (w == W_HALO) { atomicAdd(&cd.scalars[3], 1ull); return; }
  if (w & W_SUCC) return;
  const uint32_t F = w & 0x7ffffu, kk = (w >> 24) & 0x7fu;
  if (F == 1u && kk == 0) { atomicAdd(&cd.scalars[2], 1ull); return; }
  const uint32_t key = (uint32_t)__popc(F) + (kk > 0 ? 1u : 0u);
  atomicAdd(&cd.positions[key], 1ull);
  for (uint32_t m = F; m; m &= m - 1) {
    const uint32_t f = __builtin_ctz(m);
    atomicAdd(&cd.totals[f], 1ull);
    if (bykey || key <= 2) atomicAdd(&cd.counts[key * 19 + f], 1ull);
  }
  if (key == 2) {
    const uint32_t fi = __builtin_ctz(F), rest = F & (F - 1);
    atomicAdd(&cd.pair[fi * 19 + (rest ? __builtin_ctz(rest) : fi)], 1ull);
  }
  if (kk > 0) atomicAdd(&cd.rbe[key * 128 + kk], 1ull);
}

// One workgroup per chunk of kChainWords bitmap words: the chunk's PASS0 positions are compacted into an LDS
// list (popcount + workgroup scan) and the 256 threads walk the listed chains, a chain per thread, so every lane of
// a wave does the same R hops.  (Walking the set bits of one word per lane made each wave pay the busiest
// lane's chains: 15 ms at 10 GB, for ~0.2 chains per word.)  cd.counts == nullptr skips counting (eager);
// words != nullptr writes results.  A failing chain clears its bit with an atomic AND (other threads of the
// workgroup may clear bits of the same word); each thread keeps its words as first read, so the list of a
// chunk with more than kChainList chains stays the same across rounds while bits are being cleared.
constexpr int kChainWordsPerThread = 8;
constexpr int kChainWords = 256 * kChainWordsPerThread;  // 131 072 positions per chunk
constexpr int kChainList = 4096;                          // LDS list entries per round (chunk-relative u32)
__global__ __launch_bounds__(256) void k_chains(StreamView sv, int64_t x0, int64_t x1, int R,
                                                unsigned long long *__restrict__ bitmap, CountsDev cd, int bykey,
                                                uint32_t *__restrict__ words) {
  __shared__ uint32_t s_list[kChainList];
  __shared__ uint32_t s_wsum[4];
  const int64_t x0a = x0 & ~(int64_t)63;
  const int64_t nwords = (x1 - x0a + 63) >> 6;
  const int64_t nchunks = (nwords + kChainWords - 1) / kChainWords;
  const int tid = threadIdx.x, lane = lane_id(), wv = tid >> 6;
  uint32_t n_succ = 0;
  for (int64_t ch = blockIdx.x; ch < nchunks; ch += gridDim.x) {
    const int64_t w0 = ch * kChainWords + (int64_t)tid * kChainWordsPerThread;
    unsigned long long cw[kChainWordsPerThread];
    uint32_t mine = 0;
#pragma unroll
    for (int j = 0; j < kChainWordsPerThread; j++) {
      cw[j] = w0 + j < nwords ? bitmap[w0 + j] : 0ull;
      mine += (uint32_t)__popcll(cw[j]);
    }
    // workgroup exclusive scan of the per-thread counts
    uint32_t incl = mine;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t t = __shfl_up(incl, o, 64);
      if (lane >= o) incl += t;
    }
    __syncthreads();  // s_wsum / s_list of the previous chunk are no longer read
    if (lane == 63) s_wsum[wv] = incl;
    __syncthreads();
    uint32_t before = 0, total = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
      before += k < wv ? s_wsum[k] : 0u;
      total += s_wsum[k];
    }
    const uint32_t first = before + incl - mine;
    const int64_t cbase = x0a + ch * (int64_t)kChainWords * 64;
    for (uint32_t r0 = 0; r0 < total; r0 += kChainList) {
      if (mine && first < r0 + kChainList && first + mine > r0) {
        uint32_t idx = first;
#pragma unroll
        for (int j = 0; j < kChainWordsPerThread; j++) {
          for (unsigned long long m = cw[j]; m && idx < r0 + kChainList; m &= m - 1, idx++)
            if (idx >= r0) s_list[idx - r0] = (uint32_t)(((w0 + j) << 6) + __builtin_ctzll(m) - (cbase - x0a));
        }
      }
      __syncthreads();
      const uint32_t n = min((uint32_t)kChainList, total - r0);
      for (uint32_t i = tid; i < n; i += 256) {
        const int64_t p = cbase + s_list[i];
        const uint32_t w = walk_chain(sv, bitmap, x0a, x1, p, R);
        if (w & W_SUCC) n_succ++;
        else atomicAnd(&bitmap[(p - x0a) >> 6], ~(1ull << ((p - x0a) & 63)));
        if (cd.counts) count_chain_result(cd, w, bykey != 0);
        if (words) words[p - x0] = w;
      }
      __syncthreads();
    }
  }
  if (cd.counts) {
    for (int o = 32; o >= 1; o >>= 1) n_succ += __shfl_xor((int)n_succ, o, 64);
    if (lane == 0 && n_succ) atomicAdd(&cd.scalars[1], (unsigned long long)n_succ);
  }
}

// ---- chain pass, list form ------------------------------------------------------------------------------------
// Nearly every PASS0 position is a true record start whose successor (p + 4 + block_size) is the next PASS0
// position.  So the PASS0 positions are listed in order (popcount, scan, write), each gets a link bit
// ok[i] = "the next record of p_i, by walk_chain's cursor rule, is p_{i+1}, past p_i's name and CIGAR", and
// p_i's call is Success as soon as ok[i .. i+R-2] all hold: every hop of its chain lands on a PASS0 position,
// which walk_chain would take through the fast path.  Every other PASS0 position (a link missing within R-1
// hops: the stream end, a shard edge, a false-positive record start in between, a skip past the name/CIGAR)
// is walked by walk_chain itself.  Same calls and counts as k_chains; 3 streaming passes instead of R hops per
// position.
__global__ __launch_bounds__(256) void k_p0_count(const unsigned long long *__restrict__ bitmap, int64_t nwords,
                                                  int32_t *__restrict__ chunk_cnt) {
  // (coalesced: thread t counts words t + 256 j of the chunk — the order does not matter for a count)
  const int64_t cb = (int64_t)blockIdx.x * kChainWords + threadIdx.x;
  uint32_t c = 0;
#pragma unroll
  for (int j = 0; j < kChainWordsPerThread; j++) {
    const int64_t w = cb + 256 * j;
    c += w < nwords ? (uint32_t)__popcll(bitmap[w]) : 0u;
  }
  c = wave_sum(c);
  __shared__ uint32_t s_c[4];
  if (lane_id() == 0) s_c[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) chunk_cnt[blockIdx.x] = (int32_t)(s_c[0] + s_c[1] + s_c[2] + s_c[3]);
}

// The same counts from the record-0 pass's per-tile, per-wave counts (k_check_bits / k_check<MODE_COUNTS, 2>): a chunk
// is 16 whole tiles, so its count is 64 integers instead of 16 KiB of bitmap.
__global__ __launch_bounds__(256) void k_p0_count_tiles(const int32_t *__restrict__ tile_pass0, int64_t ntiles,
                                                        int64_t nch, int32_t *__restrict__ chunk_cnt) {
  const int64_t ch = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (ch >= nch) return;
  const int64_t t0 = ch * 16, t1 = min(t0 + 16, ntiles);
  int32_t c = 0;
  for (int64_t i = 4 * t0; i < 4 * t1; i++) c += tile_pass0[i];
  chunk_cnt[ch] = c;
}

// exclusive scan of the chunk counts (one workgroup): off[ch], and off[n] = total.  Thread t owns the contiguous run
// [t·per, (t + 1)·per) of the counts: it sums its run, one workgroup scan of the 1024 sums gives every run its
// base, and the run is written out (two passes over n integers instead of n / 1024 barrier-separated rounds:
// 311 -> ~20 us for the 206 K chunks of a 10 GB shard).
__global__ __launch_bounds__(1024) void k_p0_scan(const int32_t *__restrict__ cnt, int64_t n, int64_t *__restrict__ off) {
  __shared__ int64_t s_w[16];
  const int lane = lane_id(), wv = threadIdx.x >> 6;
  const int64_t per = (n + 1023) / 1024;
  const int64_t b = min((int64_t)threadIdx.x * per, n), e = min(b + per, n);
  int64_t sum = 0;
#pragma unroll 8
  for (int64_t i = b; i < e; i++) sum += cnt[i];
  int64_t incl = sum;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int64_t t = __shfl_up(incl, o, 64);
    if (lane >= o) incl += t;
  }
  if (lane == 63) s_w[wv] = incl;
  __syncthreads();
  int64_t run = incl - sum;
  for (int k = 0; k < wv; k++) run += s_w[k];
#pragma unroll 8
  for (int64_t i = b; i < e; i++) {
    off[i] = run;
    run += cnt[i];
  }
  if (threadIdx.x == 1023) off[n] = run;  // (thread 1023's run ends at n: b and e are clamped to n)
}

__global__ __launch_bounds__(256) void k_p0_list(const unsigned long long *__restrict__ bitmap, int64_t nwords,
                                                 int64_t x0a, const int64_t *__restrict__ chunk_off,
                                                 int64_t *__restrict__ list) {
  // The chunk's words go through LDS: loaded coalesced (thread t loads words t + 256 j), read back as each thread's
  // own run of 8 consecutive words (the list is written in position order, one run per thread); rows padded to 9
  // words, so the read-back is 2-way bank-conflicted instead of 16-way.  (Each thread reading its 8 words straight
  // from memory left every load instruction touching 32 lines for 512 useful bytes.)
  static_assert(kChainWordsPerThread == 8, "k_p0_list: 8-word runs");
  constexpr int kRow = kChainWordsPerThread + 1;
  __shared__ unsigned long long s_cw[256 * kRow];
  const int64_t cb = (int64_t)blockIdx.x * kChainWords;
#pragma unroll
  for (int j = 0; j < kChainWordsPerThread; j++) {
    const int i = (int)threadIdx.x + 256 * j;  // the chunk's word i: thread i / 8's word i % 8
    s_cw[(i >> 3) * kRow + (i & 7)] = cb + i < nwords ? bitmap[cb + i] : 0ull;
  }
  __syncthreads();
  const int64_t w0 = cb + (int64_t)threadIdx.x * kChainWordsPerThread;
  unsigned long long cw[kChainWordsPerThread];
  uint32_t mine = 0;
#pragma unroll
  for (int j = 0; j < kChainWordsPerThread; j++) {
    cw[j] = s_cw[threadIdx.x * kRow + j];
    mine += (uint32_t)__popcll(cw[j]);
  }
  const int lane = lane_id(), wv = threadIdx.x >> 6;
  uint32_t incl = mine;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t t = __shfl_up(incl, o, 64);
    if (lane >= o) incl += t;
  }
  __shared__ uint32_t s_w[4];
  if (lane == 63) s_w[wv] = incl;
  __syncthreads();
  uint32_t before = 0;
  for (int k = 0; k < wv; k++) before += s_w[k];
  int64_t idx = chunk_off[blockIdx.x] + before + incl - mine;
#pragma unroll
  for (int j = 0; j < kChainWordsPerThread; j++)
    for (unsigned long long m = cw[j]; m; m &= m - 1) list[idx++] = x0a + ((w0 + j) << 6) + __builtin_ctzll(m);
}

// ok[i]: p_i's record hops to p_(i+1) past its name and CIGAR.  The last entry has no successor in the list: its
// link holds when its hop leaves the checked range [x0, x1) without passing the stream end, which is what the chain
// proof (sbam_records.hip) needs of the last set bit when it skips on "no missing link" (for R = 1 no fallback walk
// checks that hop).
__global__ __launch_bounds__(256) void k_p0_links(StreamView sv, const int64_t *__restrict__ list,
                                                  const int64_t *__restrict__ n_ptr, int64_t x1,
                                                  uint8_t *__restrict__ ok) {
  const int64_t n = *n_ptr;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t p = list[i];
    const int32_t bs = g_i32(sv.u, p);
    const int32_t lrn = sv.u[p + 12];
    const int32_t nc = (int32_t)((uint32_t)sv.u[p + 16] | ((uint32_t)sv.u[p + 17] << 8));
    const int64_t c_end = p + 36 + (lrn >= 2 ? lrn : 0) + 4 * (int64_t)nc;
    const int64_t nxt = p + 4 + (int64_t)bs;
    const bool link = i + 1 < n ? list[i + 1] == nxt : (nxt >= x1 && nxt <= sv.L);
    ok[i] = (link && nxt > c_end) ? 1 : 0;
  }
}

// Success when the R-1 links from p_i hold; every other PASS0 position goes to the fallback list.  n_fb[1] counts
// the missing links between consecutive list entries and a last entry whose hop stays inside [x0, x1): with none (and no failing fallback, n_fb[2]) the success
// bitmap IS the list and every set bit hops to the next one — the chain proof of the split records
// (sbam_records.hip) then holds without another pass over the records.
__global__ __launch_bounds__(256) void k_p0_fast(const int64_t *__restrict__ list, const int64_t *__restrict__ n_ptr,
                                                 const uint8_t *__restrict__ ok, int R, CountsDev cd,
                                                 int64_t *__restrict__ fb, unsigned long long *__restrict__ n_fb) {
  const int64_t n = *n_ptr;
  uint32_t n_succ = 0, n_gap = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    bool succ = i + (R - 1) <= n - 1 || R <= 1;
    for (int k = 0; succ && k < R - 1; k++) succ = ok[i + k] != 0;
    if (succ) n_succ++;
    else fb[atomicAdd(n_fb, 1ull)] = list[i];
    n_gap += !ok[i] ? 1u : 0u;
  }
  if (__ballot(n_gap != 0)) {
    n_gap = wave_sum(n_gap);
    if (lane_id() == 0) atomicAdd(&n_fb[1], (unsigned long long)n_gap);
  }
  if (cd.counts) {
    n_succ = wave_sum(n_succ);
    if (lane_id() == 0 && n_succ) atomicAdd(&cd.scalars[1], (unsigned long long)n_succ);
  }
}

// The same for 2 <= R <= 10, 16 entries per thread: the 24 link bytes ok[i0, i0 + 24) become a 24-bit mask (one
// 16-B and one 8-B load instead of R - 1 byte loads per entry), and entry j succeeds when its R - 1 bits from j hold.
__global__ __launch_bounds__(256) void k_p0_fast16(const int64_t *__restrict__ list, const int64_t *__restrict__ n_ptr,
                                                   const uint8_t *__restrict__ ok, int R, CountsDev cd,
                                                   int64_t *__restrict__ fb, unsigned long long *__restrict__ n_fb) {
  const int64_t n = *n_ptr;
  const uint32_t need = (1u << (R - 1)) - 1u;  // R - 1 consecutive links
  uint32_t n_succ = 0, n_gap = 0;
  auto nib = [](uint32_t w) { return (((w & 0x01010101u) * 0x00204081u) >> 21) & 0xfu; };  // byte k != 0 -> bit k
  for (int64_t i0 = 16 * ((int64_t)blockIdx.x * blockDim.x + threadIdx.x); i0 < n;
       i0 += 16 * (int64_t)gridDim.x * blockDim.x) {
    uint32_t m = 0;
    if (i0 + 24 <= n) {
      const uint4 a = *reinterpret_cast<const uint4 *>(ok + i0);
      const uint2 b = *reinterpret_cast<const uint2 *>(ok + i0 + 16);
      m = nib(a.x) | nib(a.y) << 4 | nib(a.z) << 8 | nib(a.w) << 12 | nib(b.x) << 16 | nib(b.y) << 20;
    } else {
      for (int k = 0; k < 24 && i0 + k < n; k++) m |= (ok[i0 + k] != 0 ? 1u : 0u) << k;
    }
#pragma unroll
    for (int j = 0; j < 16; j++) {
      const int64_t i = i0 + j;
      if (i < n) {
        const bool succ = i + (R - 1) <= n - 1 && ((m >> j) & need) == need;
        if (succ) n_succ++;
        else fb[atomicAdd(n_fb, 1ull)] = list[i];
        n_gap += !((m >> j) & 1u) ? 1u : 0u;
      }
    }
  }
  if (__ballot(n_gap != 0)) {
    n_gap = wave_sum(n_gap);
    if (lane_id() == 0) atomicAdd(&n_fb[1], (unsigned long long)n_gap);
  }
  if (cd.counts) {
    n_succ = wave_sum(n_succ);
    if (lane_id() == 0 && n_succ) atomicAdd(&cd.scalars[1], (unsigned long long)n_succ);
  }
}

__global__ __launch_bounds__(256) void k_p0_fallback(StreamView sv, int64_t x0a, int64_t x1, int R,
                                                     unsigned long long *__restrict__ bitmap, CountsDev cd, int bykey,
                                                     const int64_t *__restrict__ fb,
                                                     unsigned long long *__restrict__ n_fb) {
  const int64_t n = (int64_t)*n_fb;
  uint32_t n_succ = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t p = fb[i];
    const uint32_t w = walk_chain(sv, bitmap, x0a, x1, p, R);
    if (w & W_SUCC) {
      n_succ++;
    } else {
      atomicAnd(&bitmap[(p - x0a) >> 6], ~(1ull << ((p - x0a) & 63)));
      atomicAdd(&n_fb[2], 1ull);
    }
    if (cd.counts) count_chain_result(cd, w, bykey != 0);
  }
  if (cd.counts) {
    n_succ = wave_sum(n_succ);
    if (lane_id() == 0 && n_succ) atomicAdd(&cd.scalars[1], (unsigned long long)n_succ);
  }
}

// ---- first record against the LDS window --------------------------------------------------------------------
// Global (address space 1) view of the stream: pointers that arrive inside a kernel-argument struct are generic,
// and generic (flat) loads make every later LDS wait also wait for them.
typedef const __attribute__((address_space(1))) uint8_t *gbytes;
SB_DEV gbytes gview(const uint8_t *p) { return (gbytes)p; }

// The staged tile: bytes, plus two bitmaps built while staging —
//   opc, residue class r (r = 0..3), interleaved (class r's dword w at 4 w + r, so op_bits addresses it from the
//     byte offset alone): bit k = "(win[4k + r] & 0xf) > 8", i.e. CIGAR op k of any op array starting at a byte
//     offset ≡ r (mod 4) is invalid (Checker.MAX_CIGAR_OP; only an op's first byte matters): one 64-bit read
//     covers 64 consecutive ops;
//   nbad: bit r = "win[r] is not an allowed read-name character" (Checker.allowedReadNameChars).
struct Tile {
  const uint8_t *win;     // staged bytes: win[r] = u[base + r], r < kWin
  const uint32_t *opc;    // 4 × kOpcWords dwords (interleaved)
  const uint32_t *nbad;   // kNameWords dwords
  int64_t base;
  const int32_t *nxt;     // stage_nxt: class r's first invalid op start at or after 256 k + r (r * kNxt + k)
  int64_t *pw = nullptr;  // k_check: the wave's first invalid op start of class r past the window (-1: not read yet)
};

// 64 bits of an LDS bitmap from bit x: two funnel shifts (v_alignbit), no branch on the bit offset
SB_DEV uint64_t bits64(const uint32_t *bm, int x) {
  const int w = x >> 5;
  const uint32_t s = (uint32_t)x & 31u;
  const uint32_t a = bm[w], b = bm[w + 1], c = bm[w + 2];
  return ((uint64_t)__builtin_amdgcn_alignbit(c, b, s) << 32) | __builtin_amdgcn_alignbit(b, a, s);
}

// Op-validity bits of the 64 ops at byte offsets c, c + 4, ... (bit i: op i invalid) from the interleaved class
// bitmap: class c & 3, bit c >> 2 -> dword 4 (c >> 7) + (c & 3), shift (c >> 2) & 31.
SB_DEV uint64_t op_bits(const uint32_t *opc, int c) {
  const int w = ((c >> 5) & ~3) | (c & 3);
  const uint32_t s = ((uint32_t)c >> 2) & 31u;
  const uint32_t a = opc[w], b = opc[w + 4], d = opc[w + 8];
  return ((uint64_t)__builtin_amdgcn_alignbit(d, b, s) << 32) | __builtin_amdgcn_alignbit(b, a, s);
}

// Any byte of the name body [rel, rel + n) outside allowedReadNameChars? (n <= 254, inside the window)
SB_DEV bool name_has_bad(const Tile &t, int rel, int32_t n) {
  for (int32_t o = 0; o < n; o += 64) {
    uint64_t m = bits64(t.nbad, rel + o);
    if (n - o < 64) m &= (1ull << (n - o)) - 1ull;
    if (m) return true;
  }
  return false;
}

// Long op arrays.  An op array whose first 64 ops are valid is rare in short-read data but the rule inside a long
// read's packed sequence (nibbles 1, 2, 4, 8 are all valid op codes, and n_cigar there is >= 0x1111), so every
// position of such a region asks for the first invalid op among thousands.  Per tile, stage_nxt keeps for each
// residue class r the first invalid op start at or after 256 k + r (k < kNxt; kNoBad: none in the window), so a
// window lookup is one 64-op bitmap read and one table read; past the window the stream is read 16 B at a time
// (k_check_bits: by the whole wave, 8 KiB per step, once per tile and class).
constexpr int kNxt = kWin / 256 + 1;
constexpr int32_t kNoBad = 0x3fffffff;
static_assert(kWin % 256 == 0 && kCheckThreads == 4 * 64, "stage_nxt: one wave per residue class");

// Fill t.nxt (after stage_tile's bitmaps are complete): wave r computes class r, lane k super-chunk k, then a suffix
// minimum across the lanes.
SB_DEV void stage_nxt(const uint32_t *s_opc, int32_t *s_nxt) {
  const int r = (int)(threadIdx.x >> 6), k = lane_id();
  int32_t v = kNoBad;
  if (k < kNxt - 1) {
    const uint64_t m = op_bits(s_opc, 256 * k + r);
    if (m) v = 256 * k + r + 4 * (int32_t)__builtin_ctzll(m);
  }
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int32_t u = __shfl_down(v, o, 64);
    if (k + o < 64) v = min(v, u);
  }
  if (k < kNxt) s_nxt[r * kNxt + k] = v;
}

// The same table built by one wave for itself (its own LDS slice; wave-level ordering only), when a tile first needs
// it: lanes k < kNxt take super-chunk k of all four classes.
__attribute__((noinline)) __device__ void wave_nxt(const uint32_t *s_opc, int32_t *nx) {
  const int k = lane_id();
  int32_t v[4];
#pragma unroll
  for (int r = 0; r < 4; r++) {
    v[r] = kNoBad;
    if (k < kNxt - 1) {
      const uint64_t m = op_bits(s_opc, 256 * k + r);
      if (m) v[r] = 256 * k + r + 4 * (int32_t)__builtin_ctzll(m);
    }
  }
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
#pragma unroll
    for (int r = 0; r < 4; r++) {
      const int32_t u = __shfl_down(v[r], o, 64);
      if (k + o < 64) v[r] = min(v[r], u);
    }
  }
  if (k < kNxt)
#pragma unroll
    for (int r = 0; r < 4; r++) nx[r * kNxt + k] = v[r];
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// First invalid op start (window-relative) at or after y (y's class), kNoBad if none before the window's end.
SB_DEV int32_t next_bad_in_window(const Tile &t, int y) {
  if (y >= kWin) return kNoBad;
  const int r = y & 3, k = (y - r + 255) >> 8;  // table entry k covers class r from 256 k + r >= y
  const int g = (256 * k + r - y) >> 2;         // the < 64 ops before it, from the bitmap
  const uint64_t m = op_bits(t.opc, y) & ((1ull << g) - 1ull);
  return m ? y + 4 * (int32_t)__builtin_ctzll(m) : t.nxt[r * kNxt + k];
}

// The first invalid op start of class r at or after the aligned position a (bytes [a, a + 16) of the stream), as a
// 4-bit mask per class of the 16-B chunk: bit j of byte r = the op at a + 4 j + r is invalid.
typedef unsigned int u32x4g __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(1))) u32x4g *g16v;
SB_DEV uint32_t bad_ops16(const u32x4g v) {
  auto bad = [](uint32_t w) { return (((w & 0x0f0f0f0fu) + 0x07070707u) >> 4) & 0x01010101u; };
  return bad(v.x) | bad(v.y) << 1 | bad(v.z) << 2 | bad(v.w) << 3;
}

// Wave-cooperative (every lane calls it with the same arguments): any invalid op among the n ops at c, c + 4, ...?
// 4 KiB of the stream per step (4 loads of 16 B per lane in flight).  Reads stay within the interior's reach or the
// stream's zero pad.
SB_DEV bool ops_bad_wave(const StreamView &sv, int64_t c, int32_t n) {
  const int r = (int)(c & 3), lane = lane_id();
  const int64_t e = c + 4 * (int64_t)n, a0 = c & ~(int64_t)15;
  const g16v src = (g16v)gview(sv.u);
  for (int64_t a = a0; a < e; a += 4096) {
    uint32_t m[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const int64_t p = a + 1024 * k + 16 * lane;
      m[k] = p < e ? (bad_ops16(src[p >> 4]) >> (8 * r)) & 0xfu : 0u;
    }
    bool hit = false;
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const int64_t p = a + 1024 * k + 16 * lane + r;  // op j of the chunk at p + 4 j
#pragma unroll
      for (int j = 0; j < 4; j++) hit |= ((m[k] >> j) & 1u) && p + 4 * j >= c && p + 4 * j < e;
    }
    if (__ballot(hit)) return true;
  }
  return false;
}

// Wave-cooperative: for each class r in `need`, nbe[r] (the wave's LDS) = the first invalid op start of class r at or
// after A0 (16-B aligned), within kScanPast bytes (else kFarAway), kScanStep bytes per step.
constexpr int64_t kScanPast = 262144;  // >= the reach of any op array from a window (4 x 65535 ops)
constexpr int64_t kFarAway = (int64_t)1 << 60;
constexpr int kTableLanes = 8;  // k_check_bits: lanes of a wave in the long-op pass that make it build the table first
constexpr int kScanStep = 2048;  // bytes per wave step: two 16-B loads per lane in flight
__attribute__((noinline)) __device__ void scan_past_window(const StreamView &sv, int64_t A0, uint32_t need,
                                                            int64_t *nbe) {
  const int lane = lane_id();
  const g16v src = (g16v)(gview(sv.u) + A0);
  uint32_t left = need;
  for (int it = 0; left && it < (int)(kScanPast / kScanStep); it++) {
    uint32_t m[kScanStep / 1024];
#pragma unroll
    for (int i = 0; i < kScanStep / 1024; i++) m[i] = bad_ops16(src[(kScanStep / 16) * it + 64 * i + lane]);
#pragma unroll
    for (int i = 0; i < kScanStep / 1024; i++) {
#pragma unroll
      for (int r = 0; r < 4; r++) {
        if ((left >> r) & 1u) {
          const uint64_t bal = __ballot(((m[i] >> (8 * r)) & 0xfu) != 0u);
          if (bal) {
            const int f = (int)__builtin_ctzll(bal);
            const uint32_t mf = ((uint32_t)__builtin_amdgcn_readlane((int)m[i], f) >> (8 * r)) & 0xfu;
            if (lane == 0) nbe[r] = A0 + kScanStep * (int64_t)it + 1024 * i + 16 * f + 4 * __builtin_ctz(mf) + r;
            left &= ~(1u << r);
          }
        }
      }
    }
  }
  if (lane == 0)
#pragma unroll
    for (int r = 0; r < 4; r++)
      if ((left >> r) & 1u) nbe[r] = kFarAway;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // (the wave reads nbe[] back from LDS)
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Index of the first op among the first `lim` ops at c, c+4, ... whose first byte has (b & 0xf) > 8, or lim.
SB_DEV int32_t first_bad_op(const Tile &t, const StreamView &sv, int64_t c, int32_t lim) {
  const int rel = (int)(c - t.base);
  const uint64_t m = op_bits(t.opc, rel);
  if (m) {
    const int32_t b = (int32_t)__builtin_ctzll(m);
    return b < lim ? b : lim;
  }
  if (lim <= 64) return lim;
  const int32_t p = next_bad_in_window(t, rel + 256);
  if (p != kNoBad) return min((p - rel) >> 2, lim);
  // past the window (this lane alone): the first invalid op start of the class at or after the window's end, read in
  // aligned 64-B steps (4 loads in flight) up to the reach of any op array or the stream's end (its zero pad covers
  // the last step), and kept for the wave's other positions in t.pw (lanes that race there store the same value)
  const int r = rel & 3;
  const int64_t e = c + 4 * (int64_t)lim;
  int64_t q = t.pw ? t.pw[r] : -1;
  if (q < 0) {
    q = kFarAway;
    const g16v src = (g16v)gview(sv.u);
    const int64_t a0 = t.base + kWin, a1 = min(a0 + kScanPast, sv.L);
    for (int64_t a = a0; a < a1; a += 64) {
      uint32_t b4 = 0;
#pragma unroll
      for (int j = 0; j < 4; j++) b4 |= ((bad_ops16(src[(a >> 4) + j]) >> (8 * r)) & 0xfu) << (4 * j);
      if (b4) {
        q = a + 4 * __builtin_ctz(b4) + r;
        break;
      }
    }
    if (t.pw) t.pw[r] = q;
  }
  return q < e ? (int32_t)((q - c) >> 2) : lim;
}

// PosChecker.getRefPosError bits with the contig length read unconditionally (clamped index) from LDS.
SB_DEV uint32_t ref_bits_lds(int32_t ri, int32_t rp, const int32_t *lensL, int32_t nref) {
  const bool in = (uint32_t)ri < (uint32_t)nref;
  const int32_t len = lensL[in ? ri : 0];
  return (ri < -1 ? 1u : 0u) | (ri >= nref ? 2u : 0u) | (rp < -1 ? 4u : 0u) | (in && rp > len ? 8u : 0u);
}

// Record 0 at x (full.Checker.scala:22-184 / eager.Checker.scala:24-126 for k = 0), fixed fields in f[],
// rel = x - tile base.  Every check is evaluated unconditionally from the tile (clamped LDS reads, no
// per-lane branches) so a wave's lanes cost the same; only the rare tails (a name body or an op array
// running past 64 checked bytes / ops) branch out to HBM.  INTERIOR: the tile lies inside [x0, x1) and ends at
// least kInteriorTail bytes before the stream end, so no read of record 0 (36 fixed bytes, <= 255 name bytes,
// <= 65535 ops) can reach EOF: the EOF arithmetic and the range checks drop out.
constexpr int64_t kInteriorTail = 262144 + 512;
template <bool EAGER, bool INTERIOR>
SB_DEV uint32_t check_first(const Tile &t, const StreamView &sv, const int32_t *lensL, int64_t x, int rel, int R,
                            const int32_t f[8]) {
  if (R == 0) return W_PASS0;  // Success(0): resolved by the chain pass
  const int32_t bs = f[0], ri = f[1], rp = f[2], bmn = f[3], fnc = f[4], ls = f[5], nri = f[6], nrp = f[7];
  const int32_t lrn = bmn & 0xff;
  const uint32_t flag = ((uint32_t)fnc) >> 16;
  const int32_t nc = fnc & 0xffff;
  const uint32_t rb0 = lensL ? ref_bits_lds(ri, rp, lensL, sv.nref) : ref_err(ri, rp, nullptr, sv.lens, sv.nref);
  const uint32_t rb1 = lensL ? ref_bits_lds(nri, nrp, lensL, sv.nref) : ref_err(nri, nrp, nullptr, sv.lens, sv.nref);
  const uint32_t Fref = (rb0 << 1) | (rb1 << 5) | (too_few_remaining(bs, lrn, nc, ls) ? (1u << 18) : 0u);
  const bool empty_mapped = (flag & 4u) == 0 && (ls == 0 || nc == 0);
  if (EAGER && (INTERIOR || x + 36 <= sv.L) && (Fref || lrn < 2 || empty_mapped))
    return Fref ? Fref : (1u << 12);  // eager: ~96 % of positions end here, skip the rest of the record
  // read name: lrn 0/1 → noReadName / emptyReadName (name not consumed); else last byte NUL, then characters
  const bool has_name = lrn >= 2;
  const bool name_eof = !INTERIOR && has_name && x + 36 + lrn > sv.L;
  const uint32_t last = t.win[rel + 35 + (has_name ? lrn : 1)];
  const bool nonnull = has_name && last != 0;
  const bool scan = has_name && last == 0;
  const int32_t nbody = lrn - 1;
  uint64_t nbm = bits64(t.nbad, rel + 36);
  if (nbody < 64) nbm &= (1ull << (nbody > 0 ? nbody : 0)) - 1ull;
  bool nonascii = scan && nbm != 0;
  if (scan && nbm == 0 && nbody > 64 && !name_eof) nonascii = name_has_bad(t, rel + 36 + 64, nbody - 64);
  // CIGAR ops: the first invalid op among min(n_cigar, ops before EOF)
  const int32_t clen = has_name ? lrn : 0;
  const int64_t c = x + 36 + clen;
  const int crel = rel + 36 + clen;
  int32_t n_eof = 0x7fffffff;
  if (!INTERIOR) {
    const int64_t n_eof64 = (sv.L - c) >> 2;
    n_eof = n_eof64 < 0 ? 0 : n_eof64 > 0x7fffffff ? 0x7fffffff : (int32_t)n_eof64;
  }
  const int32_t lim = n_eof < nc ? n_eof : nc;
  const uint64_t om = op_bits(t.opc, crel);
  int32_t bad = om ? (int32_t)__builtin_ctzll(om) : 64;
  if (om == 0 && lim > 64 && !name_eof) bad = first_bad_op(t, sv, c, lim);
  const bool inv_op = nc > 0 && bad < lim;
  const bool few_ops = !INTERIOR && nc > 0 && !inv_op && n_eof < nc;
  uint32_t F = Fref;
  F |= lrn == 0 ? (1u << 12) : 0u;
  F |= lrn == 1 ? (1u << 13) : 0u;
  F |= nonnull ? (1u << 10) : 0u;
  F |= nonascii ? (1u << 11) : 0u;
  F |= inv_op ? (1u << 15) : 0u;
  F |= few_ops ? (1u << 14) : 0u;
  F |= (empty_mapped && !inv_op && !few_ops) ? (((ls == 0) ? (1u << 16) : 0u) | ((nc == 0) ? (1u << 17) : 0u)) : 0u;
  // result, in the reference's order of early exits
  const bool fixed_eof = !INTERIOR && x + 36 > sv.L;
  uint32_t w;
  if (EAGER) {  // eager.Checker: false at the first failing group (only pass/fail and HALO matter)
    const bool fail_fixed = Fref || !has_name || empty_mapped;
    const bool fail_name = nonnull || nonascii;
    w = fixed_eof ? (sv.eof_real ? 1u : W_HALO)
        : fail_fixed ? (Fref ? Fref : (1u << 12))
        : name_eof ? (sv.eof_real ? (1u << 9) : W_HALO)
        : fail_name ? F
        : (few_ops && !sv.eof_real) ? W_HALO
        : F ? F : W_PASS0;
  } else {
    w = fixed_eof ? (sv.eof_real ? 1u : W_HALO)
        : name_eof ? (sv.eof_real ? (Fref | (1u << 9)) : W_HALO)
        : (few_ops && !sv.eof_real) ? W_HALO
        : F ? F : W_PASS0;  // record 0 passed: the 10-record chain is resolved by k_chains
  }
  return w;
}

// Stage the window of the tile at `base` (32 B per lane per step) and build the op-class and name-character
// bitmaps (struct Tile).
SB_DEV void stage_tile(const StreamView &sv, int64_t base, uint8_t *s_win, uint32_t *s_opc, uint32_t *s_nbad) {
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  typedef const __attribute__((address_space(1))) u32x4 *g16;
  const g16 src = (g16)(gview(sv.u) + base);
  u32x4 *dst = reinterpret_cast<u32x4 *>(s_win);
  uint8_t *opc8 = reinterpret_cast<uint8_t *>(s_opc);
  for (int i = threadIdx.x; i < kWin / 32; i += kCheckThreads) {
    const u32x4 a = src[2 * i], b = src[2 * i + 1];
    dst[2 * i] = a;
    dst[2 * i + 1] = b;
    const uint32_t w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    // T: bit j of byte r = byte r of w[j] is an invalid op start, so byte r of T is residue class r's 8 bits
    uint32_t T = 0, nb = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) {
      T |= ((((w[j] & 0x0f0f0f0fu) + 0x07070707u) >> 4) & 0x01010101u) << j;
      const uint32_t m = (name_bad_bytes(w[j]) >> 7) & 0x01010101u;  // bit 0 of each bad byte
      nb |= (((m * 0x00204081u) >> 21) & 0xfu) << (4 * j);
    }
#pragma unroll
    for (int r = 0; r < 4; r++) opc8[16 * (i >> 2) + 4 * r + (i & 3)] = (uint8_t)(T >> (8 * r));
    s_nbad[i] = nb;
  }
  if (threadIdx.x < 4) s_nbad[kWin / 32 + threadIdx.x] = 0;
  if (threadIdx.x < 16) s_opc[kWin / 32 + threadIdx.x] = 0;  // the 4 pad words of every class
}

// Per window byte c < kFbBytes: fb[c] = index of the first invalid CIGAR op among the ops at c, c + 4, ... (exact
// below 64; >= 64 means none among the first 64), so that a position's CIGAR test is one LDS byte read.  Thread i
// covers bytes [32 i, 32 i + 32), the 8 ops of each residue class there: the value just past the chunk comes from
// the op-class bitmap (ctz of 64 bits, capped at 64), then F_j = bad(op j) ? 0 : F_(j+1) + 1 runs backward over the
// chunk's 8 dwords, all four classes at once (one byte each).  Needs stage_tile's bitmaps (a barrier between).
constexpr int kFbBytes = ((kTile + 36 + 255 + 31) / 32) * 32;
SB_DEV void stage_fb(const uint8_t *s_win, const uint32_t *s_opc, uint8_t *s_fb) {
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  for (int i = threadIdx.x; i < kFbBytes / 32; i += kCheckThreads) {
    uint32_t F = 0;
#pragma unroll
    for (int r = 0; r < 4; r++) {
      const uint64_t om = op_bits(s_opc, 32 * i + 32 + r);
      const uint32_t z = om ? (uint32_t)__builtin_ctzll(om) : 64u;
      F |= z << (8 * r);
    }
    const u32x4 a = reinterpret_cast<const u32x4 *>(s_win)[2 * i], b = reinterpret_cast<const u32x4 *>(s_win)[2 * i + 1];
    const uint32_t w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    uint32_t o[8];
#pragma unroll
    for (int j = 7; j >= 0; j--) {
      const uint32_t bad = (((w[j] & 0x0f0f0f0fu) + 0x07070707u) >> 4) & 0x01010101u;  // (b & 0xf) > 8, bit 0
      F = (F + 0x01010101u) & ~((bad << 8) - bad);  // bad bytes -> 0xff
      o[j] = F;
    }
    reinterpret_cast<u32x4 *>(s_fb)[2 * i] = u32x4{o[0], o[1], o[2], o[3]};
    reinterpret_cast<u32x4 *>(s_fb)[2 * i + 1] = u32x4{o[4], o[5], o[6], o[7]};
  }
}

// ---- the tiled kernel -------------------------------------------------------------------------------------
enum { MODE_COUNTS = 0, MODE_EAGER = 1, MODE_WORDS = 2, MODE_BYKEY = 3 };

struct Planes {  // carry-save bit planes: per-flag counts of up to 255 values per lane
  uint32_t p[8];
  SB_DEV void clear() {
#pragma unroll
    for (int j = 0; j < 8; j++) p[j] = 0;
  }
  // add a 3-plane number (o1 weight 1, o2 weight 2, o4 weight 4)
  SB_DEV void add(uint32_t o1, uint32_t o2, uint32_t o4) {
    uint32_t c = p[0] & o1;
    p[0] ^= o1;
    uint32_t s = p[1] ^ o2 ^ c;
    c = (p[1] & o2) | (c & (p[1] ^ o2));
    p[1] = s;
    s = p[2] ^ o4 ^ c;
    c = (p[2] & o4) | (c & (p[2] ^ o4));
    p[2] = s;
#pragma unroll
    for (int j = 3; j < 8; j++) {
      const uint32_t t = p[j] & c;
      p[j] ^= c;
      c = t;
    }
  }
};

// Count one checked position into the lane's accumulators (full-check Counts semantics).
struct Acc {
  Planes pl;
  Planes kp;         // interior tiles: one-hot key planes (bit k = a position with key k; bit 0 = PASS0, ignored)
  uint64_t keyc[3];  // 8-bit counters per key (8 per word)
  uint32_t n_succ, n_tff, n_halo;
  SB_DEV void clear() {
    pl.clear();
    kp.clear();
    keyc[0] = keyc[1] = keyc[2] = 0;
    n_succ = n_tff = n_halo = 0;
  }
  // classify w; returns the counted flag word F (0 if not counted).  The rare per-key paths (keys 1-2 per flag,
  // close-call pairs) count into the workgroup's LDS tables k12 / pair; only readsBeforeError (kk > 0, chains
  // only) goes straight to global atomics.  (Global atomics from every workgroup onto the same few hundred
  // counters serialise at the memory side: 0.3 % of positions made them the checker's bottleneck.)
  template <bool BYKEY>
  SB_DEV uint32_t classify(uint32_t w, const CountsDev &cd, uint32_t *k12, uint32_t *pair, uint32_t &key_out,
                           bool &counted_out) {
    const bool succ = (w & W_SUCC) != 0;
    const bool halo = w == W_HALO;
    const bool tff = w == 1u;
    const bool counted = !succ && !halo && !tff;
    n_succ += succ;
    n_halo += halo;
    n_tff += tff;
    const uint32_t F = counted ? (w & 0x7ffffu) : 0u;
    const uint32_t kk = (w >> 24) & 0x7fu;
    const uint32_t key = (uint32_t)__popc(F) + (kk > 0 ? 1u : 0u);
    if (counted) {
      const uint64_t inc = 1ull << (8 * (key & 7));
      keyc[0] += (key >> 3) == 0 ? inc : 0ull;
      keyc[1] += (key >> 3) == 1 ? inc : 0ull;
      keyc[2] += (key >> 3) == 2 ? inc : 0ull;
      if (key <= 2 || kk > 0) {  // rare: keys 1-2 per flag, close-call pairs, readsBeforeError histogram
        if (!BYKEY && key <= 2)
          for (uint32_t m = F; m; m &= m - 1) atomicAdd(&k12[key * 19 + __builtin_ctz(m)], 1u);
        if (key == 2) {
          const uint32_t fi = __builtin_ctz(F), rest = F & (F - 1);
          atomicAdd(&pair[fi * 19 + (rest ? __builtin_ctz(rest) : fi)], 1u);
        }
        if (kk > 0) atomicAdd(&cd.rbe[key * 128 + kk], 1ull);
      }
    }
    key_out = key;
    counted_out = counted;
    return F;
  }
};

// Record-0 pass over an interior tile (every position in [x0, x1), no EOF in reach): a result is either PASS0
// (flag bits 0) or a failure with k = 0, never Success / HALO / TooFewFixedBlockBytes.  So F = w & 0x7ffff,
// key = popc(F), and the key histogram is a one-hot word added into bit planes like the flags (no per-key
// selects).  Only keys 1-2 take the rare per-flag / pair path.
SB_DEV uint32_t classify_interior(uint32_t w, uint32_t *k12, uint32_t *pair, uint32_t &onehot) {
  const uint32_t F = w & 0x7ffffu;
  const uint32_t key = (uint32_t)__popc(F);
  onehot = 1u << key;
  if (F && key <= 2) {
    for (uint32_t m = F; m; m &= m - 1) atomicAdd(&k12[key * 19 + __builtin_ctz(m)], 1u);
    if (key == 2) {
      const uint32_t fi = __builtin_ctz(F), rest = F & (F - 1);
      atomicAdd(&pair[fi * 19 + (rest ? __builtin_ctz(rest) : fi)], 1u);
    }
  }
  return F;
}

// Add a 4-plane number (weights 1, 2, 4, 8) into the planes.
SB_DEV void add_planes4(Planes &pl, uint32_t o1, uint32_t o2, uint32_t o4, uint32_t o8) {
  uint32_t c = pl.p[0] & o1;
  pl.p[0] ^= o1;
  const uint32_t o[3] = {o2, o4, o8};
#pragma unroll
  for (int j = 1; j <= 3; j++) {
    const uint32_t x = pl.p[j] ^ o[j - 1];
    const uint32_t cn = (pl.p[j] & o[j - 1]) | (c & x);
    pl.p[j] = x ^ c;
    c = cn;
  }
#pragma unroll
  for (int j = 4; j < 8; j++) {
    const uint32_t t = pl.p[j] & c;
    pl.p[j] ^= c;
    c = t;
  }
}
// 4:3 compressor of four words into (ones, twos, fours); with a held (ones, twos, fours) from the previous group
// the two are summed into a 4-plane number and added once (pairs of groups share one carry chain)
SB_DEV void add4_paired(Planes &pl, const uint32_t v[4], uint32_t (&h)[3], bool second) {
  const uint32_t x1a = v[0] ^ v[1], c1 = v[0] & v[1];
  const uint32_t x2a = v[2] ^ v[3], c2 = v[2] & v[3];
  const uint32_t o1 = x1a ^ x2a, c3 = x1a & x2a;
  const uint32_t o2 = c1 ^ c2 ^ c3, o4 = (c1 & c2) | (c3 & (c1 ^ c2));
  if (!second) {
    h[0] = o1;
    h[1] = o2;
    h[2] = o4;
    return;
  }
  const uint32_t s1 = h[0] ^ o1, k1 = h[0] & o1;
  const uint32_t s2 = h[1] ^ o2 ^ k1, k2 = (h[1] & o2) | (k1 & (h[1] ^ o2));
  const uint32_t s4 = h[2] ^ o4 ^ k2, k4 = (h[2] & o4) | (k2 & (h[2] ^ o4));
  add_planes4(pl, s1, s2, s4, k4);
}

// 4:3 compressor of four bit-plane words into (ones, twos, fours) for Planes::add
SB_DEV void add4(Planes &pl, const uint32_t v[4]) {
  const uint32_t x1a = v[0] ^ v[1], c1 = v[0] & v[1];
  const uint32_t x2a = v[2] ^ v[3], c2 = v[2] & v[3];
  const uint32_t ones = x1a ^ x2a, c3 = x1a & x2a;
  pl.add(ones, c1 ^ c2 ^ c3, (c1 & c2) | (c3 & (c1 ^ c2)));
}

// Reduce the lanes' accumulators into the workgroup's LDS totals (ballots over bit planes; wave sums).
SB_DEV void flush_acc(Acc &acc, unsigned long long *s_acc, int lane) {
#pragma unroll
  for (int f = 0; f < 19; f++) {
    uint32_t tot = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) tot += (uint32_t)__popcll(__ballot((acc.pl.p[j] >> f) & 1u)) << j;
    if (lane == 0 && tot) atomicAdd(&s_acc[f], (unsigned long long)tot);
  }
#pragma unroll
  for (int k = 0; k < 21; k++) {
    uint32_t v = wave_sum((uint32_t)(acc.keyc[k >> 3] >> (8 * (k & 7))) & 0xffu);
    if (k >= 1 && k <= 19) {
#pragma unroll
      for (int j = 0; j < 8; j++) v += (uint32_t)__popcll(__ballot((acc.kp.p[j] >> k) & 1u)) << j;
    }
    if (lane == 0 && v) atomicAdd(&s_acc[19 + k], (unsigned long long)v);
  }
  const uint32_t a = wave_sum(acc.n_succ), b = wave_sum(acc.n_tff), h = wave_sum(acc.n_halo);
  if (lane == 0) {
    if (a) atomicAdd(&s_acc[40], (unsigned long long)a);
    if (b) atomicAdd(&s_acc[41], (unsigned long long)b);
    if (h) atomicAdd(&s_acc[42], (unsigned long long)h);
  }
  acc.clear();
}

// Exact per-key flag counts (MODE_BYKEY): 19 ballots per key present in the wave.
SB_DEV void bykey_count(uint32_t *s_cnt, int lane, bool counted, uint32_t key, uint32_t F) {
  uint32_t present = wave_or(counted ? (1u << key) : 0u);
  while (present) {
    const uint32_t k = __builtin_ctz(present);
    present &= present - 1;
    const bool in = counted && key == k;
    uint32_t mycnt = 0;
#pragma unroll
    for (int ff = 0; ff < 19; ff++) {
      const unsigned long long m = __ballot(in && ((F >> ff) & 1u));
      mycnt = (lane == ff) ? (uint32_t)__popcll(m) : mycnt;
    }
    if (lane < 19 && mycnt) atomicAdd(&s_cnt[k * 19 + lane], mycnt);
  }
}

// PART 0: every tile of [x0, x1); PART 1: only the interior tiles [tlo, thi) (interior_tiles), compiled without
// the boundary path so its register budget is its own; PART 2: every tile except [tlo, thi).
template <int MODE, int PART>
__global__ __launch_bounds__(kCheckThreads, PART == 1 ? kCheckWgsInt : kCheckWgs) void k_check(
    StreamView sv, int64_t x0, int64_t x1, int R, CountsDev cd, unsigned long long *__restrict__ bitmap,
    uint32_t *__restrict__ words, int64_t tlo, int64_t thi) {
  constexpr bool EAGER = MODE == MODE_EAGER;
  constexpr bool COUNTS = MODE == MODE_COUNTS || MODE == MODE_BYKEY;
  constexpr bool BYKEY = MODE == MODE_BYKEY;
  __shared__ __attribute__((aligned(16))) uint8_t s_win[kWin + 64];
  __shared__ uint32_t s_opc[4 * kOpcWords];
  __shared__ uint32_t s_nbad[kNameWords];
  __shared__ int32_t s_lens[kLdsLens];
  __shared__ unsigned long long s_acc[19 + 21 + 3];  // totals, positions per key, succ/tff/halo
  __shared__ uint32_t s_cnt[BYKEY ? 21 * 19 : 1];
  __shared__ uint32_t s_k12[3 * 19];    // keys 0-2 × flag (non-BYKEY modes)
  __shared__ uint32_t s_pair[19 * 19];  // close-call pairs (key 2)
  __shared__ int32_t s_nxt[4 * kNxt];   // long op arrays (stage_nxt)
  __shared__ int64_t s_pw[4][4];        // ... past the window, per wave and class (first_bad_op)
  const int lane = lane_id();
  for (int i = threadIdx.x; i < 3 * 19; i += kCheckThreads) s_k12[i] = 0;
  for (int i = threadIdx.x; i < 19 * 19; i += kCheckThreads) s_pair[i] = 0;
  const int32_t *lensL = nullptr;
  if (sv.nref <= kLdsLens) {
    for (int i = threadIdx.x; i < sv.nref; i += kCheckThreads) s_lens[i] = (int32_t)sv.lens[i];
    lensL = s_lens;
  }
  for (int i = threadIdx.x; i < 19 + 21 + 3; i += kCheckThreads) s_acc[i] = 0;
  if (BYKEY)
    for (int i = threadIdx.x; i < 21 * 19; i += kCheckThreads) s_cnt[i] = 0;

  const int64_t x0a = x0 & ~(int64_t)63;
  const int64_t ntiles = (x1 - x0a + kTile - 1) / kTile;
  Acc acc;
  acc.clear();
  int since_flush = 0;

  const int64_t nskip = PART == 2 ? thi - tlo : 0;
  const int64_t tcount = PART == 1 ? thi - tlo : ntiles - nskip;
  for (int64_t ti = blockIdx.x; ti < tcount; ti += gridDim.x) {
    const int64_t t = PART == 1 ? tlo + ti : (ti >= tlo ? ti + nskip : ti);
    const int64_t base = x0a + t * kTile;
    __syncthreads();
    stage_tile(sv, base, s_win, s_opc, s_nbad);
    if (lane < 4) s_pw[threadIdx.x >> 6][lane] = -1;
    __syncthreads();
    stage_nxt(s_opc, s_nxt);
    __syncthreads();
    const Tile tl{s_win, s_opc, s_nbad, base, s_nxt, s_pw[threadIdx.x >> 6]};
    const uint32_t *w32 = reinterpret_cast<const uint32_t *>(s_win);
    uint32_t hkp[3] = {0, 0, 0}, hpl[3] = {0, 0, 0};  // held compressed counts of an even group (add4_paired)
    constexpr bool TILECNT = MODE == MODE_COUNTS && PART == 2;  // boundary tiles of the bit-sliced pass
    uint32_t tc = 0;                                             // PASS0 positions of the words this lane writes
    auto run_tile = [&](auto interior_tag) {
    constexpr bool INTERIOR = decltype(interior_tag)::value;
#pragma unroll 1
    for (int j = 0; j < kTile / (4 * kCheckThreads); j++) {
      const int g = j * kCheckThreads + threadIdx.x;  // group of 4 consecutive positions
      const int64_t xg = base + 4 * g;
      uint32_t W[10];
#pragma unroll
      for (int q = 0; q < 10; q++) W[q] = w32[g + q];
      uint32_t wd[4];
#pragma unroll
      for (int o = 0; o < 4; o++) {
        const int64_t x = xg + o;
        int32_t f[8];
#pragma unroll
        for (int q = 0; q < 8; q++) f[q] = o == 0 ? (int32_t)W[q] : (int32_t)__builtin_amdgcn_alignbyte(W[q + 1], W[q], o);
        uint32_t w = check_first<EAGER, INTERIOR>(tl, sv, lensL, x, 4 * g + o, R, f);
        if (!INTERIOR) w = (x >= x0 && x < x1) ? w : W_NONE;  // interior tiles lie inside [x0, x1)
        wd[o] = w;
      }
      if (MODE == MODE_WORDS) {
#pragma unroll
        for (int o = 0; o < 4; o++)
          if (wd[o] != W_NONE && wd[o] != W_PASS0) words[xg + o - x0] = wd[o];
      }
      // first-record-pass bits: nibble per lane → 16 lanes per 64-bit word; k_chains turns them into calls
      uint32_t nib = 0;
#pragma unroll
      for (int o = 0; o < 4; o++) nib |= (wd[o] == W_PASS0) ? (1u << o) : 0u;
      uint64_t v = 0;
      if (__ballot(nib != 0u)) {  // (a wave's 256 positions hold no record-0 pass about half the time)
        v = (uint64_t)nib << (4 * (lane & 15));
        v |= shfl_xor64(v, 1);
        v |= shfl_xor64(v, 2);
        v |= shfl_xor64(v, 4);
        v |= shfl_xor64(v, 8);
      }
      if (INTERIOR) {
        bitmap[(xg - x0a) >> 6] = v;  // the 16 lanes of a word store the same value: no branch
      } else if ((lane & 15) == 0 && xg < x1) {
        bitmap[(xg - x0a) >> 6] = v;  // word holds >= 1 position < x1
      }
      if (TILECNT && (lane & 15) == 0 && (INTERIOR || xg < x1)) tc += (uint32_t)__popcll(v);
      if (!COUNTS) continue;
      uint32_t Fo[4];
      if constexpr (INTERIOR && !BYKEY) {
        uint32_t oh[4];
        bool low = false;
#pragma unroll
        for (int o = 0; o < 4; o++) {
          Fo[o] = wd[o] & 0x7ffffu;
          oh[o] = 1u << __popc(Fo[o]);
          low |= (oh[o] & 6u) != 0;  // key 1 or 2
        }
        if (__ballot(low)) {
#pragma unroll
          for (int o = 0; o < 4; o++) {
            uint32_t oh2;
            if (oh[o] & 6u) classify_interior(wd[o], s_k12, s_pair, oh2);
          }
        }
        add4_paired(acc.kp, oh, hkp, (j & 1) != 0);
      } else {
#pragma unroll
        for (int o = 0; o < 4; o++) {
          uint32_t key = 0;
          bool counted = false;
          Fo[o] = 0;
          if (wd[o] != W_NONE && wd[o] != W_PASS0)
            Fo[o] = acc.classify<BYKEY>(wd[o], cd, s_k12, s_pair, key, counted);
          if (BYKEY) bykey_count(s_cnt, lane, counted, key, Fo[o]);
        }
      }
      if constexpr (INTERIOR && !BYKEY) add4_paired(acc.pl, Fo, hpl, (j & 1) != 0);
      else add4(acc.pl, Fo);
    }
    };
    if constexpr (PART == 1) {
      run_tile(std::integral_constant<bool, true>{});
    } else {
      if (base >= x0 && base + kTile <= x1 && base + kTile + kInteriorTail <= sv.L)
        run_tile(std::integral_constant<bool, true>{});
      else run_tile(std::integral_constant<bool, false>{});
    }
    if (TILECNT && cd.tile_pass0) {
      const uint32_t c = wave_sum(tc);
      if (lane == 0) cd.tile_pass0[t * 4 + (int)(threadIdx.x >> 6)] = (int32_t)c;
    }
    if (COUNTS) {
      if (++since_flush == kFlushTiles) {
        flush_acc(acc, s_acc, lane);
        since_flush = 0;
      }
    }
  }
  if (COUNTS) {
    flush_acc(acc, s_acc, lane);
    __syncthreads();
    if (threadIdx.x < 19 && s_acc[threadIdx.x]) atomicAdd(&cd.totals[threadIdx.x], s_acc[threadIdx.x]);
    if (threadIdx.x >= 32 && threadIdx.x < 53) {
      const int k = threadIdx.x - 32;
      if (s_acc[19 + k]) atomicAdd(&cd.positions[k], s_acc[19 + k]);
    }
    if (threadIdx.x >= 64 && threadIdx.x < 67 && s_acc[40 + threadIdx.x - 64])
      atomicAdd(&cd.scalars[1 + threadIdx.x - 64], s_acc[40 + threadIdx.x - 64]);
    if (BYKEY)
      for (int i = threadIdx.x; i < 21 * 19; i += kCheckThreads)
        if (s_cnt[i]) atomicAdd(&cd.counts[i], (unsigned long long)s_cnt[i]);
    if (!BYKEY)
      for (int i = threadIdx.x; i < 3 * 19; i += kCheckThreads)
        if (s_k12[i]) atomicAdd(&cd.counts[i], (unsigned long long)s_k12[i]);
    for (int i = threadIdx.x; i < 19 * 19; i += kCheckThreads)
      if (s_pair[i]) atomicAdd(&cd.pair[i], (unsigned long long)s_pair[i]);
  }
}

// ---- full-check Counts over interior tiles, bit-sliced ------------------------------------------------------------
// k_check<MODE_COUNTS, *> evaluates a position's 19 flags into one word and counts the words.  Here the positions
// are the bits: lane t of the workgroup owns the 32 positions 1024 j + 4 t + o (j < 8, o < 4) of a tile, and every
// per-position predicate becomes one bit of a per-lane "plane" (bit 31 - (4 j + o), appended by one v_addc:
// plane + plane + the predicate's lane mask as carry-in).  Then
//   * the reference-index predicates depend on one int32 each (PosChecker.scala:43-63): refIdx / refPos at x + 4 /
//     x + 8, nextRefIdx / nextRefPos at x + 24 / x + 28.  A predicate pass evaluates "I(y) < -1", "I(y) >= n_ref"
//     and "0 <= I(y) < n_ref && I(y + 4) > len[I(y)]" once per byte offset y into three LDS plane arrays; y = x + 4k
//     is lane t + k's position, so flags 1-8 of lane t are those arrays at t + 1, t + 2, t + 6, t + 7 (3 predicate
//     evaluations per position instead of 8);
//   * the per-record predicates (read name, CIGAR, the implied length, the EmptyMapped fields) are evaluated per
//     position (full/Checker.scala:22-184) and appended;
//   * the 32 positions' flags combine as whole planes: per-flag totals are 16 v_bcnt; the key (number of flags) is a
//     carry-save sum of 8 planes of mutually exclusive flag groups (at most one flag of each group holds at a
//     position), decoded per key with one 3-input op and counted by v_bcnt; PASS0 is the NOR of the planes,
//     transposed across 8 lanes (ds_swizzle) into bitmap dwords.
// A position with a long name or op array (past the 64 bytes / ops one bitmap read covers) is redone by check_first
// and patched into the planes.  Interior tiles only (no EOF in reach), R > 0; the contig lengths are in LDS when
// n_ref <= kLdsLens, else in the device table (round 5: many-contig references took the general k_check before).
SB_DEV uint32_t push_bit(uint32_t p, bool c) {  // (the carry-out goes to VCC: a dead SGPR-pair output made the
  uint32_t r;                                    // compiler reuse one pair and pad with s_nop between VALU writes)
  asm("v_addc_co_u32 %0, vcc, %1, %1, %2" : "=v"(r) : "v"(p), "s"(__ballot(c)) : "vcc");
  return r;
}
// One stage of an 8 x 8 transpose of nibbles across 8 lanes (nibble j of lane li -> nibble li of lane j): exchange
// with lane li ^ S the nibbles j whose bit S differs from li's.
template <int S>
SB_DEV uint32_t nibble_xpose_stage(uint32_t P, int li) {
  const uint32_t Q = (uint32_t)__builtin_amdgcn_ds_swizzle((int)P, 0x1f | (S << 10));
  constexpr uint32_t Ms = S == 4 ? 0xffff0000u : S == 2 ? 0xff00ff00u : 0xf0f0f0f0u;  // nibbles j with j & S
  const bool hi = (li & S) != 0;
  const uint32_t r = __builtin_amdgcn_alignbit(Q, Q, hi ? 4 * S : 32 - 4 * S);
  return hi ? ((P & Ms) | (r & ~Ms)) : ((P & ~Ms) | (r & Ms));
}
// Index of the lowest set bit of hi:lo, 0xffffffff if none (v_ffbl's value for 0: two ffbl, an or, a min).
SB_DEV uint32_t ffbl(uint32_t x) {  // (a cttz with a defined zero would add a compare and a select)
  uint32_t r;
  asm("v_ffbl_b32 %0, %1" : "=v"(r) : "v"(x));
  return r;
}
SB_DEV uint32_t ctz64(uint32_t lo, uint32_t hi) { return min(ffbl(lo), ffbl(hi) | 32u); }
// plane i of X[] holds flag kBitFlag[i] (the flags an interior position can fail)
constexpr int kBitFlag[16] = {1, 2, 3, 4, 5, 6, 7, 8, 10, 11, 12, 13, 15, 16, 17, 18};

// k_check_bits' op arrays of > 64 ops whose first 64 are valid (bits q of lane t's planes): the window's invalid-op
// table, then the stream past the window, read once per tile and class by the whole wave (scan_past_window; nbe: the
// wave's LDS slots; the table itself is built by the wave when a tile first needs it, wave_nxt).  A long read's packed
// sequence puts every position here.  Wave-uniform call.
// First invalid op start (window-relative) at or after y given that ops [y, y + 256) are valid (fb[y] >= 64), kNoBad
// if none before the window's end: one more first-invalid-op byte, then the table (wave_nxt) from the next entry.
SB_DEV int32_t next_bad_deep(const Tile &t, const uint8_t *fb, int y) {
  const int y2 = y + 256;
  if (y2 >= kWin) return kNoBad;
  if (y2 >= kFbBytes) return next_bad_in_window(t, y2);
  const uint32_t f = fb[y2];
  if (f < 64u) return y2 + 4 * (int32_t)f;
  const int r = y & 3, k = (y2 + 256 - r) >> 8;  // 256 k + r lies in (y2, y2 + 256]: the ops before it are valid
  return t.nxt[r * kNxt + k];
}

SB_DEV uint32_t long_ops_pass(const Tile &tl, const uint8_t *fb, const StreamView &sv, uint32_t q, uint32_t pIV, int t,
                              int64_t *nbe) {
  auto at = [&](int b, int &crel, int32_t &nc) {  // bit b's op array: window-relative start, n_cigar
    const int k = 31 - b, rel = 4 * ((k >> 2) * kCheckThreads + t) + (k & 3);
    const int32_t lrn = tl.win[rel + 12];
    nc = (int32_t)tl.win[rel + 16] | ((int32_t)tl.win[rel + 17] << 8);
    crel = rel + 36 + (lrn >= 2 ? lrn : 0);
  };
  // ops 64 .. 127 from the first-invalid-op bytes (short-read data: the rare position here finds its invalid op
  // there); a run that goes on ("deep") takes the wave's table, one that reaches the window's end ("past") the
  // stream.  A wave with many lanes here is inside a long valid run (a long read's sequence): it builds the table
  // first and resolves every position in one pass.
  const bool table = __popcll(__ballot(q != 0u)) >= kTableLanes;
  if (table) wave_nxt(tl.opc, const_cast<int32_t *>(tl.nxt));
  uint32_t deep = 0, past = 0, cls = 0;
  auto decide = [&](int b, int crel, int e, int32_t p) {
    if (p != kNoBad) {
      if (p < e) pIV |= 1u << b;
    } else if (kWin < e) {
      past |= 1u << b;
      cls |= 1u << (crel & 3);
    }
  };
  constexpr int kGroup = 2;  // (4: spills, 54.5 vs 53.8 ms on the long-read check; 2: 52.6)
  // table waves: kGroup positions at a time with every LDS read issued unconditionally (clamped addresses), so their
  // dependent chains (the record's bytes, two first-invalid-op bytes, the table) overlap instead of running one
  // position after another
  while (table && __ballot(q != 0u)) {
    int bb[kGroup], crel[kGroup], y[kGroup];
    int32_t nc[kGroup], p[kGroup];
    bool vv[kGroup];
#pragma unroll
    for (int k = 0; k < kGroup; k++) {
      vv[k] = q != 0u;
      bb[k] = vv[k] ? __builtin_ctz(q) : 0;
      q = vv[k] ? q & (q - 1u) : q;
      at(bb[k], crel[k], nc[k]);
    }
#pragma unroll
    for (int k = 0; k < kGroup; k++) {
      y[k] = crel[k] + 256;
      const int y2 = y[k] + 256, r = y[k] & 3;
      const uint32_t f = fb[min(y[k], kFbBytes - 1)], f2 = fb[min(y2, kFbBytes - 1)];
      const int32_t tb = tl.nxt[r * kNxt + min((y2 + 256 - r) >> 8, kNxt - 1)];
      // -1 / -2: the bitmap and the table from y / y2 (a first-invalid-op byte not staged there)
      p[k] = y[k] >= kWin ? kNoBad : y[k] >= kFbBytes ? -1 : f < 64u ? y[k] + 4 * (int32_t)f
             : y2 >= kWin ? kNoBad : y2 >= kFbBytes ? -2 : f2 < 64u ? y2 + 4 * (int32_t)f2 : tb;
    }
#pragma unroll
    for (int k = 0; k < kGroup; k++) {
      if (!vv[k]) continue;
      int32_t pk = p[k];
      if (pk < 0) pk = next_bad_in_window(tl, pk == -1 ? y[k] : y[k] + 256);
      decide(bb[k], crel[k], crel[k] + 4 * nc[k], pk);
    }
  }
  for (; q; q &= q - 1u) {
    const int b = __builtin_ctz(q);
    int crel;
    int32_t nc;
    at(b, crel, nc);
    const int y = crel + 256, e = crel + 4 * nc;  // (ops 0-63 are valid: pIV is clear)
    const uint32_t f = y < kFbBytes ? fb[y] : 64u;  // (>= 64: no invalid op among the 64 from y, or unknown)
    if (f < 64u) {
      if (y + 4 * (int)f < e) pIV |= 1u << b;
    } else if (y >= kWin) {
      decide(b, crel, e, kNoBad);
    } else if (y >= kFbBytes) {
      if (table) decide(b, crel, e, next_bad_in_window(tl, y));
      else deep |= 1u << b;
    } else if (y + 256 < e) {  // (else the 64 valid ops from y are the rest of the array)
      if (table) decide(b, crel, e, next_bad_deep(tl, fb, y));
      else deep |= 1u << b;
    }
  }
  if (__ballot(deep != 0u)) {
    wave_nxt(tl.opc, const_cast<int32_t *>(tl.nxt));
    for (; deep; deep &= deep - 1u) {
      const int b = __builtin_ctz(deep);
      int crel;
      int32_t nc;
      at(b, crel, nc);
      decide(b, crel, crel + 4 * nc, next_bad_in_window(tl, crel + 256));
    }
  }
  const uint32_t need = wave_or(cls);
  if (need) {
    scan_past_window(sv, tl.base + kWin, need, nbe);
    for (; past; past &= past - 1u) {
      const int b = __builtin_ctz(past);
      int crel;
      int32_t nc;
      at(b, crel, nc);
      if (nbe[crel & 3] < tl.base + crel + 4 * (int64_t)nc) pIV |= 1u << b;
    }
  }
  return pIV;
}

__global__ __launch_bounds__(kCheckThreads, kCheckWgsBits) void k_check_bits(StreamView sv, int64_t x0, int R,
                                                                                   CountsDev cd,
                                                                                   unsigned long long *__restrict__ bitmap,
                                                                                   int64_t tlo, int64_t thi) {
  __shared__ __attribute__((aligned(16))) uint8_t s_win[kWin + 64];
  __shared__ uint32_t s_opc[4 * kOpcWords];
  __shared__ uint32_t s_nbad[kNameWords];
  __shared__ __attribute__((aligned(16))) uint8_t s_fb[kFbBytes];  // first invalid op from each byte (stage_fb)
  __shared__ int32_t s_nxt[4][4 * kNxt];                            // long op arrays, per wave (wave_nxt)
  __shared__ int64_t s_nbe[4][4];                                   // ... past the window, per wave and class
  // per lane and byte offset y of its 32: I(y) < -1, I(y) >= n_ref, 0 <= I(y) < n_ref && I(y + 4) > len[I(y)],
  // byte(y) == 0, byte(y) == 1, byte(y) > 64 (I(y): the int32 at y)
  __shared__ uint32_t s_pl[6][kCheckThreads + 8];
  __shared__ unsigned long long s_acc[19 + 21];     // totals, positions per key
  __shared__ uint32_t s_k12[3 * 19];
  __shared__ uint32_t s_pair[19 * 19];
  extern __shared__ int32_t s_lens[];  // the n_ref contig lengths, then INT_MAX (dynamic, n_ref + 1 entries)
  const int t = (int)threadIdx.x, lane = lane_id(), li = t & 7;
  for (int i = t; i < 3 * 19; i += kCheckThreads) s_k12[i] = 0;
  for (int i = t; i < 19 * 19; i += kCheckThreads) s_pair[i] = 0;
  for (int i = t; i < 19 + 21; i += kCheckThreads) s_acc[i] = 0;
  const int32_t nref = sv.nref;
  // contig lengths in LDS when they fit (the dynamic allocation is n_ref + 1 entries then); else the rare probes
  // below read the device table (L2-resident, ~1 % of offsets)
  const bool lds_lens = nref <= kLdsLens;
  if (lds_lens)
    for (int i = t; i <= nref; i += kCheckThreads) s_lens[i] = i < nref ? (int32_t)sv.lens[i] : 0x7fffffff;
  const int64_t x0a = x0 & ~(int64_t)63;
  const uint32_t *w32 = reinterpret_cast<const uint32_t *>(s_win);
  // per-lane counters, two 16-bit halves per register: c < 16 = plane c's flag total, 16 + k - 1 = key k
  // (at most 32 per tile: flushed every kBitsFlush tiles)
  constexpr int kBitsFlush = 2047;
  uint32_t cnt[12];
#pragma unroll
  for (int i = 0; i < 12; i++) cnt[i] = 0;
  auto add_cnt = [&](int c, uint32_t v) { cnt[c >> 1] += (c & 1) ? v << 16 : v; };
  auto flush_cnt = [&]() {
#pragma unroll
    for (int c = 0; c < 24; c++) {
      const uint32_t v = wave_sum((cnt[c >> 1] >> (16 * (c & 1))) & 0xffffu);
      if (lane == 0 && v) atomicAdd(&s_acc[c < 16 ? kBitFlag[c] : 19 + c - 15], (unsigned long long)v);
    }
#pragma unroll
    for (int i = 0; i < 12; i++) cnt[i] = 0;
  };
  int since_flush = 0;

  for (int64_t ti = blockIdx.x; ti < thi - tlo; ti += gridDim.x) {
    const int64_t base = x0a + (tlo + ti) * kTile;
    __syncthreads();
    stage_tile(sv, base, s_win, s_opc, s_nbad);
    __syncthreads();
    stage_fb(s_win, s_opc, s_fb);
    // ---- predicate pass over the offsets 1024 j + 4 t + o; lanes t < 8 add row 8 (offsets 8192 + 4 t + o), which
    // shifts row 0 out and leaves exactly the planes of lanes 256 + t.  The contig-length test reads the length table
    // only at offsets whose int32 is a contig index (a bit loop over that plane: ~1 % of offsets)
    {
      uint32_t pa = 0, pb = 0, pz = 0, pe = 0, pg = 0;
      auto row = [&](int j) {
        const int g = j * kCheckThreads + t;
        const uint32_t W0 = w32[g], W1 = w32[g + 1];
#pragma unroll
        for (int o = 0; o < 4; o++) {
          const int32_t I = (int32_t)(o == 0 ? W0 : __builtin_amdgcn_alignbyte(W1, W0, o));
          const uint32_t by = (uint32_t)I & 0xffu;
          pa = push_bit(pa, I < -1);
          pb = push_bit(pb, I >= nref);
          pz = push_bit(pz, by == 0);
          pe = push_bit(pe, by == 1);
          pg = push_bit(pg, by > 64);
        }
      };
      // I(y + 4) > len[I(y)] where I(y) is a contig index: the bits of neither plane (-1 <= I < n_ref; I = -1
      // is tested and skipped); r0: the row of plane bit 31 (1 for lanes 256 + t)
      auto bigpos = [&](uint32_t in, int r0) {
        uint32_t pc = 0;
        for (uint32_t q = in; q; q &= q - 1u) {
          const int b = __builtin_ctz(q), k = 31 - b;
          const int y = 4 * (((k >> 2) + r0) * kCheckThreads + t) + (k & 3);
          const int32_t I = (int32_t)__builtin_amdgcn_alignbyte(w32[(y >> 2) + 1], w32[y >> 2], y & 3);
          const int32_t I4 = (int32_t)__builtin_amdgcn_alignbyte(w32[(y >> 2) + 2], w32[(y >> 2) + 1], y & 3);
          const int64_t len = lds_lens ? (int64_t)s_lens[I >= 0 ? I : 0] : sv.lens[I >= 0 ? I : 0];
          pc |= (I >= 0 && (int64_t)I4 > len) ? (1u << b) : 0u;
        }
        return pc;
      };
#pragma unroll 1
      for (int j = 0; j < 8; j++) row(j);
      s_pl[0][t] = pa;
      s_pl[1][t] = pb;
      s_pl[2][t] = bigpos(~(pa | pb), 0);
      s_pl[3][t] = pz;
      s_pl[4][t] = pe;
      s_pl[5][t] = pg;
      if (t < 8) {
        row(8);
        s_pl[0][kCheckThreads + t] = pa;
        s_pl[1][kCheckThreads + t] = pb;
        s_pl[2][kCheckThreads + t] = bigpos(~(pa | pb), 1);
        s_pl[3][kCheckThreads + t] = pz;
        s_pl[4][kCheckThreads + t] = pe;
        s_pl[5][kCheckThreads + t] = pg;
      }
    }
    __syncthreads();
    // ---- per-record predicates; the byte-local ones come from the byte planes of the lanes 3-5 to the right
    // (a field at byte offset 4q + K of position x is byte plane bit x + 4q + K: lane t + q, shifted by K)
    uint32_t pLZ = 0, pIV = 0, pTF = 0, pFL = 0;
#pragma unroll 1
    for (int j = 0; j < 8; j++) {
      const int g = j * kCheckThreads + t;
      uint32_t W[7];
#pragma unroll
      for (int q = 0; q < 7; q++) W[q] = w32[g + q];
      // flag & 4 (segment unmapped) of the 4 positions: bit 2 of bytes 18-21 (position o at nibble bit 3 - o)
      pFL = (pFL << 4) | ((W[4] >> 15) & 8u) | ((W[4] >> 24) & 4u) | ((W[5] >> 1) & 2u) | ((W[5] >> 10) & 1u);
#pragma unroll
      for (int o = 0; o < 4; o++) {
        const int rel = 4 * g + o;
        auto fld = [&](int q) { return o == 0 ? W[q] : __builtin_amdgcn_alignbyte(W[q + 1], W[q], o); };
        const int32_t bs = (int32_t)fld(0);
        const int32_t lrn = (int32_t)((W[3] >> (8 * o)) & 0xffu);
        const int32_t nc = (int32_t)(fld(4) & 0xffffu);
        const int32_t ls = (int32_t)fld(5);
        // the name's last byte (read for lrn < 2 too, unused then); first invalid op (>= 64: none among the first
        // 64); ops start at 36 + lrn, or 36 when lrn < 2: lrn = 0 reads the right byte, lrn = 1 is redone below.
        // (Round 4: both bits from one fb byte — bit 7 = "byte before is 0", set in stage_fb — was slower, 43.2 vs
        // 41.4 ms: the stage_fb work costs more than the LDS read it saves.)
        const uint32_t last = s_win[rel + 35 + lrn];
        const uint32_t obad = s_fb[rel + 36 + lrn];
        pLZ = push_bit(pLZ, last == 0);
        pIV = push_bit(pIV, obad < min((uint32_t)nc, 64u));  // an invalid op among the first min(nc, 64)
        pTF = push_bit(pTF, too_few_remaining(bs, lrn, nc, ls));
      }
    }
    // byte planes: K = 1..3 shifts a plane by K positions (bits of a nibble move up; the top K come from lane u + 1)
    auto shk = [&](int K, const uint32_t *P, int u) {
      const uint32_t M = K == 1 ? 0xeeeeeeeeu : K == 2 ? 0xccccccccu : 0x88888888u;
      return ((P[u] << K) & M) | ((P[u + 1] >> (4 - K)) & ~M);
    };
    const uint32_t *PZ = s_pl[3], *PE = s_pl[4], *PG = s_pl[5];
    const uint32_t pZ = PZ[t + 3];                                                       // l_read_name == 0
    const uint32_t pO = PE[t + 3];                                                       // l_read_name == 1
    const uint32_t z17 = shk(1, PZ, t + 4);
    const uint32_t pNC = PZ[t + 4] & z17;                                                 // n_cigar == 0
    const uint32_t pNG = ~z17 | PG[t + 4];                                                // n_cigar > 64
    const uint32_t pLS = PZ[t + 5] & shk(1, PZ, t + 5) & shk(2, PZ, t + 5) & shk(3, PZ, t + 5);  // l_seq == 0
    // l_read_name == 1: the ops start at 36, not 37
    for (uint32_t q = pO; q; q &= q - 1u) {
      const int b = __builtin_ctz(q), k = 31 - b, rel = 4 * ((k >> 2) * kCheckThreads + t) + (k & 3);
      const uint32_t nc = (uint32_t)s_win[rel + 16] | ((uint32_t)s_win[rel + 17] << 8);
      pIV = (pIV & ~(1u << b)) | (s_fb[rel + 36] < min(nc, 64u) ? (1u << b) : 0u);
    }
    // the name characters matter only where the name ends in NUL (true records and ~1/256 of the rest): those
    // positions are checked one by one, and so are the op arrays longer than 64 ops whose first 64 are valid
    const Tile tl{s_win, s_opc, s_nbad, base, s_nxt[t >> 6]};
    const uint32_t HN = ~(pZ | pO);  // l_read_name >= 2
    uint32_t pNB = 0;
    for (uint32_t q = HN & pLZ; q; q &= q - 1u) {
      const int b = __builtin_ctz(q), k = 31 - b, rel = 4 * ((k >> 2) * kCheckThreads + t) + (k & 3);
      const int32_t nbody = (int32_t)s_win[rel + 12] - 1;
      const uint64_t nbm = bits64(s_nbad, rel + 36);
      bool bad = ctz64((uint32_t)nbm, (uint32_t)(nbm >> 32)) < (uint32_t)nbody;
      if (!bad && nbody > 64) bad = name_has_bad(tl, rel + 36 + 64, nbody - 64);
      pNB |= bad ? (1u << b) : 0u;
    }
    // (op arrays of > 64 ops whose first 64 are valid: the window's invalid-op table, then the stream past the window
    // read once per tile and class by the whole wave — a long read's packed sequence puts every position here)
    if (__ballot((pNG & ~pIV) != 0u)) pIV = long_ops_pass(tl, s_fb, sv, pNG & ~pIV, pIV, t, s_nbe[t >> 6]);
    // ---- flag planes
    uint32_t X[16];
    X[0] = s_pl[0][t + 1];          // 1  refIdx < -1
    X[1] = s_pl[1][t + 1];          // 2  refIdx >= n_ref
    X[2] = s_pl[0][t + 2];          // 3  refPos < -1
    X[3] = s_pl[2][t + 1];          // 4  refPos > len[refIdx]
    X[4] = s_pl[0][t + 6];          // 5-8 the same for nextRefIdx / nextRefPos
    X[5] = s_pl[1][t + 6];
    X[6] = s_pl[0][t + 7];
    X[7] = s_pl[2][t + 6];
    X[8] = HN & ~pLZ;               // 10 name not NUL-terminated
    X[9] = HN & pLZ & pNB;          // 11 non-ASCII name
    X[10] = pZ;                     // 12 no read name
    X[11] = pO;                     // 13 empty read name
    X[12] = pIV;                    // 15 invalid CIGAR op
    X[13] = ~pFL & pLS & ~pIV;      // 16 EmptyMapped: no sequence
    X[14] = ~pFL & pNC & ~pIV;      // 17 EmptyMapped: no CIGAR ops
    X[15] = pTF;                    // 18 too few remaining bytes for the implied length
    // ---- counting: per-flag totals, then the key from 8 planes of mutually exclusive flags
#pragma unroll
    for (int i = 0; i < 16; i++) add_cnt(i, (uint32_t)__popc(X[i]));
    const uint32_t Y0 = X[0] | X[1] | X[3], Y1 = X[2];      // {1, 2, 4}: refIdx < -1 / >= n_ref / in range
    const uint32_t Y2 = X[4] | X[5] | X[7], Y3 = X[6];
    const uint32_t Y4 = X[8] | X[9] | X[10] | X[11];         // {10, 11, 12, 13}: by l_read_name and the last byte
    const uint32_t Y5 = X[12] | X[13], Y6 = X[14], Y7 = X[15];  // {15, 16}: by the invalid-op test
    auto fa = [](uint32_t a, uint32_t b, uint32_t c, uint32_t &s) {
      s = a ^ b ^ c;
      return (a & b) | (c & (a ^ b));
    };
    uint32_t s1, s2, s3, s5;
    const uint32_t c1 = fa(Y0, Y1, Y2, s1), c2 = fa(Y3, Y4, Y5, s2), c3 = fa(s1, s2, Y6, s3);
    const uint32_t b0 = s3 ^ Y7, c4 = s3 & Y7;
    const uint32_t c5 = fa(c1, c2, c3, s5);
    const uint32_t b1 = s5 ^ c4, c6 = s5 & c4;
    const uint32_t b2 = c5 ^ c6, b3 = c5 & c6;  // key = b0 + 2 b1 + 4 b2 + 8 b3 <= 8 (b3: key 8, the rest 0)
    const uint32_t K1 = b0 & ~b1 & ~b2, K2 = ~b0 & b1 & ~b2;
    add_cnt(16, (uint32_t)__popc(K1));
    add_cnt(17, (uint32_t)__popc(K2));
    add_cnt(18, (uint32_t)__popc(b0 & b1 & ~b2));
    add_cnt(19, (uint32_t)__popc(~b0 & ~b1 & b2));
    add_cnt(20, (uint32_t)__popc(b0 & ~b1 & b2));
    add_cnt(21, (uint32_t)__popc(~b0 & b1 & b2));
    add_cnt(22, (uint32_t)__popc(b0 & b1 & b2));
    add_cnt(23, (uint32_t)__popc(b3));
    if (++since_flush == kBitsFlush) {
      flush_cnt();
      since_flush = 0;
    }
    if (__ballot((K1 | K2) != 0u)) {  // keys 1-2: per-flag counts and close-call pairs (rare)
      uint32_t m = K1 | K2;
      while (m) {
        const int b = __builtin_ctz(m);
        m &= m - 1u;
        uint32_t F = 0;
#pragma unroll
        for (int i = 0; i < 16; i++) F |= ((X[i] >> b) & 1u) << kBitFlag[i];
        uint32_t oh;
        classify_interior(F, s_k12, s_pair, oh);
      }
    }
    // ---- PASS0 bits (no flag): bit 4 j + o after the reversal; an 8 x 8 nibble transpose across lanes t ^ 4, 2, 1
    // leaves lane li of each 8-lane group with row j = li of the group's 32 positions
    uint32_t P = __builtin_bitreverse32(~(Y0 | Y1 | Y2 | Y3 | Y4 | Y5 | Y6 | Y7));
    P = nibble_xpose_stage<4>(P, li);
    P = nibble_xpose_stage<2>(P, li);
    P = nibble_xpose_stage<1>(P, li);
    reinterpret_cast<uint32_t *>(bitmap)[((base - x0a) >> 5) + 32 * li + (t >> 3)] = P;
    if (cd.tile_pass0) {  // the chain pass's counts: this wave's PASS0 positions of the tile
      const uint32_t c = wave_sum((uint32_t)__popc(P));
      if (lane == 0) cd.tile_pass0[(tlo + ti) * 4 + (t >> 6)] = (int32_t)c;
    }
  }
  // per-lane counters -> workgroup -> device
  flush_cnt();
  __syncthreads();
  if (t < 19 && s_acc[t]) atomicAdd(&cd.totals[t], s_acc[t]);
  if (t >= 32 && t < 53 && s_acc[19 + t - 32]) atomicAdd(&cd.positions[t - 32], s_acc[19 + t - 32]);
  for (int i = t; i < 3 * 19; i += kCheckThreads)
    if (s_k12[i]) atomicAdd(&cd.counts[i], (unsigned long long)s_k12[i]);
  for (int i = t; i < 19 * 19; i += kCheckThreads)
    if (s_pair[i]) atomicAdd(&cd.pair[i], (unsigned long long)s_pair[i]);
}

// ---- eager record-0 pass over interior tiles, one wave per tile, with a prefilter ---------------------------------
// eager.Checker fails a position at its first failing check, and the first checks are the two reference indices
// (refIdx, nextRefIdx in [-1, n_ref): PosChecker.scala:43-63, eager/Checker.scala:24-126).  So every position is
// first tested on those two fields alone; only the survivors — true record starts and the few positions whose
// indices happen to be small — are checked in full.  Same PASS0 bitmap as k_check<MODE_EAGER, 1>.
// Round 5: no workgroup barrier (round 2-4's k_eager staged 8 KiB tiles per 256-thread workgroup, and its waves
// waited for one another at five barriers per tile and for one wave's survivor drain: 9.1 ms at 10 GB); every wave
// streams its own tiles.  Lane l holds the 16-B pieces 1024 k + 16 l of the tile (k < 8; one coalesced 16-B load per piece) and
// decides its 16 positions x = 1024 k + 16 l + j of each piece:
//   * V(y) = "the int32 at y is in [-1, n_ref)" is evaluated once per byte offset y = x + 4 of the lane's positions
//     (a 16-bit plane P_k per piece; refIdx at x + 4 — PosChecker.scala:43-63 / eager/Checker.scala:24-126);
//   * nextRefIdx at x + 24 = y + 20 is the plane of lanes l + 1 and l + 2 (wave_shl1 DPP; lanes 62-63 take the next
//     piece's lanes 0-1, and the tile's last piece the bytes past the tile, which lanes 0-3 load), so a position
//     costs one V evaluation, not two;
//   * the pieces also go to the wave's own LDS window (tile + 64 B), and the survivors S_k = P_k & (P_(l+1) >> 4 |
//     P_(l+2) << 12) (0.5 % of positions: true records and a few others) to the wave's LDS bitmap of the tile and a
//     wave-private queue; all 64 lanes check them in full from that window (a name or CIGAR ops that run past it
//     from global memory) and clear the failing ones with LDS atomics;
//   * the tile's 1 KiB of bitmap leaves as one coalesced 16-B store per lane.
// Waves never wait for one another (each has its own LDS: 16 waves per CU), so the memory system sees 16 independent
// streams per CU, and a survivor's dependent reads are LDS round trips, not memory ones.
constexpr int kEwQ = 128;                // survivor queue per wave (a tile's survivors are queued in rounds)
constexpr int kEwWaves = 4;
constexpr int kEwHalo = 64;              // bytes past the tile in the window (>= 32: nextRefIdx of the last positions)
constexpr int kEwWin = kTile + kEwHalo;  // per-wave LDS window
// The wave's layout assumes these: a tile is 8 pieces x 64 lanes x 16 B (piece k, lane l at 1024 k + 16 l; the queue
// holds tile offsets as uint16), the halo is whole 16-B pieces loaded by lanes 0 .. kEwHalo / 16 - 1 (piece 512), and
// the tile's bitmap leaves as one 16-B store per lane.
static_assert(kTile == 8 * 64 * 16, "k_eager_wave: a tile is 8 pieces of 64 lanes x 16 B");
static_assert(kEwHalo >= 32 && kEwHalo % 16 == 0 && kEwHalo <= 64 * 16, "k_eager_wave: halo of whole 16-B pieces");
static_assert(kTile / 32 == 64 * 4, "k_eager_wave: the tile's bitmap is one u32x4 per lane");
// eager.Checker record-0 checks at position rel of a wave's window (win = the tile's bytes from base), given the
// fixed fields f[]: check_first<true, true>'s pass/fail, straight from the bytes (no op-class / name-character
// bitmaps: survivors are few, and a true record's name and CIGAR are short).
// 0: fails; 1: passes; 2: passes so far, with the ops from 64 on (n64 of them at c64) left to a wave-cooperative read
// (ops_bad_wave: a long read's CIGAR has thousands of ops).
SB_DEV int eager_pass_win(const uint8_t *win, const StreamView &sv, int64_t x, int rel, const int32_t f[8],
                          int64_t &c64, int32_t &n64) {
  const int32_t bs = f[0], ri = f[1], rp = f[2], bmn = f[3], fnc = f[4], ls = f[5], nri = f[6], nrp = f[7];
  const int32_t lrn = bmn & 0xff;
  const uint32_t flag = ((uint32_t)fnc) >> 16;
  const int32_t nc = fnc & 0xffff;
  if ((uint32_t)(lrn < 2) | (uint32_t)((flag & 4u) == 0 && (ls == 0 || nc == 0)) |
      (uint32_t)too_few_remaining(bs, lrn, nc, ls))
    return 0;
  if (ref_err(ri, rp, nullptr, sv.lens, sv.nref) | ref_err(nri, nrp, nullptr, sv.lens, sv.nref)) return 0;
  const gbytes u = gview(sv.u);
  const int c0 = rel + 36 + lrn;
  if (c0 + 4 > kEwWin) {  // the name runs past the window (a position in the tile's last ~300 B): global memory
    typedef const __attribute__((address_space(1))) uint32_t *g32;
    if (u[x + 35 + lrn] != 0) return 0;
    for (int i = 0; i < lrn - 1; i += 4) {
      const int64_t a = x + 36 + i;
      const g32 q = (g32)(u + (a & ~(int64_t)3));
      const uint32_t v = __builtin_amdgcn_alignbyte(q[1], q[0], (uint32_t)a & 3u);
      const int left = lrn - 1 - i;
      const uint32_t keep = left >= 4 ? 0x80808080u : (0x80808080u >> (8 * (4 - left)));
      if (name_bad_bytes(v) & keep) return 0;
    }
  } else {
    if (win[rel + 35 + lrn] != 0) return 0;  // name not NUL-terminated
    // allowedReadNameChars, 4 name bytes per step (SWAR over an unaligned dword of the window)
    const uint32_t *w32 = reinterpret_cast<const uint32_t *>(win);
    for (int i = 0; i < lrn - 1; i += 4) {
      const int a = rel + 36 + i;
      const uint32_t w = __builtin_amdgcn_alignbyte(w32[(a >> 2) + 1], w32[a >> 2], (uint32_t)a & 3u);
      const int left = lrn - 1 - i;
      const uint32_t keep = left >= 4 ? 0x80808080u : (0x80808080u >> (8 * (4 - left)));
      if (name_bad_bytes(w) & keep) return 0;
    }
  }
  const int n1 = min(nc, 64);
  const int in_win = max(0, min(n1, (kEwWin - c0) >> 2));  // ops inside the window, then global memory
  for (int i = 0; i < in_win; i++)
    if ((win[c0 + 4 * i] & 0xfu) > 8u) return 0;
  for (int i = in_win; i < n1; i++)
    if ((u[x + 36 + lrn + 4 * (int64_t)i] & 0xfu) > 8u) return 0;
  if (nc > 64) {
    c64 = x + 36 + lrn + 256;
    n64 = nc - 64;
    return 2;
  }
  return 1;
}

// lane l ← lane l + 1's v; lane 63 ← `last` (wave_shl1 DPP, the lane past the wave keeps the old value)
SB_DEV uint32_t from_next_lane(uint32_t v, uint32_t last) {
  return (uint32_t)__builtin_amdgcn_update_dpp((int)last, (int)v, 0x130, 0xf, 0xf, false);
}

__global__ __launch_bounds__(64 * kEwWaves) void k_eager_wave(StreamView sv, int64_t x0, int R,
                                                             unsigned long long *__restrict__ bitmap, int64_t tlo,
                                                             int64_t thi) {
  __shared__ __attribute__((aligned(16))) uint8_t s_win[kEwWaves][kEwWin + 16];
  __shared__ __attribute__((aligned(16))) uint32_t s_bm[kEwWaves][kTile / 32];
  __shared__ uint16_t s_q[kEwWaves][kEwQ];
  const int lane = lane_id(), wv = (int)threadIdx.x >> 6;
  uint8_t *win = s_win[wv];
  const uint32_t *w32 = reinterpret_cast<const uint32_t *>(win);
  uint32_t *bm = s_bm[wv];
  uint16_t *q = s_q[wv];
  const uint32_t nref1 = (uint32_t)sv.nref + 1u;  // -1 <= I < n_ref  <=>  (uint32)(I + 1) < n_ref + 1
  const int64_t x0a = x0 & ~(int64_t)63;
  const gbytes u = gview(sv.u);
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  typedef const __attribute__((address_space(1))) u32x4 *g16;
  auto wave_sync = []() {  // order this wave's LDS accesses (no other wave touches its LDS)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  };
  const int64_t nt = thi - tlo;
  for (int64_t ti = (int64_t)blockIdx.x * kEwWaves + wv; ti < nt; ti += (int64_t)gridDim.x * kEwWaves) {
    const int64_t base = x0a + (tlo + ti) * kTile;
    const g16 src = (g16)(u + base);
    u32x4 pc[9];
#pragma unroll
    for (int k = 0; k < 8; k++) pc[k] = src[64 * k + lane];
    pc[8] = lane < kEwHalo / 16 ? src[512 + lane] : u32x4{0u, 0u, 0u, 0u};  // the bytes past the tile
#pragma unroll
    for (int k = 0; k < 8; k++) reinterpret_cast<u32x4 *>(win)[64 * k + lane] = pc[k];
    if (lane < kEwHalo / 16) reinterpret_cast<u32x4 *>(win)[512 + lane] = pc[8];
    // P[k] bit j = V(1024 k + 16 l + 4 + j)
    uint32_t P[9];
#pragma unroll
    for (int k = 0; k < 9; k++) {
      const uint32_t n0 = from_next_lane(pc[k].x, k < 8 ? (uint32_t)__builtin_amdgcn_readfirstlane((int)pc[k < 8 ? k + 1 : k].x) : 0u);
      const uint32_t n1 = from_next_lane(pc[k].y, k < 8 ? (uint32_t)__builtin_amdgcn_readfirstlane((int)pc[k < 8 ? k + 1 : k].y) : 0u);
      const uint32_t wd[6] = {pc[k].x, pc[k].y, pc[k].z, pc[k].w, n0, n1};
      uint32_t pl = 0;
#pragma unroll
      for (int j = 15; j >= 0; j--) {  // bit j appended last-first: pl = pl + pl + V
        const int b = 4 + j;
        const uint32_t I = (b & 3) ? __builtin_amdgcn_alignbyte(wd[(b >> 2) + 1], wd[b >> 2], b & 3) : wd[b >> 2];
        pl = push_bit(pl, I + 1u < nref1);
      }
      P[k] = pl;
    }
    // survivors: V(x + 4) && V(x + 24); x + 24 is bit j + 4 of lane l + 1's plane, or bit j - 12 of lane l + 2's
    uint32_t S[8], cnt = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) {
      const uint32_t n1 = from_next_lane(P[k], (uint32_t)__builtin_amdgcn_readfirstlane((int)P[k + 1]));
      const uint32_t n2 = from_next_lane(n1, (uint32_t)__builtin_amdgcn_readlane((int)P[k + 1], 1));
      S[k] = P[k] & ((n1 >> 4) | (n2 << 12)) & 0xffffu;
      cnt += (uint32_t)__popc(S[k]);
      reinterpret_cast<uint16_t *>(bm)[64 * k + lane] = (uint16_t)S[k];
    }
    const uint32_t incl = wave_incl_scan_u32(cnt), total = (uint32_t)__shfl((int)incl, 63, 64);
    for (uint32_t r0 = 0; r0 < total; r0 += kEwQ) {  // (one round unless the tile has > kEwQ survivors)
      uint32_t at = incl - cnt;
      if (at < r0 + kEwQ && at + cnt > r0) {
#pragma unroll
        for (int k = 0; k < 8; k++) {
          for (uint32_t m = S[k]; m; m &= m - 1, at++)
            if (at >= r0 && at < r0 + kEwQ) q[at - r0] = (uint16_t)(1024 * k + 16 * lane + __builtin_ctz(m));
        }
      }
      wave_sync();
      const uint32_t nq = min((uint32_t)kEwQ, total - r0);
      for (uint32_t i0 = 0; i0 < nq; i0 += 64) {
        const uint32_t i = i0 + (uint32_t)lane;
        int res = 1, rel = 0;
        int64_t c64 = 0;
        int32_t n64 = 0;
        if (i < nq) {
          rel = q[i];
          const int o = rel & 3, d = rel >> 2;
          int32_t f[8];
#pragma unroll
          for (int k = 0; k < 8; k++) f[k] = (int32_t)__builtin_amdgcn_alignbyte(w32[d + k + 1], w32[d + k], o);
          res = eager_pass_win(win, sv, base + rel, rel, f, c64, n64);
          if (res == 0) atomicAnd(&bm[rel >> 5], ~(1u << (rel & 31)));
        }
        // op arrays past 64 ops: the wave reads each one's remaining ops together
        for (uint64_t pm = __ballot(res == 2); pm; pm &= pm - 1ull) {
          const int fl = (int)__builtin_ctzll(pm);
          const int64_t c = (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(c64 >> 32), fl) << 32) |
                                      (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)c64, fl));
          const int32_t n = __builtin_amdgcn_readlane(n64, fl);
          if (ops_bad_wave(sv, c, n) && lane == fl) atomicAnd(&bm[rel >> 5], ~(1u << (rel & 31)));
        }
      }
      wave_sync();
    }
    const u32x4 out = reinterpret_cast<const u32x4 *>(bm)[lane];
    reinterpret_cast<u32x4 *>(bitmap + ((base - x0a) >> 6))[lane] = out;
    wave_sync();  // (the next tile's LDS writes come after every lane's reads)
  }
}

// ---- FindRecordStart ---------------------------------------------------------------------------------------
// One workgroup per start offset scans 256 positions per step with the eager checker (global reads) until the
// first true call; with a success bitmap covering [bx0, bx1) the covered prefix is read from the bitmap.
// out = found offset, -1 = None, -2 = HALO.
__global__ __launch_bounds__(kCheckThreads) void k_find_record_starts(StreamView sv, const int64_t *__restrict__ xs,
                                                                      int R, int64_t max_read_size,
                                                                      const unsigned long long *__restrict__ bitmap,
                                                                      int64_t bx0, int64_t bx1,
                                                                      int64_t *__restrict__ out) {
  __shared__ unsigned long long s_best;
  __shared__ int s_halo;
  const int64_t x0 = xs[blockIdx.x];
  if (threadIdx.x == 0) { s_best = ~0ull; s_halo = 0; }
  __syncthreads();
  if (x0 < 0) {
    if (threadIdx.x == 0) out[blockIdx.x] = -1;
    return;
  }
  const int64_t lim = min(sv.L, x0 + max_read_size);
  int64_t x = x0;
  if (bitmap && x0 >= bx0 && x0 < bx1) {
    const int64_t blim = min(lim, bx1);
    for (int64_t wb = (x0 - bx0) >> 6; bx0 + (wb << 6) < blim; wb += kCheckThreads) {
      const int64_t wi = wb + threadIdx.x;
      const int64_t wx = bx0 + (wi << 6);
      if (wx < blim) {
        unsigned long long m = bitmap[wi];
        if (wx < x0) m &= ~0ull << (x0 - wx);
        if (m) {
          const int64_t hit = wx + __ffsll((long long)m) - 1;
          if (hit < blim) atomicMin(&s_best, (unsigned long long)hit);
        }
      }
      __syncthreads();
      if (s_best != ~0ull) break;
      __syncthreads();
    }
    x = blim;
  }
  while (s_best == ~0ull && x < lim && !s_halo) {
    const int64_t p = x + threadIdx.x;
    if (p < lim) {
      const uint32_t word = check_chain<true>(sv, GlobalBytes{sv.u}, p, p, 0, R);
      if (word == W_HALO) s_halo = 1;
      else if (word & W_SUCC) atomicMin(&s_best, (unsigned long long)p);
    }
    __syncthreads();
    x += kCheckThreads;
  }
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = (s_best != ~0ull) ? (int64_t)s_best : (s_halo ? -2 : -1);
}

// ---- record chain ------------------------------------------------------------------------------------------
// counts[i] = records r with r < x_end from xs[i]; -2 when the chain left a shard's bytes (HALO), -3 truncated.
__global__ void k_record_counts(StreamView sv, const int64_t *__restrict__ xs, const int64_t *__restrict__ xe, int64_t n,
                                int64_t *__restrict__ counts) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  int64_t x = xs[i];
  const int64_t end = xe[i];
  int64_t c = 0;
  if (x >= 0) {
    while (x < end) {
      if (x + 4 > sv.L) { c = sv.eof_real ? -3 : -2; break; }
      const int32_t bs = g_i32(sv.u, x);
      if (bs < 0 || x + 4 + (int64_t)bs > sv.L) { c = sv.eof_real ? -3 : -2; break; }
      c++;
      x += 4 + (int64_t)bs;
    }
  }
  counts[i] = c;
}

__global__ void k_record_offsets(StreamView sv, int64_t x, int64_t end, int64_t *__restrict__ offs, int64_t cap,
                                 int64_t *__restrict__ n_out) {
  int64_t c = 0;
  while (x < end) {
    if (x + 4 > sv.L) { c = -3 - c; break; }
    const int32_t bs = g_i32(sv.u, x);
    if (bs < 0 || x + 4 + (int64_t)bs > sv.L) { c = -3 - c; break; }
    if (c < cap) offs[c] = x;
    c++;
    x += 4 + (int64_t)bs;
  }
  *n_out = c;
}

// ---- launch wrappers ---------------------------------------------------------------------------------------
static int check_grid(int64_t ntiles) { return (int)(ntiles < 1 ? 1 : ntiles > 2048 ? 2048 : ntiles); }
static int64_t ntiles_of(int64_t x0, int64_t x1) { return (x1 - (x0 & ~(int64_t)63) + kTile - 1) / kTile; }
// Tiles [tlo, thi) of [x0, x1) are interior (inside [x0, x1), ending >= kInteriorTail bytes before the stream end).
static void interior_tiles(const StreamView &sv, int64_t x0, int64_t x1, int64_t *tlo, int64_t *thi) {
  const int64_t x0a = x0 & ~(int64_t)63;
  const int64_t lim = x1 < sv.L - kInteriorTail ? x1 : sv.L - kInteriorTail;
  *tlo = x0 == x0a ? 0 : 1;
  *thi = lim - x0a >= kTile ? (lim - x0a) / kTile : 0;
  if (*thi < *tlo) *thi = *tlo;
}
// Grid of the grid-stride k_check<MODE, PART> launch: at least the workgroups resident on the whole device.
template <int MODE, int PART>
static int resident_grid(int64_t ntiles) {
  static std::atomic<int> cached[16];
  int dev = 0;
  (void)hipGetDevice(&dev);
  int g = cached[dev & 15].load(std::memory_order_relaxed);
  if (g <= 0) {
    int per_cu = 0, cus = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_check<MODE, PART>, kCheckThreads, 0) != hipSuccess ||
        per_cu < 1)
      per_cu = 1;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1) cus = 256;
    g = per_cu * cus;
    cached[dev & 15].store(g, std::memory_order_relaxed);
  }
  // many more workgroups than slots, ~40 tiles each: tile costs differ (data, counter flushes), and a slot that
  // finishes early takes the next workgroup (measured at 10 GB: 1280 → 121 ms, 2048 → 114, 81920 → 99)
  const int64_t want = std::max<int64_t>(g, std::min<int64_t>(ntiles / 40, 131072));
  return (int)(ntiles < 1 ? 1 : ntiles < want ? ntiles : want);
}

// Grid of k_check_bits over ntiles interior tiles (same policy as resident_grid; the occupancy depends on the
// dynamic LDS of the contig lengths).
static int bits_grid(int64_t ntiles, size_t shmem) {
  int per_cu = 0, cus = 0, dev = 0;
  (void)hipGetDevice(&dev);
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_check_bits, kCheckThreads, shmem) != hipSuccess ||
      per_cu < 1)
    per_cu = 1;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1) cus = 256;
  const int64_t want = std::max<int64_t>((int64_t)per_cu * cus, std::min<int64_t>(ntiles / 40, 131072));
  return (int)(ntiles < 1 ? 1 : ntiles < want ? ntiles : want);
}
// Record-0 pass of mode MODE over [x0, x1): interior tiles by k_check<MODE, 1>, the rest by k_check<MODE, 2>.
template <int MODE>
static void launch_split_check(StreamView sv, int64_t x0, int64_t x1, int32_t R, CountsDev cd,
                               unsigned long long *bitmap, hipStream_t s) {
  int64_t tlo, thi;
  interior_tiles(sv, x0, x1, &tlo, &thi);
  const int64_t nt = ntiles_of(x0, x1), ni = thi - tlo;
  if (ni > 0)
    hipLaunchKernelGGL((k_check<MODE, 1>), dim3(resident_grid<MODE, 1>(ni)), dim3(kCheckThreads), 0, s, sv, x0, x1, R,
                       cd, bitmap, nullptr, tlo, thi);
  if (nt > ni)
    hipLaunchKernelGGL((k_check<MODE, 2>), dim3(check_grid(nt - ni)), dim3(kCheckThreads), 0, s, sv, x0, x1, R, cd,
                       bitmap, nullptr, tlo, thi);
}
static int chain_grid(int64_t x0, int64_t x1) {
  const int64_t words = (x1 - (x0 & ~(int64_t)63) + 63) >> 6;
  const int64_t g = (words + kChainWords - 1) / kChainWords;
  return (int)(g < 1 ? 1 : g > 65535 ? 65535 : g);
}

int64_t check_tiles(int64_t x0, int64_t x1) { return x1 > x0 ? ntiles_of(x0, x1) : 0; }
hipError_t launch_check_full_counts(StreamView sv, int64_t x0, int64_t x1, int32_t R, int32_t by_key, CountsDev cd,
                                    unsigned long long *bitmap, hipStream_t s, bool *tiles_counted) {
  *tiles_counted = false;
  if (x1 <= x0) return hipSuccess;
  if (by_key) {
    hipLaunchKernelGGL((k_check<MODE_BYKEY, 0>), dim3(check_grid(ntiles_of(x0, x1))), dim3(kCheckThreads), 0, s, sv,
                       x0, x1, R, cd, bitmap, nullptr, (int64_t)0, (int64_t)0);
  } else if (R > 0) {
    // interior tiles bit-sliced (k_check_bits), the boundary tiles by k_check<MODE_COUNTS, 2>; between them every
    // tile's PASS0 count when cd.tile_pass0 is set
    *tiles_counted = cd.tile_pass0 != nullptr;
    int64_t tlo, thi;
    interior_tiles(sv, x0, x1, &tlo, &thi);
    const int64_t nt = ntiles_of(x0, x1), ni = thi - tlo;
    if (ni > 0) {
      const size_t shmem = (sv.nref <= kLdsLens ? (size_t)sv.nref + 1 : 1) * sizeof(int32_t);
      hipLaunchKernelGGL(k_check_bits, dim3(bits_grid(ni, shmem)), dim3(kCheckThreads), shmem, s, sv, x0, R, cd,
                         bitmap, tlo, thi);
    }
    if (nt > ni)
      hipLaunchKernelGGL((k_check<MODE_COUNTS, 2>), dim3(check_grid(nt - ni)), dim3(kCheckThreads), 0, s, sv, x0, x1,
                         R, cd, bitmap, nullptr, tlo, thi);
  } else {  // Success(0) everywhere, or contig lengths past the LDS table: the general pass
    hipLaunchKernelGGL((k_check<MODE_COUNTS, 0>), dim3(check_grid(ntiles_of(x0, x1))), dim3(kCheckThreads), 0, s, sv,
                       x0, x1, R, cd, bitmap, nullptr, (int64_t)0, (int64_t)0);
  }
  return hipGetLastError();
}
hipError_t launch_check_full_chains(StreamView sv, int64_t x0, int64_t x1, int32_t R, int32_t by_key, CountsDev cd,
                                    unsigned long long *bitmap, hipStream_t s) {
  if (x1 <= x0) return hipSuccess;
  hipLaunchKernelGGL(k_chains, dim3(chain_grid(x0, x1)), dim3(256), 0, s, sv, x0, x1, R, bitmap, cd, by_key, nullptr);
  return hipGetLastError();
}
int64_t chain_list_chunks(int64_t x0, int64_t x1) {
  const int64_t words = (x1 - (x0 & ~(int64_t)63) + 63) >> 6;
  return (words + kChainWords - 1) / kChainWords;
}
static_assert(kChainWords * 64 == 16 * kTile, "a chain chunk is 16 record-0 tiles");
hipError_t launch_chain_list_build(int64_t x0, int64_t x1, const unsigned long long *bitmap, const ChainScratch &cs,
                                   const int32_t *tile_pass0, hipStream_t s) {
  const int64_t x0a = x0 & ~(int64_t)63, nwords = (x1 - x0a + 63) >> 6, nch = chain_list_chunks(x0, x1);
  if (nch <= 0) return hipSuccess;
  if (tile_pass0)
    hipLaunchKernelGGL(k_p0_count_tiles, dim3((unsigned)((nch + 255) / 256)), dim3(256), 0, s, tile_pass0,
                       ntiles_of(x0, x1), nch, cs.chunk_cnt);
  else
    hipLaunchKernelGGL(k_p0_count, dim3((unsigned)nch), dim3(256), 0, s, bitmap, nwords, cs.chunk_cnt);
  hipLaunchKernelGGL(k_p0_scan, dim3(1), dim3(1024), 0, s, cs.chunk_cnt, nch, cs.chunk_off);
  return hipGetLastError();
}
hipError_t launch_chain_list_run(StreamView sv, int64_t x0, int64_t x1, int32_t R, int32_t by_key, CountsDev cd,
                                 unsigned long long *bitmap, const ChainScratch &cs, hipStream_t s) {
  const int64_t x0a = x0 & ~(int64_t)63, nwords = (x1 - x0a + 63) >> 6, nch = chain_list_chunks(x0, x1);
  if (nch <= 0) return hipSuccess;
  const int64_t *n_ptr = cs.chunk_off + nch;
  hipLaunchKernelGGL(k_p0_list, dim3((unsigned)nch), dim3(256), 0, s, bitmap, nwords, x0a, cs.chunk_off, cs.list);
  hipLaunchKernelGGL(k_p0_links, dim3(4096), dim3(256), 0, s, sv, cs.list, n_ptr, x1, cs.ok);
  (void)hipMemsetAsync(cs.n_fb, 0, 3 * sizeof(unsigned long long), s);  // fallbacks, missing links, failed fallbacks
  if (R >= 2 && R <= 10)
    hipLaunchKernelGGL(k_p0_fast16, dim3(1024), dim3(256), 0, s, cs.list, n_ptr, cs.ok, (int)R, cd, cs.fb, cs.n_fb);
  else
    hipLaunchKernelGGL(k_p0_fast, dim3(4096), dim3(256), 0, s, cs.list, n_ptr, cs.ok, (int)R, cd, cs.fb, cs.n_fb);
  hipLaunchKernelGGL(k_p0_fallback, dim3(1024), dim3(256), 0, s, sv, x0a, x1, (int)R, bitmap, cd, (int)by_key, cs.fb,
                     cs.n_fb);
  return hipGetLastError();
}
hipError_t launch_check_eager_pass0(StreamView sv, int64_t x0, int64_t x1, int32_t R, unsigned long long *bitmap,
                                    hipStream_t s) {
  if (x1 <= x0) return hipSuccess;
  if (R == 0) {  // Success(0) everywhere: no prefilter
    launch_split_check<MODE_EAGER>(sv, x0, x1, R, CountsDev{}, bitmap, s);
    return hipGetLastError();
  }
  int64_t tlo, thi;
  interior_tiles(sv, x0, x1, &tlo, &thi);
  const int64_t nt = ntiles_of(x0, x1), ni = thi - tlo;
  if (ni > 0) {  // ~10 tiles per wave: a wave that finishes early takes the next workgroup
    const int64_t g = std::max<int64_t>(1, std::min<int64_t>((ni + 10 * kEwWaves - 1) / (10 * kEwWaves), 131072));
    hipLaunchKernelGGL(k_eager_wave, dim3((unsigned)g), dim3(64 * kEwWaves), 0, s, sv, x0, (int)R, bitmap, tlo, thi);
  }
  if (nt > ni)
    hipLaunchKernelGGL((k_check<MODE_EAGER, 2>), dim3(check_grid(nt - ni)), dim3(kCheckThreads), 0, s, sv, x0, x1, R,
                       CountsDev{}, bitmap, nullptr, tlo, thi);
  return hipGetLastError();
}
hipError_t launch_check_words(StreamView sv, int64_t x0, int64_t x1, int32_t R, uint32_t *words,
                              unsigned long long *bitmap, hipStream_t s) {
  if (x1 <= x0) return hipSuccess;
  hipLaunchKernelGGL((k_check<MODE_WORDS, 0>), dim3(check_grid(ntiles_of(x0, x1))), dim3(kCheckThreads), 0, s, sv, x0,
                     x1, R, CountsDev{}, bitmap, words, (int64_t)0, (int64_t)0);
  hipLaunchKernelGGL(k_chains, dim3(chain_grid(x0, x1)), dim3(256), 0, s, sv, x0, x1, R, bitmap, CountsDev{}, 0, words);
  return hipGetLastError();
}
hipError_t launch_find_record_starts(StreamView sv, const int64_t *x0, int64_t n, int32_t R, int64_t mrs,
                                     const unsigned long long *bitmap, int64_t bx0, int64_t bx1, int64_t *out,
                                     hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_find_record_starts, dim3((unsigned)n), dim3(kCheckThreads), 0, s, sv, x0, R, mrs, bitmap, bx0,
                     bx1, out);
  return hipGetLastError();
}
hipError_t launch_record_counts(StreamView sv, const int64_t *x0, const int64_t *xe, int64_t n, int64_t *counts,
                                hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_record_counts, dim3((unsigned)((n + 63) / 64)), dim3(64), 0, s, sv, x0, xe, n, counts);
  return hipGetLastError();
}
hipError_t launch_record_offsets(StreamView sv, int64_t x0, int64_t xe, int64_t *offs, int64_t cap, int64_t *n_out,
                                 hipStream_t s) {
  hipLaunchKernelGGL(k_record_offsets, dim3(1), dim3(1), 0, s, sv, x0, xe, offs, cap, n_out);
  return hipGetLastError();
}

}  // namespace sbam
