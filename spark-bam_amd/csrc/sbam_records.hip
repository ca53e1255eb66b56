// sbam_records.hip — record chains of Hadoop splits and their decode into columns (gfx950).
//
// Reference: RecordStream._advance (check/src/main/scala/org/hammerlab/bam/iterator/RecordStream.scala:27-41)
// walks a split's records by block_size alone, from FindRecordStart's Pos while Pos < Pos(split end, 0)
// (CanLoadBam.scala:221-241, 281-334); htsjdk BAMRecordCodec.decode then reads the 32 fixed bytes after
// block_size.  A chain is inherently serial (one dependent 4-byte load per record), so a split walked by one
// lane is latency-bound.  When the full checker has left its success bitmap over the range, the chain is
// instead PROVEN equal to the bitmap's set bits in parallel, and the per-split record lists come from
// popcounts and a scan:
//
//   chain == set bits of [X0, X1)   ⇔   X0 is set, and for every set bit p in [X0, X1):
//                                        q = p + 4 + block_size(p) is in (p, L], and the bits in (p, min(q, X1))
//                                        are all clear, and bit q is set when q < X1.
//
// (⇐: starting at X0 every hop lands on the next set bit, so the walk visits exactly the set bits, in order.)
// Any violation — a false-positive call off the chain, a chain record the checker rejected, a record past EOF —
// clears the proof and the host falls back to the serial walk, which also reports the reference's errors.
// Each bitmap word is read about twice and each record's block_size once, so the proof costs a few ms at
// 10 GB where the serial walk costs ~12.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sbam_internal.h"

namespace sbam {

#define SB_DEV __device__ __forceinline__

namespace {

SB_DEV int32_t rd_i32(const uint8_t *u, int64_t x) {
  return (int32_t)((uint32_t)u[x] | ((uint32_t)u[x + 1] << 8) | ((uint32_t)u[x + 2] << 16) |
                   ((uint32_t)u[x + 3] << 24));
}

// the little-endian int32 at x from the two aligned dwords around it (the stream buffer is 4-byte aligned and
// padded past L)
SB_DEV int32_t rd_i32_aligned(const uint8_t *u, int64_t x) {
  const uint32_t *w = reinterpret_cast<const uint32_t *>(u + (x & ~(int64_t)3));
  return (int32_t)__builtin_amdgcn_alignbyte(w[1], w[0], (uint32_t)(x & 3));
}

// bit at stream offset x of a bitmap whose bit 0 is offset xa (xa 64-aligned)
SB_DEV bool bm_test(const unsigned long long *bm, int64_t xa, int64_t x) {
  const int64_t r = x - xa;
  return (bm[r >> 6] >> (r & 63)) & 1ull;
}

// any set bit in stream offsets [a, b)?
SB_DEV bool bm_any(const unsigned long long *bm, int64_t xa, int64_t a, int64_t b) {
  if (a >= b) return false;
  int64_t ra = a - xa, rb = b - xa;
  int64_t wa = ra >> 6, wb = (rb - 1) >> 6;
  const unsigned long long lo = ~0ull << (ra & 63);
  const unsigned long long hi = ~0ull >> (63 - ((rb - 1) & 63));
  if (wa == wb) return (bm[wa] & lo & hi) != 0;
  if (bm[wa] & lo) return true;
  for (int64_t w = wa + 1; w < wb; w++)
    if (bm[w]) return true;
  return (bm[wb] & hi) != 0;
}

// The hop p -> q holds: no set bit in [p + 1, min(q, X1)) and, for q < X1, bit q set.  A record's span usually
// covers a few bitmap words: those (up to 8) are loaded at once rather than one dependent load per word.
SB_DEV bool hop_ok(const unsigned long long *bm, int64_t xa, int64_t p, int64_t q, int64_t X1) {
  const int64_t e = q < X1 ? q : X1;
  const int64_t ra = p + 1 - xa, re = e - xa, rq = q - xa;  // bits [ra, re) must be clear
  const int64_t wa = ra >> 6, wl = (q < X1 ? rq : re - 1) >> 6;
  if (re <= ra || wl - wa >= 8) return !bm_any(bm, xa, p + 1, e) && (q >= X1 || bm_test(bm, xa, q));
  unsigned long long wv[8];
#pragma unroll
  for (int k = 0; k < 8; k++) wv[k] = wa + k <= wl ? bm[wa + k] : 0ull;
  bool any = false, qset = q >= X1;
#pragma unroll
  for (int k = 0; k < 8; k++) {
    const int64_t b0 = (wa + k) << 6;  // first bit of the word
    unsigned long long m = wv[k];
    m &= ra > b0 ? ~0ull << (ra - b0) : ~0ull;
    m &= re >= b0 + 64 ? ~0ull : re <= b0 ? 0ull : (1ull << (re - b0)) - 1ull;
    any |= m != 0;
    if (q < X1 && (rq >> 6) == wa + k) qset = (wv[k] >> (rq & 63)) & 1ull;
  }
  return !any && qset;
}

}  // namespace

// One thread per bitmap word of [X0, X1): every set bit p in it must hop to the next set bit (or past X1).
// exact (may be null): the chain-list counters of the check that left the bitmap ([1] missing links, [2] failed
// fallback walks, k_p0_fast): both zero means every set bit already hops to the next one (the list pass checked
// p + 4 + block_size == next PASS0 position for each), so the proof holds without reading the records again.
__global__ void k_chain_proof(const uint8_t *__restrict__ u, int64_t L, const unsigned long long *__restrict__ bm,
                              int64_t xa, int64_t X0, int64_t X1, int32_t *__restrict__ fail,
                              const unsigned long long *__restrict__ exact) {
  if (exact && exact[1] == 0 && exact[2] == 0) return;
  const int64_t w0 = (X0 - xa) >> 6, w1 = (X1 - 1 - xa) >> 6;
  for (int64_t w = w0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; w <= w1;
       w += (int64_t)gridDim.x * blockDim.x) {
    unsigned long long m = bm[w];
    const int64_t base = xa + (w << 6);
    if (base < X0) m &= ~0ull << (X0 - base);
    if (base + 64 > X1) m &= (X1 - base >= 64) ? ~0ull : ((1ull << (X1 - base)) - 1);
    bool bad = false;
    while (m && !bad) {
      const int64_t p = base + __builtin_ctzll(m);
      m &= m - 1;
      if (p + 4 > L) { bad = true; break; }
      const int32_t bs = rd_i32_aligned(u, p);
      const int64_t q = p + 4 + (int64_t)bs;
      if (bs < 0 || q > L) { bad = true; break; }
      if (!hop_ok(bm, xa, p, q, X1)) bad = true;
    }
    if (bad) atomicOr(fail, 1);
  }
}

// First index of the sorted a[0, n) whose value is >= x; called by a whole wave: 64 probes per round (a 64-ary search,
// 5 dependent loads for 10^8 entries instead of 27).
SB_DEV int64_t wave_lower_bound(const int64_t *__restrict__ a, int64_t n, int64_t x) {
  const int lane = __lane_id();
  int64_t lo = 0, hi = n;  // the answer is in [lo, hi]: a[< lo] < x, a[>= hi] >= x
  while (hi - lo > 64) {
    const int64_t step = (hi - lo + 63) / 64;
    const int64_t p = lo + (int64_t)lane * step;
    const int k = __popcll(__ballot(p < hi && a[p] < x));  // (a prefix of the lanes: a is sorted)
    if (k == 0) return lo;
    const int64_t nlo = lo + (int64_t)(k - 1) * step + 1, nhi = lo + (int64_t)k * step;
    lo = nlo;
    if (nhi < hi) hi = nhi;
  }
  const int64_t p = lo + lane;
  return lo + __popcll(__ballot(p < hi && a[p] < x));
}

// One workgroup per split: number of set bits in [xs, xe) (0 for xs < 0); fail unless xs itself is set.  When the
// bitmap is exactly the chain pass's PASS0 list (list != null and no failed fallback walk cleared a bit: exact[2] ==
// 0, k_p0_fast), the count is the number of list entries in [xs, xe): two searches instead of a pass over the bitmap.
__global__ void k_split_popcounts(const unsigned long long *__restrict__ bm, int64_t xa, const int64_t *__restrict__ xs,
                                  const int64_t *__restrict__ xe, int64_t n, int64_t *__restrict__ counts,
                                  int32_t *__restrict__ fail, const int64_t *__restrict__ list, int64_t nlist,
                                  const unsigned long long *__restrict__ exact) {
  __shared__ unsigned long long part[8];
  const int64_t i = blockIdx.x;
  if (i >= n) return;
  const int64_t a = xs[i], b = xe[i];
  if (list && exact[2] == 0) {
    if (threadIdx.x >= 64) return;
    int64_t cnt = 0;
    if (a >= 0 && a < b) {
      const int64_t ia = wave_lower_bound(list, nlist, a), ib = wave_lower_bound(list, nlist, b);
      cnt = ib - ia;
      if (threadIdx.x == 0 && !(ia < nlist && list[ia] == a)) atomicOr(fail, 1);
    }
    if (threadIdx.x == 0) counts[i] = cnt;
    return;
  }
  unsigned long long c = 0;
  if (a >= 0 && a < b) {
    const int64_t ra = a - xa, rb = b - xa;
    const int64_t wa = ra >> 6, wb = (rb - 1) >> 6;
    // 8 words in flight per thread (as a one-word loop each load waited for the one before: 0.68 ms per 10 GB)
    const int64_t step = blockDim.x;
    int64_t w = wa + threadIdx.x;
    for (; w + 7 * step <= wb; w += 8 * step) {
      unsigned long long m[8];
#pragma unroll
      for (int k = 0; k < 8; k++) m[k] = bm[w + k * step];
#pragma unroll
      for (int k = 0; k < 8; k++) {
        const int64_t wk = w + k * step;
        unsigned long long x = m[k];
        if (wk == wa) x &= ~0ull << (ra & 63);
        if (wk == wb) x &= ~0ull >> (63 - ((rb - 1) & 63));
        c += __popcll(x);
      }
    }
    for (; w <= wb; w += step) {
      unsigned long long m = bm[w];
      if (w == wa) m &= ~0ull << (ra & 63);
      if (w == wb) m &= ~0ull >> (63 - ((rb - 1) & 63));
      c += __popcll(m);
    }
    if (threadIdx.x == 0 && !bm_test(bm, xa, a)) atomicOr(fail, 1);
  }
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long t = 0;
    for (int k = 0; k < (int)(blockDim.x >> 6); k++) t += part[k];
    counts[i] = (int64_t)t;
  }
}

// One workgroup (256 threads) per split: offsets of the set bits of [xs, xe) at out[base[i] ...], in order.
__global__ void __launch_bounds__(256) k_split_offsets(const unsigned long long *__restrict__ bm, int64_t xa,
                                                       const int64_t *__restrict__ xs, const int64_t *__restrict__ xe,
                                                       const int64_t *__restrict__ base, int64_t n,
                                                       int64_t *__restrict__ out) {
  __shared__ uint32_t wsum[4];
  const int64_t i = blockIdx.x;
  if (i >= n) return;
  const int64_t a = xs[i], b = xe[i];
  if (a < 0 || a >= b) return;
  const int64_t ra = a - xa, rb = b - xa;
  const int64_t wa = ra >> 6, wb = (rb - 1) >> 6;
  int64_t run = base[i];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (int64_t w0 = wa; w0 <= wb; w0 += 256) {
    const int64_t w = w0 + threadIdx.x;
    unsigned long long m = 0;
    if (w <= wb) {
      m = bm[w];
      if (w == wa) m &= ~0ull << (ra & 63);
      if (w == wb) m &= ~0ull >> (63 - ((rb - 1) & 63));
    }
    const uint32_t pc = (uint32_t)__popcll(m);
    // inclusive scan across the wave, then across the 4 waves
    uint32_t s = pc;
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t t = __shfl_up(s, o);
      if (lane >= o) s += t;
    }
    if (lane == 63) wsum[wv] = s;
    __syncthreads();
    uint32_t before = 0, total = 0;
    for (int k = 0; k < 4; k++) {
      if (k < wv) before += wsum[k];
      total += wsum[k];
    }
    int64_t o = run + before + s - pc;
    const int64_t bx = xa + (w << 6);
    while (m) {
      out[o++] = bx + __builtin_ctzll(m);
      m &= m - 1;
    }
    run += total;
    __syncthreads();
  }
}

// Serial fallback: one lane per split walks its chain, writing offsets at out[base[i] ...].
__global__ void k_record_walk(const uint8_t *__restrict__ u, int64_t L, const int64_t *__restrict__ xs,
                              const int64_t *__restrict__ xe, const int64_t *__restrict__ base, int64_t n,
                              int64_t *__restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  int64_t x = xs[i], o = base[i];
  if (x < 0) return;
  const int64_t end = xe[i];
  while (x < end && x + 4 <= L) {
    const int32_t bs = rd_i32(u, x);
    if (bs < 0 || x + 4 + (int64_t)bs > L) break;  // the count pass already reported this chain's error
    out[o++] = x;
    x += 4 + (int64_t)bs;
  }
}

// One thread per record: Pos and the fixed fields (BAM spec §4.2; BAMRecordCodec.decode's fixed part) as columns.
__global__ void k_record_columns(const uint8_t *__restrict__ u, const int64_t *__restrict__ offs, int64_t n,
                                 const int64_t *__restrict__ bstart, const int64_t *__restrict__ buoff,
                                 const int32_t *__restrict__ busize, int64_t nblocks, int64_t file_base,
                                 RecordColumnsDev cols) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t x = offs[i];
  // Pos: last block with uoff <= x, advanced past zero-length blocks (UncompressedBytes.scala:17-19)
  int64_t lo = 0, hi = nblocks;  // first block with uoff > x
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (buoff[mid] <= x) lo = mid + 1;
    else hi = mid;
  }
  int64_t b = lo - 1;
  while (b + 1 < nblocks && x >= buoff[b] + busize[b]) b++;
  cols.block_pos[i] = file_base + bstart[b];
  cols.block_off[i] = (int32_t)(x - buoff[b]);
  uint32_t f[9];
  for (int k = 0; k < 9; k++) f[k] = (uint32_t)rd_i32(u, x + 4 * k);
  cols.block_size[i] = (int32_t)f[0];
  cols.ref_id[i] = (int32_t)f[1];
  cols.pos[i] = (int32_t)f[2];
  cols.bin_mq_nl[i] = f[3];
  cols.flag_nc[i] = f[4];
  cols.l_seq[i] = (int32_t)f[5];
  cols.next_ref_id[i] = (int32_t)f[6];
  cols.next_pos[i] = (int32_t)f[7];
  cols.tlen[i] = (int32_t)f[8];
}

// Reference span of the record at offs[i], as CanLoadBam.region reads it from htsjdk (CanLoadBam.scala:423-431):
// refID, start = pos (= getStart - 1) and the exclusive end getEnd = pos + the CIGAR's reference length (ops M, D,
// N, =, X: SAM spec §1.4.6).  An unmapped record (flag 4) has getAlignmentEnd = 0, so end = 0.  Ops past the
// stream end are not read.
__global__ void k_record_spans(const uint8_t *__restrict__ u, int64_t L, const int64_t *__restrict__ offs, int64_t n,
                               int32_t *__restrict__ ref_id, int32_t *__restrict__ start, int32_t *__restrict__ end) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t x = offs[i];
  if (x < 0 || x + 36 > L) {
    ref_id[i] = -1;
    start[i] = -1;
    end[i] = 0;
    return;
  }
  const int32_t ri = rd_i32(u, x + 4), pos = rd_i32(u, x + 8);
  const uint32_t bmn = (uint32_t)rd_i32(u, x + 12), fnc = (uint32_t)rd_i32(u, x + 16);
  const uint32_t nc = fnc & 0xffffu, flag = fnc >> 16;
  int64_t c = x + 36 + (bmn & 0xffu);
  int64_t rlen = 0;
  for (uint32_t k = 0; k < nc && c + 4 <= L; k++, c += 4) {
    const uint32_t op = (uint32_t)rd_i32(u, c);
    const uint32_t t = op & 0xfu;
    if (t == 0 || t == 2 || t == 3 || t == 7 || t == 8) rlen += op >> 4;
  }
  ref_id[i] = ri;
  start[i] = pos;
  end[i] = (flag & 4u) ? 0 : (int32_t)(pos + rlen);
}

hipError_t launch_record_spans(const uint8_t *u, int64_t L, const int64_t *offs, int64_t n, int32_t *ref_id,
                               int32_t *start, int32_t *end, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_record_spans, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, u, L, offs, n, ref_id, start,
                     end);
  return hipGetLastError();
}

hipError_t launch_chain_proof(const uint8_t *u, int64_t L, const unsigned long long *bm, int64_t xa, int64_t X0,
                              int64_t X1, int32_t *fail, const unsigned long long *exact, hipStream_t s) {
  if (X1 <= X0) return hipSuccess;
  const int64_t words = ((X1 - 1 - xa) >> 6) - ((X0 - xa) >> 6) + 1;
  int64_t g = (words + 255) / 256;
  if (g > 16384) g = 16384;
  hipLaunchKernelGGL(k_chain_proof, dim3((unsigned)g), dim3(256), 0, s, u, L, bm, xa, X0, X1, fail, exact);
  return hipGetLastError();
}
hipError_t launch_split_popcounts(const unsigned long long *bm, int64_t xa, const int64_t *xs, const int64_t *xe,
                                  int64_t n, int64_t *counts, int32_t *fail, const int64_t *list, int64_t nlist,
                                  const unsigned long long *exact, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  if (!exact) list = nullptr;
  hipLaunchKernelGGL(k_split_popcounts, dim3((unsigned)n), dim3(256), 0, s, bm, xa, xs, xe, n, counts, fail, list,
                     nlist, exact);
  return hipGetLastError();
}
hipError_t launch_split_offsets(const unsigned long long *bm, int64_t xa, const int64_t *xs, const int64_t *xe,
                                const int64_t *base, int64_t n, int64_t *out, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_split_offsets, dim3((unsigned)n), dim3(256), 0, s, bm, xa, xs, xe, base, n, out);
  return hipGetLastError();
}
hipError_t launch_record_walk(const uint8_t *u, int64_t L, const int64_t *xs, const int64_t *xe, const int64_t *base,
                              int64_t n, int64_t *out, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_record_walk, dim3((unsigned)((n + 63) / 64)), dim3(64), 0, s, u, L, xs, xe, base, n, out);
  return hipGetLastError();
}
hipError_t launch_record_columns(const uint8_t *u, const int64_t *offs, int64_t n, const int64_t *bstart,
                                 const int64_t *buoff, const int32_t *busize, int64_t nblocks, int64_t file_base,
                                 RecordColumnsDev cols, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_record_columns, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, u, offs, n, bstart, buoff,
                     busize, nblocks, file_base, cols);
  return hipGetLastError();
}

}  // namespace sbam
