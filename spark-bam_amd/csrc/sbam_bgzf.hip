// sbam_bgzf.hip — hand-written CDNA4 (gfx950) kernels for the BGZF layer of the spark-bam hot path.
//
//  * BGZF block-header scan   (Header.make bgzf/.../block/Header.scala:48-83, MetadataStream.scala:23-54,
//                              FindBlockStart.scala:8-36)
//  * batched raw-DEFLATE inflate (Stream.scala:31-71; RFC 1951 semantics of java.util.zip.Inflater)
//  The record-boundary checker and record chain live in sbam_check.hip.
//
// All byte/integer work: no MFMA (no dense contraction).  Design notes and rooflines: DESIGN.md.
#include "sbam_internal.h"

namespace sbam {

#define SB_DEV __device__ __forceinline__

// ------------------------------------------------------------------------------------------------
// wave helpers (wave64)
// ------------------------------------------------------------------------------------------------
SB_DEV int lane_id() { return __lane_id(); }
SB_DEV uint32_t wave_or(uint32_t v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v |= __shfl_xor(v, o, 64);
  return v;
}
SB_DEV uint32_t brev(uint32_t code, int len) { return __builtin_bitreverse32(code) >> (32 - len); }

// ================================================================================================
// 1. BGZF header scan
// ================================================================================================
constexpr int kScanThreads = 256;
constexpr int kScanWide = 32;  // positions per thread and iteration of k_scan_slots_wide
constexpr int kScanStep = kScanThreads * 16;  // bytes per workgroup iteration

// 16 candidate bits for positions q0..q0+15 given the 32 bytes at q0 (w[0..7] little-endian words).
// Header.make checks bytes 0-3 = 1f 8b 08 04 and 12,13,14 = 'B','C',2 (byte 15 unchecked).
SB_DEV uint32_t header_bits16(const uint32_t w[8], int64_t q0, int64_t D) {
  uint32_t bits = 0;
#pragma unroll
  for (int i = 0; i < 16; i++) {
    const int wi = i >> 2, o = i & 3;
    const uint32_t m = __builtin_amdgcn_alignbyte(w[wi + 1], w[wi], o);
    const uint32_t bc = __builtin_amdgcn_alignbyte(w[wi + 4], w[wi + 3], o) & 0x00ffffffu;
    const bool hit = (m == 0x04088b1fu) && (bc == 0x00024342u) && (q0 + i + 18 <= D);
    bits |= hit ? (1u << i) : 0u;
  }
  return bits;
}

SB_DEV void load32(const uint8_t *d, int64_t q0, uint32_t w[8]) {
  const uint4 a = *reinterpret_cast<const uint4 *>(d + q0);
  const uint4 b = *reinterpret_cast<const uint4 *>(d + q0 + 16);
  w[0] = a.x; w[1] = a.y; w[2] = a.z; w[3] = a.w;
  w[4] = b.x; w[5] = b.y; w[6] = b.z; w[7] = b.w;
}

__global__ __launch_bounds__(kScanThreads) void k_scan_count(const uint8_t *__restrict__ d, int64_t D,
                                                              int32_t *__restrict__ chunk_counts) {
  const int64_t cbase = (int64_t)blockIdx.x * kScanChunk;
  const int64_t cend = min(cbase + (int64_t)kScanChunk, D);
  int cnt = 0;
  for (int64_t it = cbase; it < cend; it += kScanStep) {
    const int64_t q0 = it + threadIdx.x * 16;
    if (q0 < cend) {
      uint32_t w[8];
      load32(d, q0, w);
      uint32_t bits = header_bits16(w, q0, D);
      if (q0 + 16 > cend) bits &= (1u << (cend - q0)) - 1u;
      cnt += __popc(bits);
    }
  }
  __shared__ int s[kScanThreads / 64];
  for (int o = 32; o >= 1; o >>= 1) cnt += __shfl_xor(cnt, o, 64);
  if (lane_id() == 0) s[threadIdx.x >> 6] = cnt;
  __syncthreads();
  if (threadIdx.x == 0) chunk_counts[blockIdx.x] = s[0] + s[1] + s[2] + s[3];
}

// Exclusive prefix over chunk counts: one workgroup (chunk count is D / 1 MiB: ~10^4 for 10 GB).
__global__ __launch_bounds__(1024) void k_scan_prefix(const int32_t *__restrict__ cnt, int64_t n,
                                                       int64_t *__restrict__ off, int64_t *__restrict__ total) {
  __shared__ int64_t s[1024];
  __shared__ int64_t carry;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (int64_t b = 0; b < n; b += 1024) {
    const int64_t i = b + threadIdx.x;
    const int64_t v = i < n ? cnt[i] : 0;
    s[threadIdx.x] = v;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {
      const int64_t t = threadIdx.x >= o ? s[threadIdx.x - o] : 0;
      __syncthreads();
      s[threadIdx.x] += t;
      __syncthreads();
    }
    if (i < n) off[i] = carry + s[threadIdx.x] - v;
    __syncthreads();
    if (threadIdx.x == 1023) carry += s[1023];
    __syncthreads();
  }
  if (threadIdx.x == 0) *total = carry;
}

SB_DEV void fill_candidate(const uint8_t *d, int64_t D, int64_t q, Candidate &c) {
  const int32_t xlen = (int32_t)d[q + 10] | ((int32_t)d[q + 11] << 8);
  const int32_t hs = 18 + xlen - 6;
  const int32_t cs = ((int32_t)d[q + 16] | ((int32_t)d[q + 17] << 8)) + 1;
  int32_t fl = 0, isz = 0;
  if (q + cs <= D) {
    const int64_t e = q + cs - 4;
    isz = (int32_t)((uint32_t)d[e] | ((uint32_t)d[e + 1] << 8) | ((uint32_t)d[e + 2] << 16) |
                    ((uint32_t)d[e + 3] << 24));
    fl |= CAND_ISIZE;
  }
  if (cs - hs - 8 == 2) fl |= CAND_EMPTY;
  c.pos = q;
  c.hsize = hs;
  c.csize = cs;
  c.isize = isz;
  c.flags = fl;
}

// Second pass: write candidates in file order at chunk_offsets[chunk] + rank.
__global__ __launch_bounds__(kScanThreads) void k_scan_write(const uint8_t *__restrict__ d, int64_t D,
                                                              const int64_t *__restrict__ chunk_off,
                                                              Candidate *__restrict__ out) {
  const int64_t cbase = (int64_t)blockIdx.x * kScanChunk;
  const int64_t cend = min(cbase + (int64_t)kScanChunk, D);
  __shared__ int s_any;
  __shared__ int s_wsum[kScanThreads / 64];
  int64_t run = chunk_off[blockIdx.x];
  for (int64_t it = cbase; it < cend; it += kScanStep) {
    const int64_t q0 = it + threadIdx.x * 16;
    uint32_t bits = 0;
    if (q0 < cend) {
      uint32_t w[8];
      load32(d, q0, w);
      bits = header_bits16(w, q0, D);
      if (q0 + 16 > cend) bits &= (1u << (cend - q0)) - 1u;
    }
    if (threadIdx.x == 0) s_any = 0;
    __syncthreads();
    if (bits) s_any = 1;
    __syncthreads();
    if (s_any) {  // rare: ordered rank = wave prefix + preceding waves
      const int c = __popc(bits);
      int incl = c;
      for (int o = 1; o < 64; o <<= 1) {
        const int t = __shfl_up(incl, o, 64);
        if (lane_id() >= o) incl += t;
      }
      if (lane_id() == 63) s_wsum[threadIdx.x >> 6] = incl;
      __syncthreads();
      int before = incl - c;
      for (int wv = 0; wv < (int)(threadIdx.x >> 6); wv++) before += s_wsum[wv];
      int64_t slot = run + before;
      while (bits) {
        const int i = __ffs(bits) - 1;
        bits &= bits - 1;
        fill_candidate(d, D, q0 + i, out[slot++]);
      }
      run += s_wsum[0] + s_wsum[1] + s_wsum[2] + s_wsum[3];
    }
    __syncthreads();
  }
}

// One-pass form (round 3): the candidates of chunk b written to its kScanSlots fixed slots, its count to
// chunk_counts[b] (slots past kScanSlots are not written; *overflow is set and the caller runs k_scan_write with the
// exact offsets instead), then k_scan_compact moves the slots into file order — the compressed bytes are read once
// instead of twice (k_scan_count + k_scan_write).  Round 4: P positions per thread and iteration (P + 16 B loaded as
// 16-B pieces, the next one's prefetched while this one's candidates are ranked), and one barrier per iteration
// without candidates (an "any candidate" flag in three rotating LDS words: the one for iteration i + 1 is cleared
// before iteration i's barrier, after every read of it in iteration i - 2).  Scan at 10 GB with P = 16 / 32 / 64:
// 2.51 / 2.14 / 2.20 ms; 16 positions with three barriers per iteration (round 3): 2.83.
template <int P>
SB_DEV void load_wide(const uint8_t *d, int64_t q0, uint32_t w[P / 4 + 4]) {
#pragma unroll
  for (int k = 0; k < P / 16 + 1; k++) {
    const uint4 a = *reinterpret_cast<const uint4 *>(d + q0 + 16 * k);
    w[4 * k] = a.x; w[4 * k + 1] = a.y; w[4 * k + 2] = a.z; w[4 * k + 3] = a.w;
  }
}
template <int P>
__global__ __launch_bounds__(kScanThreads) void k_scan_slots_wide(const uint8_t *__restrict__ d, int64_t D,
                                                                   int32_t *__restrict__ chunk_counts,
                                                                   Candidate *__restrict__ slots,
                                                                   unsigned long long *__restrict__ overflow) {
  constexpr int kW = P / 4 + 4, kScanWideStep = kScanThreads * P;  // words per thread, bytes per iteration
  static_assert(P % 16 == 0 && P <= 64 && kScanChunk % kScanWideStep == 0 && kCompPad >= P + 16, "wide scan");
  const int64_t cbase = (int64_t)blockIdx.x * kScanChunk;
  const int64_t cend = min(cbase + (int64_t)kScanChunk, D);
  __shared__ int s_any[3];
  __shared__ int s_wsum[kScanThreads / 64];
  if (threadIdx.x < 3) s_any[threadIdx.x] = 0;
  __syncthreads();
  Candidate *out = slots + (int64_t)blockIdx.x * kScanSlots;
  int run = 0, ph = 0;
  uint32_t wn[kW];
  if (cbase + threadIdx.x * P < cend) load_wide<P>(d, cbase + threadIdx.x * P, wn);
  for (int64_t it = cbase; it < cend; it += kScanWideStep) {
    const int64_t q0 = it + threadIdx.x * P;
    uint32_t w[kW];
#pragma unroll
    for (int k = 0; k < kW; k++) w[k] = wn[k];
    if (q0 + kScanWideStep < cend) load_wide<P>(d, q0 + kScanWideStep, wn);
    uint64_t bits = 0;
    if (q0 < cend) {
#pragma unroll
      for (int i = 0; i < P; i++) {
        const int wi = i >> 2, o = i & 3;
        const uint32_t m = __builtin_amdgcn_alignbyte(w[wi + 1], w[wi], o);
        const uint32_t bc = __builtin_amdgcn_alignbyte(w[wi + 4], w[wi + 3], o) & 0x00ffffffu;
        bits |= (m == 0x04088b1fu && bc == 0x00024342u) ? (1ull << i) : 0ull;
      }
      // Header.make needs 18 bytes; the chunk owns positions below cend
      const int64_t lim = min(cend - q0, D - 18 + 1 - q0);
      if (lim < P) bits &= lim > 0 ? (1ull << lim) - 1ull : 0ull;
    }
    const int nx = ph == 2 ? 0 : ph + 1;
    if (threadIdx.x == 0) s_any[nx] = 0;
    if (bits) s_any[ph] = 1;
    __syncthreads();
    const bool any = s_any[ph] != 0;
    ph = nx;
    if (any) {  // rare: ordered rank = wave prefix + preceding waves
      const int c = __popcll(bits);
      int incl = c;
      for (int o = 1; o < 64; o <<= 1) {
        const int t = __shfl_up(incl, o, 64);
        if (lane_id() >= o) incl += t;
      }
      if (lane_id() == 63) s_wsum[threadIdx.x >> 6] = incl;
      __syncthreads();
      int slot = run + incl - c;
      for (int wv = 0; wv < (int)(threadIdx.x >> 6); wv++) slot += s_wsum[wv];
      while (bits) {
        const int i = __ffsll((unsigned long long)bits) - 1;
        bits &= bits - 1;
        if (slot < kScanSlots) fill_candidate(d, D, q0 + i, out[slot]);
        slot++;
      }
      run += s_wsum[0] + s_wsum[1] + s_wsum[2] + s_wsum[3];
    }
  }
  if (threadIdx.x == 0) {
    chunk_counts[blockIdx.x] = run;
    if (run > kScanSlots) atomicOr(overflow, 1ull);
  }
}

// slots -> file order: slot j of chunk b goes to chunk_off[b] + j (j < chunk_counts[b] <= kScanSlots)
__global__ void k_scan_compact(const Candidate *__restrict__ slots, const int32_t *__restrict__ cnt,
                               const int64_t *__restrict__ off, int64_t nchunks, Candidate *__restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t b = i / kScanSlots;
  const int j = (int)(i % kScanSlots);
  if (b < nchunks && j < cnt[b]) out[off[b] + j] = slots[i];
}

// MetadataStream chain test: per candidate i (>= first), code 0 = the next header sits at cands[i+1];
// 1 = stop before emitting i (ISIZE past EOF, or empty block); 2 = emit i then EOF inside the next header;
// 3 = next header not at cands[i+1] (false positive in between, or corruption: host walks exactly).
__global__ void k_chain_verify(const Candidate *__restrict__ c, int64_t n, int64_t first, int64_t D,
                               unsigned long long *__restrict__ first_stop) {
  const int64_t i = first + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const Candidate ci = c[i];
  unsigned code;
  if (!(ci.flags & CAND_ISIZE) || (ci.flags & CAND_EMPTY)) {
    code = 1;
  } else {
    const int64_t nx = ci.pos + ci.csize;
    if (nx + 18 > D) code = 2;
    else if (i + 1 < n && c[i + 1].pos == nx) code = 0;
    else code = 3;
  }
  if (code) atomicMin(first_stop, (unsigned long long)(i * 4 + code));
}

SB_DEV int64_t cand_lower_bound(const Candidate *c, int64_t lo, int64_t hi, int64_t q) {
  while (lo < hi) {
    const int64_t m = (lo + hi) >> 1;
    if (c[m].pos < q) lo = m + 1;
    else hi = m;
  }
  return lo;
}

// FindBlockStart.apply for a batch of split starts (one thread per start).
__global__ void k_find_block_starts(const Candidate *__restrict__ c, int64_t n, int64_t D,
                                    const int64_t *__restrict__ starts, int64_t nq, int32_t nchk,
                                    int64_t *__restrict__ out) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= nq) return;
  const int64_t s = starts[t];
  const int64_t lim = s + 65536;  // Block.MAX_BLOCK_SIZE probes
  int64_t best = -1;
  const int64_t qe = max(s, D - 17);  // q + 18 > D: EOF while reading the first header → accepted
  for (int64_t j = cand_lower_bound(c, 0, n, s); j < n && c[j].pos < lim && c[j].pos < qe; j++) {
    int64_t cp = c[j].pos, idx = j;
    bool ok = true;
    for (int k = 0; k < nchk; k++) {
      if (cp + 18 > D) break;
      if (idx < 0) { ok = false; break; }
      const Candidate cc = c[idx];
      if (cp + cc.csize > D) break;
      if (cc.csize - cc.hsize - 8 == 2) break;
      cp += cc.csize;
      const int64_t nj = cand_lower_bound(c, idx + 1, n, cp);
      idx = (nj < n && c[nj].pos == cp) ? nj : -1;
    }
    if (ok) { best = c[j].pos; break; }
  }
  if (best < 0 && qe < lim) best = qe;
  out[t] = best;  // -1: HeaderSearchFailedException
}

__global__ void k_lower_bound(const Candidate *__restrict__ c, int64_t n, int64_t q, int64_t *__restrict__ out) {
  *out = cand_lower_bound(c, 0, n, q);
}

SB_DEV int64_t wave_sum64(int64_t v) {
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// The block table's columns from the verified chain, plus each workgroup's sum of uncompressed sizes for
// k_block_uoff (a negative isize counts 0, as MetadataStream's offsets do).
__global__ __launch_bounds__(256) void k_gather_blocks(const Candidate *__restrict__ c, int64_t first, int64_t n,
                                                       int64_t *__restrict__ st, int32_t *__restrict__ hs,
                                                       int32_t *__restrict__ cs, int32_t *__restrict__ us,
                                                       int64_t *__restrict__ wsum) {
  __shared__ int64_t s[4];
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int64_t u = 0;
  if (i < n) {
    const Candidate ci = c[first + i];
    st[i] = ci.pos;
    hs[i] = ci.hsize;
    cs[i] = ci.csize;
    us[i] = ci.isize;
    u = ci.isize < 0 ? 0 : ci.isize;
  }
  u = wave_sum64(u);
  if (lane_id() == 0) s[threadIdx.x >> 6] = u;
  __syncthreads();
  if (threadIdx.x == 0) wsum[blockIdx.x] = s[0] + s[1] + s[2] + s[3];
}

// Uncompressed offsets uoff[0..n] (exclusive prefix of the sizes; uoff[n] = the stream's length): each workgroup adds
// up the sums of the workgroups before it (n / 256 of them at most, from L2), then scans its own 256 blocks.
__global__ __launch_bounds__(256) void k_block_uoff(const int32_t *__restrict__ us, int64_t n,
                                                    const int64_t *__restrict__ wsum, int64_t *__restrict__ uoff) {
  __shared__ int64_t s[8];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  int64_t b = 0;
  for (int64_t k = t; k < (int64_t)blockIdx.x; k += 256) b += wsum[k];
  b = wave_sum64(b);
  if (lane == 0) s[w] = b;
  const int64_t i = (int64_t)blockIdx.x * 256 + t;
  const int64_t v = i < n ? (us[i] < 0 ? 0 : us[i]) : 0;
  int64_t x = v;  // inclusive scan within the wave
  for (int o = 1; o < 64; o <<= 1) {
    const int64_t y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) s[4 + w] = x;
  __syncthreads();
  int64_t base = s[0] + s[1] + s[2] + s[3];
  for (int k = 0; k < w; k++) base += s[4 + k];
  if (i < n) uoff[i] = base + x - v;
  if (i == n - 1) uoff[n] = base + x;
}

// ================================================================================================
// launch wrappers
// ================================================================================================

hipError_t launch_scan_count(const uint8_t *d, int64_t D, int32_t *cc, int64_t nchunks, hipStream_t s) {
  if (nchunks == 0) return hipSuccess;
  hipLaunchKernelGGL(k_scan_count, dim3((unsigned)nchunks), dim3(kScanThreads), 0, s, d, D, cc);
  return hipGetLastError();
}
hipError_t launch_scan_prefix(int32_t *cc, int64_t nchunks, int64_t *off, int64_t *total, hipStream_t s) {
  hipLaunchKernelGGL(k_scan_prefix, dim3(1), dim3(1024), 0, s, cc, nchunks, off, total);
  return hipGetLastError();
}
hipError_t launch_scan_write(const uint8_t *d, int64_t D, const int64_t *off, int64_t nchunks, Candidate *c,
                             hipStream_t s) {
  if (nchunks == 0) return hipSuccess;
  hipLaunchKernelGGL(k_scan_write, dim3((unsigned)nchunks), dim3(kScanThreads), 0, s, d, D, off, c);
  return hipGetLastError();
}
hipError_t launch_scan_slots(const uint8_t *d, int64_t D, int32_t *cc, int64_t nchunks, Candidate *slots,
                             int64_t *overflow, hipStream_t s) {
  (void)hipMemsetAsync(overflow, 0, sizeof(int64_t), s);
  if (nchunks == 0) return hipSuccess;
  hipLaunchKernelGGL(k_scan_slots_wide<kScanWide>, dim3((unsigned)nchunks), dim3(kScanThreads), 0, s, d, D, cc,
                     slots, reinterpret_cast<unsigned long long *>(overflow));
  return hipGetLastError();
}
hipError_t launch_scan_compact(const Candidate *slots, const int32_t *cc, const int64_t *off, int64_t nchunks,
                               Candidate *out, hipStream_t s) {
  const int64_t n = nchunks * kScanSlots;
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_scan_compact, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, slots, cc, off, nchunks,
                     out);
  return hipGetLastError();
}
hipError_t launch_chain_verify(const Candidate *c, int64_t n, int64_t first, int64_t D, int64_t *first_stop,
                               hipStream_t s) {
  if (n - first <= 0) return hipSuccess;
  const int64_t m = n - first;
  hipLaunchKernelGGL(k_chain_verify, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, s, c, n, first, D,
                     reinterpret_cast<unsigned long long *>(first_stop));
  return hipGetLastError();
}
hipError_t launch_find_block_starts(const uint8_t *, int64_t D, const Candidate *c, int64_t ncand, const int64_t *st,
                                    int64_t n, int32_t nchk, int64_t *out, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_find_block_starts, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, c, ncand, D, st, n,
                     nchk, out);
  return hipGetLastError();
}
hipError_t launch_lower_bound(const Candidate *c, int64_t n, int64_t q, int64_t *out, hipStream_t s) {
  hipLaunchKernelGGL(k_lower_bound, dim3(1), dim3(1), 0, s, c, n, q, out);
  return hipGetLastError();
}
hipError_t launch_gather_blocks(const Candidate *c, int64_t first, int64_t n, int64_t *st, int32_t *hs, int32_t *cs,
                                int32_t *us, int64_t *wsum, int64_t *uoff, hipStream_t s) {
  if (n == 0) return hipMemsetAsync(uoff, 0, sizeof(int64_t), s);
  const unsigned nwg = (unsigned)((n + 255) / 256);
  hipLaunchKernelGGL(k_gather_blocks, dim3(nwg), dim3(256), 0, s, c, first, n, st, hs, cs, us, wsum);
  hipLaunchKernelGGL(k_block_uoff, dim3(nwg), dim3(256), 0, s, us, n, wsum, uoff);
  return hipGetLastError();
}
}  // namespace sbam
