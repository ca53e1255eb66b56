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

__global__ void k_gather_blocks(const Candidate *__restrict__ c, int64_t first, int64_t n, int64_t *__restrict__ st,
                                int32_t *__restrict__ hs, int32_t *__restrict__ cs, int32_t *__restrict__ us) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const Candidate ci = c[first + i];
  st[i] = ci.pos;
  hs[i] = ci.hsize;
  cs[i] = ci.csize;
  us[i] = ci.isize;
}

// ================================================================================================
// 2. Inflate: one lane per BGZF block (SIMT across independent blocks), lanes pull blocks from a
//    work counter; Huffman tables per lane in an HBM scratch slot, length/distance bases in LDS.
// ================================================================================================
__constant__ uint16_t kLenBase[29] = {3,  4,  5,  6,  7,  8,  9,  10, 11,  13,  15,  17,  19,  23, 27,
                                      31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
__constant__ uint8_t kLenExtra[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
__constant__ uint16_t kDistBase[30] = {1,   2,   3,   4,   5,   7,    9,    13,   17,   25,   33,   49,   65,    97,    129,
                                       193, 257, 385, 513, 769, 1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
__constant__ uint8_t kDistExtra[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
__constant__ uint8_t kClOrder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

// per-lane scratch layout (u16 units)
constexpr int kLitRoot = 10, kDistRoot = 8, kClRoot = 7;
constexpr int kOffLit = 0, kOffDist = 1024, kOffLitCnt = 1280, kOffDistCnt = 1296, kOffLitSym = 1312,
              kOffDistSym = 1632, kOffCl = 1664, kOffLens = 1792 /* 320 bytes */, kOffClLens = 1952 /* 19 bytes */,
              kOffSlow = 1976 /* litFirst, litIndex, distFirst, distIndex, clFirst, clIndex */, kOffClCnt = 1984,
              kOffClSym = 2000 /* 19 */;
static_assert(kOffClSym + 24 <= kInflateScratchU16, "scratch layout");

// 16 counters of 9 bits packed into three u64 (7 per word): register-resident histogram.
struct Pack16 {
  uint64_t a = 0, b = 0, c = 0;
  SB_DEV void add(uint32_t l, uint64_t v) {
    const uint32_t w = (l >= 7) + (l >= 14);
    const uint64_t inc = v << (9 * (l - 7 * w));
    a += (w == 0) ? inc : 0;
    b += (w == 1) ? inc : 0;
    c += (w == 2) ? inc : 0;
  }
  SB_DEV uint32_t get(uint32_t l) const {
    const uint32_t w = (l >= 7) + (l >= 14);
    const uint64_t x = (w == 0) ? a : (w == 1) ? b : c;
    return (uint32_t)(x >> (9 * (l - 7 * w))) & 511u;
  }
};

// Canonical Huffman table (RFC 1951 §3.2.2).  Primary table of 2^root u16 entries (len<<9 | sym),
// 0 = code longer than root (or unused): decoded by the canonical slow path from cnt/sorted/slow.
// Returns 0, or -1 for an over-subscribed code.
SB_DEV int build_huff(const uint8_t *lens, int n, int root, uint16_t *tab, uint16_t *cnt_out, uint16_t *sorted,
                      uint16_t *slow) {
  Pack16 cnt;
  for (int s = 0; s < n; s++) {
    const uint32_t l = lens[s];
    if (l) cnt.add(l, 1);
  }
  int left = 1;
  for (int l = 1; l <= 15; l++) {
    left = (left << 1) - (int)cnt.get(l);
    if (left < 0) return -1;
    cnt_out[l] = (uint16_t)cnt.get(l);
  }
  Pack16 offs;
  uint32_t acc = 0;
  for (int l = 1; l <= 15; l++) {
    offs.add(l, acc);
    acc += cnt.get(l);
  }
  for (int s = 0; s < n; s++) {
    const uint32_t l = lens[s];
    if (l) {
      sorted[offs.get(l)] = (uint16_t)s;
      offs.add(l, 1);
    }
  }
  const int size = 1 << root;
  if (left > 0)
    for (int j = 0; j < size; j++) tab[j] = 0;
  uint32_t code = 0, idx = 0;
  for (int l = 1; l <= root; l++) {
    const uint32_t cl = cnt.get(l);
    for (uint32_t i = 0; i < cl; i++) {
      const uint16_t e = (uint16_t)((l << 9) | sorted[idx++]);
      for (uint32_t j = brev(code, l); j < (uint32_t)size; j += (1u << l)) tab[j] = e;
      code++;
    }
    code <<= 1;
  }
  for (int l = root + 1; l <= 15; l++) {
    const uint32_t cl = cnt.get(l);
    for (uint32_t i = 0; i < cl; i++) {
      tab[brev(code >> (l - root), root)] = 0;
      code++;
    }
    code <<= 1;
  }
  int first = 0, index = 0;
  for (int l = 1; l <= root; l++) {
    index += (int)cnt.get(l);
    first += (int)cnt.get(l);
    first <<= 1;
  }
  slow[0] = (uint16_t)first;
  slow[1] = (uint16_t)index;
  return 0;
}

// Canonical decode of a code longer than root bits (puff-style, resumed after `root` bits).
SB_DEV int slow_decode(uint64_t bb, int root, const uint16_t *cnt, const uint16_t *sorted, const uint16_t *slow,
                       uint32_t &len) {
  int code = (int)(brev((uint32_t)bb & ((1u << root) - 1u), root) << 1);
  int first = slow[0], index = slow[1];
  for (int l = root + 1; l <= 15; l++) {
    code |= (int)((bb >> (l - 1)) & 1u);
    const int count = cnt[l];
    if (code - count < first) {
      len = (uint32_t)l;
      return sorted[index + (code - first)];
    }
    index += count;
    first += count;
    first <<= 1;
    code <<= 1;
  }
  return -1;
}

enum : int { S_NEXT = 0, S_HDR = 1, S_HUFF = 2, S_COPY = 3, S_STORED = 4, S_DONE = 5, S_EXIT = 6 };

// Per-lane output ring in LDS: the last 64 output bytes of the lane's block (stride 68 B so the 64 lanes of a
// wave hit distinct banks).  Bytes are emitted into the ring and leave it as aligned 16-B global stores (or byte
// stores for a block's partial first/last chunk, which share a 16-B chunk with the neighbouring block).
// Copies with distance <= 56 read their source from the ring, longer ones from global memory (aligned 8-B pairs).
constexpr int kRingStride = 68;
constexpr int kRingNear = 56;

SB_DEV void ring_flush(uint8_t *&fp, const uint8_t *o, const uint8_t *ring, bool final) {
  for (;;) {
    const uintptr_t f = reinterpret_cast<uintptr_t>(fp), oo = reinterpret_cast<uintptr_t>(o);
    const uintptr_t cend = (f & ~(uintptr_t)15) + 16;
    if ((f & 15) == 0 && f + 16 <= oo) {
      const uint32_t *r = reinterpret_cast<const uint32_t *>(ring + (f & 63));
      *reinterpret_cast<uint4 *>(fp) = make_uint4(r[0], r[1], r[2], r[3]);
      fp += 16;
    } else if ((f & 15) != 0 && cend <= oo) {
      for (uintptr_t q = f; q < cend; q++) *reinterpret_cast<uint8_t *>(q) = ring[q & 63];
      fp = reinterpret_cast<uint8_t *>(cend);
    } else {
      if (final)
        for (uintptr_t q = f; q < oo; q++) *reinterpret_cast<uint8_t *>(q) = ring[q & 63];
      if (final) fp = const_cast<uint8_t *>(o);
      return;
    }
  }
}

enum : int32_t { INF_OK = 0, INF_SHORT = 1, INF_DATA = 2 };

__global__ __launch_bounds__(256) void k_inflate(const uint8_t *__restrict__ d, int64_t D, BlockTable bt, uint8_t *out,
                                                 uint16_t *__restrict__ scratch_all, int32_t *__restrict__ status,
                                                 int32_t *__restrict__ found, unsigned int *__restrict__ next_block,
                                                 unsigned long long *__restrict__ first_err) {
  __shared__ uint32_t s_len[32], s_dist[32];
  __shared__ __attribute__((aligned(16))) uint8_t s_ring[256 * kRingStride];
  uint8_t *ring = s_ring + threadIdx.x * kRingStride;
  if (threadIdx.x < 29) s_len[threadIdx.x] = kLenBase[threadIdx.x] | ((uint32_t)kLenExtra[threadIdx.x] << 16);
  if (threadIdx.x < 30) s_dist[threadIdx.x] = kDistBase[threadIdx.x] | ((uint32_t)kDistExtra[threadIdx.x] << 16);
  __syncthreads();

  uint16_t *scr = scratch_all + (size_t)(blockIdx.x * blockDim.x + threadIdx.x) * kInflateScratchU16;
  uint16_t *litT = scr + kOffLit, *distT = scr + kOffDist, *clT = scr + kOffCl;
  uint8_t *lens = reinterpret_cast<uint8_t *>(scr + kOffLens);
  uint8_t *cllens = reinterpret_cast<uint8_t *>(scr + kOffClLens);

  int state = S_NEXT;
  int32_t err = INF_OK;
  int64_t blk = -1;
  const uint32_t *inw = nullptr;
  const uint32_t *inlim = nullptr;  // first dword the bit reader may not load (payload + footer)
  uint64_t bb = 0;
  int bc = 0;
  uint8_t *o = nullptr, *ob = nullptr, *oe = nullptr, *fp = nullptr;
  int fin = 0, clen = 0, cdist = 0, sleft = 0;
#define RING_PUT(b) (ring[reinterpret_cast<uintptr_t>(o) & 63] = (uint8_t)(b), o++)

  for (;;) {
    if (state == S_NEXT) {
      blk = (int64_t)atomicAdd(next_block, 1u);
      if (blk >= bt.n) {
        state = S_EXIT;
      } else {
        const uintptr_t a = reinterpret_cast<uintptr_t>(d + bt.start[blk] + bt.hsize[blk]);
        inw = reinterpret_cast<const uint32_t *>(a & ~(uintptr_t)3);
        const int64_t pend = min(bt.start[blk] + bt.csize[blk], D) + 4;  // payload, 8-B footer, one dword slack
        inlim = reinterpret_cast<const uint32_t *>(reinterpret_cast<uintptr_t>(d + pend) & ~(uintptr_t)3);
        const int skip = (int)(a & 3) * 8;
        bb = (uint64_t)(*inw++) >> skip;
        bc = 32 - skip;
        ob = out + bt.uoff[blk];
        o = ob;
        fp = ob;
        const int32_t us = bt.usize[blk];
        oe = ob + us;
        fin = 0;
        err = INF_OK;
        // inflate(decBuf, 0, ISIZE): ISIZE 0 → 0 bytes, always equal; ISIZE > 64 KiB overflows decBuf.
        if (us == 0) state = S_DONE;
        else if (us < 0 || us > 65536) { err = INF_DATA; state = S_DONE; }
        else state = S_HDR;
      }
    }
    if (__all(state == S_EXIT)) break;
    if (state != S_EXIT && state != S_DONE && bc <= 32) {
      if (inw >= inlim) {  // the stream wants more input than the block holds: Inflater returns short
        err = INF_SHORT;
        state = S_DONE;
      } else {
        bb |= (uint64_t)(*inw++) << bc;
        bc += 32;
      }
    }

    if (state == S_HDR) {
      fin = (int)(bb & 1);
      const int type = (int)((bb >> 1) & 3);
      bb >>= 3;
      bc -= 3;
      if (type == 0) {  // stored
        const int drop = bc & 7;
        bb >>= drop;
        bc -= drop;
        if (bc <= 32 && inw < inlim) { bb |= (uint64_t)(*inw++) << bc; bc += 32; }
        const uint32_t ln = (uint32_t)(bb & 0xffff), nl = (uint32_t)((bb >> 16) & 0xffff);
        bb >>= 32;
        bc -= 32;
        if (ln != (~nl & 0xffffu)) { err = INF_DATA; state = S_DONE; }
        else { sleft = (int)ln; state = S_STORED; }
      } else if (type == 1) {  // fixed Huffman codes
        for (int s = 0; s < 288; s++) lens[s] = (uint8_t)(s < 144 ? 8 : s < 256 ? 9 : s < 280 ? 7 : 8);
        for (int s = 0; s < 30; s++) lens[288 + s] = 5;
        build_huff(lens, 288, kLitRoot, litT, scr + kOffLitCnt, scr + kOffLitSym, scr + kOffSlow);
        build_huff(lens + 288, 30, kDistRoot, distT, scr + kOffDistCnt, scr + kOffDistSym, scr + kOffSlow + 2);
        state = S_HUFF;
      } else if (type == 2) {  // dynamic Huffman codes
        const int hlit = (int)(bb & 31) + 257, hdist = (int)((bb >> 5) & 31) + 1, hclen = (int)((bb >> 10) & 15) + 4;
        bb >>= 14;
        bc -= 14;
        for (int i = 0; i < 19; i++) {
          if (bc <= 32 && inw < inlim) { bb |= (uint64_t)(*inw++) << bc; bc += 32; }
          uint32_t v = 0;
          if (i < hclen) { v = (uint32_t)(bb & 7); bb >>= 3; bc -= 3; }
          cllens[kClOrder[i]] = (uint8_t)v;
        }
        int ok = build_huff(cllens, 19, kClRoot, clT, scr + kOffClCnt, scr + kOffClSym, scr + kOffSlow + 4) == 0;
        const int total = hlit + hdist;
        int n = 0;
        uint32_t prev = 0;
        while (ok && n < total) {
          if (bc <= 32 && inw < inlim) { bb |= (uint64_t)(*inw++) << bc; bc += 32; }
          const uint32_t e = clT[bb & 127];
          const uint32_t l = e >> 9, sym = e & 511;
          if (l == 0) { ok = 0; break; }
          bb >>= l;
          bc -= (int)l;
          if (sym < 16) {
            lens[n++] = (uint8_t)sym;
            prev = sym;
          } else {
            int rep;
            uint32_t v;
            if (sym == 16) {
              if (n == 0) { ok = 0; break; }
              rep = 3 + (int)(bb & 3); bb >>= 2; bc -= 2; v = prev;
            } else if (sym == 17) {
              rep = 3 + (int)(bb & 7); bb >>= 3; bc -= 3; v = 0;
            } else {
              rep = 11 + (int)(bb & 127); bb >>= 7; bc -= 7; v = 0;
            }
            if (n + rep > total) { ok = 0; break; }
            for (int r = 0; r < rep; r++) lens[n++] = (uint8_t)v;
            prev = v;
          }
        }
        if (ok && lens[256] == 0) ok = 0;  // missing end-of-block code
        if (ok) ok = build_huff(lens, hlit, kLitRoot, litT, scr + kOffLitCnt, scr + kOffLitSym, scr + kOffSlow) == 0;
        if (ok)
          ok = build_huff(lens + hlit, hdist, kDistRoot, distT, scr + kOffDistCnt, scr + kOffDistSym, scr + kOffSlow + 2) == 0;
        if (ok) state = S_HUFF;
        else { err = INF_DATA; state = S_DONE; }
      } else {
        err = INF_DATA;
        state = S_DONE;
      }
    } else if (state == S_HUFF) {
      uint32_t e = litT[bb & ((1u << kLitRoot) - 1)];
      uint32_t l = e >> 9;
      int sym = (int)(e & 511);
      if (l == 0) sym = slow_decode(bb, kLitRoot, scr + kOffLitCnt, scr + kOffLitSym, scr + kOffSlow, l);
      if (sym < 0) {
        err = INF_DATA;
        state = S_DONE;
      } else {
        bb >>= l;
        bc -= (int)l;
        if (sym < 256) {
          RING_PUT(sym);
          if (o == oe) state = S_DONE;
        } else if (sym == 256) {
          if (fin) { err = (o == oe) ? INF_OK : INF_SHORT; state = S_DONE; }
          else state = S_HDR;
        } else if (sym - 257 >= 29) {
          err = INF_DATA;
          state = S_DONE;
        } else {
          const uint32_t lb = s_len[sym - 257];
          const uint32_t lx = lb >> 16;
          clen = (int)(lb & 0xffff) + (int)(bb & ((1u << lx) - 1u));
          bb >>= lx;
          bc -= (int)lx;
          if (bc <= 32 && inw < inlim) { bb |= (uint64_t)(*inw++) << bc; bc += 32; }
          uint32_t de = distT[bb & ((1u << kDistRoot) - 1)];
          uint32_t dl = de >> 9;
          int ds = (int)(de & 511);
          if (dl == 0) ds = slow_decode(bb, kDistRoot, scr + kOffDistCnt, scr + kOffDistSym, scr + kOffSlow + 2, dl);
          if (ds < 0 || ds >= 30) {
            err = INF_DATA;
            state = S_DONE;
          } else {
            bb >>= dl;
            bc -= (int)dl;
            const uint32_t db = s_dist[ds];
            const uint32_t dx = db >> 16;
            cdist = (int)(db & 0xffff) + (int)(bb & ((1u << dx) - 1u));
            bb >>= dx;
            bc -= (int)dx;
            if (cdist > (int)(o - ob)) { err = INF_DATA; state = S_DONE; }
            else state = S_COPY;
          }
        }
      }
    }
    if (state == S_COPY) {  // up to 8 bytes per step; an overlapping copy replicates its period
      const int room = (int)(oe - o);
      const int n = min(min(clen, 8), room);
      const uintptr_t src = reinterpret_cast<uintptr_t>(o) - (uintptr_t)cdist;
      const int np = min(cdist, 8);
      uint64_t pat = 0;
      if (cdist <= kRingNear) {  // source still in the ring
#pragma unroll
        for (int i = 0; i < 8; i++) pat |= (i < np) ? ((uint64_t)ring[(src + i) & 63] << (8 * i)) : 0ull;
      } else {  // source already flushed: two aligned 8-byte loads
        const uint64_t *a8 = reinterpret_cast<const uint64_t *>(src & ~(uintptr_t)7);
        const uint64_t lo = a8[0], hi = a8[1];
        const int sh = (int)(src & 7) * 8;
        pat = sh ? (lo >> sh) | (hi << (64 - sh)) : lo;
      }
      if (cdist < 8) {
        pat &= (1ull << (8 * cdist)) - 1;
        for (int p = cdist; p < 8; p <<= 1) pat |= pat << (8 * p);
      }
#pragma unroll
      for (int i = 0; i < 8; i++)
        if (i < n) RING_PUT(pat >> (8 * i));
      clen -= n;
      if (o == oe) state = S_DONE;
      else if (clen == 0) state = S_HUFF;
    } else if (state == S_STORED) {
      const int n = min(min(sleft, 4), (int)(oe - o));
      for (int i = 0; i < n; i++) RING_PUT(bb >> (8 * i));
      bb >>= 8 * n;
      bc -= 8 * n;
      sleft -= n;
      if (o == oe) state = S_DONE;
      else if (sleft == 0) {
        if (fin) { err = INF_SHORT; state = S_DONE; }
        else state = S_HDR;
      }
    }
    if (state != S_EXIT && state != S_NEXT) ring_flush(fp, o, ring, state == S_DONE);
    if (state == S_DONE) {
      if (err != INF_OK) atomicMin(first_err, (unsigned long long)blk);
      status[blk] = err;
      found[blk] = (int32_t)(o - ob);
      state = S_NEXT;
    }
  }
#undef RING_PUT
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
                                int32_t *us, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_gather_blocks, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, c, first, n, st, hs, cs, us);
  return hipGetLastError();
}
hipError_t launch_inflate(const uint8_t *d, int64_t D, BlockTable bt, uint8_t *out, uint16_t *scratch, int nlanes,
                          int32_t *status, int32_t *found, unsigned int *next_block, unsigned long long *first_err,
                          hipStream_t s) {
  if (bt.n == 0) return hipSuccess;
  (void)hipMemsetAsync(next_block, 0, sizeof(unsigned int), s);
  hipLaunchKernelGGL(k_inflate, dim3((unsigned)(nlanes / 256)), dim3(256), 0, s, d, D, bt, out, scratch, status, found,
                     next_block, first_err);
  return hipGetLastError();
}
}  // namespace sbam
