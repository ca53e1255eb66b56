// sbam_kernels.hip — hand-written CDNA4 (gfx950) kernels for the spark-bam hot path.
//
//  * BGZF block-header scan   (Header.make bgzf/.../block/Header.scala:48-83, MetadataStream.scala:23-54,
//                              FindBlockStart.scala:8-36)
//  * batched raw-DEFLATE inflate (Stream.scala:31-71; RFC 1951 semantics of java.util.zip.Inflater)
//  * exhaustive per-offset record-boundary checker, eager + full
//                             (check/.../check/eager/Checker.scala:24-126, full/Checker.scala:22-184,
//                              PosChecker.scala:43-63) with full-check Counts reduction (FullCheck.scala:141-191)
//  * FindRecordStart scan     (check/.../bam/spark/FindRecordStart.scala:30-63)
//  * record-chain walk        (check/.../bam/iterator/RecordStream.scala:27-41)
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
enum : int32_t { INF_OK = 0, INF_SHORT = 1, INF_DATA = 2 };

__global__ __launch_bounds__(256) void k_inflate(const uint8_t *__restrict__ d, int64_t D, BlockTable bt, uint8_t *out,
                                                 uint16_t *__restrict__ scratch_all, int32_t *__restrict__ status,
                                                 int32_t *__restrict__ found, unsigned int *__restrict__ next_block,
                                                 unsigned long long *__restrict__ first_err) {
  __shared__ uint32_t s_len[32], s_dist[32];
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
  uint8_t *o = nullptr, *ob = nullptr, *oe = nullptr;
  int fin = 0, clen = 0, cdist = 0, sleft = 0;

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
          *o++ = (uint8_t)sym;
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
      const uint8_t *src = o - cdist;
      const int np = min(cdist, 8);
      uint64_t pat = 0;
#pragma unroll
      for (int i = 0; i < 8; i++) pat |= (i < np) ? ((uint64_t)src[i] << (8 * i)) : 0ull;
      for (int p = cdist; p < 8; p <<= 1) pat |= pat << (8 * p);
#pragma unroll
      for (int i = 0; i < 8; i++)
        if (i < n) o[i] = (uint8_t)(pat >> (8 * i));
      o += n;
      clen -= n;
      if (o == oe) state = S_DONE;
      else if (clen == 0) state = S_HUFF;
    } else if (state == S_STORED) {
      const int n = min(min(sleft, 4), (int)(oe - o));
      for (int i = 0; i < n; i++) o[i] = (uint8_t)(bb >> (8 * i));
      bb >>= 8 * n;
      bc -= 8 * n;
      o += n;
      sleft -= n;
      if (o == oe) state = S_DONE;
      else if (sleft == 0) {
        if (fin) { err = INF_SHORT; state = S_DONE; }
        else state = S_HDR;
      }
    }
    if (state == S_DONE) {
      if (err != INF_OK) atomicMin(first_err, (unsigned long long)blk);
      status[blk] = err;
      found[blk] = (int32_t)(o - ob);
      state = S_NEXT;
    }
  }
}

// ================================================================================================
// 3. Record-boundary checker
// ================================================================================================
constexpr uint32_t W_SUCC = 0x80000000u, W_HALO = 0x00800000u;
constexpr int kCheckThreads = 256;
constexpr int kTile = 8192;  // positions per workgroup tile
constexpr int kHalo = 768;   // staged bytes past the tile: fixed fields + max read name (36 + 255) + cigar ops
constexpr int kWin = kTile + 16 + kHalo;  // staged window (multiple of 16)
static_assert(kWin % 16 == 0, "window");

// Bytes of the stream: the staged LDS window when inside it, else global memory.
struct Win {
  const uint8_t *lds;
  int64_t base;  // stream offset of lds[0]
  int wlen;
  const uint8_t *g;
  SB_DEV uint32_t byte(int64_t x) const {
    const int64_t r = x - base;
    return (r >= 0 && r < wlen) ? (uint32_t)lds[r] : (uint32_t)g[x];
  }
  SB_DEV int32_t i32(int64_t x) const {
    return (int32_t)(byte(x) | (byte(x + 1) << 8) | (byte(x + 2) << 16) | (byte(x + 3) << 24));
  }
};

SB_DEV bool name_char_ok(uint32_t b) { return (b - 33u <= 30u) || (b - 65u <= 61u); }

// PosChecker.getRefPosError as bits {negIdx, bigIdx, negPos, bigPos}; note negPos = rp < -1 in every branch.
SB_DEV uint32_t ref_err(int32_t ri, int32_t rp, const int64_t *lens, int32_t nref) {
  uint32_t f = 0;
  f |= (ri < -1) ? 1u : 0u;
  f |= (ri >= nref) ? 2u : 0u;
  f |= (rp < -1) ? 4u : 0u;
  if (ri >= 0 && ri < nref && rp >= -1) f |= ((int64_t)rp > lens[ri]) ? 8u : 0u;
  return f;
}

// full.Checker from position p with the k=0 fixed fields already loaded (f[0..7] = block_size, refID, pos,
// bin_mq_nl, flag_nc, l_seq, next_refID, next_pos).  EAGER: stop at the first failing group (the boolean
// is the same; flags returned are partial).  Returns the result word (sbam.h).
template <bool EAGER>
SB_DEV uint32_t check_from(const Win &w, const StreamView &sv, int64_t p, int R, const int32_t f0[8]) {
  int64_t s = p, a = p;
  int k = 0;
  int32_t bs = f0[0], ri = f0[1], rp = f0[2], bmn = f0[3], fnc = f0[4], ls = f0[5], nri = f0[6], nrp = f0[7];
  for (;;) {
    if (k == R) return W_SUCC | ((uint32_t)k << 24);
    if (a + 36 > sv.L) {
      if (!sv.eof_real) return W_HALO;
      if (k > 0 && s == sv.L) return W_SUCC | ((uint32_t)k << 24);
      return 1u | ((uint32_t)k << 24);
    }
    if (k > 0) {
      bs = w.i32(a); ri = w.i32(a + 4); rp = w.i32(a + 8); bmn = w.i32(a + 12);
      fnc = w.i32(a + 16); ls = w.i32(a + 20); nri = w.i32(a + 24); nrp = w.i32(a + 28);
    }
    uint32_t F = ref_err(ri, rp, sv.lens, sv.nref) << 1;
    if (EAGER && F) return (uint32_t)k << 24 | F;
    const int32_t lrn = bmn & 0xff;
    const uint32_t flag = ((uint32_t)fnc) >> 16;
    const int32_t nc = fnc & 0xffff;
    const int32_t t = (int32_t)((uint32_t)ls + 1u);
    const int32_t nsq = (int32_t)((uint32_t)(t / 2) + (uint32_t)ls);
    const int32_t implied = (int32_t)(32u + (uint32_t)lrn + 4u * (uint32_t)nc + (uint32_t)nsq);
    F |= (bs < implied) ? (1u << 18) : 0u;
    F |= ref_err(nri, nrp, sv.lens, sv.nref) << 5;
    if (EAGER) {
      if (F || lrn < 2 || ((flag & 4u) == 0 && (ls == 0 || nc == 0))) return ((uint32_t)k << 24) | (F ? F : 1u << 12);
    }
    int64_t c = a + 36;
    if (lrn == 0) {
      F |= 1u << 12;
    } else if (lrn == 1) {
      F |= 1u << 13;
    } else {
      if (c + lrn > sv.L) {
        if (!sv.eof_real) return W_HALO;
        return F | (1u << 9) | ((uint32_t)k << 24);
      }
      if (w.byte(c + lrn - 1) != 0) {
        F |= 1u << 10;
      } else {
        for (int32_t i = 0; i < lrn - 1; i++)
          if (!name_char_ok(w.byte(c + i))) {
            F |= 1u << 11;
            break;
          }
      }
      c += lrn;
      if (EAGER && F) return ((uint32_t)k << 24) | F;
    }
    bool cig_err = false;
    for (int32_t i = 0; i < nc; i++) {
      if (c + 4 > sv.L) {
        if (!sv.eof_real) return W_HALO;
        F |= 1u << 14;
        cig_err = true;
        break;
      }
      const uint32_t op = w.byte(c);
      c += 4;
      if ((op & 0xfu) > 8u) {
        F |= 1u << 15;
        cig_err = true;
        break;
      }
    }
    if (!cig_err && (flag & 4u) == 0 && (ls == 0 || nc == 0)) {
      F |= (ls == 0) ? (1u << 16) : 0u;  // EmptyMapped(emptySeq, emptyCigar) → (emptyMappedCigar, emptyMappedSeq)
      F |= (nc == 0) ? (1u << 17) : 0u;
    }
    if (F) return F | ((uint32_t)k << 24);
    const int64_t nxt = s + 4 + (int64_t)bs;
    if (nxt > c) {
      if (nxt > sv.L && !sv.eof_real) return W_HALO;
      a = nxt > sv.L ? sv.L : nxt;
    } else {
      a = c;
    }
    s = nxt;
    k++;
  }
}

// Stage stream bytes [abase, abase + kWin) into LDS (16 B per lane per step; the stream is zero padded).
SB_DEV void stage(uint8_t *s_win, const uint8_t *u, int64_t abase) {
  const uint4 *src = reinterpret_cast<const uint4 *>(u + abase);
  uint4 *dst = reinterpret_cast<uint4 *>(s_win);
  for (int i = threadIdx.x; i < kWin / 16; i += kCheckThreads) dst[i] = src[i];
}

// k=0 fixed fields of position x from the staged window: ten aligned LDS dwords + v_alignbyte.
SB_DEV void fixed_fields(const uint8_t *s_win, int64_t abase, int64_t x, int32_t f[8]) {
  const int r = (int)(x - abase);
  const uint32_t *w32 = reinterpret_cast<const uint32_t *>(s_win) + (r >> 2);
  const int o = r & 3;
  uint32_t W[9];
#pragma unroll
  for (int j = 0; j < 9; j++) W[j] = w32[j];
#pragma unroll
  for (int j = 0; j < 8; j++) f[j] = (int32_t)__builtin_amdgcn_alignbyte(W[j + 1], W[j], o);
}

enum { MODE_COUNTS = 0, MODE_EAGER = 1, MODE_WORDS = 2 };

template <int MODE>
__global__ __launch_bounds__(kCheckThreads) void k_check(StreamView sv, int64_t x0, int64_t x1, int R, CountsDev cd,
                                                         unsigned long long *__restrict__ bitmap,
                                                         uint32_t *__restrict__ words) {
  __shared__ __attribute__((aligned(16))) uint8_t s_win[kWin + 16];
  __shared__ uint32_t s_cnt[21 * 19];
  __shared__ uint32_t s_npos[21];
  const int lane = lane_id();
  if (MODE == MODE_COUNTS) {
    for (int i = threadIdx.x; i < 21 * 19; i += kCheckThreads) s_cnt[i] = 0;
    if (threadIdx.x < 21) s_npos[threadIdx.x] = 0;
  }
  unsigned long long n_succ = 0, n_tff = 0, n_halo = 0;  // lane 0 of each wave accumulates
  const int64_t ntiles = (x1 - x0 + kTile - 1) / kTile;
  for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const int64_t base = x0 + t * kTile;
    const int64_t abase = base & ~(int64_t)15;
    __syncthreads();
    stage(s_win, sv.u, abase);
    __syncthreads();
    const Win w{s_win, abase, kWin, sv.u};
    for (int j = 0; j < kTile / kCheckThreads; j++) {
      const int64_t x = base + j * kCheckThreads + threadIdx.x;
      const bool valid = x < x1;
      uint32_t word = 0;
      if (valid) {
        int32_t f[8];
        fixed_fields(s_win, abase, x, f);
        word = check_from<MODE == MODE_EAGER>(w, sv, x, R, f);
      }
      if (MODE == MODE_WORDS) {
        if (valid) words[x - x0] = word;
        continue;
      }
      const bool succ = valid && (word & W_SUCC);
      const unsigned long long sm = __ballot(succ);
      const int64_t rel = base - x0 + j * kCheckThreads + (threadIdx.x & ~63);
      if (lane == 0 && bitmap) bitmap[rel >> 6] = sm;
      if (MODE == MODE_COUNTS) {
        const bool halo = valid && word == W_HALO;
        const bool tff = valid && word == 1u;
        const bool counted = valid && !succ && !halo && !tff;
        const unsigned long long hm = __ballot(halo), tm = __ballot(tff);
        if (lane == 0) {
          n_succ += __popcll(sm);
          n_tff += __popcll(tm);
          n_halo += __popcll(hm);
        }
        const uint32_t F = word & 0x7ffffu;
        const uint32_t kk = (word >> 24) & 0x7fu;
        const uint32_t key = (uint32_t)__popc(F) + (kk > 0 ? 1u : 0u);
        uint32_t present = wave_or(counted ? (1u << key) : 0u);
        while (present) {
          const uint32_t k = __builtin_ctz(present);
          present &= present - 1;
          const bool in = counted && key == k;
          const unsigned long long km = __ballot(in);
          uint32_t mycnt = 0;
#pragma unroll
          for (int f = 0; f < 19; f++) {
            const unsigned long long m = __ballot(in && ((F >> f) & 1u));
            mycnt = (lane == f) ? (uint32_t)__popcll(m) : mycnt;
          }
          if (lane < 19 && mycnt) atomicAdd(&s_cnt[k * 19 + lane], mycnt);
          if (lane == 19) atomicAdd(&s_npos[k], (uint32_t)__popcll(km));
        }
        if (counted && kk > 0) atomicAdd(&cd.rbe[key * 128 + kk], 1ull);
        if (counted && key == 2) {  // close calls: histogram of the two failing flags
          const uint32_t fi = __builtin_ctz(F);
          const uint32_t rest = F & (F - 1);
          const uint32_t fj = rest ? __builtin_ctz(rest) : fi;  // k>0 with one flag: (fi, fi)
          atomicAdd(&cd.pair[fi * 19 + fj], 1ull);
        }
      }
    }
  }
  if (MODE == MODE_COUNTS) {
    __syncthreads();
    for (int i = threadIdx.x; i < 21 * 19; i += kCheckThreads)
      if (s_cnt[i]) atomicAdd(&cd.counts[i], (unsigned long long)s_cnt[i]);
    if (threadIdx.x < 21 && s_npos[threadIdx.x]) atomicAdd(&cd.positions[threadIdx.x], (unsigned long long)s_npos[threadIdx.x]);
    if (lane == 0) {
      if (n_succ) atomicAdd(&cd.scalars[1], n_succ);
      if (n_tff) atomicAdd(&cd.scalars[2], n_tff);
      if (n_halo) atomicAdd(&cd.scalars[3], n_halo);
    }
  }
}

// FindRecordStart.withDelta for a batch of start offsets: one workgroup per start scans 256 positions per
// step (eager checker, global reads) until the first true call; with a success bitmap covering [bx0, bx1)
// the covered prefix is read from the bitmap instead.  out = found offset, -1 = None, -2 = HALO.
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
  if (x0 < 0) { if (threadIdx.x == 0) out[blockIdx.x] = -1; return; }
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
  const Win w{nullptr, 0, 0, sv.u};
  while (s_best == ~0ull && x < lim && !s_halo) {
    const int64_t p = x + threadIdx.x;
    if (p < lim) {
      int32_t f[8];
      if (p + 36 <= sv.L) {
#pragma unroll
        for (int j = 0; j < 8; j++) f[j] = w.i32(p + 4 * j);
      } else {
#pragma unroll
        for (int j = 0; j < 8; j++) f[j] = 0;
      }
      const uint32_t word = check_from<true>(w, sv, p, R, f);
      if (word == W_HALO) s_halo = 1;
      else if (word & W_SUCC) atomicMin(&s_best, (unsigned long long)p);
    }
    __syncthreads();
    x += kCheckThreads;
  }
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = (s_best != ~0ull) ? (int64_t)s_best : (s_halo ? -2 : -1);
}

SB_DEV int32_t g_i32(const uint8_t *u, int64_t x) {
  return (int32_t)((uint32_t)u[x] | ((uint32_t)u[x + 1] << 8) | ((uint32_t)u[x + 2] << 16) | ((uint32_t)u[x + 3] << 24));
}

// Record chain per split (RecordStream._advance / PosStream): r_{j+1} = r_j + 4 + block_size while r_j < x_end.
// counts[i] = records, or -2 when the chain left a shard's loaded bytes (HALO), -3 on a truncated record.
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

// ================================================================================================
// launch wrappers
// ================================================================================================
static int check_grid(int64_t ntiles) { return (int)(ntiles < 1 ? 1 : ntiles > 2048 ? 2048 : ntiles); }

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
hipError_t launch_check_full_counts(StreamView sv, int64_t x0, int64_t x1, int32_t R, CountsDev cd,
                                    unsigned long long *bitmap, hipStream_t s) {
  if (x1 <= x0) return hipSuccess;
  const int64_t nt = (x1 - x0 + kTile - 1) / kTile;
  hipLaunchKernelGGL(k_check<MODE_COUNTS>, dim3(check_grid(nt)), dim3(kCheckThreads), 0, s, sv, x0, x1, R, cd, bitmap,
                     nullptr);
  return hipGetLastError();
}
hipError_t launch_check_eager(StreamView sv, int64_t x0, int64_t x1, int32_t R, unsigned long long *bitmap,
                              hipStream_t s) {
  if (x1 <= x0) return hipSuccess;
  const int64_t nt = (x1 - x0 + kTile - 1) / kTile;
  hipLaunchKernelGGL(k_check<MODE_EAGER>, dim3(check_grid(nt)), dim3(kCheckThreads), 0, s, sv, x0, x1, R, CountsDev{},
                     bitmap, nullptr);
  return hipGetLastError();
}
hipError_t launch_check_words(StreamView sv, int64_t x0, int64_t x1, int32_t R, uint32_t *words, hipStream_t s) {
  if (x1 <= x0) return hipSuccess;
  const int64_t nt = (x1 - x0 + kTile - 1) / kTile;
  hipLaunchKernelGGL(k_check<MODE_WORDS>, dim3(check_grid(nt)), dim3(kCheckThreads), 0, s, sv, x0, x1, R, CountsDev{},
                     nullptr, words);
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
