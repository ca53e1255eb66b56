// sbam_inflate.hip — batched raw-DEFLATE inflate of BGZF blocks for gfx950, in two kernels.
//
// Semantics: java.util.zip.Inflater(nowrap).inflate(decBuf, 0, ISIZE) on the block payload, as the reference
// calls it (bgzf/src/main/scala/org/hammerlab/bgzf/block/Stream.scala:31-71), i.e. zlib inflate():
//   * output stops at ISIZE (remaining input is ignored); ISIZE 0 returns 0 at once;
//   * the stream ending (final EOB, or input exhausted mid-symbol) before ISIZE bytes → "found" count (SHORT);
//   * invalid streams (bad block type, stored LEN/NLEN, over-subscribed / incomplete codes, missing EOB code,
//     bad repeat, invalid symbols, distance too far back) → DATA error; CRC32 is never checked.
//
// Design, two kernels with the block's "token words" (u32, below) in HBM between them:
//   k_inflate_wave    — one wavefront per BGZF block: 64 lanes decode 64 consecutive segments of the Huffman
//     stream speculatively and resynchronise (phases A/B), then write the words of the true path (phase C).
//     Blocks outside its common case go to k_inflate_slow, the exact per-lane decoder.
//   k_inflate_resolve — one wavefront per BGZF block: 64 words at a time are placed by a prefix sum and written
//     into an LDS ring holding the block's recent output; matches resolve in dependency rounds; the output leaves
//     in 16-B aligned 1 KiB groups.
#include <type_traits>

#include "sbam_internal.h"

namespace sbam {

#define SB_DEV __device__ __forceinline__

enum : int32_t { INF_OK = 0, INF_SHORT = 1, INF_DATA = 2, INF_OVERFLOW = 3 };

// ---- tokens ---------------------------------------------------------------------------------------------------
// u16 tokens, each self-describing so that the resolver can take 128 at once: t < 256 literal byte t;
// 256 <= t < 512 length t - 253, followed by its distance token 0x8000 | (distance - 1); kTokPad: padding.
constexpr uint32_t kTokPad = 0x7fffu;
constexpr uint32_t kTokDist = 0x8000u;

// Block b's main token region: the 16-B aligned region tok_region(uoff[b], b) of TokPool::main, 1 B per uncompressed
// byte (+ 32 B per block): room for (usize + 16) / 2 tokens (a token stands for >= 1 output byte, and the synthetic
// BAM needs 0.74 B per byte).  A block that needs more (up to ISIZE tokens plus 7 of padding) takes 2 ISIZE + 32 B
// of the arena (TokPool).
SB_DEV uint64_t tok_region(int64_t uoff, int64_t b) {
  return (((uint64_t)uoff + 15) & ~15ull) + 32ull * (uint64_t)b;
}
SB_DEV int32_t tok_region_cap(int32_t us) { return (us + 16) / 2; }  // tokens
SB_DEV uint64_t tok_arena_need(int32_t us) { return ((uint64_t)(2 * us + 32) + 15) & ~15ull; }

// ---- decode kernel --------------------------------------------------------------------------------------------
// Per-lane tables live in LDS, interleaved across the workgroup's lanes at dword granularity (byte b of lane L at
// ((b >> 2) * kDecThreads + L) * 4 + (b & 3)): lanes reading the same table offset never share a bank, and the
// 320-B slice lets two 256-lane workgroups — two waves per SIMD — share a CU's 160 KiB.  Everything else a lane
// needs (canonical code limits, the input window, the token chunk) is in VGPRs.
constexpr int kDecThreads = 256;
constexpr int kRows = 80;          // dwords per lane (320 B)
constexpr int kLitSorted = 0;      // bytes [0, 288): lit/len symbols in canonical order (low 8 bits)
constexpr int kClTab = 0;          //   header only: bytes [0, 128): code-length-code table (u8: len<<5 | sym)
constexpr int kLensLitRow = 32;    //   header only: rows 32..67: lit/len code lengths, 8 nibbles per row
constexpr int kLensDistRow = 68;   //   header only: rows 68..71: distance code lengths
constexpr int kDistSorted = 288;   // bytes [288, 320): distance symbols in canonical order
constexpr int kEpoch = 4;          // iterations between input-window slides and token-chunk stores
// A lane that reaches a block header parks; parked lanes build their tables together once kParkMin of the
// wave's 64 lanes wait (or none is left decoding): a table build is a serial loop of a few thousand
// instructions per lane, and builds started one lane at a time would cost the whole wave that much each.
constexpr int kParkMin = 16;

constexpr uint8_t kClOrder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

struct Slice {  // one lane's interleaved LDS slice
  uint8_t *base;
  SB_DEV uint8_t *b(int i) const { return base + (i >> 2) * (kDecThreads * 4) + (i & 3); }
  SB_DEV uint32_t *w(int row) const { return reinterpret_cast<uint32_t *>(base + row * (kDecThreads * 4)); }
};

// Compile-time loop: f(integral_constant<I>) for I in [B, E) — the index is a constant in the IR from the
// start, so the per-length arrays below stay in registers (SROA) instead of a scratch array.
template <int B, int E, class F>
SB_DEV void sfor(F &&f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    sfor<B + 1, E>(f);
  }
}

// Canonical code of one alphabet: lim[l] = left-justified (15-bit) end of the length-l codes; pk[l] =
// bse << 14 | hist << 5 | l, with bse = index (in canonical order) of the first length-l symbol minus its first
// code, and hist = index of the first length-l symbol >= 256 (symbols of one length are in increasing order,
// so the sorted table stores only their low 8 bits).  lim is non-decreasing in l, so the length of the code
// in the next 15 bits `rev` is 1 + #{l < 15 : rev >= lim[l]}: one select per length finds its pk.
struct Canon {
  uint32_t lim[16];
  int32_t pk[16];
};

// Decode the next symbol index: idx into the canonical symbol list (valid=false for an unassigned code, which
// zlib reports after consuming 1 bit — the only incomplete codes it accepts are single 1-bit codes).
SB_DEV int canon_decode(const Canon &c, uint64_t bb, int &len, bool &valid, int &hist) {
  const uint32_t rev = __builtin_bitreverse32((uint32_t)bb) >> 17;
  int32_t p = c.pk[1];
  sfor<1, 15>([&](auto I) {
    constexpr int l = decltype(I)::value;
    p = rev >= c.lim[l] ? c.pk[l + 1] : p;
  });
  const int L = p & 31;
  valid = rev < c.lim[15];
  len = valid ? L : 1;
  hist = (p >> 5) & 511;
  return valid ? (int)(rev >> (15 - L)) + (p >> 14) : 0;
}

// canon_decode over a per-lane choice of alphabet (b when useB): the second symbol slot of a step decodes a
// distance after a length and another literal/length after a literal, in one instruction stream.
SB_DEV int canon_decode_sel(const Canon &a, const Canon &b, bool useB, uint64_t bb, int &len, bool &valid,
                            int &hist) {
  const uint32_t rev = __builtin_bitreverse32((uint32_t)bb) >> 17;
  int32_t p = useB ? b.pk[1] : a.pk[1];
  sfor<1, 15>([&](auto I) {
    constexpr int l = decltype(I)::value;
    const uint32_t lim = useB ? b.lim[l] : a.lim[l];
    const int32_t pn = useB ? b.pk[l + 1] : a.pk[l + 1];
    p = rev >= lim ? pn : p;
  });
  const int L = p & 31;
  valid = rev < (useB ? b.lim[15] : a.lim[15]);
  len = valid ? L : 1;
  hist = (p >> 5) & 511;
  return valid ? (int)(rev >> (15 - L)) + (p >> 14) : 0;
}

// 15 counters of 9 bits (code lengths 1..15) in three u64: fields 0-6, 7-13, 14-15.
struct Cnt15 {
  uint64_t a = 0, b = 0, c = 0;
  SB_DEV void add(uint32_t l, uint64_t v) {
    const uint32_t w = (l >= 7) + (l >= 14);
    const uint64_t inc = v << (9 * (l - 7 * w));
    a += w == 0 ? inc : 0ull;
    b += w == 1 ? inc : 0ull;
    c += w == 2 ? inc : 0ull;
  }
  SB_DEV uint32_t get(uint32_t l) const {
    const uint32_t w = (l >= 7) + (l >= 14);
    const uint64_t x = w == 0 ? a : w == 1 ? b : c;
    return (uint32_t)(x >> (9 * (l - 7 * w))) & 511u;
  }
};

// Build the canonical structures of NW dwords of code-length nibbles (symbol s = nibble s) into the sorted
// table at sorted_off.  Returns 0, or -1 for an over-subscribed set or an incomplete one other than a single
// 1-bit code (zlib inflate_table).  A set with no codes at all is accepted (only possible for distances).
template <int NW>
SB_DEV int canon_build(const uint32_t (&lens)[NW], const Slice &sl, int sorted_off, bool lit, Canon &c) {
  Cnt15 cnt, lo;
#pragma unroll
  for (int dw = 0; dw < NW; dw++) {
    const uint32_t w = lens[dw];
#pragma unroll 1
    for (int j = 0; j < 8; j++) {
      const uint32_t v = (w >> (4 * j)) & 15u;
      if (v) {
        cnt.add(v, 1);
        if (lit && dw * 8 + j < 256) lo.add(v, 1);
      }
    }
  }
  int left = 1, maxl = 0;
  bool over = false;
  uint32_t code = 0;
  int32_t offs = 0;
  Cnt15 cur;
  sfor<1, 16>([&](auto I) {
    constexpr int l = decltype(I)::value;
    const uint32_t k = cnt.get(l);
    left = 2 * left - (int)k;
    over |= left < 0;
    maxl = k ? l : maxl;
    c.lim[l] = (code + k) << (15 - l);
    const int32_t bse = offs - (int32_t)code;
    const uint32_t hist = (uint32_t)offs + (lit ? lo.get(l) : 0u);
    c.pk[l] = (int32_t)(((uint32_t)bse << 14) | (hist << 5) | (uint32_t)l);
    cur.add(l, (uint64_t)offs);  // fill cursor
    offs += (int32_t)k;
    code = (code + k) << 1;
  });
  c.lim[0] = 0;
  c.pk[0] = 0;
  if (over || (left > 0 && maxl > 1)) return -1;
#pragma unroll
  for (int dw = 0; dw < NW; dw++) {
    const uint32_t w = lens[dw];
#pragma unroll 1
    for (int j = 0; j < 8; j++) {
      const uint32_t v = (w >> (4 * j)) & 15u;
      if (v) {
        const uint32_t pos = cur.get(v);
        cur.add(v, 1);
        *sl.b(sorted_off + (int)pos) = (uint8_t)(dw * 8 + j);
      }
    }
  }
  return 0;
}

// A[i] for a lane-dependent i < 16: a 4-level tree of v_cndmask over registers, 4 compares + 15 selects.  The
// selects are opaque asm: as plain selects the tree is recognised as an indexed load and moved to scratch memory.
SB_DEV uint32_t csel(uint64_t m, uint32_t a, uint32_t b) {  // lane bit of m set ? b : a
  uint32_t r;
  asm("v_cndmask_b32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "s"(m));
  return r;
}
SB_DEV uint32_t sel16(const uint32_t (&A)[16], uint32_t i) {
  const uint64_t m0 = __builtin_amdgcn_ballot_w64((i & 1u) != 0), m1 = __builtin_amdgcn_ballot_w64((i & 2u) != 0),
                 m2 = __builtin_amdgcn_ballot_w64((i & 4u) != 0), m3 = __builtin_amdgcn_ballot_w64((i & 8u) != 0);
  uint32_t t[8], u[4];
#pragma unroll
  for (int k = 0; k < 8; k++) t[k] = csel(m0, A[2 * k], A[2 * k + 1]);
#pragma unroll
  for (int k = 0; k < 4; k++) u[k] = csel(m1, t[2 * k], t[2 * k + 1]);
  return csel(m3, csel(m2, u[0], u[1]), csel(m2, u[2], u[3]));
}

// Token output: an 8-slot shift register (t0 low half = oldest); a full chunk moves to the pending chunk p,
// which leaves as one 16-B store at the next epoch (so stores issue together with the epoch's loads).
struct TokOut {
  uint32_t t0, t1, t2, t3;
  uint32_t p0, p1, p2, p3;
  int n;
  bool pend;
  uint64_t cur;  // byte offset of the next chunk in the pool
};

// Store one chunk into the block's token region (tok_region: room for every token the block can produce).
SB_DEV bool tok_store(TokOut &to, uint32_t a, uint32_t b, uint32_t c, uint32_t d, uint8_t *pool) {
  *reinterpret_cast<uint4 *>(pool + to.cur) = make_uint4(a, b, c, d);
  to.cur += 16;
  return true;
}

// Append one token; a completed chunk becomes pending (an older pending chunk is stored first: only at a
// block's end or when more than 8 tokens arrive within one epoch).
SB_DEV bool tok_put(TokOut &to, uint32_t t, uint8_t *pool) {
  to.t0 = __builtin_amdgcn_alignbit(to.t1, to.t0, 16);
  to.t1 = __builtin_amdgcn_alignbit(to.t2, to.t1, 16);
  to.t2 = __builtin_amdgcn_alignbit(to.t3, to.t2, 16);
  to.t3 = __builtin_amdgcn_alignbit(t, to.t3, 16);
  if (++to.n < 8) return true;
  bool ok = true;
  if (to.pend) ok = tok_store(to, to.p0, to.p1, to.p2, to.p3, pool);
  to.p0 = to.t0;
  to.p1 = to.t1;
  to.p2 = to.t2;
  to.p3 = to.t3;
  to.pend = true;
  to.n = 0;
  return ok;
}

enum : int { S_NEXT = 0, S_HDR = 1, S_HUFF = 2, S_STORED = 3, S_DONE = 4, S_EXIT = 5, S_PARK = 6 };


// Bit reader.  bb holds bc valid bits (LSB first); rp = block-relative index of the next payload dword to enter
// bb; left = payload bits not yet consumed (negative ⇒ the symbol needed bits past the payload: zlib returns
// for more input → SHORT).  While decoding symbols the dwords come from the lane's register window A (nx =
// A[rp - ws], selected ahead); while parsing a block header they come straight from HBM.
struct Bits {
  uint64_t bb;
  int bc;
  int left;
  uint32_t rp, nx;
  SB_DEV uint32_t peek(int n) const { return (uint32_t)bb & ((1u << n) - 1u); }
  SB_DEV void drop(int n) {
    bb >>= n;
    bc -= n;
    left -= n;
  }
  SB_DEV void refill_hbm(const uint32_t *src) {
    if (bc <= 32) {
      bb |= (uint64_t)src[rp] << bc;
      bc += 32;
      rp++;
    }
  }
};

__global__ __launch_bounds__(kDecThreads, 2) void k_inflate_slow(const uint8_t *__restrict__ d, int64_t D,
                                                                 BlockTable bt, TokPool tp,
                                                                 const int32_t *__restrict__ slow,
                                                                 const unsigned int *nslow,
                                                                 int32_t *__restrict__ status,
                                                                 int32_t *__restrict__ found,
                                                                 unsigned int *next_block) {
  __shared__ __attribute__((aligned(16))) uint8_t s_dec[kRows * kDecThreads * 4];
  const Slice sl{s_dec + 4 * threadIdx.x};
  const uint32_t *d32 = reinterpret_cast<const uint32_t *>(d);
  uint8_t *pool = tp.arena;  // every block of this decoder writes into an arena region of its own

  int state = S_NEXT;
  int64_t blk = -1;
  const uint32_t *src = d32;  // the block's payload, from its first (4-B aligned) dword
  uint32_t ldw = 0;           // payload dwords worth loading (payload + footer)
  Bits br{0, 0, 0, 0, 0};
  // input window: A = payload dwords [ws, ws + 16), B = the next 8 (loaded one slide ahead); the window slides
  // by 8 dwords at an epoch, so the compiler's wait for B always falls on a load issued epochs earlier
  uint32_t A[16], B[8];
  uint32_t ws = 0;
#pragma unroll
  for (int k = 0; k < 16; k++) A[k] = 0;
#pragma unroll
  for (int k = 0; k < 8; k++) B[k] = 0;
  TokOut to{0, 0, 0, 0, 0, 0, 0, 0, 0, false, 0};
  Canon lc, dc;
  int32_t o = 0, us = 0, err = INF_OK, sleft = 0, fin = 0;
  auto refill = [&]() {  // the symbol loop's refill: next dword from the register window
    if (br.bc <= 32) {
      br.bb |= (uint64_t)br.nx << br.bc;
      br.bc += 32;
      br.rp++;
      br.nx = sel16(A, br.rp - ws);
    }
  };

  for (int it = 0;; it++) {
    if (state == S_NEXT) {
      const uint32_t i = atomicAdd(next_block, 1u);
      if (i >= *nslow) {
        state = S_EXIT;
      } else {
        blk = slow[i];
        const int64_t st = bt.start[blk];
        const int32_t hs = bt.hsize[blk], cs = bt.csize[blk];
        us = bt.usize[blk];
        o = 0;
        fin = 0;
        err = INF_OK;
        const int32_t dlen = cs - hs - 8;  // Stream.scala: dataLength = compressedSize - headerSize - FOOTER_SIZE
        if (us == 0) {
          state = S_DONE;  // inflate(buf, 0, 0) returns 0
        } else if (us < 0 || us > 65536 || dlen < 0 || st + hs + dlen > D) {
          err = INF_DATA;
          state = S_DONE;
        } else {
          const uint64_t need = tok_arena_need(us);
          const uint64_t at = atomicAdd(tp.arena_used, (unsigned long long)need);
          if ((int64_t)(at + need) > tp.arena_cap) {
            err = INF_OVERFLOW;  // the host grows the arena and inflates again
            state = S_DONE;
          } else {
            tp.base[blk] = (int64_t)at;
            to.cur = at;
            to.n = 0;
            to.pend = false;
            // word pointer derived from d by arithmetic only (an integer round trip would make it a flat
            // pointer, whose loads the compiler must wait for together with every LDS access)
            const int64_t a = st + hs;
            src = d32 + (a >> 2);
            ldw = (uint32_t)(((a & 3) + dlen + 8 + 3) >> 2);
            const int skip = (int)(a & 3) * 8;
            br.bb = (uint64_t)src[0] >> skip;
            br.bc = 32 - skip;
            br.rp = 1;
            br.left = 8 * dlen;
            state = S_PARK;
          }
        }
      }
    }
    // wave-level decisions at epoch steps only (a parked or exited lane idles at most kEpoch - 1 steps)
    if ((it & (kEpoch - 1)) == 0) {
      if (__all(state == S_EXIT)) break;
      // release parked lanes together (see kParkMin)
      const uint64_t pk = __ballot(state == S_PARK);
      const uint64_t dc = __ballot(state == S_HUFF || state == S_STORED);
      if (pk && (__popcll(pk) >= kParkMin || dc == 0) && state == S_PARK) state = S_HDR;
    }

    // --- epoch (wave-uniform): slide the input window, store the pending token chunk, issue the next loads
    if ((it & (kEpoch - 1)) == 0) {
      const bool dec = state == S_HUFF || state == S_STORED;
      if (dec && br.rp - ws >= 8) {
#pragma unroll
        for (int k = 0; k < 8; k++) A[k] = A[k + 8];
#pragma unroll
        for (int k = 0; k < 8; k++) A[k + 8] = B[k];
        ws += 8;
        if (ws + 16 < ldw) {
          const uint4 *g = reinterpret_cast<const uint4 *>(src + ws + 16);
          const uint4 x0 = g[0], x1 = g[1];
          B[0] = x0.x; B[1] = x0.y; B[2] = x0.z; B[3] = x0.w;
          B[4] = x1.x; B[5] = x1.y; B[6] = x1.z; B[7] = x1.w;
        }
      }
      if (to.pend && (dec || state == S_PARK || state == S_HDR)) {
        tok_store(to, to.p0, to.p1, to.p2, to.p3, pool);
        to.pend = false;
      }
    }
    if (state == S_HDR) {
      // --- block header (RFC 1951 §3.2.3); every read checks that the payload holds the bits (else SHORT)
      br.refill_hbm(src);
      if (br.left < 3) {
        err = INF_SHORT;
        state = S_DONE;
      } else {
        fin = (int)br.peek(1);
        const int type = (int)((br.bb >> 1) & 3);
        br.drop(3);
        if (type == 0) {  // stored: skip to a byte boundary, LEN, NLEN
          br.drop(br.left & 7);
          br.refill_hbm(src);
          if (br.left < 32) {
            err = INF_SHORT;
            state = S_DONE;
          } else {
            const uint32_t ln = br.peek(16), nl = (uint32_t)(br.bb >> 16) & 0xffffu;
            br.drop(32);
            if (ln != (~nl & 0xffffu)) {
              err = INF_DATA;
              state = S_DONE;
            } else {
              sleft = (int)ln;
              state = S_STORED;
            }
          }
        } else if (type == 1) {  // fixed codes: lit 0-143:8, 144-255:9, 256-279:7, 280-287:8; dist 0-31:5
          uint32_t llit[36], ldist[4];
#pragma unroll
          for (int i = 0; i < 36; i++)
            llit[i] = i < 18 ? 0x88888888u : i < 32 ? 0x99999999u : i < 35 ? 0x77777777u : 0x88888888u;
#pragma unroll
          for (int i = 0; i < 4; i++) ldist[i] = 0x55555555u;
          canon_build<4>(ldist, sl, kDistSorted, false, dc);
          canon_build<36>(llit, sl, kLitSorted, true, lc);
          state = S_HUFF;
        } else if (type == 2) {  // dynamic codes
          br.refill_hbm(src);
          if (br.left < 14) {
            err = INF_SHORT;
            state = S_DONE;
          } else {
            const int hlit = (int)br.peek(5) + 257, hdist = (int)((br.bb >> 5) & 31) + 1,
                      hclen = (int)((br.bb >> 10) & 15) + 4;
            br.drop(14);
            int ok = 1;  // 1 ok, 0 data error, -1 short
            if (hlit > 286 || hdist > 30) ok = 0;
            // code-length code lengths, 3 bits each in kClOrder order → packed 3-bit fields by symbol
            uint64_t clp = 0;
            if (ok == 1) {
              br.refill_hbm(src);
              if (br.left < 3 * hclen) ok = -1;
              else {
#pragma unroll
                for (int i = 0; i < 19; i++) {
                  if (i == 10) br.refill_hbm(src);
                  if (i < hclen) {
                    clp |= (uint64_t)br.peek(3) << (3 * kClOrder[i]);
                    br.drop(3);
                  }
                }
              }
            }
            if (ok == 1) {
              // counts per length (8-bit fields), Kraft check: the code-length code must be complete
              uint64_t cnt = 0;
#pragma unroll
              for (int s = 0; s < 19; s++) cnt += 1ull << (8 * ((clp >> (3 * s)) & 7));
              int left = 1, maxl = 0;
              uint64_t next = 0;  // next code per length, 8-bit fields
              uint32_t code = 0;
#pragma unroll
              for (int l = 1; l <= 7; l++) {
                const int k = (int)((cnt >> (8 * l)) & 0xff);
                left = 2 * left - k;
                if (k) maxl = l;
                next |= (uint64_t)code << (8 * l);
                code = (code + (uint32_t)k) << 1;
                if (left < 0) ok = 0;
              }
              if (maxl == 0) {
                // zlib decodes every code length as 0 (1 bit each), then fails on the missing EOB code
                br.left -= hlit + hdist;
                ok = br.left < 0 ? -1 : 0;
              } else if (left > 0) {
                ok = 0;
              }
              if (ok == 1) {  // fill the 128-entry table: entries brev(code) + k·2^l
                for (int s = 0; s < 19; s++) {
                  const int l = (int)((clp >> (3 * s)) & 7);
                  if (l) {
                    const uint32_t cv = (uint32_t)((next >> (8 * l)) & 0xff);
                    next += 1ull << (8 * l);
                    const uint32_t r = __builtin_bitreverse32(cv) >> (32 - l);
                    for (uint32_t j = r; j < 128; j += 1u << l) *sl.b(kClTab + (int)j) = (uint8_t)((l << 5) | s);
                  }
                }
                // code lengths of hlit + hdist symbols (repeats may cross from the lit/len to the distance
                // lengths), one nibble each: lit/len in rows kLensLitRow.., distance in rows kLensDistRow..
#pragma unroll
                for (int r = kLensLitRow; r < kLensDistRow + 4; r++) *sl.w(r) = 0;
                const int total = hlit + hdist;
                int n = 0;
                uint32_t prev = 0, acc = 0;
                while (n < total) {
                  br.refill_hbm(src);
                  const uint32_t e = *sl.b(kClTab + (int)br.peek(7));
                  const int l = (int)(e >> 5);
                  const uint32_t sym = e & 31;
                  if (br.left < l) { ok = -1; break; }
                  br.drop(l);
                  int rep = 1;
                  uint32_t v = sym;
                  if (sym == 16) {
                    if (br.left < 2) { ok = -1; break; }
                    if (n == 0) { ok = 0; break; }
                    rep = 3 + (int)br.peek(2);
                    br.drop(2);
                    v = prev;
                  } else if (sym == 17) {
                    if (br.left < 3) { ok = -1; break; }
                    rep = 3 + (int)br.peek(3);
                    br.drop(3);
                    v = 0;
                  } else if (sym == 18) {
                    if (br.left < 7) { ok = -1; break; }
                    rep = 11 + (int)br.peek(7);
                    br.drop(7);
                    v = 0;
                  }
                  if (n + rep > total) { ok = 0; break; }
                  const uint32_t pat = v * 0x11111111u;
                  while (rep > 0) {  // up to the end of the current dword (or of the lit/len lengths) per step
                    const bool inlit = n < hlit;
                    const int i = inlit ? n : n - hlit, end = inlit ? hlit : total;
                    const int o8 = i & 7, k = min(rep, min(8 - o8, end - n));
                    const uint32_t m = (k == 8 ? 0xffffffffu : ((1u << (4 * k)) - 1u)) << (4 * o8);
                    acc |= pat & m;
                    n += k;
                    rep -= k;
                    if (((i + k) & 7) == 0 || n == end) {
                      *sl.w((inlit ? kLensLitRow : kLensDistRow) + (i >> 3)) = acc;
                      acc = 0;
                    }
                  }
                  prev = v;
                }
                if (ok == 1) {
                  uint32_t llit[36], ldist[4];
#pragma unroll
                  for (int i = 0; i < 36; i++) llit[i] = *sl.w(kLensLitRow + i);
#pragma unroll
                  for (int i = 0; i < 4; i++) ldist[i] = *sl.w(kLensDistRow + i);
                  if ((llit[32] & 15u) == 0) ok = 0;  // invalid code -- missing end-of-block
                  // distance table first (its rows do not overlap the lengths); the lit/len table then
                  // overwrites the lengths, which are in registers by now
                  if (ok == 1 && canon_build<4>(ldist, sl, kDistSorted, false, dc) != 0) ok = 0;
                  if (ok == 1 && canon_build<36>(llit, sl, kLitSorted, true, lc) != 0) ok = 0;
                }
              }
            }
            if (ok == 1) state = S_HUFF;
            else {
              err = ok == 0 ? INF_DATA : INF_SHORT;
              state = S_DONE;
            }
          }
        }
        if (state == S_HDR) {  // type 3
          err = INF_DATA;  // invalid block type
          state = S_DONE;
        }
      }
      if (state == S_HUFF || state == S_STORED) {
        // load the input window from HBM at the reader's position (one wait per header round)
        ws = br.rp;
        const uint4 *g = reinterpret_cast<const uint4 *>(src + ws);
        const uint4 x0 = g[0], x1 = g[1], x2 = g[2], x3 = g[3], y0 = g[4], y1 = g[5];
        A[0] = x0.x; A[1] = x0.y; A[2] = x0.z; A[3] = x0.w;
        A[4] = x1.x; A[5] = x1.y; A[6] = x1.z; A[7] = x1.w;
        A[8] = x2.x; A[9] = x2.y; A[10] = x2.z; A[11] = x2.w;
        A[12] = x3.x; A[13] = x3.y; A[14] = x3.z; A[15] = x3.w;
        B[0] = y0.x; B[1] = y0.y; B[2] = y0.z; B[3] = y0.w;
        B[4] = y1.x; B[5] = y1.y; B[6] = y1.z; B[7] = y1.w;
        br.nx = A[0];
      }
    } else if (state == S_HUFF) {
      // --- one literal/length symbol (+ its distance) per step
      refill();
      int L1, h1;
      bool v1;
      const int i1 = canon_decode(lc, br.bb, L1, v1, h1);
      const int sym = (int)*sl.b(kLitSorted + i1) | (i1 >= h1 ? 256 : 0);
      if (br.left < L1) {
        err = INF_SHORT;
        state = S_DONE;
      } else if (!v1 || sym > 285) {
        err = INF_DATA;  // invalid literal/length code
        state = S_DONE;
      } else {
        br.drop(L1);
        int len = 0;
        bool is_len = false;
        if (sym < 256) {
          if (!tok_put(to, (uint32_t)sym, pool)) err = INF_OVERFLOW;
          o++;
          if (o == us || err != INF_OK) state = S_DONE;
        } else if (sym == 256) {
          if (fin) {
            err = INF_SHORT;  // stream end before ISIZE bytes
            state = S_DONE;
          } else {
            state = S_PARK;
          }
        } else {
          const int k = sym - 257;
          const int lx = (k < 8 || k == 28) ? 0 : (k >> 2) - 1;
          const int lb = k < 8 ? k + 3 : k == 28 ? 258 : ((4 | (k & 3)) << lx) + 3;
          if (br.left < lx) {
            err = INF_SHORT;
            state = S_DONE;
          } else {
            len = lb + (int)br.peek(lx);
            br.drop(lx);
            is_len = true;
          }
        }
        // second slot: the distance after a length, or a second literal after a literal (taken only when it
        // is a complete, valid literal; anything else is left for the next step, which decodes it afresh)
        if (is_len || (sym < 256 && state == S_HUFF)) {
          refill();
          int L2, h2;
          bool v2;
          const int i2 = canon_decode_sel(lc, dc, is_len, br.bb, L2, v2, h2);
          const int b2 = *sl.b((is_len ? kDistSorted : kLitSorted) + i2);
          if (!is_len) {
            if (v2 && i2 < h2 && br.left >= L2) {
              br.drop(L2);
              if (!tok_put(to, (uint32_t)b2, pool)) err = INF_OVERFLOW;
              o++;
              if (o == us || err != INF_OK) state = S_DONE;
            }
          } else {
            const int ds = b2;
            if (br.left < L2) {
              err = INF_SHORT;
              state = S_DONE;
            } else if (!v2 || ds > 29) {
              err = INF_DATA;  // invalid distance code
              state = S_DONE;
            } else {
              br.drop(L2);
              const int dx = ds < 4 ? 0 : (ds >> 1) - 1;
              const int db = ds < 4 ? ds + 1 : ((2 | (ds & 1)) << dx) + 1;
              if (br.left < dx) {
                err = INF_SHORT;
                state = S_DONE;
              } else {
                const int dist = db + (int)br.peek(dx);
                br.drop(dx);
                if (dist > o) {
                  err = INF_DATA;  // invalid distance too far back
                  state = S_DONE;
                } else {
                  bool ok = true;
                  ok = ok && tok_put(to, (uint32_t)(len + 253), pool);
                  ok = ok && tok_put(to, kTokDist | (uint32_t)(dist - 1), pool);
                  if (!ok) err = INF_OVERFLOW;
                  o = min(o + len, us);
                  if (o == us || err != INF_OK) state = S_DONE;
                }
              }
            }
          }
        }
      }
    } else if (state == S_STORED) {
      // --- up to 2 stored bytes per step (byte-aligned: bb's low bits are the next byte)
      refill();
      const int n = min(min(sleft, 2), us - o);
      int m = 0;
      for (int i = 0; i < 2; i++) {
        if (i < n && br.left >= 8 && err == INF_OK) {
          if (!tok_put(to, br.peek(8), pool)) err = INF_OVERFLOW;
          br.drop(8);
          m++;
        }
      }
      o += m;
      sleft -= m;
      if (err != INF_OK) state = S_DONE;
      else if (m < n) {
        err = INF_SHORT;
        state = S_DONE;
      } else if (o == us) {
        state = S_DONE;
      } else if (sleft == 0) {
        if (fin) {
          err = INF_SHORT;
          state = S_DONE;
        } else {
          state = S_PARK;
        }
      }
    }
    if (state == S_DONE) {
      if (err != INF_OVERFLOW) {  // final (padded) chunk and any pending one leave now
        bool ok = true;
        if (to.n > 0)
          while (ok && to.n > 0) ok = tok_put(to, kTokPad, pool);
        if (ok && to.pend) ok = tok_store(to, to.p0, to.p1, to.p2, to.p3, pool);
        if (!ok) err = INF_OVERFLOW;
      }
      to.n = 0;
      to.pend = false;
      status[blk] = err;
      found[blk] = err == INF_OVERFLOW ? 0 : o;  // an overflowed block has no complete token stream
      state = S_NEXT;
    }
  }
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4a __attribute__((ext_vector_type(4), aligned(4)));  // 16-B store at a 4-B aligned address

// ---- wave decoder (fast path) -------------------------------------------------------------------------------
// One wavefront per BGZF block.  Huffman decoding is serial per stream, so the 64 lanes decode 64 consecutive
// kK-bit segments of a deflate block's data at once, each from a guessed start (its segment's first bit, in the
// literal/length state).  Huffman codes resynchronise within a few symbols: a lane whose true start (where its
// left neighbour's decode leaves that neighbour's segment) differs re-decodes from there (phase B) only until
// its path reaches one of the checkpoints its first pass (phase A) recorded every kCpSteps symbols, after which the
// first pass's counts hold.  Token and byte counts give every lane its output offset (wave prefix sums), and a
// second pass over the true segments (phase C) writes the tokens.  A first pass does not stop at an
// end-of-block or invalid symbol (in the speculative prefix such a symbol is noise): it records up to two such
// stops and keeps decoding, and phase B decides which, if any, lies on the true path.
// Block headers are decoded by the whole wave as well: every lane decodes the code-length symbol at one of 64
// consecutive bit offsets, and the true chain of symbols is followed through those 64 results.  Tables (32-bit
// entries: a 9-bit root table plus sub-tables for longer codes; 8 bits for distances) are built by the whole
// wave in LDS.  Anything outside the common case — stored or invalid blocks, incomplete codes, a stream that
// ends before ISIZE or runs past it, a distance too far back — sends the block to k_inflate_slow (the exact
// per-lane decoder), so zlib's semantics are unchanged.
namespace wd {
// 544 bits = 17 dwords: lane k's window reads start at dword 17 k + drift, so the 32 lanes of a ds_read group land
// in distinct banks (at 512 = 16 dwords, lanes k and k + 2 shared a bank: 20.9 G conflict cycles per launch at
// 10 GB, 7.0 G at 544; decode 67.0 → 63.8 ms).  An XOR-swizzled root-table index changed nothing (62.3 vs 62.6 G
// over three launches): the conflicts were the window reads'.
constexpr int kK = 544;                    // bits per lane segment
constexpr int kWinDw = 64 * kK / 32 + 16;  // staged input dwords per round (start alignment + lookahead)
// 9-bit roots for both alphabets (zlib's ENOUGH bounds: 852 literal/length and 592 distance entries with
// sub-tables), interleaved: the root entry of 9-bit prefix b in state st (0: literal/length, 1: distance after a
// length) is tab[2 b + st], so one symbol's lookup address is (bits & 511) << 3 | st << 2 with no state-dependent
// root width or table base; the sub-tables follow at kLitSubOff / kDistSubOff.  The wave's LDS is 10.0 KiB (the
// table-build counters live in the window's scratch tail), so 16 decoder waves still fit a CU (a 10-bit literal
// root: 11.4 KiB, 14 waves, decode 86 → 79 ms at 10 GB in round 2).
constexpr int kLitRoot = 9, kDistRoot = 9;
constexpr int kLitSub = 340, kDistSub = 80;  // ENOUGH - root: 852 - 512 and 592 - 512 at root 9
constexpr int kLitSubOff = 2 << kLitRoot, kDistSubOff = kLitSubOff + kLitSub;
constexpr int kTab = kDistSubOff + kDistSub;
constexpr int kCp = 12;                     // checkpoints per lane (8 × 12 and 16 × 6 symbols: within 0.2 ms of 12 × 8)
constexpr int kCpSteps = 96 / kCp;          // symbols between checkpoints
// Lanes > 0 start decoding kWarm bits before their segment, so that by the segment start their path has usually
// resynchronised with the true one: the first symbol boundary at or after the segment start ("entry") then equals
// the left neighbour's exit and phase A's counts from the entry on need no phase-B re-decode.  Decode at 10 GB:
// no warm-up 79.5 ms; 128 bits 74.8; 256: 71.6; 384: 69.6; 512 (one segment; lane 1 from the round's true start):
// 68.5; 640: 70.1; 1024: 76.7.  Round 3 (544-bit segments, register tokens, re-decode only to the rejoin point):
// 192: 70.5; 288: 65.7; 384: 59.9; 544: 51.1; 640: 49.6; 768: 49.8; 960: 52.2.
constexpr int kWarm = 640;
// Phase A keeps the tokens of its first kTR symbol steps in registers (two per VGPR, step j in half j & 1 of
// tr[j / 2]: the steps are unrolled, so every index is static).  A lane whose phase-A path is the true one (the
// common case after the warm-up) then only stores them in phase C; it decodes again only past step kTR.  With the
// round-3 v2 step (38 VALU instead of 58) the register budget is what limits kTR: 96 tokens spilled 48 VGPRs to
// scratch, 80 spill 11 (decode at 10 GB: 96 → 47.7 ms, 80 → 45.9; 72: 47.5, its phase C re-decodes more tails).
// (Round 4, measured and dropped, DESIGN.md §Inflate: the register tokens stored through LDS as whole 16-B chunks,
// 55.0 ms; the next window prefetched into registers during phase C or the table build, 44.3 ms; the register tokens
// pinned before phase C's re-decode instead of after it.)
constexpr int kTR = 80;
constexpr int kFirstFrac = 930;  // per mille: a non-final DEFLATE block's rounds are sized to this much of the rest
static_assert(kTR % 2 == 0 && kTR <= kCp * kCpSteps, "register tokens come from the unrolled checkpoint steps");
static_assert(kTR % kCpSteps == 0, "the state after step kTR (stR) is saved at a checkpoint");
constexpr int kScratchDw = 256;    // window tail that doubles as header / table-build scratch
// a block header (<= 3 + 14 + 57 + 320 * 14 bits) plus the window's start alignment fits before the scratch
static_assert(128 + 3 + 14 + 57 + 320 * 14 + 64 <= (kWinDw - kScratchDw) * 32, "header fits the window");
enum : uint32_t { K_LIT = 0, K_LEN = 1, K_DIST = 2, K_SPEC = 3, K_SUBP = 4 };  // K_SUBP: a sub-table pointer
enum : int { ST_NONE = 0, ST_EOB = 1, ST_ERR = 2, ST_OUT = 3 };
}  // namespace wd

// Table entry (u32): bits 0-3 code length, 4-7 extra bits, byte 1 the kind (alone in its byte, so a kind test is one
// byte-select compare), 16-31 value in token form, so that value + extra bits is the symbol's u16 token (literal
// byte; 253 + length base; 0x7fff + distance base; K_SPEC: 0 = end of block, 1 = invalid symbol).  A sub-table
// pointer (kind K_SUBP): bits 0-4 the sub-table's index bits (a bit-field width as it stands), 16-31 the sub-table's
// byte offset in tab.
struct WaveLds {
  uint32_t win[wd::kWinDw];
  uint32_t tab[wd::kTab];
  SB_DEV uint8_t *lens() { return reinterpret_cast<uint8_t *>(win + wd::kWinDw - wd::kScratchDw); }  // [320]
  SB_DEV uint16_t *sorted() { return reinterpret_cast<uint16_t *>(win + wd::kWinDw - wd::kScratchDw + 80); }  // [320]
  SB_DEV uint32_t *cnt() { return win + wd::kWinDw - 16; }  // [16], the scratch's last dwords
};


SB_DEV uint32_t sym_entry(uint32_t s, uint32_t l, bool dist) {
  using namespace wd;
  if (!dist) {
    if (s < 256) return l | (K_LIT << 8) | (s << 16);
    if (s == 256) return l | (K_SPEC << 8);
    if (s <= 285) {
      const uint32_t k = s - 257;
      const uint32_t x = (k < 8 || k == 28) ? 0u : (k >> 2) - 1;
      const uint32_t base = k < 8 ? k + 3 : k == 28 ? 258u : ((4u | (k & 3)) << x) + 3;
      return l | (x << 4) | (K_LEN << 8) | ((base + 253u) << 16);  // token form: 253 + length
    }
    return l | (K_SPEC << 8) | (1u << 16);
  }
  if (s < 30) {
    const uint32_t x = s < 4 ? 0u : (s >> 1) - 1;
    const uint32_t base = s < 4 ? s + 1 : ((2u | (s & 1)) << x) + 1;
    return l | (x << 4) | (K_DIST << 8) | ((base + 0x7fffu) << 16);  // token form: kTokDist | (distance - 1)
  }
  return l | (K_SPEC << 8) | (1u << 16);
}

// Canonical code of one alphabet, wave-uniform: lim[l] = left-justified (15-bit) end of the length-l codes,
// base[l] = canonical index of the first length-l code minus that code.
struct CanonW {
  uint32_t lim[16];
  int32_t base[16];
};
// code length of the 15-bit left-justified code v, known to be at most MAXL (root entries: the root bits)
template <int MAXL = 15>
SB_DEV uint32_t canon_len(const CanonW &c, uint32_t v) {
  uint32_t l = 1;
  sfor<1, MAXL>([&](auto I) { l += v >= c.lim[decltype(I)::value] ? 1u : 0u; });
  return l;
}
template <int MAXL = 15>
SB_DEV int32_t canon_base(const CanonW &c, uint32_t l) {  // c.base[l] by selects (a runtime index would
  int32_t r = 0;                                            // move the whole struct to scratch memory)
  sfor<1, MAXL + 1>([&](auto I) { r = l == (uint32_t)decltype(I)::value ? c.base[decltype(I)::value] : r; });
  return r;
}

// Wave-uniform values pinned to scalar registers, so the compiler emits uniform (scalar) control flow instead of
// exec-mask bookkeeping for branches that never diverge.
SB_DEV uint32_t uni(uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); }
SB_DEV int uni(int x) { return __builtin_amdgcn_readfirstlane(x); }
SB_DEV uint64_t uni(uint64_t x) { return ((uint64_t)uni((uint32_t)(x >> 32)) << 32) | uni((uint32_t)x); }
// Inclusive prefix sum over the wave: row_shr 1/2/4/8 within rows of 16, then row_bcast 15 / 31 across rows
// (DPP: no LDS round trip).
SB_DEV uint32_t wave_incl_scan(uint32_t x) {
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);
  return x;
}

// Decode table of one alphabet from lens[off, off + nsym), by the whole wave: root entries at tab[2 b + DIST],
// sub-tables from tab[suboff].  Returns false (wave-uniform) for a code set that is not complete (zlib rejects
// over-subscribed ones and most incomplete ones; the slow decoder handles every such block exactly) or whose
// sub-tables would not fit.
template <bool DIST>
SB_DEV bool wave_build(WaveLds &L, int off, int nsym, int suboff, int subcap) {
  constexpr int R = DIST ? wd::kDistRoot : wd::kLitRoot;
  const int lane = (int)threadIdx.x;
  uint8_t *lens = L.lens();
  uint16_t *sorted = L.sorted();
  uint32_t *cnt = L.cnt();
  if (lane < 16) cnt[lane] = 0;
  __syncthreads();
  for (int s = lane; s < nsym; s += 64) {
    const uint32_t l = lens[off + s];
    if (l) atomicAdd(&cnt[l], 1u);
  }
  __syncthreads();
  CanonW c;
  int32_t offs[16];
  int left = 1, acc = 0;
  bool over = false;
  uint32_t code = 0;
  sfor<1, 16>([&](auto I) {
    constexpr int l = decltype(I)::value;
    const uint32_t k = uni(cnt[l]);
    left = 2 * left - (int)k;
    over |= left < 0;
    c.lim[l] = (code + k) << (15 - l);
    c.base[l] = acc - (int32_t)code;
    offs[l] = acc;
    acc += (int32_t)k;
    code = (code + k) << 1;
  });
  c.lim[0] = 0;
  c.base[0] = 0;
  if (over || left != 0) return false;
  // sorted[canonical index] = symbol: a symbol's rank among the equal-length symbols below it, 64 at a time
  int32_t run[16];
  sfor<1, 16>([&](auto I) { run[decltype(I)::value] = 0; });
  for (int c0 = 0; c0 < nsym; c0 += 64) {
    const int s = c0 + lane;
    const uint32_t l = s < nsym ? lens[off + s] : 0u;
    sfor<1, 16>([&](auto I) {
      constexpr int ll = decltype(I)::value;
      const uint64_t m = __ballot(l == (uint32_t)ll);
      // (the lanes of m below this one by mbcnt: a (1 << lane) - 1 mask can be spilled and reloaded per length)
      const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
      if (l == (uint32_t)ll) sorted[off + offs[ll] + run[ll] + (int)below] = (uint16_t)s;
      run[ll] += __popcll(m);
    });
  }
  __syncthreads();
  // root entries: stream bits e (LSB first) = code prefix bitrev(e) (MSB first)
  for (int e = lane; e < (1 << R); e += 64) {
    const uint32_t v = (__builtin_bitreverse32((uint32_t)e) >> (32 - R)) << (15 - R);
    if (v < c.lim[R]) {  // a code of at most R bits
      const uint32_t l = canon_len<R>(c, v);
      L.tab[2 * e + DIST] = sym_entry(sorted[off + (int)(v >> (15 - l)) + canon_base<R>(c, l)], l, DIST);
    }
  }
  // sub-tables: one per root prefix of the codes longer than R, sized by the longest code under that prefix.  A
  // lane per prefix lays them out (offset, index bits) and marks its entries' owner; then all lanes fill the
  // entries, 64 at a time (on the synthetic BAM ~22 literal prefixes of up to 32 entries: a lane per prefix filling
  // its own ran 32 serial steps of canonical decoding).  Scratch: the window, restaged before the data rounds.
  const uint32_t P0 = c.lim[R] >> (15 - R);
  const int npre = (1 << R) - (int)P0;
  uint16_t *own = reinterpret_cast<uint16_t *>(L.win);  // [subcap] prefix index of each sub-table entry
  uint32_t *pinfo = L.win + 256;                           // [npre] offset | index bits << 16
  static_assert(wd::kLitSub <= 512 && 256 + 512 <= wd::kWinDw - wd::kScratchDw, "sub-table scratch in the window");
  int next = 0;
  for (int j0 = 0; j0 < npre; j0 += 64) {
    const int j = j0 + lane;
    const uint32_t P = P0 + (uint32_t)j;
    uint32_t sb = 0, sz = 0;
    if (j < npre) {
      sb = canon_len(c, ((P + 1) << (15 - R)) - 1) - R;
      sz = 1u << sb;
    }
    const uint32_t incl = wave_incl_scan(sz);
    const int my = next + (int)(incl - sz);
    if (j < npre && my + (int)sz <= subcap) {
      L.tab[2 * (__builtin_bitreverse32(P) >> (32 - R)) + DIST] =
          (wd::K_SUBP << 8) | sb | ((uint32_t)(4 * (suboff + my)) << 16);
      pinfo[j] = (uint32_t)my | (sb << 16);
      for (uint32_t k = 0; k < sz; k++) own[my + (int)k] = (uint16_t)j;
    }
    next += (int)__shfl(incl, 63);
  }
  __syncthreads();
  if (next <= subcap) {
    for (int e = lane; e < next; e += 64) {
      const int j = own[e];
      const uint32_t info = pinfo[j], sb = info >> 16, P = P0 + (uint32_t)j, k = (uint32_t)e - (info & 0xffffu);
      const uint32_t v = (P << (15 - R)) | ((__builtin_bitreverse32(k) >> (32 - sb)) << (15 - R - sb));
      const uint32_t l = canon_len(c, v);
      L.tab[suboff + e] = sym_entry(sorted[off + (int)(v >> (15 - l)) + canon_base(c, l)], l, DIST);
    }
  }
  __syncthreads();
  return next <= subcap;
}

// LDS byte address of a pointer into __shared__ memory
SB_DEV uint32_t lds_addr(const void *p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void *)p;
}

// One symbol of the alphabet the state st4 selects (0: literal/length, 4: distance after a length) at bit position
// pos (bits from the block's 16-B aligned base; wp = the staged window less its first bit's dword, so wp[pos >> 5]
// holds bit pos): 32 bits of lookahead from two window dwords, the root entry at byte (bits & 511) << 3 | st4 of
// tab, the sub-table entry for long codes, the extra bits.  Advances pos; returns the kind, v = the symbol's token
// (literal byte, 253 + length, 0x7fff + distance) or K_SPEC value.
typedef const __attribute__((address_space(3))) uint32_t *lds_u32;
// wp[pos >> 5] as an LDS pointer: one shift and one shift-add (the compiler's own form is a shift, a mask and an add)
SB_DEV lds_u32 win_at(const uint32_t *wp, int pos) {
  uint32_t a;
  asm("v_lshl_add_u32 %0, %1, 2, %2" : "=v"(a) : "v"((uint32_t)pos >> 5), "s"(lds_addr(wp)));
  return reinterpret_cast<lds_u32>((uintptr_t)a);
}
// The symbol whose bits start at bit pos & 31 of the dword pair hi:lo0 (see wsym).
SB_DEV uint32_t tsym(const WaveLds &L, uint32_t lo0, uint32_t hi, int &pos, uint32_t st4, uint32_t &v) {
  using namespace wd;
  const uint32_t lo = __builtin_amdgcn_alignbit(hi, lo0, (uint32_t)pos);  // (the shift is pos & 31)
  static_assert(kLitRoot == 9 && kDistRoot == 9, "interleaved 9-bit roots");
  const char *tb = reinterpret_cast<const char *>(L.tab);
  uint32_t e = *reinterpret_cast<const uint32_t *>(tb + (((lo << 3) & 0xff8u) | st4));
  if (((e >> 8) & 0xffu) == K_SUBP)
    e = *reinterpret_cast<const uint32_t *>(tb + (e >> 16) + 4u * __builtin_amdgcn_ubfe(lo, 9u, e));
  const uint32_t n = e & 15u, x = (e >> 4) & 15u;
  v = (e >> 16) + __builtin_amdgcn_ubfe(lo, n, x);
  pos += (int)(n + x);
  return (e >> 8) & 0xffu;
}
SB_DEV uint32_t wsym(const uint32_t *wp, const WaveLds &L, int &pos, uint32_t st4, uint32_t &v) {
  const lds_u32 q = win_at(wp, pos);
  return tsym(L, q[0], q[1], pos, st4, v);
}

// Wave-uniform bit reader for block headers.
struct HBits {
  uint64_t bb;
  int bc, rp, pos;
  SB_DEV void init(const uint32_t *win, int wq, int p) {
    const int rel = p - wq, w = rel >> 5, sh = rel & 31;
    bb = (((uint64_t)uni(win[w]) | ((uint64_t)uni(win[w + 1]) << 32)) >> sh);
    bc = 64 - sh;
    rp = w + 2;
    pos = p;
  }
  SB_DEV uint32_t get(const uint32_t *win, int n) {
    if (bc < 32) {
      bb |= (uint64_t)uni(win[rp]) << bc;
      bc += 32;
      rp++;
    }
    const uint32_t v = (uint32_t)bb & ((1u << n) - 1u);
    bb >>= n;
    bc -= n;
    pos += n;
    return v;
  }
};

// Stage kWinDw dwords from dword wq_dw of the block's aligned base into the window (zeros past the buffer).
// Every load is issued before the first wait: as a loop (load, wait, LDS store per 1 KiB) the compiler waited for
// each load in turn — five memory round trips per round instead of one.
SB_DEV void wave_stage(uint32_t *win, const uint32_t *base, int64_t base_dw, int wq_dw, int64_t lim_dw) {
  constexpr int kN = (wd::kWinDw + 255) / 256;
  const int lane = (int)threadIdx.x;
  __syncthreads();  // every lane is done with the previous window
  // LDS DMA (global_load_lds_dwordx4: lane l's 16 B land at the LDS base + 16 l), no VGPRs; lanes past the buffer
  // load its last 16 B instead of zeros (bits past the payload only ever end a speculative path: ST_OUT)
  {
    const int64_t last = lim_dw - 4 - base_dw;  // dword offset of the buffer's last 16 B from base
#pragma unroll
    for (int k = 0; k < kN; k++) {
      const int i = lane * 4 + 256 * k;
      if (i < wd::kWinDw) {  // (exec-masked: lanes past the window write nothing — the tables follow it)
        int64_t o = (int64_t)wq_dw + i;
        o = o > last ? last : o;
        __builtin_amdgcn_global_load_lds(base + o, win + 256 * k, 16, 0, 0);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
}
// Result of one lane's decode of its segment from a given start: counts, exit key (pos << 10 | state << 9 |
// pending length) and stop.
struct SegResult {
  uint32_t tok, byt, exit;
  int stop;
  bool bad;
};

#ifdef SBAM_WAVE_STATS
constexpr int kWaveStats = 40;  // [0, 32): k_inflate_wave, [32, 40): k_inflate_resolve
__device__ unsigned long long g_wave_stats[kWaveStats];
#define WMARK(slot) do { const uint64_t t_ = __builtin_amdgcn_s_memtime(); ws_[slot] += t_ - wt_; wt_ = t_; } while (0)
#define WADD(slot, v) ws_[slot] += (v)
extern "C" int sbam_debug_wave_stats(unsigned long long *out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_wave_stats), sizeof(g_wave_stats)) != hipSuccess) return -1;
  if (reset) {
    static const unsigned long long z[kWaveStats] = {0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_wave_stats), z, sizeof(z)) != hipSuccess) return -1;
  }
  return 0;
}
#else
#define WMARK(slot) do {} while (0)
#define WADD(slot, v) do {} while (0)
#endif
#ifdef SBAM_WAVE_STATS  // resolver phases: slot 32 + k (RMARK), 39 = steps
#define RMARK(k) do { const uint64_t t_ = __builtin_amdgcn_s_memtime(); rs_[k] += t_ - rt_; rt_ = t_; } while (0)
#else
#define RMARK(k) do {} while (0)
#endif

// ---- stored blocks (BTYPE 00) -----------------------------------------------------------------------------------
// zlib level 0 (bgzip -l 0, samtools view -u) and incompressible input at any level make stored DEFLATE blocks: LEN
// raw bytes behind a byte-aligned LEN / NLEN pair (RFC 1951 3.2.4).  A BGZF payload whose DEFLATE stream is only
// stored blocks is a copy: the wave walks the block headers (wave-uniform, one or a few per payload), then copies the
// bytes straight to the output (unaligned 16-B loads, 16-B aligned stores; byte stores for the partial 16-B chunks at
// a stored block's edges — a BGZF block's first and last chunks are shared with its neighbours) and marks the block
// done for the resolver (TokPool::base = kTokDone): no tokens, no resolve.  Anything else — a stored block after
// Huffman output, LEN != ~NLEN, data past the payload, a total other than ISIZE, more than kMaxStored blocks — goes to
// the exact decoder as before, which has zlib's semantics for every case (Stream.scala:49-54).  (Round 5 sent every
// stored block there: one lane emitting 2 literal tokens per step into the arena, then the resolver.)
constexpr int kMaxStored = 64;
constexpr int64_t kTokDone = -2;  // TokPool::base of a block already written to the output

// bitp: payload-relative bit position of the first stored block's header (BFINAL, BTYPE 00).  seg: 2 * kMaxStored
// dwords of LDS.  Returns false (nothing written) when the payload is not a clean chain of stored blocks producing
// exactly ISIZE bytes.
SB_DEV bool stored_copy(const uint8_t *__restrict__ d, int64_t a, int dlen, int bitp, int32_t us,
                        uint8_t *__restrict__ ob, int64_t U0, uint32_t *seg) {
  const int lane = (int)threadIdx.x;
  int n = 0, o = 0;
  if ((bitp + 3 + 7) / 8 > dlen) return false;
  bool fin;
  {
    const uint32_t h3 = (uint32_t)d[a + (bitp >> 3)] | (uint32_t)d[a + (bitp >> 3) + 1] << 8;
    const uint32_t hb = (h3 >> (bitp & 7)) & 7u;
    if (((hb >> 1) & 3u) != 0u) return false;
    fin = (hb & 1u) != 0u;
    bitp += 3;
  }
  for (;;) {
    const int byp = (bitp + 7) >> 3;  // LEN / NLEN start on the next byte boundary
    if (byp + 4 > dlen || n == kMaxStored) return false;
    const uint32_t len = (uint32_t)d[a + byp] | (uint32_t)d[a + byp + 1] << 8;
    const uint32_t nlen = (uint32_t)d[a + byp + 2] | (uint32_t)d[a + byp + 3] << 8;
    if ((len ^ 0xffffu) != nlen) return false;
    const int dat = byp + 4;
    if (dat + (int)len > dlen) return false;
    if (lane == 0) {
      seg[2 * n] = (uint32_t)o;
      seg[2 * n + 1] = (uint32_t)dat;
    }
    n++;
    o += (int)len;
    if (o > us) return false;
    if (fin) break;
    const int nb = dat + (int)len;  // the next block's header byte (byte-aligned after a stored block)
    if (nb >= dlen) return false;
    const uint32_t h3 = d[a + nb];
    if (((h3 >> 1) & 3u) != 0u) return false;
    fin = (h3 & 1u) != 0u;
    bitp = nb * 8 + 3;
  }
  if (o != us) return false;
  __syncthreads();  // (one wave: the segment list is visible to every lane)
  for (int j = 0; j < n; j++) {
    const int o0 = (int)seg[2 * j], o1 = j + 1 < n ? (int)seg[2 * j + 2] : us;
    const uint8_t *src = d + a + (int)seg[2 * j + 1] - o0;  // output byte x of this stored block is src[x]
    const int c0 = o0 + (int)((16 - ((U0 + o0) & 15)) & 15), c1 = o1 - (int)((U0 + o1) & 15);
    if (c0 + 16 <= c1) {
      // 16-B aligned output chunks [c0, c1): four loads in flight per lane before their stores
      int x = c0 + 16 * lane;
      for (; x + 3 * 1024 + 16 <= c1; x += 4 * 1024) {
        const u32x4 v0 = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(src + x));
        const u32x4 v1 = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(src + x + 1024));
        const u32x4 v2 = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(src + x + 2048));
        const u32x4 v3 = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(src + x + 3072));
        *reinterpret_cast<u32x4 *>(ob + x) = v0;
        *reinterpret_cast<u32x4 *>(ob + x + 1024) = v1;
        *reinterpret_cast<u32x4 *>(ob + x + 2048) = v2;
        *reinterpret_cast<u32x4 *>(ob + x + 3072) = v3;
      }
      for (; x + 16 <= c1; x += 1024)
        *reinterpret_cast<u32x4 *>(ob + x) = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(src + x));
      if (lane < c0 - o0) ob[o0 + lane] = src[o0 + lane];  // (< 16 bytes each side)
      if (lane < o1 - c1) ob[c1 + lane] = src[c1 + lane];
    } else {
      for (int x = o0 + lane; x < o1; x += 64) ob[x] = src[x];
    }
  }
  return true;
}

__global__ __launch_bounds__(64, 4) void k_inflate_wave(const uint8_t *__restrict__ d, int64_t D, BlockTable bt,
                                                     TokPool tp, int32_t *__restrict__ status,
                                                     int32_t *__restrict__ found, int32_t *__restrict__ slow,
                                                     unsigned int *nslow) {
  using namespace wd;
  __shared__ __attribute__((aligned(16))) WaveLds L;
  const int lane = (int)threadIdx.x;
  const int64_t b = blockIdx.x;
  const int64_t st0 = bt.start[b];
  const int32_t hs = bt.hsize[b], cs = bt.csize[b], us = bt.usize[b];
  const int32_t dlen = cs - hs - 8;  // Stream.scala: dataLength = compressedSize - headerSize - FOOTER_SIZE
  if (us == 0 || us < 0 || us > 65536 || dlen < 0 || st0 + hs + dlen > D) {
    if (lane == 0) {
      status[b] = us == 0 ? INF_OK : INF_DATA;  // inflate(buf, 0, 0) returns 0; else a data error
      found[b] = 0;
    }
    return;
  }
  const int64_t a = st0 + hs;
  const int64_t base_dw = (a >> 4) << 2;  // 16-B aligned dword base of the payload
  const uint32_t *base = reinterpret_cast<const uint32_t *>(d) + base_dw;
  const int64_t lim_dw = (D + kCompPad) >> 2;
  const int skip = (int)(a - base_dw * 4) * 8;
  const int pend = skip + 8 * dlen;  // payload end (bits)
  uint8_t *reg = tp.main + tok_region(bt.uoff[b], b);
  int32_t tcap = tok_region_cap(us);  // tokens the region holds (the arena region: all a block can produce)
  uint8_t *lens = L.lens();
  int pos = skip;
  int out = 0, ntok = 0;
  bool ok = true, stored = false;
#ifdef SBAM_WAVE_STATS
  uint64_t ws_[32] = {0};  // (slots 32.. are the resolver's)
  uint64_t wt_ = __builtin_amdgcn_s_memtime();
  const uint64_t wt0_ = wt_;
#endif

  for (bool fin = false; ok && !fin;) {
    // ---- block header
    int wq = (pos >> 7) << 7;
    wave_stage(L.win, base, base_dw, wq >> 5, lim_dw);
    WMARK(12);
    if (pos + 3 > pend) { ok = false; break; }
    HBits h;
    h.init(L.win, wq, pos);
    fin = h.get(L.win, 1) != 0;
    const uint32_t type = h.get(L.win, 2);
    int hlit = 288, hdist = 32;
    if (type == 1) {  // fixed codes: lit 0-143:8, 144-255:9, 256-279:7, 280-287:8; dist 0-31:5
      for (int i = lane; i < 320; i += 64)
        lens[i] = i < 144 ? 8 : i < 256 ? 9 : i < 280 ? 7 : i < 288 ? 8 : 5;
    } else if (type == 2) {
      hlit = (int)h.get(L.win, 5) + 257;
      hdist = (int)h.get(L.win, 5) + 1;
      const int hclen = (int)h.get(L.win, 4) + 4;
      if (hlit > 286 || hdist > 30) { ok = false; break; }
      uint64_t clp = 0;
      for (int i = 0; i < 19; i++)
        if (i < hclen) clp |= (uint64_t)h.get(L.win, 3) << (3 * kClOrder[i]);
      // code-length code (must be complete): left-justified 7-bit limits and the symbols in canonical order.  Lane s
      // < 19 holds symbol s's length: the counts per length are ballots, a symbol's canonical rank is a 19-step count
      // on its own lane (the wave-uniform form was a 19 x 19 compare loop per header)
      const uint32_t lsym = lane < 19 ? (uint32_t)(clp >> (3 * lane)) & 7u : 0u;
      int left = 1;
      bool over = false;
      uint32_t lim7[8], base7[8], code = 0;
      int acc = 0;
#pragma unroll
      for (int l = 1; l <= 7; l++) {
        const uint32_t k = (uint32_t)__popcll(__ballot(lsym == (uint32_t)l));
        left = 2 * left - (int)k;
        over |= left < 0;
        lim7[l] = (code + k) << (7 - l);
        base7[l] = (uint32_t)acc - code;
        acc += (int)k;
        code = (code + k) << 1;
      }
      if (over || left != 0) { ok = false; break; }
      for (int i = lane; i < 320; i += 64) lens[i] = 0;
      // every lane decodes the code-length symbol at bit b0 + lane: advance, repeat count, value kind
      uint32_t srt[4];  // symbols in canonical order, 5 bits each, 6 per dword
      {
        uint32_t r = 0;
#pragma unroll
        for (int t2 = 0; t2 < 19; t2++) {
          const uint32_t lt2 = (uint32_t)(clp >> (3 * t2)) & 7u;
          r += (lt2 != 0 && (lt2 < lsym || (lt2 == lsym && t2 < lane))) ? 1u : 0u;
        }
        // the fields are disjoint: the sum over the lanes is their OR
        const uint32_t field = lsym ? (uint32_t)lane << (5 * (r % 6)) : 0u;
#pragma unroll
        for (int q = 0; q < 4; q++)
          srt[q] = uni((uint32_t)__shfl((int)wave_incl_scan(r / 6 == (uint32_t)q ? field : 0u), 63));
      }
      // the code-length code as a 128-entry table of the next 7 stream bits (in the sorted-symbol scratch, free until
      // the table builds): length | extra bits << 3 | repeat base << 6 | value << 10 | "previous" << 14 — a window's
      // 64 decodes are one LDS read each instead of the canonical search
      uint16_t *cllut = L.sorted();
      for (int v = lane; v < 128; v += 64) {
        const uint32_t rev = __builtin_bitreverse32((uint32_t)v) >> 25;
        uint32_t l = 1;
#pragma unroll
        for (int ll = 1; ll < 7; ll++) l += rev >= lim7[ll] ? 1u : 0u;
        uint32_t bsel = 0;
#pragma unroll
        for (int ll = 1; ll <= 7; ll++) bsel = l == (uint32_t)ll ? base7[ll] : bsel;
        const uint32_t idx = (rev >> (7 - l)) + bsel;
        const uint32_t dq = idx / 6, dr = idx % 6;
        const uint32_t sw = dq == 0 ? srt[0] : dq == 1 ? srt[1] : dq == 2 ? srt[2] : srt[3];
        const uint32_t sym = (sw >> (5 * dr)) & 31u;
        const uint32_t xb = sym == 16 ? 2u : sym == 17 ? 3u : sym == 18 ? 7u : 0u;
        const uint32_t rb = sym < 16 ? 1u : sym == 18 ? 11u : 3u;
        cllut[v] = (uint16_t)(l | (xb << 3) | (rb << 6) | ((sym < 16 ? sym : 0u) << 10) | ((sym == 16 ? 1u : 0u) << 14));
      }
      __syncthreads();
      WMARK(10);
      const int total = uni(hlit + hdist);  // (uni: the compiler kept it, and the loop below, in VGPRs)
      int n = 0, p = h.pos;
      uint32_t prev = 0;
      while (n < total) {
        // lane j: the symbol at p + j
        const int q = p + lane - wq, w = q >> 5, sh = q & 31;
        const uint64_t x64 = ((uint64_t)L.win[w] | ((uint64_t)L.win[w + 1] << 32)) >> sh;
        const uint32_t bits = (uint32_t)x64;
        const uint32_t e = cllut[bits & 127u];
        const uint32_t l = e & 7u, xb = (e >> 3) & 7u;
        const uint32_t xv = __builtin_amdgcn_ubfe(bits, l, xb);
        const uint32_t rep = ((e >> 6) & 15u) + xv;
        // packed: advance (5 bits) | repeat (8) | value (4) | value is "previous" (1)
        const uint32_t info = (l + xb) | (rep << 5) | (((e >> 10) & 31u) << 13);
        // the true chain through the 64 decoded offsets: only the offsets and the running count are serial
        // (scalar readlanes); values, repeat targets and LDS writes follow for all members at once.  info2 = the
        // info of the symbol after this lane's (a shuffle), so one walk step takes two symbols: two independent
        // readlanes per step instead of one dependent readlane per symbol.
        const uint32_t nx = (uint32_t)lane + (info & 31u);
        const uint32_t info2 = (uint32_t)__shfl((int)info, (int)min(nx, 63u));
        int o = 0;
        uint64_t chain = 0;
        const int n0 = n;
        // (o, n and chain pinned to scalar registers: left to the compiler, they lived in VGPRs and every step
        // went VGPR -> readfirstlane -> readlane -> VGPR under exec-mask bookkeeping)
        while (o < 64 && n < total) {
          const uint32_t in = (uint32_t)__builtin_amdgcn_readlane((int)info, o);
          const uint32_t in2 = (uint32_t)__builtin_amdgcn_readlane((int)info2, o);
          chain = uni((uint64_t)(chain | (1ull << o)));
          n = uni(n + (int)((in >> 5) & 255u));
          const int o1 = uni(o + (int)(in & 31u));
          if (o1 < 64 && n < total) {
            chain = uni((uint64_t)(chain | (1ull << o1)));
            n = uni(n + (int)((in2 >> 5) & 255u));
            o = uni(o1 + (int)(in2 & 31u));
          } else {
            o = o1;
          }
        }
        o = uni(o);
        n = uni(n);
        const bool mem = (chain >> lane) & 1ull;
        const uint64_t below = (1ull << lane) - 1ull;
        // each member's first code-length index: n0 + the repeats of the members before it
        const uint32_t rr = mem ? (info >> 5) & 255u : 0u;
        const int nst0 = n0 + (int)(wave_incl_scan(rr) - rr);
        // value: a literal length, 0 for 17/18, and for 16 the value of the nearest member before it that has one
        // (the previous batch's last value when there is none)
        const bool isprev = (info >> 17) & 1u;
        const uint32_t own_v = (info >> 13) & 15u;
        const uint64_t hv = __ballot(mem && !isprev);
        const uint64_t hb = hv & below;
        const int src = hb ? 63 - __clzll((long long)hb) : 0;
        const uint32_t pv = (uint32_t)__shfl((int)own_v, src);
        const uint32_t v = isprev ? (hb ? pv : prev) : own_v;
        bool bad = n > total || __ballot(mem && isprev && nst0 == 0) != 0;
        if (mem && v) {
          for (int k = 0; k < (int)rr; k++) {  // <= 6 (a literal: 1; code 16: 3-6; zeros need no write)
            const int idx2 = nst0 + k;
            lens[idx2 < hlit ? idx2 : 288 + idx2 - hlit] = (uint8_t)v;
          }
        }
        const int last = chain ? 63 - __clzll((long long)chain) : 0;
        prev = uni((uint32_t)__shfl((int)v, last));
        if (bad) { ok = false; break; }
        p += o;
        if (p > pend) { ok = false; break; }
      }
      if (!ok) break;
      WMARK(11);
      h.pos = p;
      __syncthreads();
      if (lens[256] == 0) { ok = false; break; }  // no end-of-block code
    } else {  // stored from the first output byte: k_inflate_stored's copy; else (a stored block after Huffman output,
              // an invalid type) the slow decoder
      stored = type == 0 && out == 0 && ntok == 0;
      ok = false;
      break;
    }
    if (h.pos > pend) { ok = false; break; }
    WMARK(0);
    WADD(9, 1);
    if (!wave_build<true>(L, 288, hdist, kDistSubOff, kDistSub)) { ok = false; break; }
    WMARK(5);  // (the distance table; slot 1: the literal/length table)
    if (!wave_build<false>(L, 0, hlit, kLitSubOff, kLitSub)) { ok = false; break; }
    WMARK(1);

    // ---- data rounds: 64 segments of kK bits per round.  The last deflate block (BFINAL) runs to the payload's end,
    // so its rounds are sized to it: the same number of rounds with segments of kS <= kK bits spread evenly, instead
    // of a last round whose lanes past the end decode nothing of use (zlib's last block of a BGZF block is its last
    // ~7 %, one round of ~7 per block, 40 % used)
    // A non-final block's end is not known, but zlib's first block of a BGZF payload ends at 92-94 % of its bits
    // (16383 literals and matches: profiles/r05/round_model.log): its rounds are sized as if it ended at 93 % —
    // one round fewer-used lanes in the last one (decode 40.3 -> 39.5 ms at 10 GB; 95 %: 39.7, 97 %: 42.0, the
    // rounds then no longer cover the block; profiles/r05/ab/firstfrac_*.log).  Another structure only changes
    // how full the rounds are.
    int kS = kK;
    {
      const int left = fin ? pend - h.pos : (int)((int64_t)(pend - h.pos) * kFirstFrac / 1000);
      const int nr = (left + 64 * kK - 1) / (64 * kK);
      kS = nr > 0 ? min(kK, max(32, (((left + 64 * nr - 1) / (64 * nr)) + 31) & ~31)) : kK;
      kS = uni(kS);
    }
    uint32_t S = (uint32_t)h.pos << 10;  // round start: pos << 10 | state << 9 | pending match length
    for (;;) {
      const int Sp = (int)(S >> 10);
      wq = (Sp >> 7) << 7;
      wave_stage(L.win, base, base_dw, wq >> 5, lim_dw);
      const uint32_t *wp = L.win - (wq >> 5);  // wp[pos >> 5]: the staged dword holding bit pos
      WMARK(2);
      WADD(6, 1);
      const int seg_start = lane == 0 ? Sp : Sp + lane * kS;
      const int seg_end = Sp + (lane + 1) * kS;
      // ---- phase A: every lane decodes its segment from a guessed start (lane 0: the true one)
      uint32_t cp[kCp], cc[kCp];  // checkpoints: position (literal/length state) and tok | byt << 12 there
      sfor<0, kCp>([&](auto I) {
        cp[decltype(I)::value] = ~0u;
        cc[decltype(I)::value] = 0;
      });
      uint32_t s1p = ~0u, s1e = 0, s1c = 0, s2p = ~0u, s2e = 0, s2c = 0;  // stops: start, exit | kind, counts
      int nst = 0;
      uint32_t tokA = 0, bytA = 0, exitEnd, entry;
      uint32_t tr[kTR / 2];  // phase-A tokens of steps [0, kTR)
      uint32_t stR = 0, bytR = 0;  // state (exit key) and bytes after step kTR
      {
        uint32_t st4 = lane == 0 ? (S >> 7) & 4u : 0u;  // state << 2 (the table's byte offset for the state)
        uint32_t pl = lane == 0 ? (S & 511u) : 0u;
        int rp = seg_start;  // reader position
        bool go = true;
        if (seg_start >= pend && lane > 0) {
          go = false;
          nst = 1;
          s1p = (uint32_t)seg_start;
          s1e = ((uint32_t)seg_start << 10) | (uint32_t)ST_OUT;
        } else if (lane > 0 && kWarm > 0) {  // warm-up: decode (uncounted, stops ignored) up to the segment
          rp = seg_start - kWarm;
          if (rp <= Sp) {  // from the round's true start, in its true state
            rp = Sp;
            st4 = (S >> 7) & 4u;
            pl = S & 511u;
          }
          while (rp < seg_start) {
            uint32_t v;
            const uint32_t kind = wsym(wp, L, rp, st4, v);
            pl = kind == K_LEN ? v - 253u : pl;
            st4 = kind == K_LEN ? 4u : 0u;
          }
        }
        WMARK(13);
        entry = ((uint32_t)rp << 10) | (st4 << 7) | pl;
        // the window dwords W, W + 1, W + 2 of the reader (W = rp >> 5) in registers: a symbol is at most 28 bits,
        // so the next reader is in W or W + 1, and dword W + 2 of the new reader is loaded a whole step before use
        // (one LDS round trip less on a step's dependent chain: root entry, sub-table entry; decode 46.0 → 45.7 ms.
        // The same for the warm-up loop: no change)
        uint32_t wA, wB, wC;
        {
          const lds_u32 q = win_at(wp, rp);
          wA = q[0];
          wB = q[1];
          wC = q[2];
        }
        // one symbol, predicated: a lane that is done (stopped out of the data, or past its segment) decodes the
        // same symbol again and commits nothing, so the steps need no exec-mask branches
        // ST: the step's index when it is below kTR (its token goes to tr), else -1
        auto step = [&](auto ST) {
          constexpr int sj = decltype(ST)::value;
          const bool live = go && rp < seg_end;
          const uint32_t p0 = (uint32_t)rp;
          int rq = rp;
          uint32_t v;
          const uint32_t kind = tsym(L, wA, wB, rq, st4, v);
          const bool outp = rq > pend;
          const bool stp = live && (kind == K_SPEC || outp);
          if (__builtin_amdgcn_ballot_w64(stp) != 0) {  // rare: record the stop (exit in the literal state | kind) and decode on
            const uint32_t ek = ((uint32_t)rq << 10) | (uint32_t)(outp ? ST_OUT : v == 0 ? ST_EOB : ST_ERR);
            const uint32_t cn = tokA | (bytA << 12);
            const bool w1 = stp && nst == 0, w2 = stp && nst == 1;
            s1p = w1 ? p0 : s1p;
            s1e = w1 ? ek : s1e;
            s1c = w1 ? cn : s1c;
            s2p = w2 ? p0 : s2p;
            s2e = w2 ? ek : s2e;
            s2c = w2 ? cn : s2c;
            nst += stp ? 1 : 0;
            go = (stp && outp) ? false : go;
          }
          rp = live ? rq : rp;
          {
            const bool adv = (((uint32_t)rp ^ p0) >> 5) != 0u;
            wA = adv ? wB : wA;
            wB = adv ? wC : wB;
            wC = win_at(wp, rp)[2];
          }
          const bool cnt = live && !stp;
          if constexpr (sj >= 0) {  // the token (a committed step j is token j of the path: no stop before it)
            if constexpr ((sj & 1) == 0) {
              tr[sj / 2] = v;
            } else {
              tr[sj / 2] = __builtin_amdgcn_perm(v, tr[sj / 2], 0x05040100u);  // low half kept, v above
            }
          }
          // selects and carry-in adds only (no exec-mask branches): counts and the pending length.  (zlib's
          // "invalid distance too far back" is the resolver's test: k_inflate_resolve hands such a block back.)
          const bool cl = cnt && kind == K_LEN;
          const uint32_t lenv = v - 253u;
          tokA += cnt ? 1u : 0u;                                        // (v_addc with the lane mask as carry-in)
          bytA += (cl ? lenv : 0u) + ((cnt && kind == K_LIT) ? 1u : 0u);  // + length, or + 1 for a literal
          pl = cl ? lenv : pl;
          st4 = live ? (cl ? 4u : 0u) : st4;
        };
        // checkpoints every kCpSteps steps (wave-uniform, so a record costs no divergent branch): the lane's
        // position if it is at a literal/length boundary
        sfor<0, kCp>([&](auto J) {
          constexpr int jj = decltype(J)::value;
          const bool live = go && rp < seg_end;
          cp[jj] = (live && st4 == 0) ? (uint32_t)rp : ~0u;
          cc[jj] = tokA | (bytA << 12);
          if (__ballot(live) != 0) {
            if constexpr (jj * kCpSteps < kTR) {
              sfor<0, kCpSteps>([&](auto K) {
                constexpr int sj = jj * kCpSteps + decltype(K)::value;
                step(std::integral_constant<int, (sj < kTR ? sj : -1)>{});
              });
            } else {
#pragma unroll 2  // (4 and 8: the same; 1: +0.5 ms)
              for (int k = 0; k < kCpSteps; k++) step(std::integral_constant<int, -1>{});
            }
          }
          if constexpr ((jj + 1) * kCpSteps == kTR) {
            stR = ((uint32_t)rp << 10) | (st4 << 7) | pl;
            bytR = bytA;
          }
        });
        while (__ballot(go && rp < seg_end) != 0) step(std::integral_constant<int, -1>{});
        exitEnd = ((uint32_t)rp << 10) | (st4 << 7) | pl;
      }
      WMARK(3);
      // the lane's result if its guessed start is the true one: the path ends at its first stop
      const SegResult own = nst > 0 ? SegResult{s1c & 4095u, s1c >> 12, s1e & ~1023u, (int)(s1e & 3u), false}
                                    : SegResult{tokA, bytA, exitEnd, ST_NONE, false};
      // ---- phase B: lanes whose true start differs re-decode it until they reach a first-pass checkpoint
      SegResult res = own;
      uint32_t nxt = lane == 0 ? own.exit : exitEnd;  // what the right neighbour starts from (provisional)
      uint32_t bst = lane == 0 ? S : entry;
      bool ver = lane == 0;
      // where phase C finds the lane's tokens: kModeA — res is phase A's own result (tokens in tr from step 0);
      // kModeR — re-decoded from the true start up to phase A's checkpoint rjP (rjtk tokens), then phase A's path
      // from step rjs; kModeF — re-decoded to the end
      enum : int { kModeA = 0, kModeR = 1, kModeF = 2 };
      int mode = kModeA;
      uint32_t rjP = 0, rjs = 0, rjtk = 0;
      int f = 64;
      for (;;) {
        uint32_t pex = __shfl_up(nxt, 1);
        if (lane == 0) pex = S;
        bool upd = false;
        if (!ver && pex == bst) {  // the guessed start was right
          ver = true;
          upd = nxt != own.exit;
          nxt = own.exit;
          res = own;
          mode = kModeA;
        }
        const uint64_t vs = __ballot(ver && res.stop != ST_NONE);
        f = uni(vs ? __ffsll((unsigned long long)vs) - 1 : 64);
        const bool need = lane > 0 && lane <= f && pex != bst;
        if (__ballot(need || upd) == 0) break;
        WADD(7, 1);
        if (need) {
          uint32_t st4 = (pex >> 7) & 4u;
          uint32_t pl = pex & 511u, tk = 0, by = 0;
          int rp = (int)(pex >> 10);
          // the first checkpoint at or after the reader
          auto next_cp = [&](uint32_t p) {
            uint32_t m = ~0u;
            sfor<0, kCp>([&](auto I) {
              const uint32_t x = cp[decltype(I)::value];
              m = (x >= p && x < m) ? x : m;
            });
            return m;
          };
          uint32_t tcp = next_cp((uint32_t)rp);
          mode = kModeF;
          for (;;) {
            if (st4 == 0 && (uint32_t)rp == tcp) {  // on the first-pass path from here
              uint32_t cj = 0, sj = 0;
              sfor<0, kCp>([&](auto I) {
                const bool hit = cp[decltype(I)::value] == tcp;
                cj = hit ? cc[decltype(I)::value] : cj;
                sj = hit ? (uint32_t)(decltype(I)::value * kCpSteps) : sj;
              });
              const uint32_t P = tcp;
              mode = kModeR;
              rjP = P;
              rjs = sj;
              rjtk = tk;
              // the first recorded stop at or after the checkpoint ends the path
              const bool h1 = nst >= 1 && s1p >= P, h2 = !h1 && nst >= 2 && s2p >= P;
              if (h1 || h2) {
                const uint32_t se = h1 ? s1e : s2e, sc = h1 ? s1c : s2c;
                res = SegResult{tk + (sc & 4095u) - (cj & 4095u), by + (sc >> 12) - (cj >> 12), se & ~1023u,
                                (int)(se & 3u), false};
                break;
              }
              if (nst <= 2) {
                res = SegResult{tk + tokA - (cj & 4095u), by + bytA - (cj >> 12), exitEnd, ST_NONE, false};
                break;
              }
              tcp = ~0u;  // more stops than recorded, the first after P unknown: decode the rest here
              mode = kModeF;
            }
            if (rp >= seg_end) {
              res = SegResult{tk, by, ((uint32_t)rp << 10) | (st4 << 7) | pl, ST_NONE, false};
              break;
            }
            uint32_t v;
            const uint32_t kind = wsym(wp, L, rp, st4, v);
            const bool outp = rp > pend;
            if (kind == K_SPEC || outp) {
              res = SegResult{tk, by, (uint32_t)rp << 10, outp ? ST_OUT : v == 0 ? ST_EOB : ST_ERR, false};
              break;
            }
            tk++;
            by += kind == K_LIT ? 1u : kind == K_LEN ? v - 253u : 0u;
            pl = kind == K_LEN ? v - 253u : pl;
            st4 = kind == K_LEN ? 4u : 0u;
            if ((uint32_t)rp > tcp) tcp = next_cp((uint32_t)rp);
          }
          nxt = res.stop != ST_NONE ? res.exit : res.exit;
          ver = true;
          bst = pex;
        }
      }
      WMARK(4);
      // lanes 0..f carry the true path (f: the lane whose segment ends the deflate block, or 64)
      const bool act = lane <= f;
#ifdef SBAM_WAVE_STATS
      {  // token statistics of the true segments: how many lanes, how many re-decoded (phase B), token counts
        const bool viaB = act && mode != kModeA;
        WADD(23, __ballot(act && mode == kModeF) != 0 ? 1 : 0);
        WADD(14, __popcll(__ballot(act)));
        WADD(15, __popcll(__ballot(viaB)));
        WADD(16, __popcll(__ballot(act && res.tok > 64)));
        WADD(17, __popcll(__ballot(act && res.tok > 96)));
        WADD(18, __popcll(__ballot(act && res.tok > 128)));
        WADD(19, __ballot(viaB) != 0 ? 1 : 0);
        WADD(20, __ballot(act && res.tok > 96) != 0 ? 1 : 0);
        WADD(21, __ballot(act && res.tok > 64) != 0 ? 1 : 0);
        WADD(22, __ballot(act && own.stop != ST_NONE) != 0 ? 1 : 0);
      }
#endif
      const uint32_t my_tok = act ? res.tok : 0u, my_byt = act ? res.byt : 0u;
      const uint32_t itok = wave_incl_scan(my_tok), ibyt = wave_incl_scan(my_byt);
      const uint32_t tot_tok = uni((uint32_t)__shfl(itok, 63)), tot_byt = uni((uint32_t)__shfl(ibyt, 63));
      const int stop_f = f < 64 ? uni(__shfl(res.stop, f)) : ST_NONE;
      if (stop_f == ST_ERR || stop_f == ST_OUT || out + (int)tot_byt > us || __ballot(act && res.bad) != 0) {
        ok = false;
        break;
      }
      if (ntok + (int)tot_tok > tcap) {  // (rare) the block outgrows its main region: move its tokens to the arena
        const uint64_t need = tok_arena_need(us);
        uint64_t at = 0;
        if (lane == 0) at = atomicAdd(tp.arena_used, (unsigned long long)need);
        at = ((uint64_t)uni((uint32_t)__shfl((int)(at >> 32), 0)) << 32) | uni((uint32_t)__shfl((int)(uint32_t)at, 0));
        if ((int64_t)(at + need) > tp.arena_cap) {  // the exact decoder reports the overflow; the host grows the arena
          ok = false;
          break;
        }
        uint8_t *nreg = tp.arena + at;
        // the earlier rounds' token stores (this wave's) are visible to the copy's loads: a workgroup-scope fence
        // (an agent-scope __threadfence also writes back L2: measured at twice the decode time on the regions branch)
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
        const int nb = 2 * ntok, nb16 = nb & ~15;
        for (int i = 16 * lane; i < nb16; i += 1024)
          *reinterpret_cast<uint4 *>(nreg + i) = *reinterpret_cast<const uint4 *>(reg + i);
        if (lane < (nb - nb16) / 2)
          reinterpret_cast<uint16_t *>(nreg + nb16)[lane] = reinterpret_cast<const uint16_t *>(reg + nb16)[lane];
        if (lane == 0) tp.base[b] = (int64_t)at;
        reg = nreg;
        tcap = 1 << 30;
      }
      // ---- phase C: write the true segments' tokens at their offsets.  A lane re-decodes only what phase A's
      // registers do not hold: mode F its whole segment, mode R the stretch up to its rejoin checkpoint; then the
      // register tokens; then whatever lies past step kTR.
      bool tail = false;
      uint32_t tail_ti = 0, tail_st = 0;
      uint32_t r_lo = 0, r_hi = 0, r_tb = 0;  // register tokens k in [r_lo, r_hi) go to token index r_tb + k
      if (act) {
        uint32_t start = __shfl_up(nxt, 1);
        if (lane == 0) start = S;
        uint32_t ti = (uint32_t)ntok + (itok - my_tok);
        // decode from key st until the reader reaches endp (or the end-of-block symbol of lane f), writing tokens
        auto run = [&](uint32_t st, int endp) {
          uint32_t st4 = (st >> 7) & 4u;
          int rp = (int)(st >> 10);
          while (rp < endp) {
            uint32_t v;
            const uint32_t kind = wsym(wp, L, rp, st4, v);
            if (kind == K_SPEC) break;
            st4 = kind == K_LEN ? 4u : 0u;
            *reinterpret_cast<uint16_t *>(reg + 2 * ti) = (uint16_t)v;
            ti++;
          }
        };
        WMARK(24);
        run(start, mode == kModeF ? seg_end : mode == kModeR ? (int)rjP : 0);
        WMARK(25);
        // register tokens [lo, hi) of phase A's path (mode A: from step 0; mode R: from its rejoin checkpoint's
        // step), token k at index tb + k
        const uint32_t lo = mode == kModeR ? rjs : 0u;
        const uint32_t n = mode == kModeA ? res.tok : mode == kModeR ? res.tok - rjtk : 0u;
        const uint32_t hi = mode == kModeF ? 0u : min(lo + n, (uint32_t)kTR);
        const uint32_t tb = ti - lo;
        r_lo = lo;
        r_hi = hi;
        r_tb = tb;
        static_assert(kTR == 80, "one asm operand per register token dword");
        // (one statement: the spilled ones are reloaded together, one wait)
        asm volatile("" : "+v"(tr[0]), "+v"(tr[1]), "+v"(tr[2]), "+v"(tr[3]), "+v"(tr[4]), "+v"(tr[5]), "+v"(tr[6]), "+v"(tr[7]), "+v"(tr[8]), "+v"(tr[9]), "+v"(tr[10]), "+v"(tr[11]), "+v"(tr[12]), "+v"(tr[13]), "+v"(tr[14]), "+v"(tr[15]), "+v"(tr[16]), "+v"(tr[17]), "+v"(tr[18]), "+v"(tr[19]), "+v"(tr[20]), "+v"(tr[21]), "+v"(tr[22]), "+v"(tr[23]), "+v"(tr[24]), "+v"(tr[25]), "+v"(tr[26]), "+v"(tr[27]), "+v"(tr[28]), "+v"(tr[29]), "+v"(tr[30]), "+v"(tr[31]), "+v"(tr[32]), "+v"(tr[33]), "+v"(tr[34]), "+v"(tr[35]), "+v"(tr[36]), "+v"(tr[37]), "+v"(tr[38]), "+v"(tr[39]));
        {
          // 16-B stores (4-B aligned: a 2-B head when tb is odd), dwords and 2-B halves where the run starts or ends
          // inside a chunk — a lane's run is contiguous, so 8 tokens per store instruction instead of one (every
          // store instruction writes 64 lanes' separate lines)
          const uint32_t par = tb & 1u;
          uint8_t *pa = reg + 2 * ((int64_t)ti - (int64_t)lo);  // (tb may lie before the region: only k >= lo is stored)
          if (par && lo == 0 && hi > 0) *reinterpret_cast<uint16_t *>(pa) = (uint16_t)tr[0];
          u32x4a *pv = reinterpret_cast<u32x4a *>(pa + 2 * par);
          uint32_t *pw = reinterpret_cast<uint32_t *>(pa + 2 * par);
          // dword q: tokens par + 2q, par + 2q + 1
          auto dw = [&](auto Q) {
            constexpr int q = decltype(Q)::value;
            const uint32_t nx = q + 1 < kTR / 2 ? tr[q + 1 < kTR / 2 ? q + 1 : q] : 0u;
            return par ? __builtin_amdgcn_alignbit(nx, tr[q], 16) : tr[q];
          };
          sfor<0, kTR / 8>([&](auto C) {
            constexpr int c = decltype(C)::value;
            const uint32_t a0 = dw(std::integral_constant<int, 4 * c>{}), a1 = dw(std::integral_constant<int, 4 * c + 1>{});
            const uint32_t a2 = dw(std::integral_constant<int, 4 * c + 2>{}), a3 = dw(std::integral_constant<int, 4 * c + 3>{});
            const uint32_t t0 = par + 8 * c;  // the chunk's first token
            if (t0 >= lo && t0 + 8 <= hi) {
              pv[c] = u32x4a{a0, a1, a2, a3};
            } else if (t0 + 8 > lo && t0 < hi) {  // the run starts or ends in this chunk
              const uint32_t a[4] = {a0, a1, a2, a3};
#pragma unroll
              for (int k = 0; k < 4; k++) {
                const uint32_t u0 = t0 + 2 * k;
                const bool in0 = u0 >= lo && u0 < hi, in1 = u0 + 1 >= lo && u0 + 1 < hi;
                uint16_t *ph = reinterpret_cast<uint16_t *>(pw + 4 * c + k);
                if (in0 && in1) pw[4 * c + k] = a[k];
                else if (in0) ph[0] = (uint16_t)a[k];
                else if (in1) ph[1] = (uint16_t)(a[k] >> 16);
              }
            }
          });
        }
        WMARK(26);
        WMARK(27);
        // the path goes on past step kTR (no stop before it): phase A's path from step kTR (its state stR) — or, for
        // a lane that rejoined phase A only after step kTR (no register token is on its path), from the rejoin
        // checkpoint itself (a literal/length boundary, no pending length) right after the re-decoded stretch
        tail = mode != kModeF && lo + n > (uint32_t)kTR;
        tail_st = lo <= (uint32_t)kTR ? stR : rjP << 10;
        tail_ti = lo <= (uint32_t)kTR ? tb + kTR : ti;
      }
      if (tail) {
        uint32_t st4 = (tail_st >> 7) & 4u, ti = tail_ti;
        int rp = (int)(tail_st >> 10);
        while (rp < seg_end) {
          uint32_t v;
          const uint32_t kind = wsym(wp, L, rp, st4, v);
          if (kind == K_SPEC) break;
          st4 = kind == K_LEN ? 4u : 0u;
          *reinterpret_cast<uint16_t *>(reg + 2 * ti) = (uint16_t)v;
          ti++;
        }
      }
      (void)r_lo;
      (void)r_hi;
      (void)r_tb;
      WMARK(28);
      out += (int)tot_byt;
      ntok += (int)tot_tok;
      if (f < 64) {  // end of block: the next header follows lane f's end-of-block symbol
        pos = (int)(uni((uint32_t)__shfl(res.exit, f)) >> 10);
        break;
      }
      S = uni((uint32_t)__shfl(nxt, 63));
    }
  }
  if (ok && out != us) ok = false;
#ifdef SBAM_WAVE_STATS
  ws_[8] = __builtin_amdgcn_s_memtime() - wt0_;
  if (lane == 0)
    for (int i = 0; i < 29; i++) atomicAdd(&g_wave_stats[i], (unsigned long long)ws_[i]);
#endif
  if (lane == 0) {
    if (ok) {
      status[b] = INF_OK;
      found[b] = us;
    } else if (stored) {
      slow[bt.n + atomicAdd(nslow + 3, 1u)] = (int32_t)b;
    } else {
      slow[atomicAdd(nslow, 1u)] = (int32_t)b;
    }
  }
}

// The stored-only blocks k_inflate_wave listed (slow[bt.n ..], count nslow[3]): one wave each, grid-stride over the
// list.  The copy starts at the payload's first DEFLATE block; a block whose payload is not a clean stored chain from
// there (e.g. empty Huffman blocks before the stored ones, which no common encoder writes) goes to the exact
// decoder's list.
__global__ __launch_bounds__(64) void k_inflate_stored(const uint8_t *__restrict__ d, BlockTable bt, TokPool tp,
                                                      uint8_t *__restrict__ out, int32_t *__restrict__ status,
                                                      int32_t *__restrict__ found, int32_t *__restrict__ slow,
                                                      unsigned int *nslow) {
  __shared__ uint32_t seg[2 * kMaxStored];
  const unsigned n = nslow[3];
  for (unsigned i = blockIdx.x; i < n; i += gridDim.x) {
    const int64_t b = slow[bt.n + i];
    const int64_t a = bt.start[b] + bt.hsize[b], U0 = bt.uoff[b];
    const int32_t dlen = bt.csize[b] - bt.hsize[b] - 8, us = bt.usize[b];
    if (stored_copy(d, a, dlen, 0, us, out + U0, U0, seg)) {
      if (threadIdx.x == 0) {
        tp.base[b] = kTokDone;
        status[b] = INF_OK;
        found[b] = us;
      }
    } else if (threadIdx.x == 0) {
      slow[atomicAdd(nslow, 1u)] = (int32_t)b;
    }
    __syncthreads();  // (seg is reused by the next block)
  }
}

// ---- resolve kernel -------------------------------------------------------------------------------------------
// One wavefront per BGZF block; the block's recent output lives in a kRing-byte LDS ring (ring byte of output
// position p: (uoff + p) mod kRing, so ring chunks and HBM chunks share their 16-B alignment).  A step ("chunk")
// takes the next 64 words, one per lane:
//   1. a wave prefix sum of the words' output lengths gives every word its position O (a chunk is cut where a word
//      would start kSpan or more bytes after the chunk's base, and at the block's end);
//   2. the ring dwords the chunk will write are zeroed, then literal bytes are written by byte stores and match
//      bytes by LDS ORs of their (masked, shifted) dwords — lanes writing neighbouring bytes of one dword never race;
//   3. literal words are written at once; matches go in rounds: a match is ready when its source ends at or before
//      the first pending match of the chunk (the first pending one always is), ready matches copy in steps of up
//      to 16 bytes (an overlapping copy doubles its distance per step) from the ring (distance <= kNear) or, for
//      far sources, from the output already flushed to HBM;
//   4. completed output leaves in 1 KiB groups of 16-B aligned stores; a block's partial first and last 16-B chunks
//      (shared with its neighbours) leave as byte stores.
// A block's LZ77 window never leaves the chip except for the far copies; HBM sees the words once and the output
// once.  (Round 2; the round-1 design ran one lane per block with the window in HBM and was bound by the memory
// side: 16.5x the output bytes per launch.)
// (Round 4, measured and dropped: far copies deferred until the first pending match is far, 41.2 vs 38.7 ms at 10 GB
// — the deferral added rounds; four tokens per lane per step, 46.2 / 42.1 ms.)
namespace rs {
constexpr int kSpan = 1024;   // a chunk's words start within kSpan bytes of its base
constexpr int kFlush = 1024;  // output bytes per group store (64 lanes x 16 B)
}  // namespace rs

template <int RB>
struct RingGeom {
  static constexpr uint32_t kRing = 1u << RB, kMask = kRing - 1u, kDw = kRing / 4u, kDwMask = kDw - 1u;
  // ring dwords [kDw, kDw + kMirror) mirror dwords [0, kMirror): a 5-dword read from any start never wraps
  static constexpr uint32_t kMirror = 8u;
  // Near sources: the ring holds positions (E + 3 - kRing, E) while a chunk ending at E <= base + kSpan + 257 is
  // written, so every source at distance <= kNear from a word starting before base + kSpan is intact.
  static constexpr int kNear = (int)kRing - rs::kSpan - 264;
  // A far copy's 16-B loads end before O - d + L + 15 < base + kSpan + 272 - d, and the flushed mark is past
  // base - kFlush: distance >= kSpan + kFlush + 272 keeps them in HBM-resident output.
  static_assert(kNear >= rs::kSpan + rs::kFlush + 272, "far sources are in HBM");
  // A slot is flushed before a later chunk zeroes it: kRing > kSpan + 260 + kFlush.
  static_assert((int)kRing > rs::kSpan + 260 + rs::kFlush, "slots are flushed before reuse");
};

// OR one dword into the ring at (wrapped) dword i, and into its mirror when i < kMirror.
template <class G>
SB_DEV void ring_or1(uint32_t *ring, uint32_t i, uint32_t w) {
  atomicOr(ring + i, w);
  if (i < G::kMirror) atomicOr(ring + G::kDw + i, w);
}
// OR up to 5 dwords into the ring at dword q (wrapping, mirrored).  The common case uses immediate offsets.
template <class G>
SB_DEV void ring_or5(uint32_t *ring, uint32_t q, uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3, uint32_t w4) {
  if (q >= G::kMirror && q + 4u < G::kDw) {
    uint32_t *p = ring + q;
    atomicOr(p + 0, w0);
    atomicOr(p + 1, w1);
    atomicOr(p + 2, w2);
    atomicOr(p + 3, w3);
    atomicOr(p + 4, w4);
  } else {
    ring_or1<G>(ring, q & G::kDwMask, w0);
    ring_or1<G>(ring, (q + 1u) & G::kDwMask, w1);
    ring_or1<G>(ring, (q + 2u) & G::kDwMask, w2);
    ring_or1<G>(ring, (q + 3u) & G::kDwMask, w3);
    ring_or1<G>(ring, (q + 4u) & G::kDwMask, w4);
  }
}

// zlib's "invalid distance too far back" (a match reaching before the block's first output byte) is detected here,
// where every match's output position is known: the decoder's speculative phases never test it.  Such a block is
// listed in redo[] (nothing is read before its output) and the host hands it to k_inflate_slow, which reports the
// error with zlib's count, then resolves it again (list: the blocks of that second pass).
template <int RB>
__global__ __launch_bounds__(64) void k_inflate_resolve(BlockTable bt, uint8_t *__restrict__ out, TokPool pool,
                                                        const int32_t *__restrict__ found,
                                                        const int32_t *__restrict__ list, int32_t *__restrict__ redo,
                                                        unsigned int *__restrict__ nredo) {
  using G = RingGeom<RB>;
  __shared__ __attribute__((aligned(16))) uint32_t ring[G::kDw + G::kMirror];
  __shared__ __attribute__((aligned(16))) uint32_t s_keep[17 * 4];  // s_keep[4n..4n+3]: mask of the low n bytes
  uint8_t *ring8 = reinterpret_cast<uint8_t *>(ring);
  const int lane = (int)threadIdx.x;
  for (int i = lane; i < 17 * 4; i += 64) {
    const int n = i >> 2, k = i & 3, nb = n - 4 * k;  // bytes of dword k kept
    s_keep[i] = nb >= 4 ? ~0u : nb <= 0 ? 0u : (1u << (8 * nb)) - 1u;
  }
  const int64_t b = list ? list[blockIdx.x] : blockIdx.x;
  const int ae = found[b];  // output bytes of the block
  const int64_t tbase = pool.base[b];
  if (ae <= 0 || tbase == kTokDone) return;  // (kTokDone: the decoder copied a stored-only block itself)
  const int64_t U0 = bt.uoff[b];
  uint8_t *ob = out + U0;
  const uint32_t Gr = (uint32_t)U0 & G::kMask;  // ring byte of position 0
  const uint16_t *tk =
      reinterpret_cast<const uint16_t *>(tbase >= 0 ? pool.arena + tbase : pool.main + tok_region(U0, b));
  const int F0 = (int)((16 - (U0 & 15)) & 15);  // first position on a 16-B boundary
  int F = F0;                                     // flushed up to here (from F0)
  bool head = F0 == 0;                            // positions [0, F0) stored
  int Z = -(int)(Gr & 3u);                        // ring zeroed for positions [.., Z); Gr + Z is dword aligned
  int B = 0, tp = 0;                              // chunk base position, its first token
  bool toofar = false;                            // a distance past the block's first byte (zlib: data error)
  // lane i holds tokens tp + 2i and tp + 2i + 1, and sees tp + 2i + 2 (the distance of a length in its second)
  uint32_t ta = tk[2 * lane], tb = tk[2 * lane + 1], tn = tk[2 * lane + 2];
  asm volatile("" : "+v"(ta), "+v"(tb), "+v"(tn));  // (no token load pending at the loop head, from either edge)
#ifdef SBAM_WAVE_STATS
  uint64_t rs_[8] = {0};
  uint32_t it_ = 0;
  uint64_t itw_ = 0, itl_ = 0;
  uint64_t rt_ = __builtin_amdgcn_s_memtime();
  const uint64_t rt0_ = rt_;
#endif
  while (B < ae) {
    // ---- 1. positions: a lane yields up to 2 literals and at most one match (a length in its first token takes
    // the second as its distance; a length in its second takes the next lane's first)
    const bool aLit = ta < 256u, aLen = (ta >> 8) == 1u, bLit = tb < 256u, bLen = (tb >> 8) == 1u;
    const int nl = (int)aLit + (int)bLit;
    const int Lm = aLen ? (int)ta - 253 : bLen ? (int)tb - 253 : 0;
    const int d = (int)((aLen ? tb : tn) & 0x7fffu) + 1;
    const int Ln = nl + Lm;
    const int incl = (int)wave_incl_scan((uint32_t)Ln);
    const int ex = incl - Ln;
    const int O = B + ex;
    const bool take = ex < rs::kSpan && O < ae;
    const uint64_t tmask = __ballot(take);
    const int nt = __popcll(tmask);  // a prefix of the lanes (lane 0 always)
    const int E = min(B + __builtin_amdgcn_readlane(incl, nt - 1), ae);
    if (E <= B) break;  // (no output left in the tokens: never for a decoded stream)
    // the next chunk starts after the last taken lane's tokens (and the distance its second token may own)
    const int tp2 = uni(tp + 2 * nt + (int)((__ballot(bLen) >> (nt - 1)) & 1ull));
    // ---- 2. zero the ring dwords of [Z, E)
    {
      const uint32_t z0 = (Gr + (uint32_t)Z) >> 2, z1 = (Gr + (uint32_t)E + 3u) >> 2;
#pragma unroll 1
      for (uint32_t k0 = z0; k0 < z1; k0 += 64u) {  // (usually one or two rounds)
        const uint32_t k = k0 + (uint32_t)lane, i = k & G::kDwMask;
        if (k < z1) {
          ring[i] = 0u;
          if (i < G::kMirror) ring[G::kDw + i] = 0u;
        }
      }
      Z = (int)(z1 * 4u - Gr);
    }
    RMARK(0);  // positions, ring zeroing
    // ---- 3a. literals (before the match when a lane has both)
    // (byte stores: they touch only their own byte, so lanes writing neighbouring bytes of a dword never race)
    const int Ll = take ? min(nl, ae - O) : 0;
    if (Ll > 0) {
      const uint32_t lv = aLit ? (ta | (bLit ? tb << 8 : 0u)) : tb;
      const uint32_t x = (Gr + (uint32_t)O) & G::kMask;
      ring8[x] = (uint8_t)lv;
      if (x < 4u * G::kMirror) ring8[G::kRing + x] = (uint8_t)lv;
      if (Ll >= 2) {
        const uint32_t x1 = (x + 1u) & G::kMask;
        ring8[x1] = (uint8_t)(lv >> 8);
        if (x1 < 4u * G::kMirror) ring8[G::kRing + x1] = (uint8_t)(lv >> 8);
      }
    }
    RMARK(1);  // literals
    // ---- 4. output of the chunks before this one ([F, B) is final), issued before this step's loads: the stores
    // precede the next step's token loads, so waiting for those never waits for the stores (one in-order vmcnt; a
    // data-dependent store count after the loads made the compiler wait with vmcnt(0))
    if (!head && B >= F0) {  // the block's first partial 16-B chunk (shared with the previous block)
      if (lane < F0) ob[lane] = ring8[(Gr + (uint32_t)lane) & G::kMask];
      head = true;
    }
    while (B - F >= rs::kFlush) {
      const uint32_t x = (Gr + (uint32_t)(F + 16 * lane)) & G::kMask;  // 16-B aligned
      *reinterpret_cast<uint4 *>(ob + F + 16 * lane) = *reinterpret_cast<const uint4 *>(ring8 + x);
      F += rs::kFlush;
    }
    RMARK(2);  // output stores
    // ---- 3b. matches, in rounds
    const int mO = O + (bLen ? nl : 0);
    int Le = (take && Lm > 0) ? min(Lm, ae - mO) : 0;
    const bool tf = Le > 0 && d > mO;  // invalid distance too far back: no copy, the block goes to the exact decoder
    toofar |= tf;
    Le = tf ? 0 : Le;
    const bool mt = Le > 0;
    const bool far = d > G::kNear;
    const int srcEnd = mO - d + min(Le, d);
    // far sources (already in HBM, final) are loaded now, 32 B ahead; their copies wait until a near copy needs
    // them (the first pending match is far), so the loads overlap the near rounds
    u32x4 pf0 = {0u, 0u, 0u, 0u}, pf1 = {0u, 0u, 0u, 0u};
    if (mt && far) {
      pf0 = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(ob + mO - d));
      if (Le > 16) pf1 = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(ob + mO - d + 16));
    }
    // the next step's tokens, loaded after the far sources: a wait for a far source need not wait for them
    // (as raw registers, split only after the rounds: see the end of the step)
    uint32_t w2, n2;
    __builtin_memcpy(&w2, tk + tp2 + 2 * lane, 4);
    n2 = tk[tp2 + 2 * lane + 2];
    RMARK(3);  // match setup, far prefetch, next tokens issued
    uint64_t pend = __ballot(mt);
    const uint64_t below = (1ull << lane) - 1ull;
    const int mEnd = mO + Le;
    while (pend) {
      const int f = __ffsll((unsigned long long)pend) - 1;
      const int fr = __builtin_amdgcn_readlane(mO, f);
      // ready: the source ends before the first pending output, or every pending output before this lane's ends
      // at or before the source starts (pending outputs are disjoint and in lane order, so the nearest one decides)
      const uint64_t pb = pend & below;
      const int jn = pb ? 63 - __clzll((long long)pb) : lane;
      const int endj = __shfl(mEnd, jn);
      uint64_t ready = pend & __ballot(srcEnd <= fr || pb == 0 || endj <= mO - d);
      if ((ready >> lane) & 1ull) {
        int done = 0, deff = d;
        while (done < Le) {
#ifdef SBAM_WAVE_STATS
          it_++;
#endif
          const int n = min(min(Le - done, 16), deff);
          const int src = mO + done - deff;
          // the keep-mask of the first n bytes, read before the source (it was read after, a second LDS round trip
          // on every iteration's dependent chain)
          const uint4 km = *reinterpret_cast<const uint4 *>(s_keep + 4 * n);
          uint32_t v0, v1, v2, v3;
          if (far) {  // below the flushed mark: unaligned 16-B loads, past this CU's L1 (nt)
            // each path waits for its own source here (the prefetched ones: vmcnt(2), the next step's two token
            // loads may stay in flight): merged with the near path's registers, the compiler waited with vmcnt(0)
            // after the join, so every near copy also waited for the next step's tokens
            if (done >= 32) {
              const u32x4 x = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(ob + src));
              v0 = x.x; v1 = x.y; v2 = x.z; v3 = x.w;
              asm volatile("" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3));
            } else {
              const u32x4 x = done == 0 ? pf0 : pf1;
              v0 = x.x; v1 = x.y; v2 = x.z; v3 = x.w;
              asm volatile("" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3));
            }
          } else {
            const uint32_t xs = (Gr + (uint32_t)src) & G::kMask, qs = xs >> 2, ss = xs & 3u;
            const uint32_t *p = ring + qs;  // (qs + 4 < kDw + kMirror: the mirror covers the wrap)
            const uint32_t s0 = p[0], s1 = p[1], s2 = p[2], s3 = p[3], s4 = p[4];
            v0 = __builtin_amdgcn_alignbyte(s1, s0, ss);
            v1 = __builtin_amdgcn_alignbyte(s2, s1, ss);
            v2 = __builtin_amdgcn_alignbyte(s3, s2, ss);
            v3 = __builtin_amdgcn_alignbyte(s4, s3, ss);
          }
          // keep the first n bytes
          v0 &= km.x;
          v1 &= km.y;
          v2 &= km.z;
          v3 &= km.w;
          // shift to the destination's byte offset and OR in
          const uint32_t xd = (Gr + (uint32_t)(mO + done)) & G::kMask, qd = xd >> 2, s8 = (xd & 3u) * 8u;
          const uint64_t a01 = ((uint64_t)v1 << 32 | v0) << s8, a12 = ((uint64_t)v2 << 32 | v1) << s8,
                         a23 = ((uint64_t)v3 << 32 | v2) << s8, a34 = (uint64_t)v3 << s8;
          ring_or5<G>(ring, qd, (uint32_t)a01, (uint32_t)(a01 >> 32), (uint32_t)(a12 >> 32), (uint32_t)(a23 >> 32),
                      (uint32_t)(a34 >> 32));
          done += n;
          if (n == deff && deff < 16) deff *= 2;  // the copied bytes extend the period: 2·deff is a valid distance
        }
      }
      pend &= ~ready;
#ifdef SBAM_WAVE_STATS
      rs_[7]++;  // rounds
      {  // copy iterations: the wave's (the slowest lane's) and the sum over lanes
        uint32_t mx = it_, sm = it_;
        for (int o = 32; o >= 1; o >>= 1) {
          mx = max(mx, (uint32_t)__shfl_xor((int)mx, o));
          sm += (uint32_t)__shfl_xor((int)sm, o);
        }
        itw_ += mx;
        itl_ += sm;
        it_ = 0;
      }
#endif
    }
    RMARK(4);  // rounds
    B = E;
    // the wait for the next step's tokens, here: the compiler otherwise split them right after the loads (waiting
    // there), or let this step's last use of tn wait after the stores (one in-order vmcnt)
    asm volatile("" : "+v"(w2), "+v"(n2));
    ta = w2 & 0xffffu;
    tb = w2 >> 16;
    tn = n2;
    RMARK(5);  // the wait for the next tokens
#ifdef SBAM_WAVE_STATS
    rs_[6]++;  // steps
#endif
    tp = tp2;
  }
  // tail: the head (a block shorter than its first partial chunk), whole 16-B chunks, the last partial chunk
  if (!head) {
    if (lane < min(F0, ae)) ob[lane] = ring8[(Gr + (uint32_t)lane) & G::kMask];
  }
  if (ae > F0) {
    const int Ft = F + ((ae - F) & ~15);
    for (int p = F + 16 * lane; p < Ft; p += rs::kFlush)
      *reinterpret_cast<uint4 *>(ob + p) = *reinterpret_cast<const uint4 *>(ring8 + ((Gr + (uint32_t)p) & G::kMask));
    if (Ft + lane < ae) ob[Ft + lane] = ring8[(Gr + (uint32_t)(Ft + lane)) & G::kMask];
  }
  if (__ballot(toofar) != 0 && lane == 0 && redo) redo[atomicAdd(nredo, 1u)] = (int32_t)b;
#ifdef SBAM_WAVE_STATS
  // slots 32..37: phases (the tail in 37 with the total's remainder), 38: steps, 39: rounds
  const uint64_t tot_ = __builtin_amdgcn_s_memtime() - rt0_;
  if (lane == 0) {
    for (int i = 0; i < 6; i++) atomicAdd(&g_wave_stats[32 + i], (unsigned long long)rs_[i]);
    atomicAdd(&g_wave_stats[38], (unsigned long long)rs_[6]);
    atomicAdd(&g_wave_stats[39], (unsigned long long)rs_[7]);
    atomicAdd(&g_wave_stats[31], (unsigned long long)tot_);
    atomicAdd(&g_wave_stats[29], (unsigned long long)itw_);
    atomicAdd(&g_wave_stats[30], (unsigned long long)itl_);
  }
#endif
}

__global__ void k_first_error(const int32_t *__restrict__ status, int64_t n, unsigned long long *first_err) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n && status[i] != INF_OK) atomicMin(first_err, (unsigned long long)i);
}

hipError_t launch_first_error(const int32_t *status, int64_t n, unsigned long long *first_err, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_first_error, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, status, n, first_err);
  return hipGetLastError();
}


hipError_t launch_inflate_decode(const uint8_t *d, int64_t D, BlockTable bt, TokPool tok, uint8_t *out,
                                 int32_t *status, int32_t *found, int32_t *slow, unsigned int *counters,
                                 hipStream_t s) {
  // counters: [0] slow-path blocks, [1] slow-path work, [3] stored-only blocks (zeroed first: the host reads [0] back
  // even for 0 blocks).  slow: 2 x bt.n entries, the exact decoder's list from 0, the stored-only list from bt.n.
  (void)hipMemsetAsync(counters, 0, 4 * sizeof(unsigned int), s);
  if (bt.n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_inflate_wave, dim3((unsigned)bt.n), dim3(64), 0, s, d, D, bt, tok, status, found, slow,
                     counters + 0);
  hipLaunchKernelGGL(k_inflate_stored, dim3(4096), dim3(64), 0, s, d, bt, tok, out, status, found, slow,
                     counters + 0);
  hipLaunchKernelGGL(k_inflate_slow, dim3(256), dim3(kDecThreads), 0, s, d, D, bt, tok, slow, counters + 0, status,
                     found, counters + 1);
  return hipGetLastError();
}

hipError_t launch_inflate_resolve(BlockTable bt, uint8_t *out, TokPool tok, const int32_t *found,
                                  const int32_t *list, int64_t nlist, int32_t *redo, unsigned int *nredo,
                                  hipStream_t s) {
  const int64_t n = list ? nlist : bt.n;
  if (n == 0) return hipSuccess;
  // a 4 KiB ring: 8 waves per SIMD (an 8 KiB ring, 5 per SIMD: 58 ms at 10 GB; 4 KiB: 46 ms)
  hipLaunchKernelGGL(k_inflate_resolve<12>, dim3((unsigned)n), dim3(64), 0, s, bt, out, tok, found, list, redo, nredo);
  return hipGetLastError();
}

hipError_t launch_inflate_redo(const uint8_t *d, int64_t D, BlockTable bt, TokPool tok, const int32_t *list,
                               unsigned int *counters, int32_t *status, int32_t *found, hipStream_t s) {
  // counters[2]: the blocks in list; counters[1]: the exact decoder's work counter, reset
  (void)hipMemsetAsync(counters + 1, 0, sizeof(unsigned int), s);
  hipLaunchKernelGGL(k_inflate_slow, dim3(256), dim3(kDecThreads), 0, s, d, D, bt, tok, list, counters + 2, status,
                     found, counters + 1);
  return hipGetLastError();
}

}  // namespace sbam
