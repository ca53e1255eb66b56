// sbam_inflate.hip — batched raw-DEFLATE inflate of BGZF blocks for gfx950, in two kernels.
//
// Semantics: java.util.zip.Inflater(nowrap).inflate(decBuf, 0, ISIZE) on the block payload, as the reference
// calls it (bgzf/src/main/scala/org/hammerlab/bgzf/block/Stream.scala:31-71), i.e. zlib inflate():
//   * output stops at ISIZE (remaining input is ignored); ISIZE 0 returns 0 at once;
//   * the stream ending (final EOB, or input exhausted mid-symbol) before ISIZE bytes → "found" count (SHORT);
//   * invalid streams (bad block type, stored LEN/NLEN, over-subscribed / incomplete codes, missing EOB code,
//     bad repeat, invalid symbols, distance too far back) → DATA error; CRC32 is never checked.
//
// Design:
//   k_inflate_decode  — one lane per BGZF block (SIMT across independent blocks).  Huffman decoding is
//     canonical: per code length l a left-justified limit lim[l] and an index bias bse[l] live in VGPRs,
//     the symbols in canonical order live in a 640-B LDS slice per lane (256 lanes = all 160 KiB of LDS).
//     The symbol stream leaves as u16 tokens in 4 KiB pages of an HBM pool (16-B stores; lanes grab pages
//     with an atomic counter).  No lane ever reads the output, so this kernel never waits on HBM except
//     for its (prefetched) input dwords.
//   k_inflate_resolve — one lane per BGZF block again, but with no tables: 2048 lanes per CU hide the
//     latency of back-reference loads.  Tokens become bytes in a 64-B per-lane LDS ring that leaves as
//     aligned 16-B stores; copies with distance <= 40 read the ring, longer ones read HBM (4-B aligned
//     loads + v_alignbyte).  Overlapping copies double their distance per step (the period stays valid).
#include "sbam_internal.h"

namespace sbam {

#define SB_DEV __device__ __forceinline__

enum : int32_t { INF_OK = 0, INF_SHORT = 1, INF_DATA = 2, INF_OVERFLOW = 3 };

// ---- token pages ------------------------------------------------------------------------------------------
// A page is kTokPage bytes: chunk 0 holds the index of the block's next page (dword 0), chunks 1..255 hold
// tokens (8 × u16 per 16-B chunk).  Token t < 256: literal byte t.  256 <= t < 512: match of length t - 253,
// followed by the token (distance - 1).  0xffff: padding.
constexpr uint32_t kTokPad = 0xffffu;

// ---- decode kernel: per-lane LDS slice ------------------------------------------------------------------------
constexpr int kDecThreads = 256;
constexpr int kSlice = 640;        // 256 × 640 B = 160 KiB
constexpr int kLitSorted = 0;      // 288 B: lit/len symbols in canonical order (low 8 bits)
constexpr int kClTab = 0;          //   during a dynamic header: 128-entry code-length-code table (u8: len<<5 | sym)
constexpr int kLitHi = 288;        // 36 B: bit i set ⇔ canonical entry i is a symbol >= 256
constexpr int kDistSorted = 324;   // 30 B: distance symbols in canonical order
constexpr int kCnt = 416;          // 16 × u32: per-length counts, then fill cursors (builds only)
constexpr int kLens = 480;         // 160 B: code lengths, one nibble per symbol (builds only)
static_assert(kDecThreads * kSlice == 163840, "LDS budget");

constexpr uint8_t kClOrder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

// Bit reader over one block payload.  bb holds bc valid bits (LSB first); nx is the next input dword, already
// loaded (its load is issued one refill ahead, so the wave rarely waits on it); left = payload bits not yet
// consumed (negative ⇒ the symbol needed bits past the payload: zlib returns for more input → SHORT).
struct Bits {
  uint64_t bb;
  int bc;
  int left;
  uint32_t nx;
  const uint32_t *inw;
  SB_DEV void refill() {
    if (bc <= 32) {
      bb |= (uint64_t)nx << bc;
      bc += 32;
      nx = *inw++;
    }
  }
  SB_DEV uint32_t peek(int n) const { return (uint32_t)bb & ((1u << n) - 1u); }
  SB_DEV void drop(int n) {
    bb >>= n;
    bc -= n;
    left -= n;
  }
};

// Canonical code of one alphabet: lim[l] = left-justified (15-bit) end of the length-l codes, bse[l] = index
// of the first length-l symbol in canonical order minus its first code.  lim is non-decreasing in l.
struct Canon {
  uint32_t lim[16];
  int32_t bse[16];
};

// Decode the next symbol index: returns idx into the canonical symbol list (valid=false for an unassigned code,
// which zlib reports after consuming 1 bit — the only incomplete codes it accepts are single 1-bit codes).
SB_DEV int canon_decode(const Canon &c, uint64_t bb, int &len, bool &valid) {
  const uint32_t rev = __builtin_bitreverse32((uint32_t)bb) >> 17;
  int L = 1;
  int32_t B = c.bse[1];
#pragma unroll
  for (int l = 1; l < 15; l++) {  // mask arithmetic, not a select: keeps lim/bse in registers (no scratch)
    const int32_t m = -(int32_t)(rev >= c.lim[l]);
    L -= m;
    B = (c.bse[l + 1] & m) | (B & ~m);
  }
  valid = rev < c.lim[15];
  len = valid ? L : 1;
  return valid ? (int)(rev >> (15 - L)) + B : 0;
}

// Build the canonical structures of nsym code lengths (nibbles at LENS[sym0 ...]) into sorted (+hi bitmap).
// Returns 0, or -1 for an over-subscribed set or an incomplete one other than a single 1-bit code
// (zlib inflate_table).  A set with no codes at all is accepted (only possible for distances).
SB_DEV int canon_build(uint8_t *sl, int sym0, int nsym, int sorted_off, bool lit, Canon &c) {
  uint32_t *cnt = reinterpret_cast<uint32_t *>(sl + kCnt);
  const uint32_t *lens = reinterpret_cast<const uint32_t *>(sl + kLens);
#pragma unroll
  for (int i = 0; i < 16; i++) cnt[i] = 0;
  for (int s = 0; s < nsym; s++) {
    const int n = sym0 + s;
    const uint32_t v = (lens[n >> 3] >> (4 * (n & 7))) & 15u;
    if (v) atomicAdd(&cnt[v], 1u);
  }
  uint32_t k[16];
#pragma unroll
  for (int i = 0; i < 16; i++) k[i] = cnt[i];
  int left = 1, maxl = 0;
  uint32_t code = 0;
  int32_t offs = 0;
#pragma unroll
  for (int l = 1; l <= 15; l++) {
    left = 2 * left - (int)k[l];
    if (k[l]) maxl = l;
    c.lim[l] = (code + k[l]) << (15 - l);
    c.bse[l] = offs - (int32_t)code;
    cnt[l] = (uint32_t)offs;  // fill cursor
    offs += (int32_t)k[l];
    code = (code + k[l]) << 1;
    if (left < 0) return -1;
  }
  c.lim[0] = 0;
  c.bse[0] = 0;
  if (left > 0 && maxl > 1) return -1;
  if (lit) {
    uint32_t *hi = reinterpret_cast<uint32_t *>(sl + kLitHi);
#pragma unroll
    for (int i = 0; i < 9; i++) hi[i] = 0;
  }
  for (int s = 0; s < nsym; s++) {
    const int n = sym0 + s;
    const uint32_t v = (lens[n >> 3] >> (4 * (n & 7))) & 15u;
    if (v) {
      const uint32_t pos = atomicAdd(&cnt[v], 1u);
      sl[sorted_off + pos] = (uint8_t)s;
      if (lit && s >= 256) atomicOr(reinterpret_cast<uint32_t *>(sl + kLitHi) + (pos >> 5), 1u << (pos & 31));
    }
  }
  return 0;
}

// Token output: an 8-slot shift register (tk.x low half = oldest) flushed as one 16-B store per chunk.
struct TokOut {
  uint32_t t0, t1, t2, t3;
  int n;
  uint64_t cur;  // byte offset of the next chunk in the pool
  SB_DEV void put(uint32_t t) {
    t0 = __builtin_amdgcn_alignbit(t1, t0, 16);
    t1 = __builtin_amdgcn_alignbit(t2, t1, 16);
    t2 = __builtin_amdgcn_alignbit(t3, t2, 16);
    t3 = __builtin_amdgcn_alignbit(t, t3, 16);
    n++;
  }
};

// Store the full chunk; open a new page when this one is full.  Returns false on pool overflow.
SB_DEV bool tok_flush(TokOut &to, uint8_t *pool, unsigned int *pool_next, uint32_t npages) {
  *reinterpret_cast<uint4 *>(pool + to.cur) = make_uint4(to.t0, to.t1, to.t2, to.t3);
  to.cur += 16;
  to.n = 0;
  if ((to.cur & (kTokPage - 1)) == 0) {
    const uint32_t p = atomicAdd(pool_next, 1u);
    if (p >= npages) return false;
    *reinterpret_cast<uint32_t *>(pool + to.cur - kTokPage) = p;  // link from the page just filled
    to.cur = (uint64_t)p * kTokPage + 16;
  }
  return true;
}

enum : int { S_NEXT = 0, S_HDR = 1, S_HUFF = 2, S_STORED = 3, S_DONE = 4, S_EXIT = 5 };

__global__ __launch_bounds__(kDecThreads, 1) void k_inflate_decode(const uint8_t *__restrict__ d, int64_t D,
                                                                   BlockTable bt, uint8_t *__restrict__ pool,
                                                                   uint32_t npages, unsigned int *pool_next,
                                                                   int32_t *__restrict__ blk_page,
                                                                   int32_t *__restrict__ status,
                                                                   int32_t *__restrict__ found,
                                                                   unsigned int *next_block) {
  __shared__ __attribute__((aligned(16))) uint8_t s_dec[kDecThreads * kSlice];
  uint8_t *sl = s_dec + threadIdx.x * kSlice;
  const uint8_t *litS = sl + kLitSorted;
  const uint32_t *litHi = reinterpret_cast<const uint32_t *>(sl + kLitHi);
  const uint8_t *distS = sl + kDistSorted;

  int state = S_NEXT;
  int64_t blk = -1;
  Bits br{0, 0, 0, 0, nullptr};
  TokOut to{0, 0, 0, 0, 0, 0};
  Canon lc, dc;
  int32_t o = 0, us = 0, err = INF_OK, sleft = 0, fin = 0;

  for (;;) {
    if (state == S_NEXT) {
      blk = (int64_t)atomicAdd(next_block, 1u);
      if (blk >= bt.n) {
        state = S_EXIT;
      } else {
        const int64_t st = bt.start[blk];
        const int32_t hs = bt.hsize[blk], cs = bt.csize[blk];
        us = bt.usize[blk];
        o = 0;
        fin = 0;
        err = INF_OK;
        const int32_t dlen = cs - hs - 8;  // Stream.scala: dataLength = compressedSize - headerSize - FOOTER_SIZE
        blk_page[blk] = -1;
        if (us == 0) {
          state = S_DONE;  // inflate(buf, 0, 0) returns 0
        } else if (us < 0 || us > 65536 || dlen < 0 || st + hs + dlen > D) {
          err = INF_DATA;
          state = S_DONE;
        } else {
          const uint32_t p = atomicAdd(pool_next, 1u);
          if (p >= npages) {
            err = INF_OVERFLOW;
            state = S_DONE;
          } else {
            blk_page[blk] = (int32_t)p;
            to.cur = (uint64_t)p * kTokPage + 16;
            to.n = 0;
            const uintptr_t a = reinterpret_cast<uintptr_t>(d + st + hs);
            const uint32_t *w = reinterpret_cast<const uint32_t *>(a & ~(uintptr_t)3);
            const int skip = (int)(a & 3) * 8;
            br.bb = (uint64_t)w[0] >> skip;
            br.bc = 32 - skip;
            br.nx = w[1];
            br.inw = w + 2;
            br.left = 8 * dlen;
            br.refill();
            state = S_HDR;
          }
        }
      }
    }
    if (__all(state == S_EXIT)) break;

    if (state == S_HDR) {
      // --- block header (RFC 1951 §3.2.3); every read checks that the payload holds the bits (else SHORT)
      br.refill();
      if (br.left < 3) {
        err = INF_SHORT;
        state = S_DONE;
      } else {
        fin = (int)br.peek(1);
        const int type = (int)((br.bb >> 1) & 3);
        br.drop(3);
        if (type == 0) {  // stored: skip to a byte boundary, LEN, NLEN
          br.drop(br.left & 7);
          br.refill();
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
          uint32_t *lens = reinterpret_cast<uint32_t *>(sl + kLens);
          for (int i = 0; i < 18; i++) lens[i] = 0x88888888u;        // 0..143
          for (int i = 18; i < 32; i++) lens[i] = 0x99999999u;       // 144..255
          for (int i = 32; i < 35; i++) lens[i] = 0x77777777u;       // 256..279
          lens[35] = 0x88888888u;                                    // 280..287
          for (int i = 36; i < 40; i++) lens[i] = 0x55555555u;       // 288..319: 32 distance codes
          canon_build(sl, 0, 288, kLitSorted, true, lc);
          canon_build(sl, 288, 32, kDistSorted, false, dc);
          state = S_HUFF;
        } else if (type == 2) {  // dynamic codes
          br.refill();
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
              br.refill();
              if (br.left < 3 * hclen) ok = -1;
              else {
#pragma unroll
                for (int i = 0; i < 19; i++) {
                  if (i == 10) br.refill();
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
                br.drop(0);
                br.left -= hlit + hdist;
                ok = br.left < 0 ? -1 : 0;
              } else if (left > 0) {
                ok = 0;
              }
              if (ok == 1) {  // fill the 128-entry table: entries brev(code) + k·2^l
                uint8_t *clt = sl + kClTab;
                for (int s = 0; s < 19; s++) {
                  const int l = (int)((clp >> (3 * s)) & 7);
                  if (l) {
                    const uint32_t cv = (uint32_t)((next >> (8 * l)) & 0xff);
                    next += 1ull << (8 * l);
                    const uint32_t r = __builtin_bitreverse32(cv) >> (32 - l);
                    for (uint32_t j = r; j < 128; j += 1u << l) clt[j] = (uint8_t)((l << 5) | s);
                  }
                }
                // code lengths of hlit + hdist symbols (repeats may cross), one nibble each
                uint32_t *lens = reinterpret_cast<uint32_t *>(sl + kLens);
                const int total = hlit + hdist;
                int n = 0;
                uint32_t prev = 0, acc = 0;
                while (n < total) {
                  br.refill();
                  const uint32_t e = clt[br.peek(7)];
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
                  for (int r = 0; r < rep; r++) {
                    acc |= v << (4 * (n & 7));
                    if ((n & 7) == 7) {
                      lens[n >> 3] = acc;
                      acc = 0;
                    }
                    n++;
                  }
                  prev = v;
                }
                if (ok == 1) {
                  if (n & 7) lens[n >> 3] = acc;
                  if (((lens[32] & 15u) == 0)) ok = 0;  // invalid code -- missing end-of-block
                }
                if (ok == 1 && canon_build(sl, 0, hlit, kLitSorted, true, lc) != 0) ok = 0;
                if (ok == 1 && canon_build(sl, hlit, hdist, kDistSorted, false, dc) != 0) ok = 0;
              }
            }
            if (ok == 1) state = S_HUFF;
            else {
              err = ok == 0 ? INF_DATA : INF_SHORT;
              state = S_DONE;
            }
          }
        } else {
          err = INF_DATA;  // invalid block type
          state = S_DONE;
        }
      }
    } else if (state == S_HUFF) {
      // --- one literal/length symbol (+ its distance) per step
      br.refill();
      int L1;
      bool v1;
      const int i1 = canon_decode(lc, br.bb, L1, v1);
      const uint32_t hb = (litHi[i1 >> 5] >> (i1 & 31)) & 1u;
      const int sym = (int)litS[i1] | (int)(hb << 8);
      if (br.left < L1) {
        err = INF_SHORT;
        state = S_DONE;
      } else if (!v1 || sym > 285) {
        err = INF_DATA;  // invalid literal/length code
        state = S_DONE;
      } else {
        br.drop(L1);
        if (sym < 256) {
          to.put((uint32_t)sym);
          o++;
          if (o == us) state = S_DONE;
        } else if (sym == 256) {
          if (fin) {
            err = INF_SHORT;  // stream end before ISIZE bytes
            state = S_DONE;
          } else {
            state = S_HDR;
          }
        } else {
          const int k = sym - 257;
          const int lx = (k < 8 || k == 28) ? 0 : (k >> 2) - 1;
          const int lb = k < 8 ? k + 3 : k == 28 ? 258 : ((4 | (k & 3)) << lx) + 3;
          if (br.left < lx) {
            err = INF_SHORT;
            state = S_DONE;
          } else {
            const int len = lb + (int)br.peek(lx);
            br.drop(lx);
            br.refill();
            int L2;
            bool v2;
            const int i2 = canon_decode(dc, br.bb, L2, v2);
            const int ds = distS[i2];
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
                  if (to.n == 7) to.put(kTokPad);
                  if (to.n == 8 && !tok_flush(to, pool, pool_next, npages)) {
                    err = INF_OVERFLOW;
                    state = S_DONE;
                  }
                  to.put((uint32_t)(len + 253));
                  to.put((uint32_t)(dist - 1));
                  o = min(o + len, us);
                  if (o == us) state = S_DONE;
                }
              }
            }
          }
        }
      }
    } else if (state == S_STORED) {
      // --- up to 4 stored bytes per step (byte-aligned: bb's low bits are the next byte)
      br.refill();
      const int n = min(min(sleft, 4), us - o);
      int m = 0;
      for (int i = 0; i < 4; i++) {
        if (i < n && br.left >= 8) {
          to.put(br.peek(8));
          br.drop(8);
          if (to.n == 8 && !tok_flush(to, pool, pool_next, npages)) err = INF_OVERFLOW;
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
          state = S_HDR;
        }
      }
    }
    if (state != S_DONE && state != S_EXIT && state != S_NEXT && to.n == 8 &&
        !tok_flush(to, pool, pool_next, npages)) {
      err = INF_OVERFLOW;
      state = S_DONE;
    }
    if (state == S_DONE) {
      if (to.n > 0 && err != INF_OVERFLOW) {
        while (to.n < 8) to.put(kTokPad);
        *reinterpret_cast<uint4 *>(pool + to.cur) = make_uint4(to.t0, to.t1, to.t2, to.t3);
        to.n = 0;
      }
      to.n = 0;
      status[blk] = err;
      found[blk] = err == INF_OVERFLOW ? 0 : o;  // an overflowed block has no complete token stream
      state = S_NEXT;
    }
  }
}

// ---- resolve kernel -------------------------------------------------------------------------------------------
constexpr int kResThreads = 256;
constexpr int kRing = 72;     // per-lane ring stride (64 B used): 18 dwords ⇒ ≤2-way bank conflicts, 8-B aligned
constexpr int kNear = 40;     // copies with (effective) distance <= kNear read the ring

struct TokIn {
  uint32_t t0, t1, t2, t3;
  int n;          // tokens left in t0..t3
  uint64_t cur;   // byte offset of the next chunk in the pool
  uint32_t pnext; // next page of this block
  SB_DEV uint32_t get(const uint8_t *pool) {
    if (n == 0) {
      if ((cur & (kTokPage - 1)) == 0) {
        pnext = *reinterpret_cast<const uint32_t *>(pool + cur);
        cur += 16;
      }
      const uint4 v = *reinterpret_cast<const uint4 *>(pool + cur);
      t0 = v.x;
      t1 = v.y;
      t2 = v.z;
      t3 = v.w;
      cur += 16;
      if ((cur & (kTokPage - 1)) == 0) cur = (uint64_t)pnext * kTokPage;
      n = 8;
    }
    const uint32_t t = t0 & 0xffffu;
    t0 = __builtin_amdgcn_alignbit(t1, t0, 16);
    t1 = __builtin_amdgcn_alignbit(t2, t1, 16);
    t2 = __builtin_amdgcn_alignbit(t3, t2, 16);
    t3 >>= 16;
    n--;
    return t;
  }
};

__global__ __launch_bounds__(kResThreads, 8) void k_inflate_resolve(BlockTable bt, uint8_t *out,
                                                                    const uint8_t *__restrict__ pool,
                                                                    const int32_t *__restrict__ blk_page,
                                                                    const int32_t *__restrict__ found,
                                                                    unsigned int *next_block) {
  __shared__ __attribute__((aligned(16))) uint8_t s_ring[kResThreads * kRing];
  uint8_t *ring = s_ring + threadIdx.x * kRing;
  uint32_t *ring32 = reinterpret_cast<uint32_t *>(ring);

  bool active = false, exited = false;
  uint8_t *a = nullptr, *ae = nullptr, *fl = nullptr;
  TokIn ti{0, 0, 0, 0, 0, 0, 0};
  int crem = 0, eff = 0, npad = 0;

  for (;;) {
    if (!active && !exited) {
      const int64_t b = (int64_t)atomicAdd(next_block, 1u);
      if (b >= bt.n) {
        exited = true;
      } else {
        const int32_t f = found[b];
        const int32_t pg = blk_page[b];
        if (f > 0 && pg >= 0) {
          a = out + bt.uoff[b];
          ae = a + f;
          fl = a;
          ti.n = 0;
          ti.cur = (uint64_t)pg * kTokPage;
          crem = 0;
          npad = 0;
          active = true;
        }
      }
    }
    if (__all(exited)) break;
    if (!active) continue;

    if (crem == 0) {
      const uint32_t t = ti.get(pool);
      if (t < 256) {
        ring[reinterpret_cast<uintptr_t>(a) & 63] = (uint8_t)t;
        a++;
      } else if (t != kTokPad) {
        crem = (int)t - 253;
        eff = (int)ti.get(pool) + 1;
      }
      npad = t == kTokPad ? npad + 1 : 0;
      if (npad > 8) active = false;  // never for a decoded stream: a guard against reading past its end
    }
    if (crem > 0) {
      const int n = min(min(crem, 16), min(eff, (int)(ae - a)));
      const uintptr_t src = reinterpret_cast<uintptr_t>(a) - (uintptr_t)eff;
      uint32_t v0, v1, v2, v3;
      const int sh = (int)(src & 3);
      if (eff <= kNear) {  // source in the ring: 5 dwords around it
        const int q = (int)((src & 63) >> 2);
        const uint32_t s0 = ring32[q & 15], s1 = ring32[(q + 1) & 15], s2 = ring32[(q + 2) & 15],
                       s3 = ring32[(q + 3) & 15], s4 = ring32[(q + 4) & 15];
        v0 = __builtin_amdgcn_alignbyte(s1, s0, sh);
        v1 = __builtin_amdgcn_alignbyte(s2, s1, sh);
        v2 = __builtin_amdgcn_alignbyte(s3, s2, sh);
        v3 = __builtin_amdgcn_alignbyte(s4, s3, sh);
      } else {  // source already stored to HBM (it lies below the flushed mark)
        const uint32_t *g = reinterpret_cast<const uint32_t *>(src & ~(uintptr_t)3);
        const uint4 x = *reinterpret_cast<const uint4 *>(g);
        const uint32_t x4 = g[4];
        v0 = __builtin_amdgcn_alignbyte(x.y, x.x, sh);
        v1 = __builtin_amdgcn_alignbyte(x.z, x.y, sh);
        v2 = __builtin_amdgcn_alignbyte(x.w, x.z, sh);
        v3 = __builtin_amdgcn_alignbyte(x4, x.w, sh);
      }
      // write 16 bytes at a (bytes past a + n are scratch, rewritten before they are flushed):
      // head bytes up to the next dword boundary, then 4 aligned dwords
      const uintptr_t aa = reinterpret_cast<uintptr_t>(a);
      const int h = (int)((4 - (aa & 3)) & 3);
#pragma unroll
      for (int k = 0; k < 3; k++)
        if (k < h) ring[(aa + k) & 63] = (uint8_t)(v0 >> (8 * k));
      const uint32_t w0 = __builtin_amdgcn_alignbyte(v1, v0, h), w1 = __builtin_amdgcn_alignbyte(v2, v1, h),
                     w2 = __builtin_amdgcn_alignbyte(v3, v2, h), w3 = __builtin_amdgcn_alignbyte(0u, v3, h);
      const int q = (int)(((aa + h) & 63) >> 2);
      ring32[q & 15] = w0;
      ring32[(q + 1) & 15] = w1;
      ring32[(q + 2) & 15] = w2;
      ring32[(q + 3) & 15] = w3;
      a += n;
      crem -= n;
      if (n == eff && eff < 16) eff *= 2;  // the copied bytes extend the period: distance 2·eff is valid
    }
    // flush: a block's partial first chunk (shared with the previous block) as bytes, then aligned 16-B chunks
    {
      const uintptr_t f = reinterpret_cast<uintptr_t>(fl);
      if (f & 15) {
        const uintptr_t hd = (f & ~(uintptr_t)15) + 16;
        if (reinterpret_cast<uintptr_t>(a) >= hd || a == ae) {
          const uintptr_t lim = reinterpret_cast<uintptr_t>(a) < hd ? reinterpret_cast<uintptr_t>(a) : hd;
          for (uintptr_t x = f; x < lim; x++) *reinterpret_cast<uint8_t *>(x) = ring[x & 63];
          fl = reinterpret_cast<uint8_t *>(lim);
        }
      }
      while ((reinterpret_cast<uintptr_t>(fl) & 15) == 0 && a - fl >= 16) {
        const uint2 lo = *reinterpret_cast<const uint2 *>(ring + (reinterpret_cast<uintptr_t>(fl) & 63));
        const uint2 hi = *reinterpret_cast<const uint2 *>(ring + ((reinterpret_cast<uintptr_t>(fl) + 8) & 63));
        *reinterpret_cast<uint4 *>(fl) = make_uint4(lo.x, lo.y, hi.x, hi.y);
        fl += 16;
      }
      if (a == ae) {  // tail (shared with the next block) as bytes
        for (uint8_t *x = fl; x < ae; x++) *x = ring[reinterpret_cast<uintptr_t>(x) & 63];
        fl = ae;
        active = false;
      }
    }
  }
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

hipError_t launch_inflate_tokens(const uint8_t *d, int64_t D, BlockTable bt, uint8_t *out, uint8_t *pool,
                                 uint32_t npages, int32_t *blk_page, int32_t *status, int32_t *found,
                                 unsigned int *counters, int dec_wgs, int res_wgs, hipStream_t s) {
  if (bt.n == 0) return hipSuccess;
  // counters: [0] decode work, [1] pool pages used, [2] resolve work
  (void)hipMemsetAsync(counters, 0, 3 * sizeof(unsigned int), s);
  hipLaunchKernelGGL(k_inflate_decode, dim3((unsigned)dec_wgs), dim3(kDecThreads), 0, s, d, D, bt, pool, npages,
                     counters + 1, blk_page, status, found, counters + 0);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_inflate_resolve, dim3((unsigned)res_wgs), dim3(kResThreads), 0, s, bt, out, pool, blk_page,
                     found, counters + 2);
  return hipGetLastError();
}

}  // namespace sbam
