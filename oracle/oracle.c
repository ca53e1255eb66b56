/*
 * oracle.c — CPU restatement of spark-bam's split/check/decode hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product path (spark-bam_amd/) links,
 * loads or calls this file.  It is the checker the parity tests, smoke() and
 * bench.py's cpu_baseline leg compare the HIP path against.
 *
 * The reference (Scala 2.11 / Spark / htsjdk) cannot be compiled or run in this
 * image (no JDK, scalac, sbt; no network) — see DESIGN.md §Oracle.  This file
 * restates its algorithm function by function, citing the Scala file:line it
 * follows (paths relative to the reference root).  It is pinned by the
 * reference's own fixtures and golden outputs (tests/test_oracle_*.py):
 *   - .blocks / .records sidecars of every test BAM
 *   - cli/src/test/resources/output/full-check/ per-flag totals
 *   - ComputeSplitsTest / LoadBAMTest split and partition goldens
 *   - full/CheckerTest point cases, FindBlockStartTest, FindRecordStartTest
 *
 * Third-party arithmetic: raw-DEFLATE decoding is done by the system zlib
 * (1.2.11), the same library family as the JDK's java.util.zip.Inflater that the
 * reference calls at bgzf/.../block/Stream.scala:49-54.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <zlib.h>

#define OR_OK 0
#define OR_ERR_HEADER_PARSE 1   /* HeaderParseException        (HeaderParseException.scala) */
#define OR_ERR_HEADER_SEARCH 2  /* HeaderSearchFailedException (FindBlockStart.scala:31-35) */
#define OR_ERR_INFLATE 3        /* IOException "Expected N decompressed bytes, found M" (Stream.scala:52-54) */
#define OR_ERR_CAPACITY 4
#define OR_ERR_NOT_BAM 5        /* require(... == "BAM\1") (bam/header/Header.scala:44-46) */

static inline uint32_t u16le(const uint8_t *d, int64_t i) { return (uint32_t)d[i] | ((uint32_t)d[i + 1] << 8); }
static inline int32_t i32le(const uint8_t *d, int64_t i) {
  return (int32_t)((uint32_t)d[i] | ((uint32_t)d[i + 1] << 8) | ((uint32_t)d[i + 2] << 16) | ((uint32_t)d[i + 3] << 24));
}

/* ------------------------------------------------------------------------------------------------
 * BGZF layer
 * ---------------------------------------------------------------------------------------------- */

/* Header.make (bgzf/.../block/Header.scala:48-83).  Returns 0 if the 18 bytes at d[c..c+18) parse,
 * else 1 with idx, actual, expected describing the
 * HeaderParseException(idx, actual, expected). Byte 15 is not checked; BC is assumed first subfield. */
static int header_make(const uint8_t *d, int64_t c, int32_t *hsize, int32_t *csize, int32_t *idx, int32_t *actual,
                       int32_t *expected) {
  static const int idxs[7] = {0, 1, 2, 3, 12, 13, 14};
  static const int exps[7] = {31, 139, 8, 4, 66, 67, 2};
  for (int j = 0; j < 7; j++) {
    if (d[c + idxs[j]] != (uint8_t)exps[j]) {
      if (idx) *idx = idxs[j];
      if (actual) *actual = (int8_t)d[c + idxs[j]]; /* Scala Byte is signed */
      if (expected) *expected = (int8_t)(uint8_t)exps[j];
      return 1;
    }
  }
  int32_t xlen = (int32_t)u16le(d, c + 10);
  *hsize = 18 + xlen - 6;
  *csize = (int32_t)u16le(d, c + 16) + 1;
  return 0;
}

/* MetadataStream._advance (bgzf/.../block/MetadataStream.scala:23-54), iterated from `from`.
 * Stops (like the Scala iterator's None) on EOF inside the 18-B header, on an ISIZE read past EOF,
 * and on the first block whose deflate payload is 2 bytes (empty block / EOF marker).
 * Returns the number of blocks emitted, or -1 on HeaderParseException (err_* filled). */
int64_t or_metadata_stream(const uint8_t *d, int64_t D, int64_t from, int64_t max_blocks, int64_t *start,
                           int32_t *csize, int32_t *usize, int32_t *hsize, int64_t *err_pos, int32_t *err_idx,
                           int32_t *err_actual, int32_t *err_expected) {
  int64_t c = from, n = 0;
  while (n < max_blocks) {
    if (c + 18 > D) break; /* EOFException in Header(ch) → None */
    int32_t hs, cs, ei, ea, ee;
    if (header_make(d, c, &hs, &cs, &ei, &ea, &ee)) {
      if (err_pos) *err_pos = c;
      if (err_idx) *err_idx = ei;
      if (err_actual) *err_actual = ea;
      if (err_expected) *err_expected = ee;
      return -1;
    }
    if (c + cs > D) break; /* ch.getInt of ISIZE past EOF → EOFException → None */
    int32_t isize = i32le(d, c + cs - 4);
    if (cs - hs - 8 == 2) break; /* dataLength == 2: empty block ends the stream (:131-133) */
    if (start) start[n] = c;
    if (csize) csize[n] = cs;
    if (usize) usize[n] = isize;
    if (hsize) hsize[n] = hs;
    n++;
    c += cs;
  }
  return n;
}

/* FindBlockStart.apply (bgzf/.../block/FindBlockStart.scala:8-36): first start+pos, pos < 65536
 * (Block.MAX_BLOCK_SIZE), at which MetadataStream.take(n) raises no HeaderParseException.
 * Returns OR_OK with *out, or OR_ERR_HEADER_SEARCH. */
int or_find_block_start(const uint8_t *d, int64_t D, int64_t start, int32_t n, int64_t *out) {
  for (int64_t pos = 0; pos < 65536; pos++) {
    int64_t c = start + pos;
    int ok = 1;
    for (int32_t j = 0; j < n; j++) {
      if (c + 18 > D) break;
      int32_t hs, cs;
      if (header_make(d, c, &hs, &cs, 0, 0, 0)) {
        ok = 0;
        break;
      }
      if (c + cs > D) break;
      if (cs - hs - 8 == 2) break;
      c += cs;
    }
    if (ok) {
      *out = start + pos;
      return OR_OK;
    }
  }
  return OR_ERR_HEADER_SEARCH;
}

/* StreamI._advance (bgzf/.../block/Stream.scala:31-71) over the blocks of or_metadata_stream:
 * raw inflate (Inflater(nowrap=true)) of each payload [c+hsize, c+csize-8) into ISIZE bytes; the
 * count produced must equal ISIZE.  CRC32 is never checked (as in the reference).  Writes the
 * concatenated stream to out (capacity out_cap) and per-block uncompressed offsets to uoff.
 * Returns total uncompressed bytes, or -1 (err_block = failing block index, err_found = bytes). */
int64_t or_inflate_blocks(const uint8_t *d, int64_t nblocks, const int64_t *start, const int32_t *csize,
                          const int32_t *usize, const int32_t *hsize, uint8_t *out, int64_t out_cap, int64_t *uoff,
                          int64_t *err_block, int64_t *err_found) {
  int64_t total = 0;
  z_stream zs;
  for (int64_t b = 0; b < nblocks; b++) {
    if (uoff) uoff[b] = total;
    if (total + usize[b] > out_cap) {
      if (err_block) *err_block = b;
      if (err_found) *err_found = -2;
      return -1;
    }
    memset(&zs, 0, sizeof(zs));
    if (inflateInit2(&zs, -15) != Z_OK) return -1;
    zs.next_in = (Bytef *)(d + start[b] + hsize[b]);
    zs.avail_in = (uInt)(csize[b] - hsize[b] - 8);
    zs.next_out = out + total;
    zs.avail_out = (uInt)usize[b];
    int rc = inflate(&zs, Z_FINISH);
    int64_t produced = (int64_t)usize[b] - zs.avail_out;
    inflateEnd(&zs);
    if ((rc != Z_STREAM_END && rc != Z_BUF_ERROR && rc != Z_OK) || produced != usize[b]) {
      if (err_block) *err_block = b;
      if (err_found) *err_found = produced;
      return -1;
    }
    total += usize[b];
  }
  return total;
}

/* ------------------------------------------------------------------------------------------------
 * BAM header (check/.../bam/header/Header.scala:26-60)
 * ---------------------------------------------------------------------------------------------- */

/* Parses "BAM\1", l_text, skips text, n_ref × (l_name, name, l_ref).  Returns n_ref (lengths written
 * up to cap) and *end_off = uncompressed offset just past the header, or -OR_ERR_NOT_BAM. */
int32_t or_bam_header(const uint8_t *u, int64_t L, int64_t *lens, int32_t cap, int64_t *end_off) {
  if (L < 12 || memcmp(u, "BAM\1", 4) != 0) return -OR_ERR_NOT_BAM;
  int64_t x = 4;
  int32_t l_text = i32le(u, x);
  x += 4 + (int64_t)l_text;
  int32_t n_ref = i32le(u, x);
  x += 4;
  for (int32_t i = 0; i < n_ref; i++) {
    int32_t l_name = i32le(u, x);
    x += 4 + (int64_t)l_name;
    int32_t l_ref = i32le(u, x);
    x += 4;
    if (i < cap) lens[i] = l_ref;
  }
  *end_off = x;
  return n_ref;
}

/* ------------------------------------------------------------------------------------------------
 * Record-boundary checker
 * ---------------------------------------------------------------------------------------------- */

/* Result word: bits 0..18 = Flags in bitset order (check/.../full/error/Flags.scala:201-223),
 * bits 24..30 = readsBeforeError / Success.readsParsed, bit 31 = Success. */
#define F_TOO_FEW_FIXED 0
#define F_NEG_IDX 1
#define F_BIG_IDX 2
#define F_NEG_POS 3
#define F_BIG_POS 4
#define F_NEG_NIDX 5
#define F_BIG_NIDX 6
#define F_NEG_NPOS 7
#define F_BIG_NPOS 8
#define F_FEW_NAME 9
#define F_NON_NULL 10
#define F_NON_ASCII 11
#define F_NO_NAME 12
#define F_EMPTY_NAME 13
#define F_FEW_CIGAR 14
#define F_BAD_CIGAR 15
#define F_EMPTY_MAPPED_CIGAR 16
#define F_EMPTY_MAPPED_SEQ 17
#define F_FEW_REMAINING 18
#define W_SUCCESS 0x80000000u
#define W_K(k) (((uint32_t)(k) & 0x7f) << 24)

/* Checker.allowedReadNameChars = ('!' to '?') ++ ('A' to '~')  (check/.../check/Checker.scala:12-17) */
static inline int name_char_ok(uint8_t b) { return (b >= 33 && b <= 63) || (b >= 65 && b <= 126); }

/* PosChecker.getRefPosError (check/.../check/PosChecker.scala:43-63) as 4 bits
 * {negIdx, bigIdx, negPos, bigPos} in that order. */
static inline uint32_t ref_err(int32_t ri, int32_t rp, const int64_t *lens, int32_t nref) {
  if (ri < -1) return 1u | (rp < -1 ? 4u : 0u);
  if (ri >= nref) return 2u | (rp < -1 ? 4u : 0u);
  if (rp < -1) return 4u;
  if (ri >= 0 && (int64_t)rp > lens[ri]) return 8u;
  return 0u;
}

/* full.Checker.apply + build (check/.../check/full/Checker.scala:22-184) at uncompressed offset p of
 * the stream u[0..L).  Java int32 arithmetic (wrap, '/' toward zero) where the Scala uses Int;
 * offsets are int64 (nextOffset is a Long, :53). */
static inline uint32_t check_full_core(const uint8_t *u, int64_t L, const int64_t *lens, int32_t nref, int64_t p,
                                       int32_t R, int *hit) {
  int64_t s = p, a = p;
  int32_t k = 0;
  for (;;) {
    if (k == R) return W_SUCCESS | W_K(k); /* :27-28 */
    if (a + 36 > L) {                     /* readFully(buf) fails (:31-48) */
      *hit = 1;
      if (k > 0 && s == L) return W_SUCCESS | W_K(k);
      return (1u << F_TOO_FEW_FIXED) | W_K(k);
    }
    int32_t bs = i32le(u, a), ri = i32le(u, a + 4), rp = i32le(u, a + 8), bmn = i32le(u, a + 12);
    int32_t fnc = i32le(u, a + 16), ls = i32le(u, a + 20), nri = i32le(u, a + 24), nrp = i32le(u, a + 28);
    uint32_t F = ref_err(ri, rp, lens, nref) << F_NEG_IDX;
    int32_t lrn = bmn & 0xff;                      /* :57 */
    uint32_t flag = ((uint32_t)fnc) >> 16;         /* :61 */
    int32_t nc = fnc & 0xffff;                     /* :63 */
    int32_t t = (int32_t)((uint32_t)ls + 1u);      /* (seqLen + 1) in Int */
    int32_t nsq = (int32_t)((uint32_t)(t / 2) + (uint32_t)ls); /* (seqLen+1)/2 + seqLen (:68) */
    int32_t implied = (int32_t)(32u + (uint32_t)lrn + 4u * (uint32_t)nc + (uint32_t)nsq);
    if (bs < implied) F |= 1u << F_FEW_REMAINING; /* :70-71 */
    F |= ref_err(nri, nrp, lens, nref) << F_NEG_NIDX;
    int64_t c = a + 36;
    if (lrn == 0) {
      F |= 1u << F_NO_NAME;
    } else if (lrn == 1) {
      F |= 1u << F_EMPTY_NAME;
    } else {
      if (c + lrn > L) { /* readFully(readNameBuffer) EOF → TooFewBytesForReadName, cigar unevaluated (:140-144) */
        *hit = 1;
        F |= 1u << F_FEW_NAME;
        return F | W_K(k);
      }
      if (u[c + lrn - 1] != 0) {
        F |= 1u << F_NON_NULL;
      } else {
        for (int32_t i = 0; i < lrn - 1; i++)
          if (!name_char_ok(u[c + i])) {
            F |= 1u << F_NON_ASCII;
            break;
          }
      }
      c += lrn;
    }
    int cig_err = 0; /* :111-136 */
    for (int32_t i = 0; i < nc; i++) {
      if (c + 4 > L) {
        *hit = 1;
        F |= 1u << F_FEW_CIGAR;
        cig_err = 1;
        break;
      }
      uint8_t op = u[c];
      c += 4;
      if ((op & 0xf) > 8) {
        F |= 1u << F_BAD_CIGAR;
        cig_err = 1;
        break;
      }
    }
    if (!cig_err && (flag & 4u) == 0 && (ls == 0 || nc == 0)) {
      /* EmptyMapped(emptySeq, emptyCigar) feeds (emptyMappedCigar, emptyMappedSeq): swapped names
       * (full/Checker.scala:123-129, error/CigarOpsError.scala:22-24) */
      if (ls == 0) F |= 1u << F_EMPTY_MAPPED_CIGAR;
      if (nc == 0) F |= 1u << F_EMPTY_MAPPED_SEQ;
    }
    if (F) return F | W_K(k);
    int64_t nxt = s + 4 + (int64_t)bs; /* :53, :167-172 */
    if (nxt > L) *hit = 1;
    if (nxt > c)
      a = nxt > L ? L : nxt; /* skip past EOF: parity unpinned; clamp */
    else
      a = c;
    s = nxt;
    k++;
  }
}

uint32_t or_check_full(const uint8_t *u, int64_t L, const int64_t *lens, int32_t nref, int64_t p, int32_t R) {
  int hit = 0;
  return check_full_core(u, L, lens, nref, p, R, &hit);
}

/* eager.Checker.apply (check/.../check/eager/Checker.scala:24-126): same checks, boolean result;
 * it succeeds exactly when the full checker returns Success. */
int or_check_eager(const uint8_t *u, int64_t L, const int64_t *lens, int32_t nref, int64_t p, int32_t R) {
  return (or_check_full(u, L, lens, nref, p, R) & W_SUCCESS) != 0;
}

/* Batch: words for positions [p0, p1). */
void or_check_full_range(const uint8_t *u, int64_t L, const int64_t *lens, int32_t nref, int64_t p0, int64_t p1,
                         int32_t R, uint32_t *words) {
  for (int64_t p = p0; p < p1; p++) words[p - p0] = or_check_full(u, L, lens, nref, p, R);
}

/* Counts reduction (check/.../full/error/Counts.scala; cli/.../full/FullCheck.scala:141-191):
 * results equal to Flags.TooFewFixedBlockBytes (flag 0 only, k=0) are dropped; every other Flags
 * result is keyed by numNonZeroFields = popcount(flags) + (k > 0).
 *   counts[key*19 + f]  += flag f set                  (key 0..20)
 *   npos[key]           += 1
 *   rbe[key*128 + k]    += 1 if k > 0 (readsBeforeError histogram)
 * plus n_success. */
void or_counts_range(const uint8_t *u, int64_t L, const int64_t *lens, int32_t nref, int64_t p0, int64_t p1,
                     int32_t R, int64_t *counts, int64_t *npos, int64_t *rbe, int64_t *n_success) {
  for (int64_t p = p0; p < p1; p++) {
    uint32_t w = or_check_full(u, L, lens, nref, p, R);
    if (w & W_SUCCESS) {
      (*n_success)++;
      continue;
    }
    uint32_t F = w & 0x7ffff;
    uint32_t k = (w >> 24) & 0x7f;
    if (F == 1u && k == 0) continue;
    int key = __builtin_popcount(F) + (k > 0);
    npos[key]++;
    for (int f = 0; f < 19; f++)
      if (F & (1u << f)) counts[key * 19 + f]++;
    if (k > 0) rbe[key * 128 + k]++;
  }
}

/* FindRecordStart.withDelta (check/.../bam/spark/FindRecordStart.scala:30-63) in flat offsets:
 * first x in [x0, min(L, x0+max_read_size)) with eager(x); returns x or -1 (None). */
int64_t or_find_record_start(const uint8_t *u, int64_t L, const int64_t *lens, int32_t nref, int64_t x0,
                             int32_t R, int64_t max_read_size) {
  for (int64_t i = 0; i < max_read_size; i++) {
    int64_t x = x0 + i;
    if (x >= L) return -1;
    if (or_check_eager(u, L, lens, nref, x, R)) return x;
  }
  return -1;
}

/* RecordStream / PosStream chain (check/.../bam/iterator/RecordStream.scala:27-41, PosStream.scala:14-22):
 * r0 = x0, r_{j+1} = r_j + 4 + block_size(r_j), while r_j < x_end and a full 4-byte block_size is
 * readable.  Writes up to cap offsets; returns the number of records (truncated record at EOF
 * ends the stream: UnexpectedEOF, RecordStream.scala:35-36,44-46). */
int64_t or_record_chain(const uint8_t *u, int64_t L, int64_t x0, int64_t x_end, int64_t *out, int64_t cap) {
  int64_t n = 0, x = x0;
  while (x < x_end && x + 4 <= L) {
    int32_t bs = i32le(u, x);
    if (x + 4 + (int64_t)bs > L) break;
    if (n < cap && out) out[n] = x;
    n++;
    x = x + 4 + (int64_t)bs;
  }
  return n;
}

/* ------------------------------------------------------------------------------------------------
 * Windowed forms for oracle runs over files larger than memory (tools/pin_bench_digests.py).  The
 * stream is held as a window u[0..L) that is a prefix of the rest of the file: a position's result
 * equals the whole file's unless its evaluation reached the window's end (one of the `> L` tests
 * above fired), which these functions count in *hits so that the caller can widen the window.
 * ---------------------------------------------------------------------------------------------- */

/* or_counts_range + the close-call pair histogram of key-2 results (FullCheck.scala:141-191: the
 * first two flags, or (flag, flag) when the second non-zero field is readsBeforeError) and the
 * TooFewFixedBlockBytes-only results dropped from the Counts.  scal = {n_success, n_too_few_fixed, hits}. */
void or_counts_window(const uint8_t *u, int64_t L, const int64_t *lens, int32_t nref, int64_t p0, int64_t p1,
                      int32_t R, int64_t *counts, int64_t *npos, int64_t *rbe, int64_t *pair, int64_t *scal) {
  for (int64_t p = p0; p < p1; p++) {
    int hit = 0;
    uint32_t w = check_full_core(u, L, lens, nref, p, R, &hit);
    scal[2] += hit;
    if (w & W_SUCCESS) {
      scal[0]++;
      continue;
    }
    uint32_t F = w & 0x7ffff;
    uint32_t k = (w >> 24) & 0x7f;
    if (F == 1u && k == 0) {
      scal[1]++;
      continue;
    }
    int key = __builtin_popcount(F) + (k > 0);
    npos[key]++;
    for (int f = 0; f < 19; f++)
      if (F & (1u << f)) counts[key * 19 + f]++;
    if (k > 0) rbe[key * 128 + k]++;
    if (key == 2) {
      int f0 = __builtin_ctz(F);
      uint32_t rest = F & (F - 1);
      int f1 = rest ? __builtin_ctz(rest) : f0;
      pair[f0 * 19 + f1]++;
    }
  }
}

/* or_find_record_start with the window-end test counted in *hits. */
int64_t or_find_record_start_window(const uint8_t *u, int64_t L, const int64_t *lens, int32_t nref, int64_t x0,
                                    int32_t R, int64_t max_read_size, int64_t *hits) {
  for (int64_t i = 0; i < max_read_size; i++) {
    int64_t x = x0 + i;
    if (x >= L) {
      (*hits)++;
      return -1;
    }
    int hit = 0;
    uint32_t w = check_full_core(u, L, lens, nref, x, R, &hit);
    *hits += hit;
    if (w & W_SUCCESS) return x;
  }
  return -1;
}
