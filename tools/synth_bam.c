/*
 * synth_bam.c — deterministic synthetic BAM generator for the benchmark workloads.
 *
 * Produces a BGZF "tile": a run of BAM records, Illumina-like (150 bp paired reads by default), cut into
 * htsjdk-style 65498-byte uncompressed payloads and compressed with zlib level 6 (raw DEFLATE, BGZF header
 * with the BC subfield, CRC32, ISIZE).  Records are NOT block-aligned (they straddle blocks), except that the
 * tile ends on a record boundary, so a file = header blocks + tile × k + EOF marker is a valid BAM whose record
 * chain runs through every tile seam.  read_len > 1000 gives fixed-length long reads with a few ops;
 * read_len == 0 is the long-read config of SURVEY §8(d) #5 (ONT/PacBio-like, bam_long_record): log-normal
 * lengths 10–50 kb (median 20 kb), 200–3000 CIGAR ops, names up to 63 characters, unpaired, and ~5% of
 * records larger than a 64 KiB BGZF block.
 *
 * Contig set: the 84 GRCh37 contigs of the reference's 2.bam header (ContigLengthsTest.scala:15-102).  A short-read
 * tile visits all 84 in order, an equal run of records on each (positions wrap inside the contig, so the smallest
 * GL contigs stay in range); synth_unplaced makes the WGS tail of unplaced pairs (refID = pos = -1 for the read and
 * its mate) that a coordinate-sorted BAM ends with.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <math.h>
#include <zlib.h>

#define PAYLOAD 65498

static const char *kNames[] = {
    "1", "2", "3", "4", "5", "6", "7", "8", "9", "10", "11", "12", "13", "14", "15", "16", "17", "18", "19", "20",
    "21", "22", "X", "Y", "MT", "GL000207.1", "GL000226.1", "GL000229.1", "GL000231.1", "GL000210.1", "GL000239.1",
    "GL000235.1", "GL000201.1", "GL000247.1", "GL000245.1", "GL000197.1", "GL000203.1", "GL000246.1", "GL000249.1",
    "GL000196.1", "GL000248.1", "GL000244.1", "GL000238.1", "GL000202.1", "GL000234.1", "GL000232.1", "GL000206.1",
    "GL000240.1", "GL000236.1", "GL000241.1", "GL000243.1", "GL000242.1", "GL000230.1", "GL000237.1", "GL000233.1",
    "GL000204.1", "GL000198.1", "GL000208.1", "GL000191.1", "GL000227.1", "GL000228.1", "GL000214.1", "GL000221.1",
    "GL000209.1", "GL000218.1", "GL000220.1", "GL000213.1", "GL000211.1", "GL000199.1", "GL000217.1", "GL000216.1",
    "GL000215.1", "GL000205.1", "GL000219.1", "GL000224.1", "GL000223.1", "GL000195.1", "GL000212.1", "GL000222.1",
    "GL000200.1", "GL000193.1", "GL000194.1", "GL000225.1", "GL000192.1"};
static const int64_t kLens[] = {
    249250621, 243199373, 198022430, 191154276, 180915260, 171115067, 159138663, 146364022, 141213431, 135534747,
    135006516, 133851895, 115169878, 107349540, 102531392, 90354753, 81195210, 78077248, 59128983, 63025520,
    48129895, 51304566, 155270560, 59373566, 16569, 4262, 15008, 19913, 27386, 27682, 33824, 34474, 36148, 36422,
    36651, 37175, 37498, 38154, 38502, 38914, 39786, 39929, 39939, 40103, 40531, 40652, 41001, 41933, 41934, 42152,
    43341, 43523, 43691, 45867, 45941, 81310, 90085, 92689, 106433, 128374, 129120, 137718, 155397, 159169, 161147,
    161802, 164239, 166566, 169874, 172149, 172294, 172545, 174588, 179198, 179693, 180455, 182896, 186858, 186861,
    187035, 189789, 191469, 211173, 547496};
#define NREF 84

/* splitmix64 */
typedef struct { uint64_t s; } rng_t;
static inline uint64_t rnext(rng_t *r) {
  uint64_t z = (r->s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
static inline uint32_t runi(rng_t *r, uint32_t n) { return (uint32_t)(((rnext(r) >> 32) * (uint64_t)n) >> 32); }

typedef struct { uint8_t *p; int64_t n, cap; } buf_t;
static void bput(buf_t *b, const void *src, int64_t n) {
  if (b->n + n > b->cap) {
    int64_t c = b->cap ? b->cap : 1 << 20;
    while (c < b->n + n) c *= 2;
    b->p = (uint8_t *)realloc(b->p, (size_t)c);
    b->cap = c;
  }
  memcpy(b->p + b->n, src, (size_t)n);
  b->n += n;
}
static void bput32(buf_t *b, uint32_t v) { bput(b, &v, 4); }
static void bput16(buf_t *b, uint16_t v) { bput(b, &v, 2); }

/* SAM spec reg2bin (0-based, end exclusive) */
static int reg2bin(int beg, int end) {
  --end;
  if (beg >> 14 == end >> 14) return ((1 << 15) - 1) / 7 + (beg >> 14);
  if (beg >> 17 == end >> 17) return ((1 << 12) - 1) / 7 + (beg >> 17);
  if (beg >> 20 == end >> 20) return ((1 << 9) - 1) / 7 + (beg >> 20);
  if (beg >> 23 == end >> 23) return ((1 << 6) - 1) / 7 + (beg >> 23);
  if (beg >> 26 == end >> 26) return ((1 << 3) - 1) / 7 + (beg >> 26);
  return 0;
}

static void bam_header(buf_t *b) {
  const char *text = "@HD\tVN:1.5\tSO:coordinate\n@RG\tID:grp1\tSM:synthetic\tPL:ILLUMINA\n";
  bput(b, "BAM\1", 4);
  bput32(b, (uint32_t)strlen(text));
  bput(b, text, (int64_t)strlen(text));
  bput32(b, NREF);
  for (int i = 0; i < NREF; i++) {
    bput32(b, (uint32_t)strlen(kNames[i]) + 1);
    bput(b, kNames[i], (int64_t)strlen(kNames[i]) + 1);
    bput32(b, (uint32_t)kLens[i]);
  }
}

static const uint8_t kQualBins[8] = {2, 6, 15, 22, 27, 33, 37, 40};
static const uint8_t kQualCdf[8] = {2, 5, 12, 22, 35, 55, 130, 255}; /* skewed high, /255 */

/* One record; read_len query bases.  ctx: running coordinate state. */
typedef struct { int32_t ref; int32_t pos; uint64_t serial; int64_t left, per; } coord_t;

static void bam_record(buf_t *b, rng_t *r, coord_t *co, int read_len, uint8_t *rec) {
  int n = 0;
  char name[64];
  const uint64_t pair = co->serial / 2;
  const int second = (int)(co->serial & 1);
  rng_t pr = {pair * 0x9E3779B97F4A7C15ull + 12345};
  snprintf(name, sizeof name, "SYN:1:FC:%u:%u:%u:%u", 1 + runi(&pr, 8), 1101 + runi(&pr, 1128), runi(&pr, 30000),
           runi(&pr, 200000));
  const int lrn = (int)strlen(name) + 1;
  const int unmapped = runi(r, 1000) < 5;
  co->pos += (int32_t)runi(r, 40);
  if (co->left-- <= 0) { co->ref = (co->ref + 1) % NREF; co->pos = 400; co->left = co->per - 1; }
  if (co->pos + 2400 > kLens[co->ref]) co->pos = 400; /* mates stay inside [50, len) */
  const int32_t pos = co->pos;
  const int32_t mpos = second ? pos - 250 - (int32_t)runi(&pr, 100) : pos + 250 + (int32_t)runi(&pr, 100);
  uint32_t cig[8];
  int nc = 0;
  int ref_span = read_len;
  if (unmapped) {
    nc = 0;
  } else if (read_len > 1000) { /* long read: many ops */
    int rem = read_len;
    nc = 0;
    ref_span = 0;
    while (rem > 0 && nc < 7) {
      int m = rem > 4000 ? 1000 + (int)runi(r, 3000) : rem;
      cig[nc++] = ((uint32_t)m << 4) | 0; /* M */
      ref_span += m;
      rem -= m;
      if (rem > 0 && nc < 7) {
        int ins = 1 + (int)runi(r, 5);
        if (ins > rem) ins = rem;
        cig[nc++] = ((uint32_t)ins << 4) | 1; /* I */
        rem -= ins;
      }
    }
    if (rem > 0) { cig[nc - 1] += (uint32_t)rem << 4; if ((cig[nc - 1] & 0xf) == 0) ref_span += rem; }
  } else if (runi(r, 10) < 9) {
    nc = 1;
    cig[0] = ((uint32_t)read_len << 4) | 0;
  } else {
    const int kind = (int)runi(r, 4);
    const int a = 10 + (int)runi(r, (uint32_t)(read_len - 30));
    if (kind == 0) { cig[0] = (uint32_t)a << 4 | 4; cig[1] = (uint32_t)(read_len - a) << 4 | 0; nc = 2; ref_span = read_len - a; }
    else if (kind == 1) { const int i = 1 + (int)runi(r, 4); cig[0] = (uint32_t)a << 4; cig[1] = (uint32_t)i << 4 | 1; cig[2] = (uint32_t)(read_len - a - i) << 4; nc = 3; ref_span = read_len - i; }
    else if (kind == 2) { const int d = 1 + (int)runi(r, 4); cig[0] = (uint32_t)a << 4; cig[1] = (uint32_t)d << 4 | 2; cig[2] = (uint32_t)(read_len - a) << 4; nc = 3; ref_span = read_len + d; }
    else { const int s1 = 5 + (int)runi(r, 10), s2 = 5 + (int)runi(r, 10), m = read_len - s1 - s2;
      cig[0] = (uint32_t)s1 << 4 | 4; cig[1] = (uint32_t)m << 4; cig[2] = (uint32_t)s2 << 4 | 4; nc = 3; ref_span = m; }
  }
  uint16_t flag = 1 | 2 | (second ? 128 : 64) | (second ? 16 : 32);
  if (unmapped) flag = (uint16_t)((flag & ~2) | 4);
  const uint8_t mapq = unmapped ? 0 : (uint8_t)runi(r, 61);
  const int bin = reg2bin(pos, pos + (ref_span > 0 ? ref_span : 1));
  /* fixed fields */
#define W32(v) do { uint32_t t_ = (uint32_t)(v); memcpy(rec + n, &t_, 4); n += 4; } while (0)
#define W16(v) do { uint16_t t_ = (uint16_t)(v); memcpy(rec + n, &t_, 2); n += 2; } while (0)
#define W8(v) do { rec[n++] = (uint8_t)(v); } while (0)
  W32(0); /* block_size placeholder */
  W32(co->ref);
  W32(pos);
  W8(lrn); W8(mapq); W16(bin);
  W16(nc); W16(flag);
  W32(read_len);
  W32(co->ref);
  W32(mpos);
  W32(second ? -(int32_t)(pos - mpos + 150) : (int32_t)(mpos - pos + 150));
  memcpy(rec + n, name, (size_t)lrn); n += lrn;
  for (int i = 0; i < nc; i++) W32(cig[i]);
  static const uint8_t codes[4] = {1, 2, 4, 8};
  for (int i = 0; i < read_len; i += 2) {
    uint8_t hi = runi(r, 1000) == 0 ? 15 : codes[rnext(r) & 3];
    uint8_t lo = (i + 1 < read_len) ? (runi(r, 1000) == 0 ? 15 : codes[rnext(r) & 3]) : 0;
    W8((hi << 4) | lo);
  }
  uint8_t prevq = 37;
  for (int i = 0; i < read_len; i++) { /* binned qualities with runs (Markov: repeat the previous bin 60%) */
    if (runi(r, 10) >= 6 || i == 0) {
      const uint32_t u = runi(r, 256);
      int k = 0;
      while (k < 7 && u > kQualCdf[k]) k++;
      prevq = kQualBins[k];
    }
    W8(prevq);
  }
  /* tags: NM:c MD:Z AS:C XS:C RG:Z */
  const int nm = (int)runi(r, 4);
  W8('N'); W8('M'); W8('c'); W8(nm);
  W8('M'); W8('D'); W8('Z');
  n += sprintf((char *)rec + n, "%d", read_len > 1000 ? 1000 : read_len); rec[n++] = 0;
  W8('A'); W8('S'); W8('C'); W8(read_len > 255 ? 255 : read_len - 5 * nm);
  W8('X'); W8('S'); W8('C'); W8(runi(r, 100));
  W8('R'); W8('G'); W8('Z'); memcpy(rec + n, "grp1", 5); n += 5;
  const uint32_t bs = (uint32_t)(n - 4);
  memcpy(rec, &bs, 4);
  bput(b, rec, n);
  co->serial++;
}

/* Long-read record.  Length: 20 kb · exp(0.45·z), z ≈ N(0,1) from 12 uniforms,
 * clipped to [10 000, 50 000].  CIGAR: soft clips at both ends, then alternating M and I/D ops until
 * 200–3000 ops; query-consuming ops sum to the read length.  Unpaired (next_refID −1), 0.5% unmapped. */
static void bam_long_record(buf_t *b, rng_t *r, coord_t *co, uint8_t *rec, uint32_t *cig) {
  int n = 0;
  double z = -6.0;
  for (int i = 0; i < 12; i++) z += (double)(rnext(r) >> 11) * (1.0 / 9007199254740992.0);
  double lf = 20000.0 * exp(0.45 * z);
  int read_len = lf < 10000.0 ? 10000 : lf > 50000.0 ? 50000 : (int)lf;
  char name[80];
  static const char hex[] = "0123456789abcdef";
  int ln = 0;
  for (int i = 0; i < 36; i++) name[ln++] = (i == 8 || i == 13 || i == 18 || i == 23) ? '-' : hex[rnext(r) & 15];
  const int extra = (int)runi(r, 28); /* names of 36..63 characters */
  if (extra) {
    name[ln++] = '_';
    for (int i = 1; i < extra; i++) name[ln++] = (char)('A' + runi(r, 26));
  }
  name[ln] = 0;
  const int lrn = ln + 1;
  const int unmapped = runi(r, 1000) < 5;
  co->pos += (int32_t)runi(r, 400);
  if (co->pos + 120000 > kLens[co->ref]) { co->ref = (co->ref + 1) % 25; co->pos = 10000; }
  const int32_t pos = co->pos;
  int nc = 0, ref_span = 0;
  if (!unmapped) {
    int target = 201 + (int)runi(r, 2800);
    if (target > read_len / 4) target = read_len / 4;
    const int s1 = 10 + (int)runi(r, 190), s2 = 10 + (int)runi(r, 190);
    const int pairs = (target - 3) / 2; /* S, M + (I|D) pairs, a final M, S: 2·pairs + 3 <= target ops */
    int q = read_len - s1 - s2;         /* query bases for M and I ops */
    cig[nc++] = ((uint32_t)s1 << 4) | 4;
    for (int k = 0; k < pairs; k++) {
      const int left = pairs - k;       /* M ops still to place, including this one (+ the final M) */
      int m = q / (left + 1);
      m = m < 1 ? 1 : m - 1 + (int)runi(r, 3);
      if (m > q - left) m = q - left;
      if (m < 1) m = 1;
      cig[nc++] = (uint32_t)m << 4;
      ref_span += m;
      q -= m;
      const int l = 1 + (int)runi(r, 4);
      if (runi(r, 2) && q - l >= left) { cig[nc++] = ((uint32_t)l << 4) | 1; q -= l; }
      else { cig[nc++] = ((uint32_t)l << 4) | 2; ref_span += l; }
    }
    cig[nc++] = (uint32_t)q << 4; /* q >= 1 by construction */
    ref_span += q;
    cig[nc++] = ((uint32_t)s2 << 4) | 4;
  }
  const uint16_t flag = (uint16_t)(unmapped ? 4 : (runi(r, 2) ? 16 : 0));
  const uint8_t mapq = unmapped ? 0 : (uint8_t)runi(r, 61);
  const int bin = reg2bin(pos, pos + (ref_span > 0 ? ref_span : 1));
  W32(0);
  W32(co->ref);
  W32(pos);
  W8(lrn); W8(mapq); W16(bin);
  W16(nc); W16(flag);
  W32(read_len);
  W32(-1);
  W32(-1);
  W32(0);
  memcpy(rec + n, name, (size_t)lrn); n += lrn;
  for (int i = 0; i < nc; i++) W32(cig[i]);
  static const uint8_t codes[4] = {1, 2, 4, 8};
  for (int i = 0; i < read_len; i += 2) {
    uint8_t hi = codes[rnext(r) & 3];
    uint8_t lo = (i + 1 < read_len) ? codes[rnext(r) & 3] : 0;
    W8((hi << 4) | lo);
  }
  uint8_t prevq = 20;
  for (int i = 0; i < read_len; i++) { /* unbinned qualities 2..41 with runs */
    if (runi(r, 10) >= 7) prevq = (uint8_t)(2 + runi(r, 40));
    W8(prevq);
  }
  W8('N'); W8('M'); W8('i'); W32(runi(r, 2000));
  W8('A'); W8('S'); W8('i'); W32(read_len - (int)runi(r, 2000));
  W8('R'); W8('G'); W8('Z'); memcpy(rec + n, "grp1", 5); n += 5;
  const uint32_t bs = (uint32_t)(n - 4);
  memcpy(rec, &bs, 4);
  bput(b, rec, n);
  co->serial++;
}
/* Unplaced pair member (both reads unmapped, no coordinates): refID = pos = next refID = next pos = -1,
 * bin 4680 (reg2bin(-1, 0)), no CIGAR, flag 77 / 141. */
static void bam_unplaced_record(buf_t *b, rng_t *r, coord_t *co, int read_len, uint8_t *rec) {
  int n = 0;
  char name[64];
  const int second = (int)(co->serial & 1);
  rng_t pr = {(co->serial / 2) * 0x9E3779B97F4A7C15ull + 777};
  snprintf(name, sizeof name, "SYN:1:FC:%u:%u:%u:%u", 1 + runi(&pr, 8), 1101 + runi(&pr, 1128), runi(&pr, 30000),
           runi(&pr, 200000));
  const int lrn = (int)strlen(name) + 1;
  W32(0);
  W32(-1);
  W32(-1);
  W8(lrn); W8(0); W16(4680);
  W16(0); W16(second ? 141 : 77);
  W32(read_len);
  W32(-1);
  W32(-1);
  W32(0);
  memcpy(rec + n, name, (size_t)lrn); n += lrn;
  static const uint8_t codes[5] = {1, 2, 4, 8, 15};
  for (int i = 0; i < read_len; i += 2) {
    uint8_t hi = codes[runi(r, 5)];
    uint8_t lo = (i + 1 < read_len) ? codes[runi(r, 5)] : 0;
    W8((hi << 4) | lo);
  }
  for (int i = 0; i < read_len; i++) W8(2 + runi(r, 10));
  W8('R'); W8('G'); W8('Z'); memcpy(rec + n, "grp1", 5); n += 5;
  const uint32_t bs = (uint32_t)(n - 4);
  memcpy(rec, &bs, 4);
  bput(b, rec, n);
  co->serial++;
}
#undef W32
#undef W16
#undef W8

static void bgzf_block(const uint8_t *src, int len, int level, buf_t *out_blk) {
  uint8_t cbuf[65536 + 1024];
  z_stream zs;
  memset(&zs, 0, sizeof zs);
  deflateInit2(&zs, level, Z_DEFLATED, -15, 8, Z_DEFAULT_STRATEGY);
  zs.next_in = (Bytef *)src;
  zs.avail_in = (uInt)len;
  zs.next_out = cbuf;
  zs.avail_out = sizeof cbuf;
  deflate(&zs, Z_FINISH);
  int clen = (int)zs.total_out;
  deflateEnd(&zs);
  if (clen + 26 > 65536) { /* incompressible: stored */
    memset(&zs, 0, sizeof zs);
    deflateInit2(&zs, 0, Z_DEFLATED, -15, 8, Z_DEFAULT_STRATEGY);
    zs.next_in = (Bytef *)src; zs.avail_in = (uInt)len; zs.next_out = cbuf; zs.avail_out = sizeof cbuf;
    deflate(&zs, Z_FINISH);
    clen = (int)zs.total_out;
    deflateEnd(&zs);
  }
  const uint8_t hdr[16] = {0x1f, 0x8b, 8, 4, 0, 0, 0, 0, 0, 0xff, 6, 0, 'B', 'C', 2, 0};
  bput(out_blk, hdr, 16);
  bput16(out_blk, (uint16_t)(clen + 25));
  bput(out_blk, cbuf, clen);
  bput32(out_blk, (uint32_t)crc32(0L, src, (uInt)len));
  bput32(out_blk, (uint32_t)len);
}

typedef struct {
  const uint8_t *u;
  int64_t ulen;
  int64_t b0, b1;
  int level;
  buf_t *outs;
} job_t;

static void *worker(void *arg) {
  job_t *j = (job_t *)arg;
  for (int64_t b = j->b0; b < j->b1; b++) {
    const int64_t off = b * PAYLOAD;
    const int len = (int)((j->ulen - off) < PAYLOAD ? (j->ulen - off) : PAYLOAD);
    bgzf_block(j->u + off, len, j->level, &j->outs[b]);
  }
  return NULL;
}

static int64_t compress_stream(const uint8_t *u, int64_t ulen, int level, int threads, uint8_t **out) {
  const int64_t nb = (ulen + PAYLOAD - 1) / PAYLOAD;
  buf_t *outs = (buf_t *)calloc((size_t)(nb ? nb : 1), sizeof(buf_t));
  if (threads < 1) threads = 1;
  pthread_t *th = (pthread_t *)calloc((size_t)threads, sizeof(pthread_t));
  job_t *jobs = (job_t *)calloc((size_t)threads, sizeof(job_t));
  for (int t = 0; t < threads; t++) {
    jobs[t] = (job_t){u, ulen, nb * t / threads, nb * (t + 1) / threads, level, outs};
    pthread_create(&th[t], NULL, worker, &jobs[t]);
  }
  for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
  int64_t total = 0;
  for (int64_t b = 0; b < nb; b++) total += outs[b].n;
  uint8_t *o = (uint8_t *)malloc((size_t)(total ? total : 1));
  int64_t p = 0;
  for (int64_t b = 0; b < nb; b++) {
    memcpy(o + p, outs[b].p, (size_t)outs[b].n);
    p += outs[b].n;
    free(outs[b].p);
  }
  free(outs);
  free(th);
  free(jobs);
  *out = o;
  return total;
}

/* ---- exported API ------------------------------------------------------------------------------ */

const uint8_t kEof[28] = {0x1f, 0x8b, 8, 4, 0, 0, 0, 0, 0, 0xff, 6, 0, 'B', 'C', 2, 0, 0x1b, 0, 3, 0, 0, 0, 0, 0, 0, 0, 0, 0};

int synth_contigs(int32_t *n, int64_t *lens) {
  *n = NREF;
  if (lens) memcpy(lens, kLens, sizeof kLens);
  return 0;
}

/* Header blocks (BGZF) of the synthetic BAM. */
int64_t synth_header(uint8_t **out) {
  buf_t h = {0};
  bam_header(&h);
  int64_t n = compress_stream(h.p, h.n, 6, 1, out);
  free(h.p);
  return n;
}

/* A tile of records with ~target_u uncompressed bytes (ends on a record boundary), compressed.
 * *n_records, *u_len receive the record count and uncompressed length. */
int64_t synth_tile(uint64_t seed, int64_t target_u, int read_len, int level, int threads, uint8_t **out,
                   int64_t *n_records, int64_t *u_len) {
  rng_t r = {seed};
  buf_t u = {0};
  coord_t co = {0, 10000, seed * 1000003ull, 0, 1};
  if (read_len) { /* an equal run of records on each of the 84 contigs */
    co.per = target_u / ((int64_t)read_len * 2 + 110) / NREF;
    if (co.per < 1) co.per = 1;
    co.left = co.per;
    co.pos = 400;
  }
  int64_t nrec = 0;
  uint8_t *rec = (uint8_t *)malloc((size_t)(read_len ? 4 * read_len + 4096 : 4 * 50000 + 4 * 3000 + 4096));
  uint32_t *cig = (uint32_t *)malloc(4 * 3008);
  while (u.n < target_u) {
    if (read_len) bam_record(&u, &r, &co, read_len, rec);
    else bam_long_record(&u, &r, &co, rec, cig);
    nrec++;
  }
  free(cig);
  free(rec);
  int64_t n = compress_stream(u.p, u.n, level, threads, out);
  if (n_records) *n_records = nrec;
  if (u_len) *u_len = u.n;
  free(u.p);
  return n;
}

/* The unplaced tail: ~target_u uncompressed bytes of unmapped pairs without coordinates, compressed. */
int64_t synth_unplaced(uint64_t seed, int64_t target_u, int read_len, int level, int threads, uint8_t **out,
                       int64_t *n_records, int64_t *u_len) {
  rng_t r = {seed ^ 0x0DDBA11ull};
  buf_t u = {0};
  coord_t co = {-1, -1, seed * 1000003ull + 1, 0, 1};
  int64_t nrec = 0;
  uint8_t *rec = (uint8_t *)malloc((size_t)(4 * read_len + 4096));
  while (u.n < target_u || (nrec & 1)) {
    bam_unplaced_record(&u, &r, &co, read_len, rec);
    nrec++;
  }
  free(rec);
  int64_t n = compress_stream(u.p, u.n, level, threads, out);
  if (n_records) *n_records = nrec;
  if (u_len) *u_len = u.n;
  free(u.p);
  return n;
}

void synth_free(void *p) { free(p); }
const uint8_t *synth_eof(void) { return kEof; }
