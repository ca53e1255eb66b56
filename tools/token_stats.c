/* Token statistics of a BGZF file's DEFLATE streams (analysis tool, not part of the product path): literal and
 * match counts, match-length and distance histograms, and how many match bytes lie beyond the resolver's on-chip
 * ring (k_inflate_resolve's kNear).  A plain canonical-Huffman inflater (RFC 1951) over each block's payload.
 *   gcc -O2 -o /tmp/token_stats tools/token_stats.c && /tmp/token_stats file.bam [near]            */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef struct { const uint8_t *p; int64_t n, bit; } Br;
static int need(Br *b, int k) { return b->bit + k <= 8 * b->n; }
static uint32_t bits(Br *b, int k) {
  uint32_t v = 0;
  for (int i = 0; i < k; i++, b->bit++) v |= (uint32_t)((b->p[b->bit >> 3] >> (b->bit & 7)) & 1) << i;
  return v;
}
typedef struct { uint16_t cnt[16], sym[320]; } Huff;
static int build(Huff *h, const uint8_t *len, int n) {
  uint16_t off[16];
  memset(h->cnt, 0, sizeof h->cnt);
  for (int i = 0; i < n; i++) h->cnt[len[i]]++;
  h->cnt[0] = 0;
  off[1] = 0;
  for (int l = 1; l < 15; l++) off[l + 1] = off[l] + h->cnt[l];
  for (int i = 0; i < n; i++)
    if (len[i]) h->sym[off[len[i]]++] = (uint16_t)i;
  return 0;
}
static int decode(Br *b, const Huff *h) {
  int code = 0, first = 0, idx = 0;
  for (int l = 1; l <= 15; l++) {
    if (!need(b, 1)) return -1;
    code |= (int)bits(b, 1);
    int c = h->cnt[l];
    if (code - c < first) return h->sym[idx + (code - first)];
    idx += c;
    first = (first + c) << 1;
    code <<= 1;
  }
  return -1;
}
static const uint16_t lbase[29] = {3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
static const uint8_t lext[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
static const uint16_t dbase[30] = {1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129, 193, 257, 385, 513, 769, 1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
static const uint8_t dext[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};

static uint64_t n_lit, n_match, b_match, n_far, b_far, n_blocks, n_bytes, dhist[16], lhist[10];
static int kNear = 2808;
static uint64_t n_hdr, hdr_maxlen[16];

static int inflate_block(const uint8_t *p, int64_t n) {
  Br b = {p, n, 0};
  int fin = 0;
  int64_t out = 0;
  while (!fin) {
    if (!need(&b, 3)) return -1;
    fin = (int)bits(&b, 1);
    int type = (int)bits(&b, 2);
    Huff hl, hd;
    uint8_t len[320];
    if (type == 0) {
      b.bit = (b.bit + 7) & ~7;
      int l = (int)bits(&b, 16);
      bits(&b, 16);
      b.bit += 8 * l;
      out += l;
      n_lit += l;
      continue;
    } else if (type == 1) {
      for (int i = 0; i < 288; i++) len[i] = i < 144 ? 8 : i < 256 ? 9 : i < 280 ? 7 : 8;
      build(&hl, len, 288);
      for (int i = 0; i < 30; i++) len[i] = 5;
      build(&hd, len, 30);
    } else if (type == 2) {
      static const uint8_t ord[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};
      int hlit = (int)bits(&b, 5) + 257, hdist = (int)bits(&b, 5) + 1, hclen = (int)bits(&b, 4) + 4;
      uint8_t cl[19] = {0};
      for (int i = 0; i < hclen; i++) cl[ord[i]] = (uint8_t)bits(&b, 3);
      Huff hc;
      build(&hc, cl, 19);
      int i = 0;
      while (i < hlit + hdist) {
        int s = decode(&b, &hc);
        if (s < 0) return -1;
        if (s < 16) len[i++] = (uint8_t)s;
        else {
          int r = s == 16 ? 3 + (int)bits(&b, 2) : s == 17 ? 3 + (int)bits(&b, 3) : 11 + (int)bits(&b, 7);
          uint8_t v = s == 16 ? len[i - 1] : 0;
          while (r--) len[i++] = v;
        }
      }
      uint8_t dl[32];
      memcpy(dl, len + hlit, (size_t)hdist);
      /* root-9 sub-table shape of the literal/length code: the longest code, the widest sub-table */
      int ml = 0;
      for (int k = 0; k < hlit; k++) ml = len[k] > ml ? len[k] : ml;
      n_hdr++;
      hdr_maxlen[ml]++;
      build(&hl, len, hlit);
      build(&hd, dl, hdist);
    } else return -1;
    for (;;) {
      int s = decode(&b, &hl);
      if (s < 0) return -1;
      if (s < 256) { n_lit++; out++; continue; }
      if (s == 256) break;
      int L = lbase[s - 257] + (int)bits(&b, lext[s - 257]);
      int ds = decode(&b, &hd);
      if (ds < 0) return -1;
      int d = dbase[ds] + (int)bits(&b, dext[ds]);
      n_match++;
      b_match += (uint64_t)L;
      int k = 0;
      while ((1 << (k + 1)) <= d && k < 15) k++;
      dhist[k]++;
      lhist[L < 4 ? 0 : L < 8 ? 1 : L < 16 ? 2 : L < 32 ? 3 : L < 64 ? 4 : L < 128 ? 5 : L < 258 ? 6 : 7]++;
      if (d > kNear) { n_far++; b_far += (uint64_t)L; }
      out += L;
    }
  }
  n_bytes += (uint64_t)out;
  return 0;
}

int main(int argc, char **argv) {
  if (argc < 2) { fprintf(stderr, "usage: token_stats file.bam [near]\n"); return 2; }
  if (argc > 2) kNear = atoi(argv[2]);
  FILE *f = fopen(argv[1], "rb");
  if (!f) return 1;
  fseek(f, 0, SEEK_END);
  int64_t n = ftell(f);
  fseek(f, 0, SEEK_SET);
  uint8_t *d = malloc((size_t)n);
  if (fread(d, 1, (size_t)n, f) != (size_t)n) return 1;
  fclose(f);
  for (int64_t c = 0; c + 18 <= n;) {
    const int xlen = d[c + 10] | d[c + 11] << 8;
    const int bsize = (d[c + 16] | d[c + 17] << 8) + 1;  /* the BC subfield (first extra field in BGZF) */
    const int hs = 12 + xlen;
    if (inflate_block(d + c + hs, bsize - hs - 8) < 0) { fprintf(stderr, "bad block at %lld\n", (long long)c); return 1; }
    n_blocks++;
    c += bsize;
  }
  const uint64_t tok = n_lit + 2 * n_match;
  printf("{\"blocks\": %llu, \"bytes\": %llu, \"literals\": %llu, \"matches\": %llu, \"match_bytes\": %llu, "
         "\"tokens\": %llu, \"tokens_per_byte\": %.4f, \"mean_match\": %.2f, \"near\": %d, \"far_matches\": %llu, "
         "\"far_match_frac\": %.4f, \"far_bytes_frac\": %.4f,\n \"dist_log2_hist\": [",
         (unsigned long long)n_blocks, (unsigned long long)n_bytes, (unsigned long long)n_lit,
         (unsigned long long)n_match, (unsigned long long)b_match, (unsigned long long)tok, (double)tok / (double)n_bytes,
         (double)b_match / (double)(n_match ? n_match : 1), kNear, (unsigned long long)n_far,
         (double)n_far / (double)(n_match ? n_match : 1), (double)b_far / (double)n_bytes);
  for (int k = 0; k < 16; k++) printf("%s%llu", k ? ", " : "", (unsigned long long)dhist[k]);
  printf("],\n \"len_hist_3_4_8_16_32_64_128_258\": [");
  for (int k = 0; k < 8; k++) printf("%s%llu", k ? ", " : "", (unsigned long long)lhist[k]);
  printf("],\n \"headers\": %llu, \"lit_max_code_len_hist\": [", (unsigned long long)n_hdr);
  for (int k = 0; k < 16; k++) printf("%s%llu", k ? ", " : "", (unsigned long long)hdr_maxlen[k]);
  printf("]}\n");
  return 0;
}
