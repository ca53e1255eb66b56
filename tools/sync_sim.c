// sync_sim — CPU model of k_inflate_wave's speculative segment decoding (tools only, not product code).
//
// For every dynamic/fixed DEFLATE block of a BGZF file it replays the wave decoder's round structure (64 lanes x
// K-bit segments, lanes > 0 warm up W bits before their segment in the literal/length state) against the true
// symbol path and counts, per round, the wave-uniform step counts that set the decoder's time: the warm-up (max
// over lanes), phase A (max over lanes), and the phase-B re-decode a lane whose guessed entry is off the true
// path needs before it rejoins its phase-A path — detected at the first common symbol boundary ("bitmask") or
// only at a phase-A checkpoint every 8 symbols ("checkpoint", the round-3 design).
//
//   sync_sim FILE.bam K W1 [W2 ...]      prints one line per W
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
  uint16_t sym;
  uint8_t len;
} ent;
static ent LT[1 << 15], DT[1 << 15];
static const uint8_t *P;
static int64_t PLEN;

static inline uint32_t bits_at(int64_t p) {
  uint64_t v = 0;
  const int64_t by = p >> 3;
  for (int i = 0; i < 8; i++) v |= (uint64_t)(by + i < PLEN && by + i >= 0 ? P[by + i] : 0) << (8 * i);
  return (uint32_t)(v >> (p & 7));
}
static const uint16_t LBASE[29] = {3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
static const uint8_t LEXT[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
static const uint8_t DEXT[32] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13, 0, 0};

static int build(ent *T, const uint8_t *lens, int n) {  // 0 ok, -1 incomplete/over
  int cnt[16] = {0}, next[16];
  for (int i = 0; i < n; i++) cnt[lens[i]]++;
  cnt[0] = 0;
  int left = 1;
  for (int l = 1; l < 16; l++) {
    left = 2 * left - cnt[l];
    if (left < 0) return -1;
  }
  if (left) return -1;
  int code = 0;
  for (int l = 1; l < 16; l++) {
    next[l] = code;
    code = (code + cnt[l]) << 1;
  }
  memset(T, 0, sizeof(ent) << 15);
  for (int s = 0; s < n; s++) {
    const int l = lens[s];
    if (!l) continue;
    const int c = next[l]++;
    int r = 0;
    for (int i = 0; i < l; i++) r |= ((c >> i) & 1) << (l - 1 - i);
    for (int f = r; f < (1 << 15); f += 1 << l) {
      T[f].sym = (uint16_t)s;
      T[f].len = (uint8_t)l;
    }
  }
  return 0;
}

// one symbol at p in state st (0 literal/length, 1 distance): returns kind 0 lit, 1 len, 2 dist, 3 EOB, 4 invalid
static inline int dsym(int64_t *p, int *st) {
  const uint32_t b = bits_at(*p);
  if (*st == 0) {
    const ent e = LT[b & 0x7fff];
    const int s = e.sym;
    int adv = e.len, kind;
    if (s < 256) kind = 0;
    else if (s == 256) kind = 3;
    else if (s <= 285) {
      kind = 1;
      adv += LEXT[s - 257];
    } else kind = 4;
    *p += adv;
    *st = kind == 1;
    return kind;
  }
  const ent e = DT[b & 0x7fff];
  const int s = e.sym;
  *p += e.len + (s < 30 ? DEXT[s] : 0);
  *st = 0;
  return s < 30 ? 2 : 4;
}

static int64_t *tpos;
static int8_t *tst;
static int ntrue, tcap;
static uint8_t *mA[2];  // phase-A symbol starts per state, bit offsets [seg_start, seg_end + 64)
static long long warm_sum, a_sum, b_sum, bcp_sum, rounds, lanes_b, lanes_bcp, rounds_b, lanes_f, lanes_tot, sym_true;
static long long bhist[8];
static long long n_lit, n_match, len_sum, lhist[6], dhist[6], dfar[4];
static int last_len;

static void sim_block(int64_t p0, int64_t pend, int K, int W) {
  // true path
  ntrue = 0;
  int64_t p = p0;
  int st = 0;
  for (;;) {
    if (ntrue + 2 >= tcap) {
      tcap = tcap ? 2 * tcap : 1 << 16;
      tpos = realloc(tpos, sizeof(int64_t) * tcap);
      tst = realloc(tst, tcap);
    }
    tpos[ntrue] = p;
    tst[ntrue] = (int8_t)st;
    ntrue++;
    const int64_t q = p;
    const int k = dsym(&p, &st);
    if (k == 0) n_lit++;
    if (k == 1) {  // length value
      const uint32_t b = bits_at(q);
      const ent e = LT[b & 0x7fff];
      const int ls = e.sym - 257;
      last_len = LBASE[ls] + (int)((b >> e.len) & ((1u << LEXT[ls]) - 1u));
      n_match++;
      len_sum += last_len;
      lhist[last_len <= 4 ? 0 : last_len <= 16 ? 1 : last_len <= 32 ? 2 : last_len <= 64 ? 3 : last_len <= 128 ? 4 : 5]++;
    }
    if (k == 2) {
      const uint32_t b = bits_at(q);
      const ent e = DT[b & 0x7fff];
      static const uint16_t DB[30] = {1,2,3,4,5,7,9,13,17,25,33,49,65,97,129,193,257,385,513,769,1025,1537,2049,3073,4097,6145,8193,12289,16385,24577};
      const int dv = DB[e.sym] + (int)((b >> e.len) & ((1u << DEXT[e.sym]) - 1u));
      dhist[dv <= 4 ? 0 : dv <= 16 ? 1 : dv <= 64 ? 2 : dv <= 1024 ? 3 : dv <= 2808 ? 4 : 5]++;
      dfar[dv <= 6904 ? 0 : dv <= 15096 ? 1 : dv <= 24000 ? 2 : 3]++;
    }
    if (k == 3 || k == 4 || p > pend) break;
  }
  tpos[ntrue] = p;  // end (after EOB)
  tst[ntrue] = 0;
  sym_true += ntrue;
  int ti = 0;  // true index of the round start
  while (ti < ntrue) {
    const int64_t Sp = tpos[ti];
    const int Sst = tst[ti];
    int wmax = 0, amax = 0, bmax = 0, bcpmax = 0, anyb = 0;
    int lti = ti;  // true index of the lane's true entry
    for (int lane = 0; lane < 64; lane++) {
      const int64_t ss = lane == 0 ? Sp : Sp + (int64_t)lane * K, se = Sp + (int64_t)(lane + 1) * K;
      while (lti < ntrue && tpos[lti] < ss) lti++;
      if (lti >= ntrue) break;  // the block ended in an earlier segment
      lanes_tot++;
      int64_t rp;
      int s;
      int wsteps = 0;
      if (lane == 0) {
        rp = Sp;
        s = Sst;
      } else {
        rp = ss - W;
        s = 0;
        if (rp <= Sp) {
          rp = Sp;
          s = Sst;
        }
        while (rp < ss) {
          dsym(&rp, &s);
          wsteps++;
        }
      }
      const int64_t ent_p = rp;
      const int ent_s = s;
      // phase A
      const int span = (int)(se - ss) + 64;
      memset(mA[0], 0, (size_t)span);
      memset(mA[1], 0, (size_t)span);
      int64_t cpp[64];
      int ncp = 0, asteps = 0;
      while (rp < se) {
        if (asteps % 8 == 0 && ncp < 64) cpp[ncp++] = s == 0 ? rp : -1;
        mA[s][rp - ss] = 1;
        dsym(&rp, &s);
        asteps++;
      }
      if (wsteps > wmax) wmax = wsteps;
      if (asteps > amax) amax = asteps;
      if (tpos[lti] == ent_p && tst[lti] == ent_s) continue;  // mode A
      // bitmask rejoin: true symbols from the entry until one is a phase-A start in the same state
      int nb = 0, j = lti;
      while (j < ntrue && tpos[j] < se && !mA[tst[j]][tpos[j] - ss]) {
        nb++;
        j++;
      }
      if (!(j < ntrue && tpos[j] < se)) lanes_f++;
      int nc = 0;
      j = lti;
      for (; j < ntrue && tpos[j] < se; j++, nc++) {
        int hit = 0;
        for (int c = 0; c < ncp; c++) hit |= cpp[c] == tpos[j] && tst[j] == 0;
        if (hit) break;
      }
      lanes_b++;
      anyb = 1;
      bhist[nb < 2 ? 0 : nb < 4 ? 1 : nb < 8 ? 2 : nb < 16 ? 3 : nb < 32 ? 4 : nb < 64 ? 5 : 6]++;
      if (nb > bmax) bmax = nb;
      if (nc > bcpmax) bcpmax = nc;
    }
    rounds++;
    rounds_b += anyb;
    warm_sum += wmax;
    a_sum += amax;
    b_sum += bmax;
    bcp_sum += bcpmax;
    // next round: the first true boundary at or after Sp + 64 K
    const int64_t e = Sp + 64LL * K;
    while (ti < ntrue && tpos[ti] < e) ti++;
  }
}

int main(int argc, char **argv) {
  if (argc < 4) {
    fprintf(stderr, "usage: sync_sim FILE K W...\n");
    return 2;
  }
  FILE *fh = fopen(argv[1], "rb");
  if (!fh) return 1;
  fseek(fh, 0, SEEK_END);
  const long n = ftell(fh);
  fseek(fh, 0, SEEK_SET);
  uint8_t *d = malloc((size_t)n);
  if (fread(d, 1, (size_t)n, fh) != (size_t)n) return 1;
  fclose(fh);
  const int K = atoi(argv[2]);
  mA[0] = malloc((size_t)K + 64);
  mA[1] = malloc((size_t)K + 64);
  for (int wi = 3; wi < argc; wi++) {
    const int W = atoi(argv[wi]);
    warm_sum = a_sum = b_sum = bcp_sum = rounds = lanes_b = rounds_b = lanes_f = lanes_tot = sym_true = 0;
    memset(bhist, 0, sizeof bhist);
    long nblk = 0, skipped = 0;
    for (long off = 0; off + 18 <= n;) {
      const int xlen = d[off + 10] | d[off + 11] << 8;
      const int bsize = (d[off + 16] | d[off + 17] << 8) + 1;
      const int hs = 12 + xlen;
      P = d + off + hs;
      PLEN = bsize - hs - 8;
      off += bsize;
      if (PLEN <= 2) continue;
      nblk++;
      int64_t p = 0;
      for (int fin = 0; !fin;) {
        fin = bits_at(p) & 1;
        const int type = (bits_at(p) >> 1) & 3;
        p += 3;
        uint8_t lens[320];
        int hlit = 288, hdist = 32;
        if (type == 1) {
          for (int i = 0; i < 320; i++) lens[i] = i < 144 ? 8 : i < 256 ? 9 : i < 280 ? 7 : i < 288 ? 8 : 5;
        } else if (type == 2) {
          hlit = (int)(bits_at(p) & 31) + 257;
          hdist = (int)((bits_at(p) >> 5) & 31) + 1;
          const int hclen = (int)((bits_at(p) >> 10) & 15) + 4;
          p += 14;
          static const uint8_t ord[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};
          uint8_t cl[19] = {0};
          for (int i = 0; i < hclen; i++, p += 3) cl[ord[i]] = bits_at(p) & 7;
          ent CT[1 << 15];
          if (build(CT, cl, 19)) { skipped++; break; }
          memset(lens, 0, sizeof lens);
          uint8_t all[320];
          int k = 0;
          while (k < hlit + hdist) {
            const ent e = CT[bits_at(p) & 0x7fff];
            p += e.len;
            if (e.sym < 16) all[k++] = (uint8_t)e.sym;
            else if (e.sym == 16) {
              int r = 3 + (bits_at(p) & 3);
              p += 2;
              while (r-- && k < 320) { all[k] = all[k - 1]; k++; }
            } else if (e.sym == 17) {
              int r = 3 + (bits_at(p) & 7);
              p += 3;
              while (r-- && k < 320) all[k++] = 0;
            } else {
              int r = 11 + (bits_at(p) & 127);
              p += 7;
              while (r-- && k < 320) all[k++] = 0;
            }
          }
          memcpy(lens, all, (size_t)hlit);
          memcpy(lens + 288, all + hlit, (size_t)hdist);
        } else {
          skipped++;
          break;
        }
        if (build(LT, lens, 288 < hlit ? 288 : hlit) || build(DT, lens + 288, hdist)) {
          skipped++;
          break;
        }
        sim_block(p, PLEN * 8, K, W);
        p = tpos[ntrue];
      }
    }
    printf("K=%d W=%d blocks=%ld skipped=%ld rounds=%lld sym/round=%.1f | per round: warm %.1f  A %.1f  B(bitmask) %.2f  "
           "B(cp8) %.2f | lanes re-decoding %.3f%% (no rejoin %.4f%%), rounds with any %.1f%% | B hist <2,<4,<8,<16,<32,<64,>=64:",
           K, W, nblk, skipped, rounds, (double)sym_true / rounds, (double)warm_sum / rounds, (double)a_sum / rounds,
           (double)b_sum / rounds, (double)bcp_sum / rounds, 100.0 * lanes_b / lanes_tot, 100.0 * lanes_f / lanes_tot,
           100.0 * rounds_b / rounds);
    for (int i = 0; i < 7; i++) printf(" %lld", bhist[i]);
    printf("\n");
    printf("tokens: lit %lld match %lld (mean len %.1f) | len <=4,<=16,<=32,<=64,<=128,>128: %lld %lld %lld %lld %lld %lld | dist <=4,<=16,<=64,<=1024,<=2808,>2808: %lld %lld %lld %lld %lld %lld\n",
           n_lit, n_match, (double)len_sum / n_match, lhist[0], lhist[1], lhist[2], lhist[3], lhist[4], lhist[5],
           dhist[0], dhist[1], dhist[2], dhist[3], dhist[4], dhist[5]);
    printf("far split: <=6904 (8K ring) %lld, <=15096 (16K ring) %lld, <=24000 %lld, more %lld\n", dfar[0], dfar[1], dfar[2], dfar[3]);
    memset(dfar, 0, sizeof dfar);
    n_lit = n_match = len_sum = 0;
    memset(lhist, 0, sizeof lhist);
    memset(dhist, 0, sizeof dhist);
    fflush(stdout);
  }
  return 0;
}
