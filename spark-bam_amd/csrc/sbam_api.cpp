// sbam_api.cpp — C-ABI (include/sbam.h) over the HIP kernels: device memory, stage orchestration,
// Pos mapping, split assembly and error records.  Host code mirrors the reference's control flow:
//   Channels / FindBlockStart / FindRecordStart / loadReadsAndPositions / loadSplitsAndReads
//   (load/src/main/scala/org/hammerlab/bam/spark/load/CanLoadBam.scala:173-334),
//   full-check Counts folding (cli/src/main/scala/org/hammerlab/bam/check/full/FullCheck.scala:141-191).
#include "../../include/sbam.h"

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "sbam_internal.h"

using namespace sbam;

struct sbam_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  int64_t D = 0, base = 0, file_size = 0;
  uint8_t *d_comp = nullptr;
  size_t comp_cap = 0;
  // list-form chain pass scratch (launch_chain_list_*)
  int32_t *d_ccnt = nullptr;
  int32_t *d_tcnt = nullptr;  // record-0 pass: PASS0 positions per tile and wave (CountsDev::tile_pass0)
  size_t tcnt_cap = 0;
  int64_t *d_coff2 = nullptr, *d_plist = nullptr, *d_pfb = nullptr;
  uint8_t *d_pok = nullptr;
  unsigned long long *d_nfb = nullptr;
  size_t ccnt_cap = 0, coff2_cap = 0, plist_cap = 0, pfb_cap = 0, pok_cap = 0, nfb_cap = 0;
  // candidates from the header scan
  Candidate *d_cand = nullptr;
  int64_t ncand = -1;
  size_t cand_cap = 0;
  int32_t *d_cc = nullptr;
  int64_t *d_coff = nullptr;
  size_t cc_cap = 0, coff_cap = 0;
  Candidate *d_slots = nullptr;  // one-pass scan: kScanSlots per chunk
  size_t slots_cap = 0;
  // per-call query scratch (split starts / answers): kept, since hipMalloc + hipFree per call cost ~0.5 ms of
  // host time each (a device-wide synchronisation) between the kernels of a step
  int64_t *d_qa = nullptr, *d_qb = nullptr;
  size_t qa_cap = 0, qb_cap = 0, lens_cap = 0;
  // block table (relative offsets), device + host
  int64_t nblocks = -1;
  int64_t *d_bstart = nullptr, *d_buoff = nullptr;
  int32_t *d_bh = nullptr, *d_bc = nullptr, *d_bu = nullptr;
  size_t bcap[5] = {0, 0, 0, 0, 0};
  std::vector<int64_t> h_bstart, h_buoff;
  std::vector<int32_t> h_bc, h_bu;
  // the fast scan's table comes back behind the GPU, into pinned staging (the stream's length first, then the
  // columns); host_blocks() moves it into h_* when the host first reads them (sbam_inflate: while the decoder runs)
  uint8_t *h_stage = nullptr;
  size_t stage_cap = 0;
  hipEvent_t blk_ev[3] = {nullptr, nullptr, nullptr};  // [0]: the length copied, [1]: the columns copied, [2]: built
  hipStream_t copy_stream = nullptr;  // the columns' copy runs here, beside the decoder
  bool blk_pending = false;
  // uncompressed stream
  uint8_t *d_u = nullptr;
  size_t u_cap = 0;
  int64_t L = -1;
  int32_t *d_status = nullptr, *d_found = nullptr;
  size_t status_cap = 0, found_cap = 0;
  // contig lengths
  int32_t nref = -1;
  int64_t *d_lens = nullptr;
  std::vector<int64_t> h_lens;
  sbam_pos header_end{0, 0, 0};
  // success bitmap of the latest full/eager check
  unsigned long long *d_bitmap = nullptr;
  size_t bitmap_cap = 0;
  int64_t bm_x0 = 0, bm_x1 = 0;
  bool bm_valid = false;
  bool bm_list = false;  // the bitmap came from the list-form chain pass: d_nfb[1..2] describe its links
  int64_t plist_n = 0;   // (and d_plist[0, plist_n) its PASS0 positions)
  int32_t bm_R = -1;
  // inflate scratch: token pages of the decode → resolve path
  uint8_t *d_pool = nullptr;  // main token regions (inflate_token_bytes)
  size_t pool_cap = 0;
  uint8_t *d_arena = nullptr;  // token arena (TokPool): blocks whose tokens outgrow their main region
  size_t arena_cap = 0;        // bytes (the allocation has 1 KiB more: the resolver's token lookahead)
  int64_t *d_tokbase = nullptr;
  size_t tokbase_cap = 0;
  int32_t *d_slow = nullptr;  // blocks the wave decoder hands to the exact per-lane decoder
  size_t slow_cap = 0;
  unsigned int *d_icnt = nullptr;  // slow-path blocks, slow-path work, resolve work, stored-only blocks
  int64_t inflate_slow = -1;       // blocks the last sbam_inflate decoded on the exact per-lane path
  // split chains: per-split first record / chain end / count / record base (grow-only)
  int64_t *d_sx = nullptr, *d_se = nullptr, *d_sn = nullptr, *d_sb = nullptr;
  size_t sx_cap = 0, se_cap = 0, sn_cap = 0, sb_cap = 0;
  // decoded records of the last sbam_load_records (offset column + RecordColumnsDev in one arena)
  int64_t *d_roff = nullptr;
  size_t roff_cap = 0;
  uint8_t *d_rcols = nullptr;
  size_t rcols_cap = 0;
  RecordColumnsDev rcols{};
  int64_t n_loaded = -1;
  // small device scratch
  int64_t *d_small = nullptr;  // 64 int64
  unsigned long long *d_counts = nullptr;
  // timing
  std::map<std::string, std::pair<hipEvent_t, hipEvent_t>> ev;
  // sbam_load's copy pieces in flight (hipEventDisableTiming events, created on first use)
  hipEvent_t load_ev[4] = {nullptr, nullptr, nullptr, nullptr};
  sbam_error err{};
  std::string path = "<bytes>";  // Path.toString in exception messages (sbam_set_path)
};

namespace {

constexpr size_t kCountsWords = 21 * 19 + 21 + 21 * 128 + 19 * 19 + 4 + 19;

int set_err(sbam_ctx *c, int code, const char *fmt, ...) {
  c->err.code = code;
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(c->err.message, sizeof(c->err.message), fmt, ap);
  va_end(ap);
  return code;
}

#define HIPCHK(ctx, expr)                                                                     \
  do {                                                                                        \
    hipError_t e_ = (expr);                                                                   \
    if (e_ != hipSuccess) return set_err(ctx, SBAM_ERR_HIP, "%s: %s", #expr, hipGetErrorString(e_)); \
  } while (0)

template <class T>
hipError_t dalloc(T **p, size_t n) {
  return hipMalloc(reinterpret_cast<void **>(p), std::max<size_t>(n, 1) * sizeof(T));
}
template <class T>
void dfree(T *&p) {
  if (p) (void)hipFree(p);
  p = nullptr;
}
// SBAM_LOG_GROW=1: report every reallocation of an existing buffer (the streamed pipe's stalls)
bool log_grow() {
  static const bool on = [] {
    const char *e = std::getenv("SBAM_LOG_GROW");
    return e && *e && *e != '0';
  }();
  return on;
}
// grow-only device buffer: reused across sbam_reset() so a re-run allocates nothing
template <class T>
hipError_t ensure(T **p, size_t *cap, size_t n) {
  if (*p && *cap >= n) return hipSuccess;
  if (*p && log_grow())
    std::fprintf(stderr, "[sbam] grow %zu -> %zu bytes\n", *cap * sizeof(T), std::max<size_t>(n, 1) * sizeof(T));
  dfree(*p);
  *cap = 0;
  hipError_t e = dalloc(p, n);
  if (e == hipSuccess) *cap = std::max<size_t>(n, 1);
  return e;
}

struct Timer {  // HIP events around a launch family on the ctx stream
  sbam_ctx *c;
  std::pair<hipEvent_t, hipEvent_t> *e;
  Timer(sbam_ctx *c_, const char *name) : c(c_) {
    auto it = c->ev.find(name);
    if (it == c->ev.end()) {
      std::pair<hipEvent_t, hipEvent_t> p;
      (void)hipEventCreate(&p.first);
      (void)hipEventCreate(&p.second);
      it = c->ev.emplace(name, p).first;
    }
    e = &it->second;
    (void)hipEventRecord(e->first, c->stream);
  }
  ~Timer() { (void)hipEventRecord(e->second, c->stream); }
};

StreamView view(sbam_ctx *c) {
  return StreamView{c->d_u, c->L, c->d_lens, c->nref, (c->base + c->D >= c->file_size) ? 1 : 0};
}

// Header.make details at relative offset q (for HeaderParseException).
int header_parse_error(sbam_ctx *c, int64_t q) {
  uint8_t h[18] = {0};
  const int64_t n = std::min<int64_t>(18, c->D - q);
  if (n > 0) (void)hipMemcpy(h, c->d_comp + q, (size_t)n, hipMemcpyDeviceToHost);
  static const int idxs[7] = {0, 1, 2, 3, 12, 13, 14};
  static const int exps[7] = {31, 139, 8, 4, 66, 67, 2};
  for (int j = 0; j < 7; j++)
    if (h[idxs[j]] != (uint8_t)exps[j]) {
      c->err.idx = idxs[j];
      c->err.actual = (int8_t)h[idxs[j]];
      c->err.expected = (int8_t)(uint8_t)exps[j];
      c->err.position = c->base + q;
      return set_err(c, SBAM_ERR_HEADER_PARSE, "Position %d: %d != %d", idxs[j], (int)(int8_t)h[idxs[j]],
                     (int)(int8_t)(uint8_t)exps[j]);
    }
  return set_err(c, SBAM_ERR_HEADER_PARSE, "header parse failure at %lld", (long long)(c->base + q));
}

// NoReadFoundException(path, start, maxReadSize) (FindRecordStart.scala:11-28, 66-71)
int no_read_found(sbam_ctx *c, int64_t start, int32_t max_read_size) {
  c->err.position = start;
  c->err.expected = max_read_size;
  return set_err(c, SBAM_ERR_NO_READ_FOUND, "Failed to find a valid read-start in %d attempts in %s from %lld",
                 max_read_size, c->path.c_str(), (long long)start);
}

// h_* of a table whose copy the fast scan left in flight (sbam_scan_blocks)
int host_blocks(sbam_ctx *c) {
  if (!c->blk_pending) return SBAM_OK;
  HIPCHK(c, hipEventSynchronize(c->blk_ev[1]));
  const int64_t nb = c->nblocks;
  const int64_t *st = reinterpret_cast<const int64_t *>(c->h_stage + 8), *uo = st + nb;
  const int32_t *cs = reinterpret_cast<const int32_t *>(uo + nb + 1), *us = cs + nb;
  c->h_bstart.assign(st, st + nb);
  c->h_buoff.assign(uo, uo + nb + 1);
  c->h_bc.assign(cs, cs + nb);
  c->h_bu.assign(us, us + nb);
  c->blk_pending = false;
  return SBAM_OK;
}
// the scanned stream's uncompressed length (waits only for its own 8-byte copy)
int block_total(sbam_ctx *c, int64_t *L) {
  if (!c->blk_pending) {
    *L = c->h_buoff[c->nblocks];
    return SBAM_OK;
  }
  HIPCHK(c, hipEventSynchronize(c->blk_ev[0]));
  *L = *reinterpret_cast<const int64_t *>(c->h_stage);
  return SBAM_OK;
}
// a scanned block table, with its host copy in h_*
int ensure_blocks(sbam_ctx *c) {
  if (c->nblocks < 0) return set_err(c, SBAM_ERR_STATE, "sbam_scan_blocks has not run");
  return host_blocks(c);
}
int ensure_stream(sbam_ctx *c) {
  if (c->L < 0) return set_err(c, SBAM_ERR_STATE, "sbam_inflate has not run");
  if (c->nref < 0) return set_err(c, SBAM_ERR_STATE, "contig lengths unknown (sbam_header / sbam_set_contig_lengths)");
  return host_blocks(c);
}

// block index whose (relative) start == q, or -1
int64_t block_at(const sbam_ctx *c, int64_t q) {
  auto it = std::lower_bound(c->h_bstart.begin(), c->h_bstart.end(), q);
  if (it == c->h_bstart.end() || *it != q) return -1;
  return it - c->h_bstart.begin();
}
sbam_pos pos_of(const sbam_ctx *c, int64_t x, int64_t *hint = nullptr) {
  // last block with uoff <= x and usize > 0 containing x; x at a block end normalises to (next, 0).  hint: the block
  // of the previous (smaller) query — the search gallops from it (split starts ascend: 4767 full binary searches
  // over a 3 MB table were 0.2 ms of host time per 10 GB step)
  int64_t lo = 0, hi = c->nblocks;
  if (hint && *hint >= 0 && *hint < c->nblocks && c->h_buoff[*hint] <= x) {
    int64_t step = 1;
    lo = *hint;
    while (lo + step < c->nblocks && c->h_buoff[lo + step] <= x) {
      lo += step;
      step *= 2;
    }
    hi = std::min(lo + step, c->nblocks);
  }
  auto it = std::upper_bound(c->h_buoff.begin() + lo, c->h_buoff.begin() + hi, x);
  int64_t b = (it - c->h_buoff.begin()) - 1;
  if (hint && b >= 0) *hint = b;
  while (b >= 0 && b < c->nblocks && x >= c->h_buoff[b] + c->h_bu[b]) b++;
  if (b < 0 || b >= c->nblocks) {
    const int64_t endp = c->nblocks > 0 ? c->h_bstart[c->nblocks - 1] + c->h_bc[c->nblocks - 1] : 0;
    return sbam_pos{c->base + endp, 0, 0};
  }
  return sbam_pos{c->base + c->h_bstart[b], (int32_t)(x - c->h_buoff[b]), 0};
}

int ensure_bitmap(sbam_ctx *c, int64_t x0, int64_t x1) {
  const size_t words = (size_t)((x1 - (x0 & ~(int64_t)63) + 63) / 64) + 1;
  if (words > c->bitmap_cap) {
    if (c->d_bitmap && log_grow()) std::fprintf(stderr, "[sbam] grow bitmap %zu -> %zu words\n", c->bitmap_cap, words);
    dfree(c->d_bitmap);
    HIPCHK(c, dalloc(&c->d_bitmap, words));
    c->bitmap_cap = words;
  }
  return SBAM_OK;
}

}  // namespace

extern "C" {

const char *sbam_version(void) { return "sbam-mi355x 0.1 (gfx950)"; }

int sbam_open(int device, const uint8_t *data, int64_t len, int64_t base_offset, int64_t file_size, sbam_ctx **out) {
  if (!out || (!data && len > 0) || len < 0 || base_offset < 0 || file_size < base_offset + len) return SBAM_ERR_ARG;
  sbam_ctx *c = new sbam_ctx();
  *out = c;
  c->device = device;
  c->D = len;
  c->base = base_offset;
  c->file_size = file_size;
  HIPCHK(c, hipSetDevice(device));
  HIPCHK(c, hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
  HIPCHK(c, ensure(&c->d_comp, &c->comp_cap, (size_t)len + kCompPad));
  HIPCHK(c, hipMemsetAsync(c->d_comp + len, 0, kCompPad, c->stream));
  if (len) HIPCHK(c, hipMemcpyAsync(c->d_comp, data, (size_t)len, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, dalloc(&c->d_small, 64));
  HIPCHK(c, dalloc(&c->d_counts, kCountsWords));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return SBAM_OK;
}

void sbam_close(sbam_ctx *c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  dfree(c->d_comp);
  dfree(c->d_ccnt);
  dfree(c->d_tcnt);
  dfree(c->d_coff2);
  dfree(c->d_plist);
  dfree(c->d_pfb);
  dfree(c->d_pok);
  dfree(c->d_nfb);
  dfree(c->d_cand);
  dfree(c->d_cc);
  dfree(c->d_coff);
  dfree(c->d_slots);
  dfree(c->d_qa);
  dfree(c->d_qb);
  dfree(c->d_status);
  dfree(c->d_found);
  dfree(c->d_bstart);
  dfree(c->d_buoff);
  dfree(c->d_bh);
  dfree(c->d_bc);
  dfree(c->d_bu);
  dfree(c->d_u);
  dfree(c->d_lens);
  dfree(c->d_bitmap);
  dfree(c->d_pool);
  dfree(c->d_arena);
  dfree(c->d_tokbase);
  dfree(c->d_slow);
  dfree(c->d_icnt);
  dfree(c->d_small);
  dfree(c->d_counts);
  dfree(c->d_sx);
  dfree(c->d_se);
  dfree(c->d_sn);
  dfree(c->d_sb);
  dfree(c->d_roff);
  dfree(c->d_rcols);
  for (auto &kv : c->ev) {
    (void)hipEventDestroy(kv.second.first);
    (void)hipEventDestroy(kv.second.second);
  }
  for (hipEvent_t e : c->load_ev)
    if (e) (void)hipEventDestroy(e);
  if (c->copy_stream) (void)hipStreamSynchronize(c->copy_stream);
  for (hipEvent_t e : c->blk_ev)
    if (e) (void)hipEventDestroy(e);
  if (c->copy_stream) (void)hipStreamDestroy(c->copy_stream);
  if (c->h_stage) (void)hipHostFree(c->h_stage);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

const sbam_error *sbam_last_error(const sbam_ctx *c) { return c ? &c->err : nullptr; }

int sbam_set_path(sbam_ctx *c, const char *path) {
  if (!c || !path) return SBAM_ERR_ARG;
  c->path = path;
  return SBAM_OK;
}

int sbam_load(sbam_ctx *c, const uint8_t *data, int64_t len, int64_t base_offset, int64_t file_size) {
  if (!c || (!data && len > 0) || len < 0 || base_offset < 0 || file_size < base_offset + len) return SBAM_ERR_ARG;
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipStreamSynchronize(c->stream));  // the previous window's work is done with d_comp
  HIPCHK(c, ensure(&c->d_comp, &c->comp_cap, (size_t)len + kCompPad));
  HIPCHK(c, hipMemsetAsync(c->d_comp + len, 0, kCompPad, c->stream));
  // in 8 MiB pieces with at most kInFlight queued: a multi-GB copy queued whole would hold the copy engine, and the
  // small copies of another context's kernels running meanwhile (results, tables) would wait behind it
  // (tools/e2e_probe.py: a window's compute 56 -> 98 ms while the next window's 2.5 GB copy ran); a few pieces in
  // flight keep the engine busy without a host round trip between pieces
  constexpr int64_t kPiece = 8ll << 20;
  constexpr int kInFlight = 3;
  for (hipEvent_t &e : c->load_ev)
    if (!e) HIPCHK(c, hipEventCreateWithFlags(&e, hipEventDisableTiming));
  int64_t k = 0;
  for (int64_t o = 0; o < len; o += kPiece, k++) {
    if (k >= kInFlight) HIPCHK(c, hipEventSynchronize(c->load_ev[(k - kInFlight) % 4]));
    const int64_t n = std::min(kPiece, len - o);
    HIPCHK(c, hipMemcpyAsync(c->d_comp + o, data + o, (size_t)n, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipEventRecord(c->load_ev[k % 4], c->stream));
  }
  HIPCHK(c, hipStreamSynchronize(c->stream));
  // another file (or a range from its start): its contig lengths must come from sbam_header /
  // sbam_set_contig_lengths again; a later window of the same file keeps them
  if (base_offset == 0 || file_size != c->file_size) c->nref = -1;
  c->D = len;
  c->base = base_offset;
  c->file_size = file_size;
  return sbam_reset(c);
}

int sbam_reserve(sbam_ctx *c, int64_t comp_bytes, int64_t n_blocks, int64_t ubytes, int64_t n_records) {
  if (!c || comp_bytes < 0 || n_blocks < 0 || ubytes < 0 || n_records < 0) return SBAM_ERR_ARG;
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  if (c->copy_stream) HIPCHK(c, hipStreamSynchronize(c->copy_stream));
  // Any stage buffer that grows is a fresh allocation whose contents are gone, so a context that has already run a
  // stage drops its stages (sbam_reset) when one grows: a later query re-runs them instead of reading uninitialised
  // device memory.  The resident compressed bytes and the contig lengths are kept.
  bool grew = false;
  auto grow = [&](auto **p, size_t *cap, size_t n) {  // (a buffer never allocated held no stage's data)
    grew |= *p != nullptr && *cap < std::max<size_t>(n, 1);
    return ensure(p, cap, n);
  };
  if ((size_t)comp_bytes + kCompPad > c->comp_cap) {  // keep the resident bytes (sbam_load replaces them anyway)
    uint8_t *p = nullptr;
    HIPCHK(c, dalloc(&p, (size_t)comp_bytes + kCompPad));
    if (c->D + kCompPad > 0) HIPCHK(c, hipMemcpy(p, c->d_comp, (size_t)c->D + kCompPad, hipMemcpyDeviceToDevice));
    dfree(c->d_comp);
    c->d_comp = p;
    c->comp_cap = (size_t)comp_bytes + kCompPad;
  }
  const int64_t nchunks = (comp_bytes + kScanChunk - 1) / kScanChunk;
  HIPCHK(c, grow(&c->d_cc, &c->cc_cap, nchunks));
  HIPCHK(c, grow(&c->d_coff, &c->coff_cap, nchunks));
  HIPCHK(c, grow(&c->d_slots, &c->slots_cap, (size_t)nchunks * kScanSlots));
  // candidates: every block's header plus the rare false positives inside payloads
  HIPCHK(c, grow(&c->d_cand, &c->cand_cap, (size_t)(n_blocks + n_blocks / 8 + 1024)));
  HIPCHK(c, grow(&c->d_bstart, &c->bcap[0], n_blocks + 1));
  HIPCHK(c, grow(&c->d_bh, &c->bcap[1], n_blocks + 1));
  HIPCHK(c, grow(&c->d_bc, &c->bcap[2], n_blocks + 1));
  HIPCHK(c, grow(&c->d_bu, &c->bcap[3], n_blocks + 1));
  HIPCHK(c, grow(&c->d_buoff, &c->bcap[4], n_blocks + 1 + (n_blocks + 255) / 256));  // (+ the scan's sums)
  HIPCHK(c, grow(&c->d_u, &c->u_cap, (size_t)ubytes + kStreamPad));
  HIPCHK(c, grow(&c->d_status, &c->status_cap, n_blocks));
  HIPCHK(c, grow(&c->d_found, &c->found_cap, n_blocks));
  HIPCHK(c, grow(&c->d_pool, &c->pool_cap, inflate_token_bytes(ubytes, n_blocks)));
  if (inflate_arena_bytes(ubytes) > c->arena_cap) {
    HIPCHK(c, grow(&c->d_arena, &c->arena_cap, inflate_arena_bytes(ubytes) + 1024));
    c->arena_cap -= 1024;
  }
  HIPCHK(c, grow(&c->d_tokbase, &c->tokbase_cap, n_blocks));
  HIPCHK(c, grow(&c->d_slow, &c->slow_cap, 2 * n_blocks));  // (the exact decoder's list, then the stored-only list)
  grew |= c->d_bitmap != nullptr && (size_t)((ubytes + 63) / 64) + 1 > c->bitmap_cap;
  if (int rc = ensure_bitmap(c, 0, ubytes)) return rc;
  HIPCHK(c, grow(&c->d_tcnt, &c->tcnt_cap, (size_t)(4 * check_tiles(0, ubytes) + 8)));  // (x0 may add a tile)
  if (n_records > 0) {  // the chain pass's PASS0 list (about one entry per record) and loadReads' offsets
    const size_t n = (size_t)(n_records + n_records / 8 + 4096);
    HIPCHK(c, grow(&c->d_plist, &c->plist_cap, n));
    HIPCHK(c, grow(&c->d_pfb, &c->pfb_cap, n));
    HIPCHK(c, grow(&c->d_pok, &c->pok_cap, n));
    HIPCHK(c, grow(&c->d_roff, &c->roff_cap, n));
    // loadReads' columns (sbam_load_records: an int64 column and ten int32 ones, 256-B aligned)
    const size_t stride = (n * 8 + 255) & ~(size_t)255, stride4 = (n * 4 + 255) & ~(size_t)255;
    HIPCHK(c, grow(&c->d_rcols, &c->rcols_cap, stride + 10 * stride4));
  }
  if (grew && (c->ncand >= 0 || c->nblocks >= 0 || c->L >= 0 || c->n_loaded >= 0)) return sbam_reset(c);
  return SBAM_OK;
}

int sbam_reset(sbam_ctx *c) {
  if (!c) return SBAM_ERR_ARG;
  c->ncand = -1;
  c->nblocks = -1;
  c->blk_pending = false;
  c->L = -1;
  c->inflate_slow = -1;
  c->bm_valid = false;
  c->n_loaded = -1;
  c->err = sbam_error{};
  return SBAM_OK;
}

double sbam_last_kernel_ms(sbam_ctx *c, const char *kernel) {
  auto it = c->ev.find(kernel);
  if (it == c->ev.end()) return -1.0;
  (void)hipEventSynchronize(it->second.second);
  float ms = -1.f;
  if (hipEventElapsedTime(&ms, it->second.first, it->second.second) != hipSuccess) return -1.0;
  return ms;
}

// ---- candidates (scan) ---------------------------------------------------------------------------
static int scan_candidates(sbam_ctx *c) {
  if (c->ncand >= 0) return SBAM_OK;
  Timer t(c, "scan");
  const int64_t nchunks = (c->D + kScanChunk - 1) / kScanChunk;
  HIPCHK(c, ensure(&c->d_cc, &c->cc_cap, nchunks));
  HIPCHK(c, ensure(&c->d_coff, &c->coff_cap, nchunks));
  HIPCHK(c, ensure(&c->d_slots, &c->slots_cap, (size_t)nchunks * kScanSlots));
  // one pass into per-chunk slots (+ counts, exact even past the slots); d_small[0] = total, [1] = overflow
  HIPCHK(c, launch_scan_slots(c->d_comp, c->D, c->d_cc, nchunks, c->d_slots, c->d_small + 1, c->stream));
  HIPCHK(c, launch_scan_prefix(c->d_cc, nchunks, c->d_coff, c->d_small, c->stream));
  int64_t tot_ovf[2] = {0, 0};
  HIPCHK(c, hipMemcpyAsync(tot_ovf, c->d_small, 2 * sizeof(int64_t), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  const int64_t total = tot_ovf[0];
  HIPCHK(c, ensure(&c->d_cand, &c->cand_cap, total));
  if (tot_ovf[1] == 0) {
    HIPCHK(c, launch_scan_compact(c->d_slots, c->d_cc, c->d_coff, nchunks, c->d_cand, c->stream));
  } else {  // a chunk with more than kScanSlots candidates (blocks under 2 KiB): the exact second pass
    HIPCHK(c, launch_scan_write(c->d_comp, c->D, c->d_coff, nchunks, c->d_cand, c->stream));
  }
  HIPCHK(c, hipStreamSynchronize(c->stream));
  c->ncand = total;
  return SBAM_OK;
}

int sbam_find_block_starts(sbam_ctx *c, const int64_t *starts, int64_t n, int32_t nchk, int64_t *out) {
  if (!c || (!starts && n) || (!out && n) || nchk < 0) return SBAM_ERR_ARG;
  HIPCHK(c, hipSetDevice(c->device));
  int rc = scan_candidates(c);
  if (rc) return rc;
  std::vector<int64_t> rel(n);
  for (int64_t i = 0; i < n; i++) {
    rel[i] = starts[i] - c->base;
    if (rel[i] < 0 || rel[i] > c->D) return set_err(c, SBAM_ERR_ARG, "split start %lld outside loaded bytes", (long long)starts[i]);
  }
  HIPCHK(c, ensure(&c->d_qa, &c->qa_cap, (size_t)n));
  HIPCHK(c, ensure(&c->d_qb, &c->qb_cap, (size_t)n));
  int64_t *d_q = c->d_qa, *d_o = c->d_qb;
  HIPCHK(c, hipMemcpyAsync(d_q, rel.data(), n * sizeof(int64_t), hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, launch_find_block_starts(c->d_comp, c->D, c->d_cand, c->ncand, d_q, n, nchk, d_o, c->stream));
  HIPCHK(c, hipMemcpyAsync(out, d_o, n * sizeof(int64_t), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  for (int64_t i = 0; i < n; i++) {
    if (out[i] < 0) {
      // HeaderSearchFailedException(path, start, positionsAttempted = MAX_BLOCK_SIZE) (FindBlockStart.scala:16-35)
      c->err.position = starts[i];
      c->err.actual = 65536;
      return set_err(c, SBAM_ERR_HEADER_SEARCH, "%s: failed to find BGZF header in %d bytes from %lld",
                     c->path.c_str(), 65536, (long long)starts[i]);
    }
    out[i] += c->base;
  }
  return SBAM_OK;
}

int sbam_scan_blocks(sbam_ctx *c, int64_t *n_blocks) {
  if (!c) return SBAM_ERR_ARG;
  HIPCHK(c, hipSetDevice(c->device));
  int rc = scan_candidates(c);
  if (rc) return rc;
  int64_t start_rel = 0;
  if (c->base > 0) {  // a shard starts at the first block at/after its first byte
    int64_t s = c->base, o = 0;
    rc = sbam_find_block_starts(c, &s, 1, 5, &o);
    if (rc) return rc;
    start_rel = o - c->base;
  }
  Timer t(c, "chain");
  std::vector<int64_t> st;
  std::vector<int32_t> hs, cs, us;
  int64_t first = 0;
  HIPCHK(c, launch_lower_bound(c->d_cand, c->ncand, start_rel, c->d_small, c->stream));
  HIPCHK(c, hipMemcpyAsync(&first, c->d_small, sizeof(int64_t), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  int64_t nb = 0;
  bool fast = true;
  if (start_rel + 18 > c->D) {
    nb = 0;  // EOF before the first header: empty stream
  } else {
    Candidate c0{};
    if (first < c->ncand) HIPCHK(c, hipMemcpy(&c0, c->d_cand + first, sizeof(Candidate), hipMemcpyDeviceToHost));
    if (first >= c->ncand || c0.pos != start_rel) return header_parse_error(c, start_rel);
    const unsigned long long none = ~0ull;
    HIPCHK(c, hipMemcpyAsync(c->d_small + 1, &none, sizeof(none), hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, launch_chain_verify(c->d_cand, c->ncand, first, c->D, c->d_small + 1, c->stream));
    unsigned long long stop = 0;
    HIPCHK(c, hipMemcpyAsync(&stop, c->d_small + 1, sizeof(stop), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    const int64_t si = (int64_t)(stop >> 2);
    const int code = (int)(stop & 3);
    if (code == 1) nb = si - first;
    else if (code == 2) nb = si - first + 1;
    else fast = false;  // a candidate that is not the next header: walk exactly on the host
  }
  c->h_bstart.clear();
  c->h_bc.clear();
  c->h_bu.clear();
  if (c->copy_stream) HIPCHK(c, hipEventSynchronize(c->blk_ev[1]));  // (the last table's copy has read its columns)
  HIPCHK(c, ensure(&c->d_bstart, &c->bcap[0], nb + 1));
  HIPCHK(c, ensure(&c->d_bh, &c->bcap[1], nb + 1));
  HIPCHK(c, ensure(&c->d_bc, &c->bcap[2], nb + 1));
  HIPCHK(c, ensure(&c->d_bu, &c->bcap[3], nb + 1));
  if (fast) {
    // columns and offsets built on the device; the host's copy is queued behind them, not waited for
    const int64_t nwg = (nb + 255) / 256;
    HIPCHK(c, ensure(&c->d_buoff, &c->bcap[4], nb + 1 + nwg));
    HIPCHK(c, launch_gather_blocks(c->d_cand, first, nb, c->d_bstart, c->d_bh, c->d_bc, c->d_bu, c->d_buoff + nb + 1,
                                   c->d_buoff, c->stream));
    const size_t need = 8 + (size_t)nb * 8 + (size_t)(nb + 1) * 8 + (size_t)nb * 8;
    if (c->stage_cap < need) {
      HIPCHK(c, hipStreamSynchronize(c->stream));  // (an earlier table's copy may still target the old staging)
      if (c->h_stage) (void)hipHostFree(c->h_stage);
      c->h_stage = nullptr;
      c->stage_cap = 0;
      HIPCHK(c, hipHostMalloc(reinterpret_cast<void **>(&c->h_stage), need + need / 8, hipHostMallocDefault));
      c->stage_cap = need + need / 8;
    }
    for (hipEvent_t &e : c->blk_ev)
      if (!e) HIPCHK(c, hipEventCreateWithFlags(&e, hipEventDisableTiming));
    if (!c->copy_stream) HIPCHK(c, hipStreamCreateWithFlags(&c->copy_stream, hipStreamNonBlocking));
    int64_t *st = reinterpret_cast<int64_t *>(c->h_stage + 8), *uo = st + nb;
    int32_t *cs = reinterpret_cast<int32_t *>(uo + nb + 1), *us = cs + nb;
    HIPCHK(c, hipMemcpyAsync(c->h_stage, c->d_buoff + nb, 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipEventRecord(c->blk_ev[0], c->stream));
    HIPCHK(c, hipEventRecord(c->blk_ev[2], c->stream));
    HIPCHK(c, hipStreamWaitEvent(c->copy_stream, c->blk_ev[2], 0));
    HIPCHK(c, hipMemcpyAsync(uo, c->d_buoff, (nb + 1) * 8, hipMemcpyDeviceToHost, c->copy_stream));
    if (nb) {
      HIPCHK(c, hipMemcpyAsync(st, c->d_bstart, nb * 8, hipMemcpyDeviceToHost, c->copy_stream));
      HIPCHK(c, hipMemcpyAsync(cs, c->d_bc, nb * 4, hipMemcpyDeviceToHost, c->copy_stream));
      HIPCHK(c, hipMemcpyAsync(us, c->d_bu, nb * 4, hipMemcpyDeviceToHost, c->copy_stream));
    }
    HIPCHK(c, hipEventRecord(c->blk_ev[1], c->copy_stream));
    c->blk_pending = true;
  } else {
    std::vector<Candidate> hc(c->ncand);
    HIPCHK(c, hipMemcpy(hc.data(), c->d_cand, c->ncand * sizeof(Candidate), hipMemcpyDeviceToHost));
    int64_t q = start_rel, i = first;
    std::vector<int32_t> h_h;
    for (;;) {  // MetadataStream._advance, exactly (MetadataStream.scala:23-54)
      if (q + 18 > c->D) break;
      while (i < c->ncand && hc[i].pos < q) i++;
      if (i >= c->ncand || hc[i].pos != q) return header_parse_error(c, q);
      const Candidate &k = hc[i];
      if (!(k.flags & CAND_ISIZE) || (k.flags & CAND_EMPTY)) break;
      c->h_bstart.push_back(k.pos);
      c->h_bc.push_back(k.csize);
      c->h_bu.push_back(k.isize);
      h_h.push_back(k.hsize);
      q += k.csize;
    }
    nb = (int64_t)c->h_bstart.size();
    HIPCHK(c, ensure(&c->d_bstart, &c->bcap[0], nb + 1));
    HIPCHK(c, ensure(&c->d_bh, &c->bcap[1], nb + 1));
    HIPCHK(c, ensure(&c->d_bc, &c->bcap[2], nb + 1));
    HIPCHK(c, ensure(&c->d_bu, &c->bcap[3], nb + 1));
    HIPCHK(c, hipMemcpy(c->d_bstart, c->h_bstart.data(), nb * 8, hipMemcpyHostToDevice));
    HIPCHK(c, hipMemcpy(c->d_bh, h_h.data(), nb * 4, hipMemcpyHostToDevice));
    HIPCHK(c, hipMemcpy(c->d_bc, c->h_bc.data(), nb * 4, hipMemcpyHostToDevice));
    HIPCHK(c, hipMemcpy(c->d_bu, c->h_bu.data(), nb * 4, hipMemcpyHostToDevice));
    c->h_buoff.resize(nb + 1);
    int64_t acc = 0;
    for (int64_t b = 0; b < nb; b++) {
      c->h_buoff[b] = acc;
      acc += (c->h_bu[b] < 0) ? 0 : c->h_bu[b];
    }
    c->h_buoff[nb] = acc;
    HIPCHK(c, ensure(&c->d_buoff, &c->bcap[4], nb + 1));
    HIPCHK(c, hipMemcpyAsync(c->d_buoff, c->h_buoff.data(), (nb + 1) * 8, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
  }
  c->nblocks = nb;
  if (n_blocks) *n_blocks = nb;
  return SBAM_OK;
}

int sbam_get_blocks(sbam_ctx *c, int64_t *start, int32_t *csize, int32_t *usize, int64_t *uoff, int64_t cap) {
  if (!c) return SBAM_ERR_ARG;
  int rc = ensure_blocks(c);
  if (rc) return rc;
  if (cap < c->nblocks) return set_err(c, SBAM_ERR_ARG, "capacity %lld < %lld blocks", (long long)cap, (long long)c->nblocks);
  for (int64_t b = 0; b < c->nblocks; b++) {
    if (start) start[b] = c->base + c->h_bstart[b];
    if (csize) csize[b] = c->h_bc[b];
    if (usize) usize[b] = c->h_bu[b];
    if (uoff) uoff[b] = c->h_buoff[b];
  }
  return SBAM_OK;
}

int sbam_inflate(sbam_ctx *c, int64_t *usz) {
  if (!c) return SBAM_ERR_ARG;
  if (c->nblocks < 0) return set_err(c, SBAM_ERR_STATE, "sbam_scan_blocks has not run");
  int rc = SBAM_OK;  // (the table's host copy is picked up below, while the decoder runs)
  HIPCHK(c, hipSetDevice(c->device));
  int64_t L = 0;
  rc = block_total(c, &L);
  if (rc) return rc;
  HIPCHK(c, ensure(&c->d_u, &c->u_cap, (size_t)L + kStreamPad));
  HIPCHK(c, hipMemsetAsync(c->d_u + L, 0, kStreamPad, c->stream));
  const int64_t nb = c->nblocks;
  HIPCHK(c, ensure(&c->d_status, &c->status_cap, nb));
  HIPCHK(c, ensure(&c->d_found, &c->found_cap, nb));
  int32_t *d_status = c->d_status, *d_found = c->d_found;
  const unsigned long long none = ~0ull;
  BlockTable bt{c->d_bstart, c->d_bh, c->d_bc, c->d_bu, c->d_buoff, nb};
  // token pool (TokPool): main regions at 1 B per output byte, the arena for blocks that need more
  HIPCHK(c, ensure(&c->d_pool, &c->pool_cap, inflate_token_bytes(L, nb)));
  if (!c->d_arena || c->arena_cap < inflate_arena_bytes(L)) {
    HIPCHK(c, ensure(&c->d_arena, &c->arena_cap, inflate_arena_bytes(L) + 1024));
    c->arena_cap -= 1024;
  }
  HIPCHK(c, ensure(&c->d_tokbase, &c->tokbase_cap, nb));
  HIPCHK(c, ensure(&c->d_slow, &c->slow_cap, 2 * nb));  // (the exact decoder's list, then the stored-only list)
  if (!c->d_icnt) HIPCHK(c, dalloc(&c->d_icnt, 4));
  unsigned long long *d_used = reinterpret_cast<unsigned long long *>(c->d_small + 16);
  unsigned long long ferr = 0;
  unsigned int cnt3[3] = {0, 0, 0};  // slow-path blocks, -, blocks the resolver handed back
  for (;;) {
    const TokPool tp{c->d_pool, c->d_arena, (int64_t)c->arena_cap, d_used, c->d_tokbase};
    HIPCHK(c, hipMemsetAsync(c->d_tokbase, 0xff, nb * sizeof(int64_t), c->stream));  // every block: main region
    HIPCHK(c, hipMemsetAsync(d_used, 0, sizeof(unsigned long long), c->stream));
    {
      Timer t(c, "inflate");
      {
        Timer t1(c, "inflate_decode");
        HIPCHK(c, launch_inflate_decode(c->d_comp, c->D, bt, tp, c->d_u, d_status, d_found, c->d_slow, c->d_icnt, c->stream));
      }
      Timer t2(c, "inflate_resolve");
      // (the slow list is consumed by now: the resolver's redo list reuses d_slow, its count is d_icnt[2])
      HIPCHK(c, launch_inflate_resolve(bt, c->d_u, tp, d_found, nullptr, 0, c->d_slow, c->d_icnt + 2, c->stream));
    }
    // the table's host copy, while the kernels run (before the copies of the results below: copies into pageable
    // memory wait for the stream)
    rc = host_blocks(c);
    if (rc) return rc;
    HIPCHK(c, hipMemcpyAsync(c->d_small + 2, &none, 8, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, launch_first_error(d_status, nb, reinterpret_cast<unsigned long long *>(c->d_small + 2), c->stream));
    HIPCHK(c, hipMemcpyAsync(&ferr, c->d_small + 2, 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(cnt3, c->d_icnt, 12, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (cnt3[2] > 0) {  // a distance past its block's start ("invalid distance too far back"): the exact decoder
      HIPCHK(c, launch_inflate_redo(c->d_comp, c->D, bt, tp, c->d_slow, c->d_icnt, d_status, d_found, c->stream));
      HIPCHK(c, launch_inflate_resolve(bt, c->d_u, tp, d_found, c->d_slow, cnt3[2], nullptr, nullptr, c->stream));
      HIPCHK(c, hipMemcpyAsync(c->d_small + 2, &none, 8, hipMemcpyHostToDevice, c->stream));
      HIPCHK(c, launch_first_error(d_status, nb, reinterpret_cast<unsigned long long *>(c->d_small + 2), c->stream));
      HIPCHK(c, hipMemcpyAsync(&ferr, c->d_small + 2, 8, hipMemcpyDeviceToHost, c->stream));
      HIPCHK(c, hipStreamSynchronize(c->stream));
    }
    if (ferr == ~0ull) break;
    int32_t st = 0;
    unsigned long long used = 0;
    HIPCHK(c, hipMemcpy(&st, d_status + ferr, 4, hipMemcpyDeviceToHost));
    HIPCHK(c, hipMemcpy(&used, d_used, 8, hipMemcpyDeviceToHost));
    if (st != 3 /* INF_OVERFLOW */ || used <= c->arena_cap) break;
    // the arena was too small for the blocks that needed it (used counts every request): grow it, inflate again
    if (log_grow()) std::fprintf(stderr, "[sbam] token arena %zu -> %llu bytes\n", c->arena_cap, used);
    HIPCHK(c, ensure(&c->d_arena, &c->arena_cap, (size_t)used + (used >> 3) + 1024));
    c->arena_cap -= 1024;
  }
  c->inflate_slow = cnt3[0] + cnt3[2];
  if (ferr != ~0ull) {
    int32_t found = 0;
    HIPCHK(c, hipMemcpy(&found, d_found + ferr, 4, hipMemcpyDeviceToHost));
    c->err.position = c->base + c->h_bstart[ferr];
    c->err.expected = c->h_bu[ferr];
    c->err.actual = found;
    return set_err(c, SBAM_ERR_INFLATE, "Expected %d decompressed bytes, found %d", c->h_bu[ferr], found);
  }
  c->L = L;
  c->bm_valid = false;
  if (usz) *usz = L;
  return SBAM_OK;
}

int sbam_inflate_fallbacks(sbam_ctx *c, int64_t *n) {
  if (!c || !n) return SBAM_ERR_ARG;
  if (c->L < 0 || c->inflate_slow < 0) return set_err(c, SBAM_ERR_STATE, "sbam_inflate has not run");
  *n = c->inflate_slow;
  return SBAM_OK;
}

int sbam_read_uncompressed(sbam_ctx *c, int64_t off, int64_t len, uint8_t *out) {
  if (!c || off < 0 || len < 0) return SBAM_ERR_ARG;
  if (c->L < 0) return set_err(c, SBAM_ERR_STATE, "sbam_inflate has not run");
  if (off + len > c->L) return set_err(c, SBAM_ERR_ARG, "range past the stream end");
  HIPCHK(c, hipSetDevice(c->device));
  if (len) HIPCHK(c, hipMemcpy(out, c->d_u + off, (size_t)len, hipMemcpyDeviceToHost));
  return SBAM_OK;
}

int sbam_pos_to_offset(sbam_ctx *c, sbam_pos p, int64_t *off) {
  if (!c || !off) return SBAM_ERR_ARG;
  int rc = ensure_blocks(c);
  if (rc) return rc;
  const int64_t b = block_at(c, p.block_pos - c->base);
  if (b < 0 || p.offset < 0 || p.offset > c->h_bu[b]) return set_err(c, SBAM_ERR_ARG, "no block at %lld", (long long)p.block_pos);
  *off = c->h_buoff[b] + p.offset;
  return SBAM_OK;
}

int sbam_offset_to_pos(sbam_ctx *c, int64_t off, sbam_pos *p) {
  if (!c || !p) return SBAM_ERR_ARG;
  int rc = ensure_blocks(c);
  if (rc) return rc;
  *p = pos_of(c, off);
  return SBAM_OK;
}

// ---- BAM header -----------------------------------------------------------------------------------
int sbam_set_contig_lengths(sbam_ctx *c, int32_t n_ref, const int64_t *lengths) {
  if (!c || n_ref < 0 || (n_ref && !lengths)) return SBAM_ERR_ARG;
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, ensure(&c->d_lens, &c->lens_cap, (size_t)n_ref));
  if (n_ref) HIPCHK(c, hipMemcpyAsync(c->d_lens, lengths, n_ref * 8, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  c->h_lens.assign(lengths, lengths + n_ref);
  c->nref = n_ref;
  c->bm_valid = false;
  return SBAM_OK;
}

int sbam_header(sbam_ctx *c, int32_t *n_ref, int64_t *lengths, int32_t cap, sbam_pos *end_pos) {
  if (!c) return SBAM_ERR_ARG;
  if (c->L < 0) return set_err(c, SBAM_ERR_STATE, "sbam_inflate has not run");
  if (c->base != 0) return set_err(c, SBAM_ERR_STATE, "header lives in the file's first block (shard: sbam_set_contig_lengths)");
  if (int rc = host_blocks(c)) return rc;
  auto rd = [&](int64_t off, int64_t n, void *dst) -> bool {
    if (off < 0 || off + n > c->L) return false;
    return hipMemcpy(dst, c->d_u + off, (size_t)n, hipMemcpyDeviceToHost) == hipSuccess;
  };
  char magic[4];
  if (!rd(0, 4, magic) || memcmp(magic, "BAM\1", 4) != 0)
    return set_err(c, SBAM_ERR_NOT_BAM, "requirement failed");
  int32_t l_text = 0, nr = 0;
  if (!rd(4, 4, &l_text)) return set_err(c, SBAM_ERR_NOT_BAM, "truncated header");
  int64_t x = 8 + (int64_t)l_text;
  if (!rd(x, 4, &nr)) return set_err(c, SBAM_ERR_NOT_BAM, "truncated header");
  x += 4;
  std::vector<int64_t> lens;
  for (int32_t i = 0; i < nr; i++) {
    int32_t l_name = 0, l_ref = 0;
    if (!rd(x, 4, &l_name)) return set_err(c, SBAM_ERR_NOT_BAM, "truncated header");
    x += 4 + (int64_t)l_name;
    if (!rd(x, 4, &l_ref)) return set_err(c, SBAM_ERR_NOT_BAM, "truncated header");
    x += 4;
    lens.push_back(l_ref);
  }
  int rc = sbam_set_contig_lengths(c, nr, lens.data());
  if (rc) return rc;
  c->header_end = pos_of(c, x);
  if (n_ref) *n_ref = nr;
  if (lengths)
    for (int32_t i = 0; i < nr && i < cap; i++) lengths[i] = lens[i];
  if (end_pos) *end_pos = c->header_end;
  return SBAM_OK;
}

// Copy a device bitmap covering [x0 & ~63, x1) out as bits relative to x0.
static int copy_bitmap_out(sbam_ctx *c, int64_t x0, int64_t x1, uint64_t *out) {
  const int64_t x0a = x0 & ~(int64_t)63, sh = x0 - x0a;
  const size_t nwa = (size_t)((x1 - x0a + 63) / 64), nw = (size_t)((x1 - x0 + 63) / 64);
  if (!nw) return SBAM_OK;
  if (!sh) {
    HIPCHK(c, hipMemcpyAsync(out, c->d_bitmap, nw * 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return SBAM_OK;
  }
  std::vector<uint64_t> t(nwa + 1, 0);
  HIPCHK(c, hipMemcpyAsync(t.data(), c->d_bitmap, nwa * 8, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  for (size_t i = 0; i < nw; i++) out[i] = (t[i] >> sh) | (t[i + 1] << (64 - sh));
  const int64_t tail = (x1 - x0) & 63;
  if (tail) out[nw - 1] &= (1ull << tail) - 1;
  return SBAM_OK;
}

// ---- checkers ------------------------------------------------------------------------------------
static int check_range_args(sbam_ctx *c, int64_t x0, int64_t x1, int32_t R) {
  int rc = ensure_stream(c);
  if (rc) return rc;
  if (x0 < 0 || x1 < x0 || x1 > c->L) return set_err(c, SBAM_ERR_ARG, "range [%lld, %lld) outside stream of %lld", (long long)x0, (long long)x1, (long long)c->L);
  if (R < 0 || R > SBAM_MAX_READS_TO_CHECK) return set_err(c, SBAM_ERR_ARG, "reads_to_check %d out of range", R);
  return SBAM_OK;
}

static hipError_t run_chains(sbam_ctx *c, int64_t x0, int64_t x1, int32_t R, int32_t by_key, CountsDev cd,
                             const int32_t *tile_pass0 = nullptr);

int sbam_check_eager(sbam_ctx *c, int64_t x0, int64_t x1, int32_t R, uint64_t *bitmap) {
  if (!c) return SBAM_ERR_ARG;
  int rc = check_range_args(c, x0, x1, R);
  if (rc) return rc;
  HIPCHK(c, hipSetDevice(c->device));
  rc = ensure_bitmap(c, x0, x1);
  if (rc) return rc;
  {
    Timer t(c, "check_eager");
    {
      Timer t0(c, "check_eager_pass0");
      HIPCHK(c, launch_check_eager_pass0(view(c), x0, x1, R, c->d_bitmap, c->stream));
    }
    HIPCHK(c, run_chains(c, x0, x1, R, 0, CountsDev{}));
  }
  HIPCHK(c, hipStreamSynchronize(c->stream));
  if (bitmap) {
    int rc2 = copy_bitmap_out(c, x0, x1, bitmap);
    if (rc2) return rc2;
  }
  c->bm_x0 = x0 & ~(int64_t)63;
  c->bm_x1 = x1;
  c->bm_R = R;
  c->bm_valid = true;
  return SBAM_OK;
}

int sbam_check_full_words(sbam_ctx *c, int64_t x0, int64_t x1, int32_t R, uint32_t *words) {
  if (!c || !words) return SBAM_ERR_ARG;
  int rc = check_range_args(c, x0, x1, R);
  if (rc) return rc;
  HIPCHK(c, hipSetDevice(c->device));
  uint32_t *d_w = nullptr;
  HIPCHK(c, dalloc(&d_w, x1 - x0));
  rc = ensure_bitmap(c, x0, x1);
  if (rc) return rc;
  {
    Timer t(c, "check_words");
    HIPCHK(c, launch_check_words(view(c), x0, x1, R, d_w, c->d_bitmap, c->stream));
  }
  c->bm_list = false;
  c->bm_x0 = x0 & ~(int64_t)63;
  c->bm_x1 = x1;
  c->bm_R = R;
  c->bm_valid = true;
  if (x1 > x0) HIPCHK(c, hipMemcpyAsync(words, d_w, (x1 - x0) * 4, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  dfree(d_w);
  return SBAM_OK;
}

// Chain pass after a record-0 pass: the list form (launch_chain_list_*) when the PASS0 positions fit its
// scratch (a position list of up to 1/32 of the range), else the per-chunk k_chains walk.
static hipError_t run_chains(sbam_ctx *c, int64_t x0, int64_t x1, int32_t R, int32_t by_key, CountsDev cd,
                             const int32_t *tile_pass0) {
  const int64_t nch = chain_list_chunks(x0, x1);
  const int64_t cap = (x1 - x0) / 32 + 4096;
  hipError_t e;
  if ((e = ensure(&c->d_ccnt, &c->ccnt_cap, (size_t)std::max<int64_t>(nch, 1))) != hipSuccess) return e;
  if ((e = ensure(&c->d_coff2, &c->coff2_cap, (size_t)nch + 1)) != hipSuccess) return e;
  ChainScratch cs{c->d_ccnt, c->d_coff2, nullptr, nullptr, nullptr, nullptr};
  if ((e = launch_chain_list_build(x0, x1, c->d_bitmap, cs, tile_pass0, c->stream)) != hipSuccess) return e;
  int64_t total = 0;
  if ((e = hipMemcpyAsync(&total, c->d_coff2 + nch, 8, hipMemcpyDeviceToHost, c->stream)) != hipSuccess) return e;
  if ((e = hipStreamSynchronize(c->stream)) != hipSuccess) return e;
  c->bm_list = false;
  if (total > cap) return launch_check_full_chains(view(c), x0, x1, R, by_key, cd, c->d_bitmap, c->stream);
  const size_t n = (size_t)std::max<int64_t>(total, 1);
  if ((e = ensure(&c->d_plist, &c->plist_cap, n)) != hipSuccess) return e;
  if ((e = ensure(&c->d_pfb, &c->pfb_cap, n)) != hipSuccess) return e;
  if ((e = ensure(&c->d_pok, &c->pok_cap, n)) != hipSuccess) return e;
  if ((e = ensure(&c->d_nfb, &c->nfb_cap, 3)) != hipSuccess) return e;
  cs.list = c->d_plist;
  cs.ok = c->d_pok;
  cs.fb = c->d_pfb;
  cs.n_fb = c->d_nfb;
  c->bm_list = true;
  c->plist_n = total;
  return launch_chain_list_run(view(c), x0, x1, R, by_key, cd, c->d_bitmap, cs, c->stream);
}

int sbam_check_full_counts(sbam_ctx *c, int64_t x0, int64_t x1, int32_t R, int32_t by_key, sbam_counts *out,
                           uint64_t *bitmap) {
  if (!c || !out) return SBAM_ERR_ARG;
  int rc = check_range_args(c, x0, x1, R);
  if (rc) return rc;
  HIPCHK(c, hipSetDevice(c->device));
  rc = ensure_bitmap(c, x0, x1);
  if (rc) return rc;
  HIPCHK(c, hipMemsetAsync(c->d_counts, 0, kCountsWords * 8, c->stream));
  CountsDev cd;
  cd.counts = c->d_counts;
  cd.positions = cd.counts + 21 * 19;
  cd.rbe = cd.positions + 21;
  cd.pair = cd.rbe + 21 * 128;
  cd.scalars = cd.pair + 19 * 19;
  cd.totals = cd.scalars + 4;
  HIPCHK(c, ensure(&c->d_tcnt, &c->tcnt_cap, (size_t)std::max<int64_t>(4 * check_tiles(x0, x1), 1)));
  cd.tile_pass0 = c->d_tcnt;
  bool tiles = false;
  {
    Timer t(c, "check_full");
    {
      Timer t0(c, "check_pass0");
      HIPCHK(c, launch_check_full_counts(view(c), x0, x1, R, by_key, cd, c->d_bitmap, c->stream, &tiles));
    }
    Timer t1(c, "check_chains");
    HIPCHK(c, run_chains(c, x0, x1, R, by_key, cd, tiles ? c->d_tcnt : nullptr));
  }
  std::vector<unsigned long long> h(kCountsWords);
  HIPCHK(c, hipMemcpyAsync(h.data(), c->d_counts, kCountsWords * 8, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  if (bitmap) {
    int rc2 = copy_bitmap_out(c, x0, x1, bitmap);
    if (rc2) return rc2;
  }
  memset(out, 0, sizeof(*out));
  const unsigned long long *p = h.data();
  for (int k = 0; k < 21; k++)
    for (int f = 0; f < 19; f++) out->counts[k][f] = (int64_t)p[k * 19 + f];
  p += 21 * 19;
  for (int k = 0; k < 21; k++) out->positions[k] = (int64_t)p[k];
  p += 21;
  for (int k = 0; k < 21; k++)
    for (int r = 0; r < 128; r++) out->reads_before_error[k][r] = (int64_t)p[k * 128 + r];
  p += 21 * 128;
  for (int i = 0; i < 19; i++)
    for (int j = 0; j < 19; j++) out->pair_hist[i][j] = (int64_t)p[i * 19 + j];
  p += 19 * 19;
  out->n_positions = x1 - x0;
  out->n_success = (int64_t)p[1];
  out->n_too_few_fixed = (int64_t)p[2];
  out->n_halo = (int64_t)p[3];
  p += 4;
  for (int f = 0; f < 19; f++) out->totals[f] = (int64_t)p[f];
  c->bm_x0 = x0 & ~(int64_t)63;
  c->bm_x1 = x1;
  c->bm_R = R;
  c->bm_valid = true;
  if (out->n_halo) {
    c->err.actual = out->n_halo;
    return set_err(c, SBAM_ERR_HALO, "%lld positions need bytes past the shard", (long long)out->n_halo);
  }
  return SBAM_OK;
}

static int find_record_starts(sbam_ctx *c, const std::vector<int64_t> &x0, int32_t R, int64_t mrs, bool use_bm,
                              std::vector<int64_t> &out) {
  const int64_t n = (int64_t)x0.size();
  out.assign(n, -1);
  if (!n) return SBAM_OK;
  HIPCHK(c, ensure(&c->d_qa, &c->qa_cap, (size_t)n));
  HIPCHK(c, ensure(&c->d_qb, &c->qb_cap, (size_t)n));
  int64_t *d_x = c->d_qa, *d_o = c->d_qb;
  HIPCHK(c, hipMemcpyAsync(d_x, x0.data(), n * 8, hipMemcpyHostToDevice, c->stream));
  const bool bm = use_bm && c->bm_valid && c->bm_R == R;
  {
    Timer t(c, "find_record");
    HIPCHK(c, launch_find_record_starts(view(c), d_x, n, R, mrs, bm ? c->d_bitmap : nullptr, c->bm_x0, c->bm_x1, d_o,
                                        c->stream));
  }
  HIPCHK(c, hipMemcpyAsync(out.data(), d_o, n * 8, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return SBAM_OK;
}

int sbam_find_record_start(sbam_ctx *c, int64_t block_start, int32_t R, int32_t mrs, int32_t *found, sbam_pos *pos,
                           int32_t *delta) {
  if (!c || !found) return SBAM_ERR_ARG;
  int rc = ensure_stream(c);
  if (rc) return rc;
  HIPCHK(c, hipSetDevice(c->device));
  *found = 0;
  const int64_t b = block_at(c, block_start - c->base);
  if (b < 0) return SBAM_OK;  // EOF-marker block / past the stream: the uncompressed stream is empty → None
  std::vector<int64_t> x0{c->h_buoff[b]}, out;
  rc = find_record_starts(c, x0, R, mrs, true, out);
  if (rc) return rc;
  if (out[0] == -2) return set_err(c, SBAM_ERR_HALO, "record search left the shard");
  if (out[0] < 0) return SBAM_OK;
  *found = 1;
  if (pos) *pos = pos_of(c, out[0]);
  if (delta) *delta = (int32_t)(out[0] - x0[0]);
  return SBAM_OK;
}

// ---- splits ----------------------------------------------------------------------------------------
int sbam_file_splits(int64_t file_size, int64_t split_size, int64_t *starts, int64_t *ends, int64_t cap, int64_t *n_out) {
  if (split_size <= 0 || file_size < 0 || !n_out) return SBAM_ERR_ARG;
  // FileInputFormat.getSplits: while (bytesRemaining / splitSize > SPLIT_SLOP) emit; then the remainder.
  int64_t n = 0, off = 0, rem = file_size;
  while ((double)rem / (double)split_size > 1.1) {
    if (n < cap && starts) { starts[n] = off; ends[n] = off + split_size; }
    n++;
    off += split_size;
    rem -= split_size;
  }
  if (rem > 0) {
    if (n < cap && starts) { starts[n] = off; ends[n] = file_size; }
    n++;
  }
  *n_out = n;
  return SBAM_OK;
}

// FindBlockStart → FindRecordStart for Hadoop splits [first, first+count): first-record offsets xs and chain
// ends xe = offset of Pos(split end, 0) (CanLoadBam.scala:195-241).
static int split_starts(sbam_ctx *c, const sbam_split_args *a, int64_t first, int64_t count, std::vector<int64_t> &xs,
                        std::vector<int64_t> &xe) {
  int64_t ns = 0;
  sbam_file_splits(c->file_size, a->split_size, nullptr, nullptr, 0, &ns);
  if (first + count > ns) return set_err(c, SBAM_ERR_ARG, "split range past %lld splits", (long long)ns);
  std::vector<int64_t> st(ns), en(ns);
  sbam_file_splits(c->file_size, a->split_size, st.data(), en.data(), ns, &ns);
  std::vector<int64_t> q(st.begin() + first, st.begin() + first + count), bs(count);
  int rc = sbam_find_block_starts(c, q.data(), count, a->bgzf_blocks_to_check, bs.data());
  if (rc) return rc;
  std::vector<int64_t> x0(count);
  xe.assign(count, 0);
  // block_at / x_end_of for every split: the queries ascend, so each search gallops from the previous answer
  // (10 240 independent binary searches over the host block table took ~1 ms of host time per 10 GB step)
  const int64_t nbh = (int64_t)c->h_bstart.size();
  auto first_ge = [&](int64_t from, int64_t q) {  // first index >= from with h_bstart[index] >= q
    int64_t lo = from, step = 1, hi = from;
    while (hi < nbh && c->h_bstart[hi] < q) {
      lo = hi + 1;
      hi += step;
      step *= 2;
    }
    return (int64_t)(std::lower_bound(c->h_bstart.begin() + lo, c->h_bstart.begin() + std::min(hi, nbh), q) -
                     c->h_bstart.begin());
  };
  int64_t ib = 0, ie = 0;
  for (int64_t i = 0; i < count; i++) {
    const int64_t qb = bs[i] - c->base, qe = en[first + i] - c->base;
    const bool sorted = i == 0 || (bs[i] >= bs[i - 1] && en[first + i] >= en[first + i - 1]);
    ib = first_ge(sorted ? ib : 0, qb);
    ie = first_ge(sorted ? ie : 0, qe);
    const int64_t b = (ib < nbh && c->h_bstart[ib] == qb) ? ib : -1;  // block_at
    if (b < 0) {  // FindRecordStart on the EOF marker: empty stream → None → NoReadFoundException
      return no_read_found(c, bs[i], a->max_read_size);
    }
    x0[i] = c->h_buoff[b];
    xe[i] = ie < nbh ? c->h_buoff[ie] : c->L;  // flat offset of Pos(first block starting at or past the end, 0)
  }
  rc = find_record_starts(c, x0, a->reads_to_check, a->max_read_size, a->use_success_bitmap != 0, xs);
  if (rc) return rc;
  for (int64_t i = 0; i < count; i++) {
    if (xs[i] == -2) return set_err(c, SBAM_ERR_HALO, "record search left the shard");
    if (xs[i] < 0) {
      return no_read_found(c, bs[i], a->max_read_size);
    }
  }
  return SBAM_OK;
}

// Record counts of the chains [xs[i], xe[i]) (RecordStream.scala:27-41).  With try_bitmap and a success bitmap
// covering them, the chains are proven equal to the bitmap's set bits (sbam_records.hip) and counted by
// popcount; else (or if the proof fails) each chain is walked.  Leaves xs/xe on the device (d_sx, d_se).
static int split_counts(sbam_ctx *c, bool try_bitmap, const std::vector<int64_t> &xs, const std::vector<int64_t> &xe,
                        std::vector<int64_t> &cnt, bool *proved) {
  const int64_t n = (int64_t)xs.size();
  *proved = false;
  cnt.assign(n, 0);
  if (!n) return SBAM_OK;
  HIPCHK(c, ensure(&c->d_sx, &c->sx_cap, n));
  HIPCHK(c, ensure(&c->d_se, &c->se_cap, n));
  HIPCHK(c, ensure(&c->d_sn, &c->sn_cap, n));
  HIPCHK(c, hipMemcpyAsync(c->d_sx, xs.data(), n * 8, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(c->d_se, xe.data(), n * 8, hipMemcpyHostToDevice, c->stream));
  const int64_t X0 = *std::min_element(xs.begin(), xs.end());
  const int64_t X1 = *std::max_element(xe.begin(), xe.end());
  Timer t(c, "records");
  if (try_bitmap && c->bm_valid && X0 >= c->bm_x0 && X1 <= c->bm_x1) {
    int32_t *d_fail = reinterpret_cast<int32_t *>(c->d_small + 8);
    const int64_t xa = c->bm_x0 & ~(int64_t)63;
    HIPCHK(c, hipMemsetAsync(d_fail, 0, 4, c->stream));
    // SBAM_FORCE_PROOF=1 (measurement): run the proof even when the list pass found every link, as a bitmap with one
    // false-positive PASS0 site anywhere in the range would (bench.py's loadReads line reports both)
    const char *fp = std::getenv("SBAM_FORCE_PROOF");
    const bool force = fp && *fp && *fp != '0';
    HIPCHK(c, launch_chain_proof(c->d_u, c->L, c->d_bitmap, xa, X0, X1, d_fail,
                                 (c->bm_list && !force) ? c->d_nfb : nullptr, c->stream));
    HIPCHK(c, launch_split_popcounts(c->d_bitmap, xa, c->d_sx, c->d_se, n, c->d_sn, d_fail, c->d_plist, c->plist_n,
                                     c->bm_list ? c->d_nfb : nullptr, c->stream));
    int32_t fail = 1;
    HIPCHK(c, hipMemcpyAsync(&fail, d_fail, 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(cnt.data(), c->d_sn, n * 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (!fail) {
      *proved = true;
      return SBAM_OK;
    }
  }
  HIPCHK(c, launch_record_counts(view(c), c->d_sx, c->d_se, n, c->d_sn, c->stream));
  HIPCHK(c, hipMemcpyAsync(cnt.data(), c->d_sn, n * 8, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  for (int64_t i = 0; i < n; i++) {
    if (cnt[i] == -2) return set_err(c, SBAM_ERR_HALO, "record chain left the shard");
    if (cnt[i] < 0) return set_err(c, SBAM_ERR_INFLATE, "UnexpectedEOF in record stream");
  }
  return SBAM_OK;
}

int sbam_split_records(sbam_ctx *c, const sbam_split_args *a, int64_t first, int64_t count, sbam_pos *first_pos,
                       int32_t *found, int64_t *n_records) {
  if (!c || !a || first < 0 || count < 0) return SBAM_ERR_ARG;
  int rc = ensure_stream(c);
  if (rc) return rc;
  HIPCHK(c, hipSetDevice(c->device));
  std::vector<int64_t> xs, xe, cnt;
  rc = split_starts(c, a, first, count, xs, xe);
  if (rc) return rc;
  bool proved = false;
  rc = split_counts(c, a->use_success_bitmap != 0, xs, xe, cnt, &proved);
  if (rc) return rc;
  int64_t hint = 0;
  for (int64_t i = 0; i < count; i++) {
    if (first_pos) first_pos[i] = pos_of(c, xs[i], &hint);
    if (found) found[i] = cnt[i] > 0;
    if (n_records) n_records[i] = cnt[i];
  }
  return SBAM_OK;
}

int sbam_compute_splits(sbam_ctx *c, const sbam_split_args *a, sbam_split *splits, int64_t cap, int64_t *n_out) {
  if (!c || !a || !n_out) return SBAM_ERR_ARG;
  int64_t ns = 0;
  sbam_file_splits(c->file_size, a->split_size, nullptr, nullptr, 0, &ns);
  std::vector<sbam_pos> fp(ns);
  std::vector<int32_t> fd(ns);
  int rc = sbam_split_records(c, a, 0, ns, fp.data(), fd.data(), nullptr);
  if (rc) return rc;
  std::vector<sbam_pos> firsts;
  for (int64_t i = 0; i < ns; i++)
    if (fd[i]) firsts.push_back(fp[i]);
  const int64_t n = (int64_t)firsts.size();
  *n_out = n;
  if (cap < n) return set_err(c, SBAM_ERR_ARG, "capacity %lld < %lld splits", (long long)cap, (long long)n);
  for (int64_t i = 0; i < n; i++) {
    splits[i].start = firsts[i];
    splits[i].end = (i + 1 < n) ? firsts[i + 1] : sbam_pos{c->file_size, 0, 0};
  }
  return SBAM_OK;
}

int sbam_record_offsets(sbam_ctx *c, int64_t x0, int64_t x_end, int64_t *offsets, int64_t cap, int64_t *n_out) {
  if (!c || !n_out || x0 < 0) return SBAM_ERR_ARG;
  int rc = ensure_stream(c);
  if (rc) return rc;
  HIPCHK(c, hipSetDevice(c->device));
  int64_t *d_o = nullptr;
  HIPCHK(c, dalloc(&d_o, cap));
  HIPCHK(c, launch_record_offsets(view(c), x0, std::min(x_end, c->L), d_o, cap, c->d_small + 4, c->stream));
  int64_t n = 0;
  HIPCHK(c, hipMemcpyAsync(&n, c->d_small + 4, 8, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  if (n < 0) n = -(n + 3);
  if (offsets && n) HIPCHK(c, hipMemcpy(offsets, d_o, std::min(n, cap) * 8, hipMemcpyDeviceToHost));
  dfree(d_o);
  *n_out = n;
  return SBAM_OK;
}

int sbam_record_spans(sbam_ctx *c, const int64_t *offsets, int64_t n, int32_t *ref_id, int32_t *start, int32_t *end) {
  if (!c || n < 0 || (n && (!offsets || !ref_id || !start || !end))) return SBAM_ERR_ARG;
  if (n == 0) return SBAM_OK;
  int rc = ensure_stream(c);
  if (rc) return rc;
  HIPCHK(c, hipSetDevice(c->device));
  int64_t *d_o = nullptr;
  int32_t *d_r = nullptr;
  HIPCHK(c, dalloc(&d_o, n));
  HIPCHK(c, dalloc(&d_r, 3 * n));
  HIPCHK(c, hipMemcpyAsync(d_o, offsets, n * 8, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, launch_record_spans(c->d_u, c->L, d_o, n, d_r, d_r + n, d_r + 2 * n, c->stream));
  HIPCHK(c, hipMemcpyAsync(ref_id, d_r, n * 4, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipMemcpyAsync(start, d_r + n, n * 4, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipMemcpyAsync(end, d_r + 2 * n, n * 4, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  dfree(d_o);
  dfree(d_r);
  return SBAM_OK;
}

// ---- record decode ---------------------------------------------------------------------------------------
int sbam_load_records(sbam_ctx *c, const sbam_split_args *a, int64_t first, int64_t count, int64_t *split_counts_out,
                      int64_t *n_records) {
  if (!c || !a || first < 0 || count < 0) return SBAM_ERR_ARG;
  int rc = ensure_stream(c);
  if (rc) return rc;
  HIPCHK(c, hipSetDevice(c->device));
  c->n_loaded = -1;
  std::vector<int64_t> xs, xe, cnt;
  rc = split_starts(c, a, first, count, xs, xe);
  if (rc) return rc;
  bool proved = false;
  rc = split_counts(c, a->use_success_bitmap != 0, xs, xe, cnt, &proved);
  if (rc) return rc;
  std::vector<int64_t> base(count + 1, 0);
  for (int64_t i = 0; i < count; i++) base[i + 1] = base[i] + cnt[i];
  const int64_t N = base[count];
  HIPCHK(c, ensure(&c->d_sb, &c->sb_cap, count + 1));
  HIPCHK(c, ensure(&c->d_roff, &c->roff_cap, N));
  // column arena: block_pos (8 B) + 10 × 4 B, each column 256-B aligned
  const size_t stride = ((size_t)std::max<int64_t>(N, 1) * 8 + 255) & ~(size_t)255;
  const size_t stride4 = ((size_t)std::max<int64_t>(N, 1) * 4 + 255) & ~(size_t)255;
  HIPCHK(c, ensure(&c->d_rcols, &c->rcols_cap, stride + 10 * stride4));
  {
    uint8_t *p = c->d_rcols;
    RecordColumnsDev &k = c->rcols;
    k.block_pos = reinterpret_cast<int64_t *>(p);
    int32_t *q[10];
    for (int j = 0; j < 10; j++) q[j] = reinterpret_cast<int32_t *>(p + stride + j * stride4);
    k.block_off = q[0]; k.block_size = q[1]; k.ref_id = q[2]; k.pos = q[3];
    k.bin_mq_nl = reinterpret_cast<uint32_t *>(q[4]); k.flag_nc = reinterpret_cast<uint32_t *>(q[5]);
    k.l_seq = q[6]; k.next_ref_id = q[7]; k.next_pos = q[8]; k.tlen = q[9];
  }
  HIPCHK(c, hipMemcpyAsync(c->d_sb, base.data(), (count + 1) * 8, hipMemcpyHostToDevice, c->stream));
  {
    Timer t(c, "load_records");
    if (proved)
      HIPCHK(c, launch_split_offsets(c->d_bitmap, c->bm_x0 & ~(int64_t)63, c->d_sx, c->d_se, c->d_sb, count, c->d_roff,
                                     c->stream));
    else
      HIPCHK(c, launch_record_walk(c->d_u, c->L, c->d_sx, c->d_se, c->d_sb, count, c->d_roff, c->stream));
    HIPCHK(c, launch_record_columns(c->d_u, c->d_roff, N, c->d_bstart, c->d_buoff, c->d_bu, c->nblocks, c->base,
                                    c->rcols, c->stream));
  }
  HIPCHK(c, hipStreamSynchronize(c->stream));
  c->n_loaded = N;
  if (split_counts_out)
    for (int64_t i = 0; i < count; i++) split_counts_out[i] = cnt[i];
  if (n_records) *n_records = N;
  return SBAM_OK;
}

int sbam_get_record_columns(sbam_ctx *c, int64_t i0, int64_t n, const sbam_record_columns *o) {
  if (!c || !o || i0 < 0 || n < 0) return SBAM_ERR_ARG;
  if (c->n_loaded < 0) return set_err(c, SBAM_ERR_STATE, "sbam_load_records has not run");
  if (i0 + n > c->n_loaded)
    return set_err(c, SBAM_ERR_ARG, "records [%lld, %lld) past %lld loaded", (long long)i0, (long long)(i0 + n),
                   (long long)c->n_loaded);
  if (!n) return SBAM_OK;
  HIPCHK(c, hipSetDevice(c->device));
  const RecordColumnsDev &k = c->rcols;
  struct { void *dst; const void *src; size_t w; } cp[] = {
      {o->offset, c->d_roff, 8}, {o->block_pos, k.block_pos, 8}, {o->block_off, k.block_off, 4},
      {o->block_size, k.block_size, 4}, {o->ref_id, k.ref_id, 4}, {o->pos, k.pos, 4},
      {o->bin_mq_nl, k.bin_mq_nl, 4}, {o->flag_nc, k.flag_nc, 4}, {o->l_seq, k.l_seq, 4},
      {o->next_ref_id, k.next_ref_id, 4}, {o->next_pos, k.next_pos, 4}, {o->tlen, k.tlen, 4}};
  for (auto &e : cp)
    if (e.dst)
      HIPCHK(c, hipMemcpyAsync(e.dst, static_cast<const uint8_t *>(e.src) + i0 * e.w, n * e.w, hipMemcpyDeviceToHost,
                               c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return SBAM_OK;
}

int sbam_record_columns_device(sbam_ctx *c, sbam_record_columns *d, int64_t *n_records) {
  if (!c || !d) return SBAM_ERR_ARG;
  if (c->n_loaded < 0) return set_err(c, SBAM_ERR_STATE, "sbam_load_records has not run");
  const RecordColumnsDev &k = c->rcols;
  *d = sbam_record_columns{c->d_roff, k.block_pos, k.block_off, k.block_size, k.ref_id, k.pos,
                           k.bin_mq_nl, k.flag_nc, k.l_seq, k.next_ref_id, k.next_pos, k.tlen};
  if (n_records) *n_records = c->n_loaded;
  return SBAM_OK;
}

}  // extern "C"
