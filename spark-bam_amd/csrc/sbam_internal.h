// sbam_internal.h — launch wrappers shared by the kernels (sbam_kernels.hip) and the C-ABI host
// layer (sbam_api.cpp).  Not part of the public ABI (include/sbam.h is).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdlib>
#include <stdint.h>

namespace sbam {

// One BGZF header candidate found by the byte scan (Header.make, bgzf/.../block/Header.scala:48-83).
struct Candidate {
  int64_t pos;    // offset in the loaded buffer
  int32_t hsize;  // 18 + XLEN - 6
  int32_t csize;  // BSIZE + 1
  int32_t isize;  // ISIZE (valid when flags & CAND_ISIZE)
  int32_t flags;  // CAND_*
};
enum : int32_t { CAND_ISIZE = 1, CAND_EMPTY = 2 };

// Device view of the BGZF block table (struct of arrays; offsets relative to the loaded buffer).
struct BlockTable {
  const int64_t *start;
  const int32_t *hsize;
  const int32_t *csize;
  const int32_t *usize;
  const int64_t *uoff;
  int64_t n;
};

// The decode -> resolve token pool.  Block b's u16 tokens live in its main region (1 B per uncompressed byte,
// tok_region in sbam_inflate.hip: room for (usize + 16) / 2 tokens) unless base[b] >= 0: then at arena + base[b],
// a region of 2 usize + 32 B taken from the arena by a block that needs more (the exact decoder's blocks, and
// blocks whose wave decode outgrows the main region: they move there).  arena_used counts every request, also
// those past arena_cap (the block then reports INF_OVERFLOW and the host grows the arena and inflates again).
struct TokPool {
  uint8_t *main;
  uint8_t *arena;
  int64_t arena_cap;
  unsigned long long *arena_used;
  int64_t *base;
};

// Stream under check: uncompressed bytes u[0, L) (+ zero pad), contig lengths, EOF semantics.
struct StreamView {
  const uint8_t *u;
  int64_t L;
  const int64_t *lens;  // contig lengths (device)
  int32_t nref;
  int32_t eof_real;  // 1: L is the file's end; 0: a shard, reads past L are HALO
};

struct CountsDev {  // mirrors sbam_counts (int64 fields) in device memory
  unsigned long long *counts;  // [21][19]
  unsigned long long *positions;  // [21]
  unsigned long long *rbe;  // [21][128]
  unsigned long long *pair;  // [19][19]
  unsigned long long *scalars;  // n_positions, n_success, n_too_few_fixed, n_halo
  unsigned long long *totals;   // [19] per-flag totals over every counted position
  // [ntiles][4]: the record-0 pass's PASS0 positions per tile and wave (set only for the bit-sliced pass, which then
  // writes every tile's; the chain pass's chunk counts come from these instead of a second read of the bitmap)
  int32_t *tile_pass0 = nullptr;
};

// Device columns of decoded records (sbam_records.hip); mirrors sbam_record_columns minus the offsets.
struct RecordColumnsDev {
  int64_t *block_pos;
  int32_t *block_off, *block_size, *ref_id, *pos;
  uint32_t *bin_mq_nl, *flag_nc;
  int32_t *l_seq, *next_ref_id, *next_pos, *tlen;
};

constexpr int kScanChunk = 1 << 20;  // bytes per workgroup in the BGZF candidate scan
constexpr int kScanSlots = 512;      // candidate slots per chunk in the one-pass scan (>= 2 KiB per block)
constexpr int kStreamPad = 16384;  // zero pad behind the uncompressed stream (>= checker LDS window)
constexpr int kCompPad = 256;  // zero pad behind the compressed bytes (bit-reader / input-ring lookahead)

hipError_t launch_scan_count(const uint8_t *d, int64_t D, int32_t *chunk_counts, int64_t nchunks, hipStream_t s);
hipError_t launch_scan_slots(const uint8_t *d, int64_t D, int32_t *chunk_counts, int64_t nchunks, Candidate *slots,
                             int64_t *overflow, hipStream_t s);
hipError_t launch_scan_compact(const Candidate *slots, const int32_t *chunk_counts, const int64_t *chunk_offsets,
                               int64_t nchunks, Candidate *out, hipStream_t s);
hipError_t launch_scan_prefix(int32_t *chunk_counts, int64_t nchunks, int64_t *chunk_offsets, int64_t *total,
                              hipStream_t s);
hipError_t launch_scan_write(const uint8_t *d, int64_t D, const int64_t *chunk_offsets, int64_t nchunks,
                             Candidate *cands, hipStream_t s);
hipError_t launch_chain_verify(const Candidate *cands, int64_t ncand, int64_t first, int64_t D, int64_t *first_stop,
                               hipStream_t s);
hipError_t launch_find_block_starts(const uint8_t *d, int64_t D, const Candidate *cands, int64_t ncand,
                                    const int64_t *starts, int64_t n, int32_t blocks_to_check, int64_t *out,
                                    hipStream_t s);
// (+ uoff[0..n]: the uncompressed offsets, computed on the device; wsum: (n + 255) / 256 int64 of scratch)
hipError_t launch_gather_blocks(const Candidate *cands, int64_t first, int64_t n, int64_t *start, int32_t *hsize,
                                int32_t *csize, int32_t *usize, int64_t *wsum, int64_t *uoff, hipStream_t s);
// Inflate (sbam_inflate.hip): entropy decode into per-block token regions (wave-parallel fast path, per-lane
// exact path for the blocks it hands over), then LZ77 resolve into `out`.  tok: inflate_token_bytes(L, nb) bytes;
// slow: nb int32; counters: 3 × u32 device scratch, reset by the decode launch.
inline size_t inflate_token_bytes(int64_t L, int64_t nb) {
  // main regions (+1 KiB: the resolver reads up to 2 x 64 + 1 tokens past a step's start)
  return (((size_t)L + 15) & ~(size_t)15) + 32 * (size_t)nb + 1024;
}
// default arena: 1/16 of the uncompressed bytes (the synthetic BAM needs none; stored blocks need 2 B per byte)
// (SBAM_ARENA_MB overrides it: tests of the arena's growth)
inline size_t inflate_arena_bytes(int64_t L) {
  const char *e = std::getenv("SBAM_ARENA_MB");
  if (e && *e) return (size_t)std::atoll(e) << 20;
  return (size_t)L / 16 + (1u << 20);
}
hipError_t launch_inflate_decode(const uint8_t *d, int64_t D, BlockTable bt, TokPool tok, uint8_t *out,
                                 int32_t *status, int32_t *found, int32_t *slow, unsigned int *counters,
                                 hipStream_t s);
// list (nlist blocks) or every block; blocks with a distance past their first byte are appended to redo[*nredo]
hipError_t launch_inflate_resolve(BlockTable bt, uint8_t *out, TokPool tok, const int32_t *found,
                                  const int32_t *list, int64_t nlist, int32_t *redo, unsigned int *nredo,
                                  hipStream_t s);
// the exact decoder over list[0 .. counters[2]) (the resolver's redo list)
hipError_t launch_inflate_redo(const uint8_t *d, int64_t D, BlockTable bt, TokPool tok, const int32_t *list,
                               unsigned int *counters, int32_t *status, int32_t *found, hipStream_t s);
// first_err = min block index with status != 0 (caller presets ~0)
hipError_t launch_first_error(const int32_t *status, int64_t n, unsigned long long *first_err, hipStream_t s);
hipError_t launch_lower_bound(const Candidate *c, int64_t n, int64_t q, int64_t *out, hipStream_t s);
// Bitmaps cover [x0 & ~63, x1): bit (x - (x0 & ~63)) = call at x (0 for x < x0).
// *tiles_counted: whether cd.tile_pass0 now holds every tile's PASS0 count (the bit-sliced pass ran)
hipError_t launch_check_full_counts(StreamView sv, int64_t x0, int64_t x1, int32_t R, int32_t by_key, CountsDev cd,
                                    unsigned long long *bitmap, hipStream_t s, bool *tiles_counted);
int64_t check_tiles(int64_t x0, int64_t x1);  // record-0 pass tiles of [x0, x1)
// (launch_check_full_counts runs the record-0 pass; launch_check_full_chains then resolves the PASS0 chains)
hipError_t launch_check_full_chains(StreamView sv, int64_t x0, int64_t x1, int32_t R, int32_t by_key, CountsDev cd,
                                    unsigned long long *bitmap, hipStream_t s);
// list-form chain pass (sbam_check.hip): scratch owned by the context
struct ChainScratch {
  int32_t *chunk_cnt;             // [nchunks]
  int64_t *chunk_off;             // [nchunks + 1]; [nchunks] = number of PASS0 positions
  int64_t *list;                  // PASS0 positions in order
  uint8_t *ok;                    // link bits
  int64_t *fb;                    // fallback positions
  unsigned long long *n_fb;       // fallback count
};
int64_t chain_list_chunks(int64_t x0, int64_t x1);
// tile_pass0 (or nullptr: count the bitmap): the record-0 pass's per-tile counts (CountsDev::tile_pass0)
hipError_t launch_chain_list_build(int64_t x0, int64_t x1, const unsigned long long *bitmap, const ChainScratch &cs,
                                   const int32_t *tile_pass0, hipStream_t s);
hipError_t launch_chain_list_run(StreamView sv, int64_t x0, int64_t x1, int32_t R, int32_t by_key, CountsDev cd,
                                 unsigned long long *bitmap, const ChainScratch &cs, hipStream_t s);
hipError_t launch_check_eager_pass0(StreamView sv, int64_t x0, int64_t x1, int32_t R, unsigned long long *bitmap,
                                    hipStream_t s);
hipError_t launch_check_words(StreamView sv, int64_t x0, int64_t x1, int32_t R, uint32_t *words,
                              unsigned long long *bitmap, hipStream_t s);
hipError_t launch_find_record_starts(StreamView sv, const int64_t *x0, int64_t n, int32_t R, int64_t max_read_size,
                                     const unsigned long long *bitmap, int64_t bitmap_x0, int64_t bitmap_x1,
                                     int64_t *out, hipStream_t s);
hipError_t launch_record_counts(StreamView sv, const int64_t *x0, const int64_t *x_end, int64_t n, int64_t *counts,
                                hipStream_t s);
hipError_t launch_record_offsets(StreamView sv, int64_t x0, int64_t x_end, int64_t *offsets, int64_t cap,
                                 int64_t *n_out, hipStream_t s);
// Record chains of splits and record decode (sbam_records.hip).  Bitmaps as for the checker: bit (x - xa) = call
// at x, xa 64-aligned.  fail: i32 device flag, set to 1 when the chain is not the bitmap's set bits.
hipError_t launch_chain_proof(const uint8_t *u, int64_t L, const unsigned long long *bm, int64_t xa, int64_t X0,
                              int64_t X1, int32_t *fail, const unsigned long long *exact, hipStream_t s);
// (list, nlist, exact: the chain pass's PASS0 list and counters when the bitmap came from it, else nullptr)
hipError_t launch_split_popcounts(const unsigned long long *bm, int64_t xa, const int64_t *xs, const int64_t *xe,
                                  int64_t n, int64_t *counts, int32_t *fail, const int64_t *list, int64_t nlist,
                                  const unsigned long long *exact, hipStream_t s);
hipError_t launch_split_offsets(const unsigned long long *bm, int64_t xa, const int64_t *xs, const int64_t *xe,
                                const int64_t *base, int64_t n, int64_t *out, hipStream_t s);
hipError_t launch_record_walk(const uint8_t *u, int64_t L, const int64_t *xs, const int64_t *xe, const int64_t *base,
                              int64_t n, int64_t *out, hipStream_t s);
hipError_t launch_record_spans(const uint8_t *u, int64_t L, const int64_t *offs, int64_t n, int32_t *ref_id,
                               int32_t *start, int32_t *end, hipStream_t s);
hipError_t launch_record_columns(const uint8_t *u, const int64_t *offs, int64_t n, const int64_t *bstart,
                                 const int64_t *buoff, const int32_t *busize, int64_t nblocks, int64_t file_base,
                                 RecordColumnsDev cols, hipStream_t s);

}  // namespace sbam
