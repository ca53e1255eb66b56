/*
 * sbam.h — C ABI of the MI355X-native spark-bam hot path (libsbam.so).
 *
 * Plain C types only (fixed-width ints, caller-owned host buffers, opaque handle), so a JVM
 * binding (JDK 22 Panama downcalls, or a JNI shim) or ctypes can call it directly; INTEGRATION.md
 * shows the reference-side binding for each entry point.  Every entry point names the reference
 * interface it replaces (paths relative to the spark-bam repository root).
 *
 * Threading / ownership (mirrors the reference's per-Spark-task channels, Channels.scala:15-26,
 * CallPartition.scala:35-37): one handle per task/file-shard, reentrant per handle, no global
 * mutable state, device memory owned by the handle and freed by sbam_close().  Errors are int
 * status codes plus a per-handle error record whose message text equals the reference exception's.
 */
#ifndef SBAM_H
#define SBAM_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes ---------------------------------------------------------------------------- */
#define SBAM_OK 0
#define SBAM_ERR_HEADER_PARSE 1   /* HeaderParseException        bgzf/.../block/HeaderParseException.scala:6-11 */
#define SBAM_ERR_HEADER_SEARCH 2  /* HeaderSearchFailedException bgzf/.../block/FindBlockStart.scala:31-35;
                                     error.position = start, error.actual = positionsAttempted              */
#define SBAM_ERR_INFLATE 3        /* IOException "Expected N decompressed bytes, found M" Stream.scala:52-54 */
#define SBAM_ERR_NO_READ_FOUND 4  /* NoReadFoundException        check/.../bam/spark/FindRecordStart.scala:66-71;
                                     error.position = start, error.expected = maxReadSize                   */
#define SBAM_ERR_NOT_BAM 5        /* require(magic == "BAM\1")   check/.../bam/header/Header.scala:44-46      */
#define SBAM_ERR_ARG 6            /* invalid argument / capacity too small                                  */
#define SBAM_ERR_HIP 7            /* HIP runtime failure (device, allocation, launch)                       */
#define SBAM_ERR_STATE 8          /* stage called out of order (e.g. check before inflate)                  */
#define SBAM_ERR_HALO 9           /* a check needed bytes past a shard's loaded range (grow the halo)       */

typedef struct sbam_ctx sbam_ctx;

/* Virtual position: Pos(blockPos, offset), bgzf/src/main/scala/org/hammerlab/bgzf/Pos.scala:12 */
typedef struct {
  int64_t block_pos;
  int32_t offset;
  int32_t reserved;
} sbam_pos;

/* Split(start, end), check/src/main/scala/org/hammerlab/bam/spark/Split.scala:9-13 */
typedef struct {
  sbam_pos start;
  sbam_pos end;
} sbam_split;

typedef struct {
  int32_t code;      /* SBAM_ERR_* */
  int32_t idx;       /* HeaderParseException idx */
  int64_t actual;    /* HeaderParseException actual / inflate "found" */
  int64_t expected;  /* HeaderParseException expected / inflate "expected" */
  int64_t position;  /* compressed (or split-start) offset the error refers to */
  char message[512]; /* reference exception message text */
} sbam_error;

/* full-check reductions (check/.../full/error/Counts.scala:8-130; cli/.../full/FullCheck.scala:141-191).
 * Results equal to Flags.TooFewFixedBlockBytes (flag 0 alone, readsBeforeError 0) are dropped (counted in
 * n_too_few_fixed); every other Flags result is keyed by numNonZeroFields = popcount(flags) +
 * (readsBeforeError > 0). Flag index order = Flags.scala:201-223 bitset order. */
#define SBAM_NUM_FLAGS 19
#define SBAM_NUM_KEYS 21
#define SBAM_MAX_READS_TO_CHECK 127
typedef struct {
  int64_t totals[SBAM_NUM_FLAGS];                           /* per flag, all keys ("Total error counts") */
  int64_t counts[SBAM_NUM_KEYS][SBAM_NUM_FLAGS];            /* per key, per flag: keys 1-2 always, all with by_key */
  int64_t positions[SBAM_NUM_KEYS];                         /* positions per key */
  int64_t reads_before_error[SBAM_NUM_KEYS][SBAM_MAX_READS_TO_CHECK + 1];
  int64_t pair_hist[SBAM_NUM_FLAGS][SBAM_NUM_FLAGS];        /* key-2 positions by (flag i < flag j) */
  int64_t n_positions;                                      /* positions checked */
  int64_t n_success;                                        /* positions whose call is true */
  int64_t n_too_few_fixed;                                  /* dropped TooFewFixedBlockBytes results */
  int64_t n_halo;                                           /* positions that needed bytes past the shard */
} sbam_counts;

/* Per-position result word of the full checker (full/Checker.scala:22-184):
 * bits 0..18 = Flags bits, bits 24..30 = readsBeforeError (or Success.readsParsed), bit 31 = Success. */
#define SBAM_WORD_SUCCESS 0x80000000u
#define SBAM_WORD_HALO 0x00800000u /* bit 23: result unknown, chain left the shard's loaded bytes */

/* ---- lifetime ------------------------------------------------------------------------------- */

/* Open a BAM file (or a shard of one) on a GPU: copies `len` compressed bytes that sit at file offset
 * `base_offset` of a file of `file_size` bytes into HBM.  For a whole file pass base_offset 0 and
 * file_size == len.  Replaces Channels(path) (load/.../spark/load/Channels.scala:15-26). */
int sbam_open(int device, const uint8_t *data, int64_t len, int64_t base_offset, int64_t file_size,
              sbam_ctx **out);
void sbam_close(sbam_ctx *ctx);
/* Replace the resident compressed bytes of an open context with another byte range (of the same or another
 * file) and drop every derived stage, keeping the device allocations: the streaming form of sbam_open for
 * inputs larger than HBM, one byte-range window after another (a Spark task re-opening its channel at the
 * next split range).  `data` may be pinned host memory; the copy is on the context's stream, so a second
 * context can load the next window while this one computes.  Contig lengths persist only for a later window
 * of the same file (base_offset > 0 and the same file_size); otherwise sbam_header / sbam_set_contig_lengths
 * must run again before a check. */
int sbam_load(sbam_ctx *ctx, const uint8_t *data, int64_t len, int64_t base_offset, int64_t file_size);
/* Size a context's device buffers for windows of up to comp_bytes compressed bytes, n_blocks BGZF blocks,
 * ubytes uncompressed bytes and n_records records (0: leave the record-sized buffers alone), so that no later
 * sbam_load / stage reallocates: the buffers are grow-only, and growing one is a hipFree + hipMalloc of up to
 * tens of GB that synchronises the device (a streamed Spark task whose next split range is larger than any
 * before it).  Allocates nothing that is already large enough.  The resident compressed bytes and contig lengths
 * are kept; when any stage buffer grows on a context that has already run a stage, every derived stage is
 * dropped (as sbam_reset) and later queries re-run them.  (No reference counterpart: the JVM channel has no
 * device memory; CanLoadBam.scala:281-334 re-opens a channel per split.) */
int sbam_reserve(sbam_ctx *ctx, int64_t comp_bytes, int64_t n_blocks, int64_t ubytes, int64_t n_records);
const sbam_error *sbam_last_error(const sbam_ctx *ctx);
/* The path (Path.toString) that exception messages name, as the reference's HeaderSearchFailedException /
 * NoReadFoundException format it (HeaderSearchFailedException.scala:7-12, FindRecordStart.scala:66-71);
 * default "<bytes>". */
int sbam_set_path(sbam_ctx *ctx, const char *path);
/* Drop every derived stage (block table, stream, bitmap) but keep the compressed bytes and the device
 * allocations, so the pipeline can be re-run from the resident input without allocating (bench). */
int sbam_reset(sbam_ctx *ctx);
const char *sbam_version(void);

/* ---- BGZF layer -------------------------------------------------------------------------------- */

/* FindBlockStart.apply for a batch of split starts (bgzf/.../block/FindBlockStart.scala:8-36).
 * out[i] = first start[i]+pos, pos < 65536, at which `blocks_to_check` BGZF headers chain. */
int sbam_find_block_starts(sbam_ctx *ctx, const int64_t *starts, int64_t n, int32_t blocks_to_check, int64_t *out);

/* MetadataStream from the shard's first block (offset 0 of a whole file; FindBlockStart(base_offset)
 * of a shard) to the end of the stream (MetadataStream.scala:23-54): builds the device block table.
 * *n_blocks receives the block count. */
int sbam_scan_blocks(sbam_ctx *ctx, int64_t *n_blocks);

/* Copy the block table (IndexBlocks format: start, compressedSize, uncompressedSize;
 * bgzf/.../index/IndexBlocks.scala:40-44) plus each block's offset in the uncompressed stream. */
int sbam_get_blocks(sbam_ctx *ctx, int64_t *start, int32_t *csize, int32_t *usize, int64_t *uoff, int64_t cap);

/* Inflate every block of the table into the device-resident uncompressed stream
 * (Stream.scala:31-71 with Inflater(nowrap=true)); *uncompressed_size receives its length. */
int sbam_inflate(sbam_ctx *ctx, int64_t *uncompressed_size);

/* Blocks the last sbam_inflate handed from the wave-parallel decoder to the exact per-lane one (stored or
 * invalid blocks, incomplete codes, streams that end before ISIZE or run past it); for parity tests and profiles. */
int sbam_inflate_fallbacks(sbam_ctx *ctx, int64_t *n);

/* Copy uncompressed bytes [off, off+len) of the stream to the host. */
int sbam_read_uncompressed(sbam_ctx *ctx, int64_t off, int64_t len, uint8_t *out);

/* Pos <-> flat uncompressed offset (UncompressedBytes.scala:17-19,65-78). */
int sbam_pos_to_offset(sbam_ctx *ctx, sbam_pos pos, int64_t *offset);
int sbam_offset_to_pos(sbam_ctx *ctx, int64_t offset, sbam_pos *pos);

/* ---- BAM header (check/.../bam/header/Header.scala:26-60; ContigLengths.scala:33-55) ---------- */

/* n_ref and contig lengths (cap entries), end_pos = Header.endPos.  Must follow sbam_inflate on a
 * whole file; a shard takes them from sbam_set_contig_lengths (the broadcast in CanLoadBam.scala:179-180). */
int sbam_header(sbam_ctx *ctx, int32_t *n_ref, int64_t *lengths, int32_t cap, sbam_pos *end_pos);
int sbam_set_contig_lengths(sbam_ctx *ctx, int32_t n_ref, const int64_t *lengths);

/* ---- record-boundary checkers --------------------------------------------------------------- */

/* eager.Checker at every uncompressed offset in [x0, x1) (check/.../check/eager/Checker.scala:24-126):
 * bit i of bitmap (LSB-first within uint64 words) = call at x0+i.  bitmap may be NULL (device-only). */
int sbam_check_eager(sbam_ctx *ctx, int64_t x0, int64_t x1, int32_t reads_to_check, uint64_t *bitmap);

/* full.Checker result words for [x0, x1) (check/.../check/full/Checker.scala:22-184). */
int sbam_check_full_words(sbam_ctx *ctx, int64_t x0, int64_t x1, int32_t reads_to_check, uint32_t *words);

/* full.Checker over [x0, x1) reduced to full-check Counts + success bitmap (device-resident; copied
 * to success_bitmap when non-NULL).  Replaces the per-position RDD + reduceByKey of FullCheck.scala:117-191.
 * by_key = 0 fills what the full-check report prints (totals, keys 1-2 per flag, positions per key, close-call
 * pairs, readsBeforeError); by_key = 1 also fills counts[k][f] for every key (negativesByNumNonzeroFields). */
int sbam_check_full_counts(sbam_ctx *ctx, int64_t x0, int64_t x1, int32_t reads_to_check, int32_t by_key,
                           sbam_counts *counts, uint64_t *success_bitmap);

/* FindRecordStart.withDelta (check/.../bam/spark/FindRecordStart.scala:30-63) from Pos(block_start, 0):
 * *found = 0 means None. */
int sbam_find_record_start(sbam_ctx *ctx, int64_t block_start, int32_t reads_to_check, int32_t max_read_size,
                           int32_t *found, sbam_pos *pos, int32_t *delta);

/* ---- splits and records (load/.../spark/load/CanLoadBam.scala:173-334) ----------------------- */

typedef struct {
  int64_t split_size;         /* MaxSplitSize (hadoop FileSplits max split size)  */
  int32_t bgzf_blocks_to_check; /* default 5  (bgzf/.../block/package.scala:20-21) */
  int32_t reads_to_check;     /* default 10 (check/.../check/package.scala:17-18)  */
  int32_t max_read_size;      /* default 10_000_000 (check/.../check/package.scala:28-29) */
  int32_t use_success_bitmap; /* 1: reuse the bitmap of a preceding sbam_check_full_counts over the stream */
} sbam_split_args;

/* Hadoop FileSplits of the whole file (FileInputFormat rule, SPLIT_SLOP 1.1): n_out splits [start, end). */
int sbam_file_splits(int64_t file_size, int64_t split_size, int64_t *starts, int64_t *ends, int64_t cap,
                     int64_t *n_out);

/* For Hadoop splits [first, first+count) of the file: FindBlockStart → FindRecordStart → record chain
 * with Pos < (end, 0).  Writes each split's first-record position (found[i]=0 when the split is empty or
 * past the shard) and record count (= the partition size of loadReads / loadReadsAndPositions). */
int sbam_split_records(sbam_ctx *ctx, const sbam_split_args *args, int64_t first, int64_t count, sbam_pos *first_pos,
                       int32_t *found, int64_t *n_records);

/* loadSplitsAndReads' splits for the whole file (CanLoadBam.scala:245-279): first positions of the non-empty
 * partitions paired by sliding2(Pos(fileSize, 0)). */
int sbam_compute_splits(sbam_ctx *ctx, const sbam_split_args *args, sbam_split *splits, int64_t cap, int64_t *n_out);

/* Record chain from flat offset x0 while offset < x_end (RecordStream.scala:27-41): record start offsets
 * (cap entries) and *n_out records; record bytes are stream[off, off+4+block_size). */
int sbam_record_offsets(sbam_ctx *ctx, int64_t x0, int64_t x_end, int64_t *offsets, int64_t cap, int64_t *n_out);

/* Reference spans of the records at the n stream offsets (loadBamIntervals' region filter, CanLoadBam.scala:
 * 107-135, 423-431): ref_id, start = POS (0-based) and end = POS + the CIGAR's reference length (M/D/N/=/X),
 * i.e. [getStart - 1, getEnd); unmapped records (flag 4) get end = 0, htsjdk's getAlignmentEnd. */
int sbam_record_spans(sbam_ctx *ctx, const int64_t *offsets, int64_t n, int32_t *ref_id, int32_t *start, int32_t *end);

/* ---- record decode: loadReads / loadReadsAndPositions (CanLoadBam.scala:221-241, 281-334) ------------- */

/* Per-record columns: the record's flat stream offset, its Pos, and the BAM fixed fields (SAM spec §4.2, the
 * part htsjdk BAMRecordCodec.decode reads eagerly: RecordStream.scala:16-33).  Record bytes are
 * stream[offset, offset + 4 + block_size) (sbam_read_uncompressed).  Any pointer may be NULL (not copied). */
typedef struct {
  int64_t *offset;
  int64_t *block_pos;   /* Pos.blockPos */
  int32_t *block_off;   /* Pos.offset   */
  int32_t *block_size;
  int32_t *ref_id;
  int32_t *pos;
  uint32_t *bin_mq_nl;  /* bin << 16 | MAPQ << 8 | l_read_name */
  uint32_t *flag_nc;    /* FLAG << 16 | n_cigar_op */
  int32_t *l_seq;
  int32_t *next_ref_id;
  int32_t *next_pos;
  int32_t *tlen;
} sbam_record_columns;

/* Records of Hadoop splits [first, first+count) — the partitions of loadReadsAndPositions, in split order —
 * decoded into device-resident columns owned by ctx (valid until the next load, reset or close).
 * split_counts[count] (may be NULL) receives the partition sizes, *n_records their sum.  With
 * use_success_bitmap and a preceding full check over the range, the chains are proven equal to the checker's
 * success bitmap and listed in parallel; otherwise (or when the proof fails) each split's chain is walked. */
int sbam_load_records(sbam_ctx *ctx, const sbam_split_args *args, int64_t first, int64_t count, int64_t *split_counts,
                      int64_t *n_records);

/* Copy records [i0, i0+n) of the last sbam_load_records into caller-owned host columns. */
int sbam_get_record_columns(sbam_ctx *ctx, int64_t i0, int64_t n, const sbam_record_columns *out);

/* Device pointers of the last sbam_load_records' columns (for in-process GPU consumers; no copy). */
int sbam_record_columns_device(sbam_ctx *ctx, sbam_record_columns *dev, int64_t *n_records);

/* ---- timing support for bench/profiling -------------------------------------------------------- */
/* Device time (ms, HIP events on the library's stream) of the most recent launch of a named kernel
 * family: "scan", "inflate", "check_full", "check_eager", "records", "load_records". Returns -1 if none. */
double sbam_last_kernel_ms(sbam_ctx *ctx, const char *kernel);

#ifdef __cplusplus
}
#endif
#endif /* SBAM_H */
