// fpm_kernels.hpp — launch interface between the C-ABI (fpm_api.cpp) and the
// gfx950 kernels (sketch.hip, dist.hip, fingerprint.hip).  Host-only types.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fpm {

// One tile = a contiguous byte range of the packed, separator-delimited sequence
// buffer, all of it from one sketch group.  Every k-mer start of the tile lies
// in [byte_off, byte_off + n_bytes - k]; windows that cross a 0x00 separator are
// invalid by construction (0x00 is never in an alphabet).
struct TileDesc {
    uint64_t byte_off;
    uint32_t n_bytes;
    uint32_t out_row;   // row of the output (or temp) matrix this tile writes
    uint32_t thr_slot;  // 0: keep every hash; i > 0: keep hashes <= thr[i - 1] (long groups)
    uint32_t pad;       // the tile's group (read by the -M multiplicity pass only)
};

struct SketchKParams {
    uint32_t k;
    uint32_t s;             // sketch size (row stride of the output matrix)
    uint32_t seed;
    uint32_t use64;
    uint32_t canonical;
    uint32_t preserve_case;
    uint32_t compl_acgt;    // every alphabet byte is one of A C G T: complement by bit ops
    uint8_t alphabet[256];  // 1 = valid (after uppercasing)
    uint8_t complement[256];
};

// Pairwise merge of two ascending distinct lists into the first s distinct of
// their union (bottom-s of a union = bottom-s of the union of bottom-s sets).
struct MergeDesc {
    const uint64_t *a; const uint32_t *alen;
    const uint64_t *b; const uint32_t *blen;   // b == nullptr: copy a
    uint64_t *c; uint32_t *clen;
};

// numer / denom output cells of the dist grid: u32, or u16 (c16) when the sketch size fits
// (fpm_dist_dev16: counts <= s <= 65535, 4 bytes per pair instead of 8)
struct Counts {
    void *numer = nullptr, *denom = nullptr;
    bool c16 = false;
};

// Tile capacity classes (k-mer starts per tile).
constexpr int kTileClasses = 6;
constexpr uint32_t kTileCap[kTileClasses] = {256, 512, 1024, 2048, 4096, 8192};

// class-4 (4096-window) tiles that all carry a bound (thr_slot != 0): survivors only; tiles
// with more than the kernel holds are appended to d_redo (count *d_redo_n, zeroed by the
// caller) for launch_sketch_tiles
hipError_t launch_sketch_tiles_thr(const uint8_t *d_seq, const TileDesc *d_tiles, uint32_t n_tiles,
                                   const SketchKParams &p, const uint64_t *d_thr, uint64_t *d_out,
                                   uint32_t *d_count, TileDesc *d_redo, uint32_t *d_redo_n,
                                   hipStream_t st);
// the tiles a launch_sketch_tiles_thr pass listed (d_redo[0 .. *d_redo_n), at most max_tiles),
// through the plain P = 4096 kernel, the count read on the device
hipError_t launch_sketch_redo(const uint8_t *d_seq, const TileDesc *d_redo, const uint32_t *d_redo_n,
                              uint32_t max_tiles, const SketchKParams &p, const uint64_t *d_thr,
                              uint64_t *d_out, uint32_t *d_count, hipStream_t st);
// survivors one THR tile holds (kBlock * kSurv + kSurvShared, sketch.hip)
constexpr uint32_t kThrTileKeys = 1024;
hipError_t launch_sketch_tiles(int cls, const uint8_t *d_seq, const TileDesc *d_tiles,
                               uint32_t n_tiles, const SketchKParams &p, const uint64_t *d_thr,
                               uint64_t *d_out, uint32_t *d_count, hipStream_t st);
// -M: pass 0 counts / first positions of the final hashes, pass 1 the final maximum up to T_top
hipError_t launch_sketch_mult(int cls, int pass, const uint8_t *d_seq, const TileDesc *d_tiles,
                              uint32_t n_tiles, const SketchKParams &p, const uint64_t *d_rows,
                              const uint32_t *d_count, uint32_t *d_mult,
                              unsigned long long *d_first, const uint64_t *d_ttop, hipStream_t st);
hipError_t launch_mult_ttop(const uint32_t *d_count, uint32_t n_groups, uint32_t s,
                            const unsigned long long *d_first, uint64_t *d_ttop, hipStream_t st);
// thr_safe[i] = s-th smallest of sample row srow[i] when it holds s hashes, else no bound;
// thr[i] = its kt[i]-th smallest (d_kt null: thr = thr_safe)
hipError_t launch_sketch_threshold(const uint32_t *d_srow, uint32_t n_slots, const uint64_t *d_rows,
                                   const uint32_t *d_count, uint32_t s, const uint32_t *d_kt,
                                   uint64_t *d_thr, uint64_t *d_thr_safe, hipStream_t st);
// slots whose group (slot_group[i]) ended with fewer than s hashes under thr < thr_safe:
// listed (d_short_slots, count *d_n_short, zeroed by the caller), with `raise` thr raised to
// thr_safe
// samples (sample row srow[i]) left with fewer than s hashes under their a-priori bound
// d_sbound[i] (< ~0): listed (count *d_n_short, zeroed by the caller), with `raise` the bound
// lifted to ~0
hipError_t launch_sketch_sample_short(const uint32_t *d_srow, uint32_t n_slots,
                                      const uint32_t *d_count, uint32_t s, uint64_t *d_sbound,
                                      uint32_t *d_n_short, uint32_t *d_short_slots, bool raise,
                                      hipStream_t st);
hipError_t launch_sketch_short(const uint32_t *d_slot_group, uint32_t n_slots,
                               const uint32_t *d_count, uint32_t s, uint64_t *d_thr,
                               const uint64_t *d_thr_safe, uint32_t *d_n_short,
                               uint32_t *d_short_slots, bool raise, hipStream_t st);
uint32_t merge_small_cap();   // list length merge_small_kernel stages in LDS
// one long group's sketch selected from its bounded tile lists (rows row_ids[row_begin ..
// row_begin + n_rows)) into out_row; slot: its bound thr[slot] (0xFFFFFFFF: none, the
// sample pass of long groups)
struct SelDesc { uint32_t row_begin, n_rows, out_row, slot; };
uint32_t group_select_cap();   // keys one selection stages in LDS (sketch sizes up to ~0.85 x)
// *failed |= 1 when a group's keys below the cut do not fit (the caller merges instead)
hipError_t launch_group_select(const SelDesc *d_desc, uint32_t n, const uint32_t *d_row_ids,
                               uint64_t *d_rows, uint32_t *d_count, uint32_t s,
                               const uint64_t *d_thr, uint32_t *d_failed, hipStream_t st);
// small: the round's lists are estimated short (merge_small_kernel; exact for any length)
// merge_small_kernel launches whose lists overflowed its LDS cap since the last call (reset)
hipError_t merge_small_spills(uint64_t *count);
hipError_t launch_merge(const MergeDesc *d_desc, uint32_t n, uint32_t s, bool small,
                        hipStream_t st);

hipError_t launch_fp_hash(const uint64_t *d_vals, const uint64_t *d_line_off, uint64_t n_lines,
                          uint32_t seed, uint32_t use64, void *d_out, hipStream_t st);

hipError_t launch_compare_grid(const void *d_ref, const uint32_t *d_ref_len, uint64_t ref_stride,
                               uint32_t n_ref, const void *d_qry, const uint32_t *d_qry_len,
                               uint64_t qry_stride, uint32_t n_qry, uint32_t hash_bytes,
                               uint32_t sketch_size, Counts cnt, hipStream_t st);

// dense walk of u32 lists on 16-bit rank images (dist.hip), for 64 <= min(S, stride) <= 1023;
// scratch from compare_grid_img_scratch
bool compare_grid_img_ok(uint32_t hash_bytes, uint32_t sketch_size, uint64_t ref_stride,
                         uint64_t qry_stride);
void compare_grid_img_scratch(uint32_t n_qry, uint32_t sketch_size, uint64_t ref_stride,
                              uint64_t qry_stride, size_t *ublk_bytes, size_t *bimg_bytes);
hipError_t launch_compare_grid_img(const void *d_ref, const uint32_t *d_ref_len,
                                   uint64_t ref_stride, uint32_t n_ref, const void *d_qry,
                                   const uint32_t *d_qry_len, uint64_t qry_stride, uint32_t n_qry,
                                   uint32_t sketch_size, void *ublk, void *bimg, Counts cnt,
                                   hipStream_t st);
// the record rows of one side of a candidate walk (launch_record_rows): values, positions,
// counts, row stride; val == nullptr: none (the walk starts at (0, 0))
struct RecRows {
    const void *val = nullptr;
    const uint32_t *pos = nullptr, *len = nullptr;
    uint64_t stride = 0;
};
// the literal walk of each candidate pair; with record rows of both sides (unsorted lists),
// only the stretches where both running maxima equal a shared record are walked
hipError_t launch_walk_candidates(const uint64_t *d_cand, const unsigned long long *d_n_cand,
                                  uint64_t cap, const void *d_ref, const uint32_t *d_ref_len,
                                  uint64_t ref_stride, uint32_t n_ref, const void *d_qry,
                                  const uint32_t *d_qry_len, uint64_t qry_stride,
                                  uint32_t hash_bytes, uint32_t S, Counts cnt, RecRows rec_ref,
                                  RecRows rec_qry, hipStream_t st);

// bucket index over ref hashes (dist_index.hip)
constexpr uint32_t kIdxL1 = 10;        // level-1 partition bits
constexpr uint32_t kIdxTile = 16384;   // the most matrix cells per level-1 tile (~16 entries per partition)
struct IdxGeom {
    uint32_t l2;       // level-2 bits (1..14)
    uint32_t nbits;    // bucket bits = kIdxL1 + l2
    uint32_t rbits;    // ref-id bits in a u32 entry
    uint32_t fbits;    // key-fingerprint bits in a u32 entry (32 - rbits, >= 8)
    uint32_t ntiles;   // level-1 tiles
    uint32_t tile;     // matrix cells per level-1 tile (<= kIdxTile, a multiple of 1024)
    // device pointer: the largest indexed key (idx_kmax_kernel), from which every kernel
    // derives the bucket scale (bucket_of / key_fp in dist_index.hip)
    const unsigned long long *kmax;
    // level-1 partition capacity of the one-pass scatter (tent holds kParts x cap entries,
    // each tile appends to its partitions by one atomic per partition); 0 = the exact
    // two-pass build (histogram + scan, tent holds E entries)
    uint32_t cap;
};
// entries of the level-1 staging buffer `tent` the build needs
uint64_t idx_tent_words(const IdxGeom &g, uint64_t E);
hipError_t launch_idx_build(const void *d_ref, const uint32_t *d_ref_len, uint64_t stride,
                            uint32_t n_ref, uint32_t hash_bytes, IdxGeom g, uint32_t *tile_hist,
                            uint32_t *tile_off, uint32_t *scan_s, uint64_t *tent,
                            uint32_t *dir, uint32_t *entries, uint32_t *unsorted,
                            unsigned long long *self_events, unsigned long long *zero,
                            uint32_t nzero, unsigned long long *acc, uint32_t *part_fill,
                            uint32_t *overflow, hipStream_t st,
                            unsigned long long *zero_x = nullptr);
// zero[0..nzero) (and *zero_x when given) is cleared first; acc[0..1]: two words that start at
// zero and are left at zero.
// One-pass build (g.cap != 0): part_fill holds 2^kIdxL1 u32 (cleared by the build), *overflow
// (inside zero[]) is set when a partition exceeded cap: the index is then unusable and the
// caller rebuilds with g.cap = 0
uint64_t scan_scratch_words(uint64_t n);
// copy n (<= kPubWords - 1) u64 counters into host-mapped memory, then write `seq` into its
// last word (system-scope fence between): the host spins on that word
constexpr uint32_t kPubWords = 128;
hipError_t launch_publish(const unsigned long long *d_src, uint32_t n, unsigned long long *h_dst,
                          unsigned long long seq, hipStream_t st);
// each row's records among its first min(len, S, out_stride) entries (the strict increases of
// its running maximum: sorted and distinct; dist_index.hip), the index / probe input for
// unsorted lists: only pairs sharing a record value can count anything in the literal walk
// (pos_out, may be null: each record's position in its row, at the same offsets; unsorted,
// may be null: set to 1 when some row is not strictly increasing, the index build's test)
hipError_t launch_record_rows(const void *in, const uint32_t *in_len, uint64_t in_stride,
                              uint32_t n, uint32_t hash_bytes, uint32_t S, void *out,
                              uint32_t *pos_out, uint32_t *out_len, uint64_t out_stride,
                              hipStream_t st, uint32_t *unsorted = nullptr);
hipError_t launch_exscan(const uint32_t *in, uint32_t *out, uint32_t *out2, uint64_t n,
                         uint32_t *scratch, uint32_t *total, hipStream_t st);
hipError_t launch_probe_count(const void *d_qry, const uint32_t *d_qry_len, uint64_t stride,
                              uint32_t n_qry, uint32_t hash_bytes, IdxGeom g, const uint32_t *dir,
                              unsigned long long *events, uint32_t *unsorted, hipStream_t st);
// The final values of a pair that shares no hash: (0, min(S, la+lb)), distance 1 (0 when
// both lists are empty, numer == denom), p-value 1 and the -d / -v filters
// (CommandDistance.cpp:404-419 at numer = 0).  launch_dist_fill writes them to every cell
// of the grid; the candidate cells are then rewritten by the candidate compare and
// launch_dist_cand_finalize.
struct PairFill {
    double *dist = nullptr, *pval = nullptr;
    uint8_t *pass = nullptr;
    double max_dist = -1, max_pvalue = -1;
};
// flat: the fill over the flattened grid (line-aligned wave stores, ~6.5 TB/s alone), else
// row-aligned workgroups (~4.8 TB/s alone, gentler on a latency-bound kernel beside it).
// fill.dist == nullptr: the numer / denom defaults only (the compact output)
hipError_t launch_dist_fill(const uint32_t *d_ref_len, uint32_t n_ref, const uint32_t *d_qry_len,
                            uint32_t n_qry, uint32_t S, Counts cnt, const PairFill &fill,
                            hipStream_t st, bool flat = true);
// A compact grid's counts written ahead of its dist call (fpm_dist_list_prefill): (0, S) in
// every cell; then, once the lists are known, denom = la + lb where la + lb < S
hipError_t launch_dist_counts_const(uint16_t *numer, uint16_t *denom, uint64_t cells, uint32_t S,
                                    hipStream_t st);
hipError_t launch_dist_counts_fixup(const uint32_t *d_ref_len, uint32_t n_ref,
                                    const uint32_t *d_qry_len, uint32_t n_qry, uint32_t S,
                                    uint16_t *denom, hipStream_t st);
// `defaults`: also write (0, min(S, la+lb)) to every numer / denom cell of the row (off
// when launch_dist_fill already did)
hipError_t launch_probe_rows(const void *d_qry, const uint32_t *d_qry_len, uint64_t stride,
                             uint32_t n_qry, uint32_t n_ref, uint32_t hash_bytes, IdxGeom g,
                             const uint32_t *dir, const uint32_t *entries,
                             const uint32_t *d_ref_len, uint32_t S, bool sym, bool defaults,
                             bool self_set, Counts cnt, uint64_t *cand,
                             unsigned long long *n_cand, uint64_t *row_seg,
                             const uint32_t *d_qry_it_len, uint32_t *q_unsorted,
                             unsigned long long *events, uint64_t cap, uint32_t *cand_over,
                             hipStream_t st, uint32_t q_lo = 0);
// (q_lo, n_qry: the query rows [q_lo, q_lo + n_qry) of the grid)
// (d_qry_it_len non-null: the probed query rows are launch_record_rows copies of length
// d_qry_it_len[q]; d_qry_len stays the original list lengths for the default cells)
// (self_set: the query set is the indexed ref set, same buffers: buckets of one entry are
// the row's own hash and are not read)
// sorted-distinct candidates: one workgroup per query row, one wave per pair
hipError_t launch_merge_rows(const uint64_t *d_cand, const uint64_t *row_seg, uint32_t n_qry,
                             const uint64_t *d_ref, const uint32_t *d_ref_len, uint64_t ref_stride,
                             uint32_t n_ref, const uint64_t *d_qry, const uint32_t *d_qry_len,
                             uint64_t qry_stride, uint32_t S, bool sym, Counts cnt,
                             uint32_t *d_cnum, uint32_t *d_cden, hipStream_t st, uint32_t q_lo = 0);
// (d_cnum, d_cden non-null: results go to candidate slot c instead of the grid cells;
// q_lo, n_qry: the query rows [q_lo, q_lo + n_qry), whose probe has run)

// -fp CFL text: newline index, then one lane per line (fingerprint.hip)
uint32_t text_blocks(uint64_t len);
hipError_t launch_fp_nl_count(const uint8_t *d_text, uint64_t len, uint32_t *blk_cnt,
                              uint32_t *blk_off, uint32_t *scan_s, hipStream_t st);
hipError_t launch_fp_nl_scatter(const uint8_t *d_text, uint64_t len, const uint32_t *blk_off,
                                uint64_t *d_line_start, hipStream_t st);
// the References of a parsed -fp file (heads: line 0 and new_id == 1): per-block head counts +
// their exclusive scan (blk_off[nb] = the total), then the ordered heads, each Reference's
// length (the first line's count twice, Sketch.cpp:117, 134) and its ID bounds
uint32_t fp_head_blocks(uint64_t n_lines);
hipError_t launch_fp_heads(const uint8_t *d_new_id, uint64_t n_lines, uint32_t *blk_cnt,
                           uint32_t *blk_off, uint32_t *scan_s, hipStream_t st);
hipError_t launch_fp_refs(const uint8_t *d_new_id, uint64_t n_lines, const uint32_t *blk_off,
                          uint64_t n_refs, const uint32_t *d_n_vals, const uint64_t *d_id_off,
                          const uint32_t *d_id_len, uint64_t *d_first, uint64_t *d_length,
                          uint64_t *d_ref_id_off, uint32_t *d_ref_id_len, hipStream_t st);
hipError_t launch_fp_lines(const uint8_t *d_text, uint64_t len, const uint64_t *d_line_start,
                           uint64_t n_nl, uint64_t n_lines, uint32_t seed, uint32_t use64,
                           uint64_t *id_off, uint32_t *id_len, uint32_t *n_vals, void *hash,
                           uint8_t *new_id, hipStream_t st);

// FASTA text -> packed records (seqparse.hip).  The text buffer holds each file from a
// kSpChunk-aligned offset, '\n' bytes after it; reset[c] = 1 on a file's first chunk.
constexpr uint32_t kSpChunk = 4096;
size_t seq_xf_bytes();    // per-chunk summary
size_t seq_cin_bytes();   // per-chunk input state / counts
// summaries + chunk scan; d_totals = {records, sequence bytes, '+' in sequence text}
hipError_t launch_seq_scan(const uint8_t *d_text, const uint8_t *d_reset, uint32_t n_chunks,
                           void *d_xf, void *d_cin, uint64_t *d_totals, hipStream_t st);
// record table (header '>' position, header '\n' position, packed offset, length) and the
// packed records (sequence bytes + 0x00 each) in d_out
hipError_t launch_seq_emit(const uint8_t *d_text, uint32_t n_chunks, const void *d_cin,
                           uint64_t n_rec, uint64_t total_kept, uint64_t *d_hdr_pos,
                           uint64_t *d_hdr_end, uint64_t *d_kept_at, uint64_t *d_seq_off,
                           uint64_t *d_seq_len, uint8_t *d_out, hipStream_t st);

// FASTQ, 4-line records verified against kseq_read's quality rules (seqparse.hip).
// d_seg = (offset, length) per file in the text; d_file_lines = (first line, lines) per file
hipError_t launch_fq_files(const uint64_t *d_line_start, uint64_t n_starts, const uint64_t *d_seg,
                           uint32_t n_seg, uint64_t *d_file_lines, hipStream_t st);
// record table in d_rec (hdr_pos | hdr_end | kept_at | seq_off | seq_len), *d_fail != 0 when a
// record does not read the 4-line way; d_scan holds (n_rec + 1023) / 1024 u64, *d_total = bases
hipError_t launch_fq_records(const uint8_t *d_text, const uint64_t *d_line_start,
                             const uint64_t *d_seg, const uint64_t *d_file_lines,
                             const uint64_t *d_rec_base, uint32_t n_seg, uint64_t n_rec,
                             uint64_t *d_rec, uint64_t *d_scan, uint64_t *d_total, uint32_t *d_fail,
                             uint8_t *d_out, hipStream_t st);
hipError_t launch_fq_emit(const uint8_t *d_text, uint64_t n_rec, uint64_t *d_rec, uint8_t *d_out,
                          hipStream_t st);

// triangle -fp positional compare (dist.hip)
hipError_t launch_positional_grid(const void *d_ref, const uint32_t *d_ref_len,
                                  uint64_t ref_stride, uint32_t n_ref, const void *d_qry,
                                  const uint32_t *d_qry_len, uint64_t qry_stride, uint32_t n_qry,
                                  uint32_t hash_bytes, double max_dist, double max_pvalue,
                                  uint32_t *d_numer, uint32_t *d_denom, double *d_dist,
                                  double *d_pvalue, uint8_t *d_pass, hipStream_t st);

// The transposed grid of a rectangular compare (fpm_refset_dist_mirror_dev): cell (r, q) at
// r * n_qry + q holds the pair "query r of the ref set against ref q of the query set".  For
// sorted distinct lists (numer, denom) is symmetric, and so are distance and p-value.
struct MirrorOut {
    Counts cnt;
    double *dist = nullptr, *pval = nullptr;
    uint8_t *pass = nullptr;
    uint32_t n_qry = 0;
};
// distance / p-value / pass of the candidate cells only (after the candidate compare), and
// of each mirror cell (r, q) when `sym`, or of its cell in the transposed grid `mir` (when
// mir.dist is set); the other cells hold the probe's PairFill values
hipError_t launch_dist_cand_finalize(const uint64_t *d_cand, const unsigned long long *d_n_cand,
                                     uint64_t cap, bool sym, const uint32_t *d_cnum,
                                     const uint32_t *d_cden, Counts cnt,
                                     const uint64_t *d_ref_length,
                                     const uint64_t *d_qry_length, uint32_t n_ref,
                                     uint32_t kmer_size, double kmer_space, double max_dist,
                                     double max_pvalue, double *d_dist, double *d_pvalue,
                                     uint8_t *d_pass, const MirrorOut &mir, hipStream_t st);
// distance and p-value of n cells from their u16 / u32 counts and per-cell genome lengths
hipError_t launch_pvalue_batch(const void *numer, const void *denom, uint32_t count_bytes,
                               const uint64_t *len_ref, const uint64_t *len_qry, uint64_t n,
                               uint32_t kmer_size, double kmer_space, double *dist,
                               double *pvalue, hipStream_t st);
hipError_t launch_dist_finalize(Counts cnt, const uint64_t *d_ref_length, const uint64_t *d_qry_length,
                                uint32_t n_ref, uint32_t n_qry, uint32_t kmer_size,
                                double kmer_space, double max_dist, double max_pvalue,
                                double *d_dist, double *d_pvalue, uint8_t *d_pass,
                                hipStream_t st);

// The compact dist output's list of cells with numer > 0 (fpm_dist_list_dev): entry i =
// (qry[i], ref[i]) with its distance / p-value / pass; *count (device) counts every entry,
// those at index >= cap are not written.
struct CellList {
    uint32_t *qry = nullptr, *ref = nullptr;
    double *dist = nullptr, *pval = nullptr;
    uint8_t *pass = nullptr;
    unsigned long long *count = nullptr;
    uint64_t cap = 0;
};
// candidates: scatter (numer, denom) (mirror cell with `sym`; transposed grid mcnt with its own
// list mlist) and list the cells with numer > 0; d_cnum == nullptr: counts read from the grid
hipError_t launch_dist_cand_list(const uint64_t *d_cand, const unsigned long long *d_n_cand,
                                 uint64_t cap, bool sym, const uint32_t *d_cnum,
                                 const uint32_t *d_cden, Counts cnt, const uint64_t *d_ref_length,
                                 const uint64_t *d_qry_length, uint32_t n_ref, uint32_t kmer_size,
                                 double kmer_space, double max_dist, double max_pvalue,
                                 const CellList &list, Counts mcnt, uint32_t m_nqry,
                                 const CellList &mlist, hipStream_t st);
// every cell of a computed grid with numer > 0 into the list
hipError_t launch_dist_grid_list(Counts cnt, uint32_t n_ref, uint32_t n_qry,
                                 const uint64_t *d_ref_length, const uint64_t *d_qry_length,
                                 uint32_t kmer_size, double kmer_space, double max_dist,
                                 double max_pvalue, const CellList &list, hipStream_t st);

}  // namespace fpm
