/*
 * fpmash.h — the drop-in C ABI of the MI355X (gfx950) sketch + dist hot path.
 *
 * Plain C: pointers, sizes and int status codes; no C++ or torch types.  Every
 * entry point names the fp-mash interface (file:line under
 * /root/reference/mash/src/mash) whose work it takes over.  The host side
 * (fp-mash_amd/host: the Command/Sketch/-fp surface) and the Python binding
 * (fp-mash_amd/fpmash) call only these symbols; INTEGRATION.md shows the binding
 * a maintainer adds to the reference.
 *
 * Conventions
 *  - Return FPM_OK (0) on success, a negative FPM_E* code otherwise; the message
 *    is in fpm_last_error() (thread-local).  The reference has no status codes on
 *    this path (it prints and exit(1)s: Sketch.cpp:75-76, 1446-1463); the host
 *    maps a non-zero status to that behaviour.
 *  - `*_dev` entry points take DEVICE pointers and a hipStream_t passed as
 *    void* (NULL = the context's stream) and never synchronise; the others take
 *    host buffers, stage them, run, copy back and synchronise.
 *  - Hashes are returned as uint64_t; with use64 == 0 the value is the low 32
 *    bits of h1, zero-extended (hash_u.hash32, hash.h:17-21).
 *  - There is no CPU fallback: with no usable gfx950 device every compute call
 *    fails with FPM_ENODEV.
 *  - A context is bound to one device; contexts are independent and may be used
 *    from different threads (one thread per context at a time).
 */
#ifndef FPMASH_H
#define FPMASH_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FPM_OK 0
#define FPM_EINVAL (-1)
#define FPM_ENODEV (-2)
#define FPM_EHIP (-3)
#define FPM_ENOMEM (-4)

#define FPM_ABI_VERSION 1

typedef struct fpm_ctx fpm_ctx;
typedef struct fpm_sketch_job fpm_sketch_job;

/* Sketch::Parameters (Sketch.h:40-113) as filled by sketchParameterSetup
 * (sketchParameterSetup.cpp:9-126) and setAlphabetFromString (Sketch.cpp:1260-1289). */
typedef struct fpm_sketch_params {
    uint32_t kmer_size;      /* 1..32 (Command.cpp:183-185) */
    uint32_t sketch_size;    /* minHashesPerWindow, s */
    uint32_t seed;           /* hash seed (default 42) */
    uint32_t use64;          /* alphabetSize^k > 2^32 */
    uint32_t noncanonical;   /* -n / -a / -z / -fp */
    uint32_t preserve_case;  /* -Z */
    uint8_t alphabet[256];   /* parameters.alphabet[] (1 = in alphabet) */
} fpm_sketch_params;

/* ---- context / device --------------------------------------------------- */
int fpm_abi_version(void);
/* The build id of this libfpmash.so: the first 16 hex digits of a SHA-256 over the sources it
 * was compiled from (csrc/, include/fpmash.h, the Makefile), also embedded in the file as the
 * text "fpm-build-id:<id>" so a profile can be stamped with the build it measured without
 * loading the library (tools/pmc_traffic.py, bench.py's roofline check). */
const char *fpm_build_id(void);
const char *fpm_last_error(void);
int fpm_device_count(int *count);
int fpm_ctx_create(int device, fpm_ctx **out);
void fpm_ctx_destroy(fpm_ctx *ctx);
void *fpm_ctx_stream(fpm_ctx *ctx);          /* the context's hipStream_t */
int fpm_ctx_synchronize(fpm_ctx *ctx);
/* Extra streams and events on the context's device, for callers that overlap independent
 * batches (e.g. the sketch of batch i+1 beside the dist of batch i): every call above takes
 * a stream argument.  Handles are the library's own hipStream_t / hipEvent_t (the HIP runtime
 * libfpmash links, which need not be the one another framework in the process bundles). */
int fpm_stream_create(fpm_ctx *ctx, void **stream);
int fpm_stream_destroy(fpm_ctx *ctx, void *stream);
int fpm_event_create(fpm_ctx *ctx, void **event);
int fpm_event_destroy(fpm_ctx *ctx, void *event);
int fpm_event_record(fpm_ctx *ctx, void *event, void *stream);
int fpm_stream_wait_event(fpm_ctx *ctx, void *stream, void *event);
/* first-use costs of a process up front: the pinned staging ring and one small DMA each way
 * (~15-25 ms in a fresh process, paid by the first staged upload otherwise).  Optional; for a caller that can run it beside other start-up work (the CLI's
 * device warm-up thread). */
int fpm_ctx_warm(fpm_ctx *ctx);

/* device memory helpers (for bindings that own no allocator) */
int fpm_malloc(fpm_ctx *ctx, void **dptr, size_t bytes);
int fpm_free(fpm_ctx *ctx, void *dptr);
int fpm_memcpy_h2d(fpm_ctx *ctx, void *dst, const void *src, size_t bytes);
int fpm_memcpy_d2h(fpm_ctx *ctx, void *dst, const void *src, size_t bytes);
/* device-to-device copy, ordered on the context stream (e.g. sketch rows into a buffer
 * handed to a collective) */
int fpm_memcpy_d2d(fpm_ctx *ctx, void *dst, const void *src, size_t bytes);
int fpm_memset(fpm_ctx *ctx, void *dptr, int value, size_t bytes);

/* Per-kernel timing with HIP events recorded on the launch stream.
 * kernel ids: sketch tiles, sketch merge, fp hash, compare walk, finalize,
 * dist index build (insert + scan + scatter + probe count), dist row probe. */
#define FPM_K_SKETCH 0
#define FPM_K_MERGE 1
#define FPM_K_FPHASH 2
#define FPM_K_COMPARE 3
#define FPM_K_FINALIZE 4
#define FPM_K_INDEX 5
#define FPM_K_PROBE 6
#define FPM_K_FPTEXT 7
#define FPM_K_FILL 8
#define FPM_K_SEQPARSE 9
#define FPM_K_COUNT 10
/* one-pass bucket-index builds (dist_index.hip) that overflowed a level-1 slot and were
 * redone by the exact two-pass build, since the context was created */
int fpm_ctx_index_rebuilds(fpm_ctx *ctx, uint64_t *count);
/* dist calls whose probe was enqueued behind the index build before the host read the
 * build's counters (a call of the previous sparse call's shape): kept (hits) or dropped and
 * redone on the path the counters chose (misses), since the context was created */
int fpm_ctx_spec_stats(fpm_ctx *ctx, uint64_t *hits, uint64_t *misses);
int fpm_ctx_set_timing(fpm_ctx *ctx, int enable);
int fpm_ctx_reset_timing(fpm_ctx *ctx);
/* total milliseconds and launch count since the last reset (synchronises) */
int fpm_ctx_kernel_time(fpm_ctx *ctx, int kernel, double *total_ms, uint64_t *launches);
/* merges routed to the small-list kernel whose lists overflowed its LDS cap (searched in global
 * memory instead: same results, slower) since the last call on this device; resets it */
int fpm_merge_small_spills(fpm_ctx *ctx, uint64_t *count);

/* dist strategy: FPM_DIST_AUTO picks the inverted-index path unless the shared-hash
 * events exceed pairs*S/4; DENSE walks every pair; SPARSE always uses the index.
 * All three give identical results. */
#define FPM_DIST_AUTO 0
#define FPM_DIST_DENSE 1
#define FPM_DIST_SPARSE 2
int fpm_ctx_set_dist_mode(fpm_ctx *ctx, int mode);
/* statistics of the last compare: path (0 dense walk, 1 index + literal walk of the
 * candidates, 2 index + sorted-set merge of the candidates), posting events, candidates */
int fpm_ctx_last_dist_stats(fpm_ctx *ctx, int *sparse, uint64_t *events, uint64_t *candidates);

/* ---- k-mer sketch ------------------------------------------------------------
 * Replaces addMinHashes (Sketch.cpp:664-735) + MinHashHeap::tryInsert
 * (MinHashHeap.cpp:68-146) + setMinHashesForReference/HashSet::toHashList
 * (Sketch.cpp:1291-1297, HashSet.cpp:78-118), as driven by sketchSequence
 * (Sketch.cpp:1490-1517, -i: one sketch per record) and sketchFile
 * (Sketch.cpp:1299-1488, default: one sketch per file = group of records).
 *
 * Records: seq[rec_off[r] .. rec_off[r+1]).  Records shorter than k are skipped
 * (Sketch.cpp:488-492, 1373-1377).  group_of_rec == NULL: record r is sketch r
 * (n_groups is ignored); else record r belongs to sketch group_of_rec[r] and
 * records of a group are streamed in record order.
 * Output: sketch g's ascending distinct hashes at out_hashes[g*sketch_size ..],
 * out_count[g] of them (= min(s, distinct k-mers)).
 */
int fpm_sketch_batch(fpm_ctx *ctx, const fpm_sketch_params *p, const char *seq,
                     const uint64_t *rec_off, uint32_t n_rec, const uint32_t *group_of_rec,
                     uint32_t n_groups, uint64_t *out_hashes, uint32_t *out_count);

/* Staged form for device-resident pipelines: stage() packs and uploads the
 * sequence and the tile plan (H2D), run() launches the kernels only (inputs
 * already in HBM), device_output() exposes the [n_groups][s] u64 result matrix
 * and the u32 counts on the device, fetch() copies them back. */
int fpm_sketch_stage(fpm_ctx *ctx, const fpm_sketch_params *p, const char *seq,
                     const uint64_t *rec_off, uint32_t n_rec, const uint32_t *group_of_rec,
                     uint32_t n_groups, fpm_sketch_job **job);
int fpm_sketch_run(fpm_sketch_job *job, void *stream);
int fpm_sketch_device_output(fpm_sketch_job *job, uint64_t **d_hashes, uint32_t **d_count,
                             uint32_t *n_groups, uint32_t *row_stride);
int fpm_sketch_fetch(fpm_sketch_job *job, uint64_t *out_hashes, uint32_t *out_count);
/* -M: the multiplicity of every hash of the final sketches, as MinHashHeap counts them
 * (MinHashHeap.cpp:68-146 with multiplicityMinimum 1: occurrences from a hash's first one on;
 * the final maximum of a full sketch stops counting once the heap holds the final set), the
 * counts32 that sketch -M writes (Sketch.cpp:584-596).  After run() on the same stream;
 * out_mult: n_groups x sketch_size u32, row g's first out_count[g] entries in hash order. */
int fpm_sketch_mult(fpm_sketch_job *job, void *stream, uint32_t *out_mult);
/* bytes the run() kernels read + write by algorithm (for roofline accounting) */
int fpm_sketch_job_info(fpm_sketch_job *job, uint64_t *seq_bytes, uint64_t *n_tiles,
                        uint64_t *n_kmers);
/* Tiles of the last run() that the survivors-only tile kernel could not keep and the plain
 * kernel redid (a test hook beside the MinHashHeap restatement, MinHashHeap.cpp:68-146, the
 * result does not depend on it): -1 when the job does not use that kernel (no long groups, or
 * s too large for their bound to leave few survivors per tile).  Waits for the device. */
int fpm_sketch_job_redo_tiles(fpm_sketch_job *job, int32_t *n_redo);
/* Long groups of the last run() that their tight bound (the sample's kt-th smallest hash,
 * kt ~ f s + 8 sqrt(f s) + 32 for a sampled share f of the group's tiles) left with fewer
 * than s hashes, so their tiles and selection ran again under the sample's s-th smallest
 * (values repeated across the group's tiles): a test hook; the sketches are MinHashHeap's
 * either way (MinHashHeap.cpp:68-146).  -1 when the job has no tight bounds (no long
 * groups, or s beyond the one-workgroup selection). */
int fpm_sketch_job_short_groups(fpm_sketch_job *job, int32_t *n_short);
/* Samples of the last fpm_sketch_run that the a-priori sample bound (~1.25 s + 16 sqrt s of
 * the sample's windows below it) left with fewer than s distinct hashes and that were redone
 * unbounded (a test hook, like the two above; every run starts from the staged bounds).  -1
 * when the job's samples carry no a-priori bound. */
int fpm_sketch_job_sample_short(fpm_sketch_job *job, int32_t *n_short);
void fpm_sketch_job_free(fpm_sketch_job *job);

/* Bottom-s of the union of n_lists sketches (device rows of stride s, ascending and
 * distinct, counts[i] entries each) into d_out / d_out_count: the final min-merge when one
 * sketch is computed in parts (a genome or read set split over GPUs, then all-gathered).
 * MinHashHeap keeps the s smallest distinct hashes of one stream (MinHashHeap.cpp:68-146);
 * the s smallest of a union are the s smallest of the union of the parts' s smallest. */
int fpm_sketch_merge_dev(fpm_ctx *ctx, const uint64_t *d_lists, const uint32_t *d_counts,
                         uint32_t n_lists, uint32_t s, uint64_t *d_out, uint32_t *d_out_count,
                         void *stream);

/* ---- FASTA text on the device ------------------------------------------------------
 * Replaces the main-thread kseq loop that feeds sketching (kseq_read, kseq.h:170-208, in
 * sketchFileBySequence / sketchFile, Sketch.cpp:478-522, 1299-1488): the n_seg file images
 * (one per input file, already inflated) go to the device, where records are found (a '>'
 * or '@' that is the first such byte of its line starts one; the header runs to the next
 * '\n'; the sequence is every isgraph byte up to the next record) and their sequence bytes
 * are packed for the sketch kernels without returning to the host.
 * quality_lines = 1 when a '+' occurs in sequence text (FASTQ: kseq then reads quality
 * lines, which this parser does not restate): the caller parses such input on the host.
 * fpm_seq_records: per record, its file, the header's byte offset ('>' / '@') in that file,
 * the header line's length (to its '\n' or the end of the file) and the sequence length.
 * fpm_sketch_stage_seq: a sketch job over the parsed records (group_of_rec[r] as in
 * fpm_sketch_stage, FPM_NO_GROUP = not sketched, e.g. records shorter than k); the job
 * takes over the packed records (stage once per parse). */
typedef struct fpm_seqtext fpm_seqtext;
#define FPM_NO_GROUP 0xFFFFFFFFu
int fpm_seq_parse(fpm_ctx *ctx, const char *const *seg_text, const uint64_t *seg_len,
                  uint32_t n_seg, fpm_seqtext **job, uint64_t *n_records, int *quality_lines);
int fpm_seq_records(fpm_seqtext *job, uint32_t *seg_of_rec, uint64_t *hdr_off, uint64_t *hdr_len,
                    uint64_t *seq_len);
int fpm_sketch_stage_seq(fpm_ctx *ctx, const fpm_sketch_params *p, fpm_seqtext *seq,
                         const uint32_t *group_of_rec, uint32_t n_groups, fpm_sketch_job **job);
void fpm_seq_free(fpm_seqtext *job);

/* ---- -fp k-finger lines ------------------------------------------------------
 * Replaces the per-line getHashFingerPrint of Sketch::initFromFingerprints
 * (Sketch.cpp:131 -> hash.cpp:45-73): line l hashes the 8*n little-endian bytes
 * of vals[line_off[l] .. line_off[l+1]).  use64 == 0 (the -fp setting) writes
 * uint32_t, else uint64_t, into out. */
int fpm_fp_hash_lines(fpm_ctx *ctx, const uint64_t *vals, const uint64_t *line_off,
                      uint64_t n_lines, uint32_t seed, uint32_t use64, void *out);
int fpm_fp_hash_lines_dev(fpm_ctx *ctx, const uint64_t *d_vals, const uint64_t *d_line_off,
                          uint64_t n_lines, uint32_t seed, uint32_t use64, void *d_out,
                          void *stream);

/* ---- -fp text ------------------------------------------------------------------
 * Replaces the parse loop of Sketch::initFromFingerprints (Sketch.cpp:82-101: getline,
 * `iss >> id`, `while (iss >> v)` over u64 values) and its per-line getHashFingerPrint
 * (:131): the whole file image goes to the device, lines are split on '\n' (a last line
 * without '\n' counts), at most max_lines are parsed (the caller passes what is left of
 * the 1,000,000-line budget, :37, :82).  Per line: the ID token (byte offset, length),
 * the number of values, the line hash (u32, or u64 when use64), and new_id = 1 when the
 * ID differs from the previous line's, 0 when equal, 2 on line 0 (the caller compares
 * it with the previous file's last ID).  Grouping lines into References stays with the
 * caller (it owns names/comments).  fetch may be given NULL for outputs it does not need. */
typedef struct fpm_fptext fpm_fptext;
int fpm_fp_text_stage(fpm_ctx *ctx, const char *text, uint64_t text_len, uint64_t max_lines,
                      uint32_t seed, uint32_t use64, fpm_fptext **job, uint64_t *n_lines);
int fpm_fp_text_fetch(fpm_fptext *job, uint64_t *id_off, uint32_t *id_len, uint32_t *n_vals,
                      void *hash, uint8_t *new_id);
/* The References the staged file's lines make (Sketch.cpp:104-145, the grouping of
 * initFromFingerprints): one at line 0 (the caller checks its ID against the previous file's
 * last ID: equal IDs across files crash the reference, :131) and one wherever the ID changes.
 * Per Reference: its first line, its ID (byte offset, length in the text) and its length (the
 * first line's value count, :117, plus every line's, :134).  Computed on the device on the
 * first call; *n_refs is always set, the arrays are filled when cap >= *n_refs (a first call
 * with cap 0 sizes them).  With it a caller fetches only the hashes (fpm_fp_text_fetch with
 * the other outputs NULL): 4 B per line instead of 21. */
int fpm_fp_text_refs(fpm_fptext *job, uint64_t cap, uint64_t *n_refs, uint64_t *first_line,
                     uint64_t *id_off, uint32_t *id_len, uint64_t *length);
void fpm_fp_text_free(fpm_fptext *job);

/* ---- dist ---------------------------------------------------------------------
 * Replaces compare()/compareSketches()/pValue() (CommandDistance.cpp:335-450) over
 * the whole ref x query grid that CommandDistance::run chunks (:224-261).
 * Sketch lists are rows of dense matrices (row stride in elements) holding
 * hash_bytes = 8 (u64) or 4 (u32) values; lists may be unsorted and carry
 * duplicates (-fp), the walk is the reference's literal one.  sketch_size =
 * min(s_ref, s_query) (:342-344).  Outputs are query-major: index q*n_ref + r. */
int fpm_compare_grid(fpm_ctx *ctx, const void *ref, const uint32_t *ref_len,
                     uint64_t ref_stride, uint32_t n_ref, const void *qry,
                     const uint32_t *qry_len, uint64_t qry_stride, uint32_t n_qry,
                     uint32_t hash_bytes, uint32_t sketch_size, uint32_t *out_numer,
                     uint32_t *out_denom);
int fpm_compare_grid_dev(fpm_ctx *ctx, const void *d_ref, const uint32_t *d_ref_len,
                         uint64_t ref_stride, uint32_t n_ref, const void *d_qry,
                         const uint32_t *d_qry_len, uint64_t qry_stride, uint32_t n_qry,
                         uint32_t hash_bytes, uint32_t sketch_size, uint32_t *d_numer,
                         uint32_t *d_denom, void *stream);
/* distance (:404-419), p-value (:433-450, FP64) and the -d/-v filter (:421-429);
 * ref_length/qry_length are Reference::length (k-mer space scaling of pValue).
 * max_dist / max_pvalue < 0 disable the filter.  pass may be NULL. */
int fpm_dist_finalize_dev(fpm_ctx *ctx, const uint32_t *d_numer, const uint32_t *d_denom,
                          const uint64_t *d_ref_length, const uint64_t *d_qry_length,
                          uint32_t n_ref, uint32_t n_qry, uint32_t kmer_size,
                          double kmer_space, double max_dist, double max_pvalue,
                          double *d_dist, double *d_pvalue, uint8_t *d_pass, void *stream);
/* Distance and p-value of n independent cells from their counts (u16 when count_bytes = 2,
 * u32 when 4) and per-cell genome lengths, device pointers, stream-ordered, no -d / -v
 * filters: the values the compact output (fpm_dist_list_dev) leaves out, for the cells a
 * caller wants.  Replaces the per-pair distance + pValue of CommandDistance.cpp:404-419,
 * 433-450 (SURVEY §8(b)'s optional fpm_pvalue_batch).  d_dist / d_pvalue may each be NULL. */
int fpm_pvalue_batch_dev(fpm_ctx *ctx, const void *d_numer, const void *d_denom,
                         uint32_t count_bytes, const uint64_t *d_len_ref,
                         const uint64_t *d_len_qry, uint64_t n, uint32_t kmer_size,
                         double kmer_space, double *d_dist, double *d_pvalue, void *stream);
/* compare + finalize in one call on device buffers (= fpm_compare_grid_dev followed by
 * fpm_dist_finalize_dev on the same stream). */
int fpm_dist_dev(fpm_ctx *ctx, const void *d_ref, const uint32_t *d_ref_len,
                 const uint64_t *d_ref_length, uint64_t ref_stride, uint32_t n_ref,
                 const void *d_qry, const uint32_t *d_qry_len, const uint64_t *d_qry_length,
                 uint64_t qry_stride, uint32_t n_qry, uint32_t hash_bytes, uint32_t sketch_size,
                 uint32_t kmer_size, double kmer_space, double max_dist, double max_pvalue,
                 uint32_t *d_numer, uint32_t *d_denom, double *d_dist, double *d_pvalue,
                 uint8_t *d_pass, void *stream);
/* fpm_dist_dev with u16 numer / denom cells (every count is <= sketch_size <= 65535): the
 * same results in 4 bytes per pair instead of 8 (the grid's counts as SURVEY.md §8(b)
 * sizes them); FPM_EINVAL when sketch_size > 65535. */
int fpm_dist_dev16(fpm_ctx *ctx, const void *d_ref, const uint32_t *d_ref_len,
                   const uint64_t *d_ref_length, uint64_t ref_stride, uint32_t n_ref,
                   const void *d_qry, const uint32_t *d_qry_len, const uint64_t *d_qry_length,
                   uint64_t qry_stride, uint32_t n_qry, uint32_t hash_bytes, uint32_t sketch_size,
                   uint32_t kmer_size, double kmer_space, double max_dist, double max_pvalue,
                   uint16_t *d_numer, uint16_t *d_denom, double *d_dist, double *d_pvalue,
                   uint8_t *d_pass, void *stream);
/* ---- compact dist output (the grid as u16 numer / denom) ----------
 * compareSketches' (numer, denom) for every cell of the n_qry x n_ref grid as u16 cells (4 B
 * per pair, query-major), and distance / p-value / pass only for the cells that share hashes
 * (numer > 0): an unordered list, each such cell exactly once.  A cell not in the list has
 * numer 0, and compareSketches / pValue give it closed-form values (CommandDistance.cpp:
 * 404-408 and 435-437 at common = 0): distance 0 when denom == 0 (two empty lists), else 1;
 * p-value 1; pass = (max_dist < 0 || distance <= max_dist) && (max_pvalue < 0 || 1 <=
 * max_pvalue).  Listed cells hold what fpm_dist_dev16 writes for them.
 * The list lives in caller device memory: entry i is (qry[i], ref[i], dist[i], pvalue[i],
 * pass[i]) (pass may be NULL).  *count is a DEVICE u64 the call resets and then sets to the
 * number of cells with numer > 0; entries at index >= cap are not written, so a caller that
 * reads *count > cap after the stream work repeats the call with cap >= *count. */
typedef struct fpm_cell_list {
    uint32_t *qry, *ref;
    double *dist, *pvalue;
    uint8_t *pass;
    uint64_t cap;
    uint64_t *count;
} fpm_cell_list;
int fpm_dist_list_dev(fpm_ctx *ctx, const void *d_ref, const uint32_t *d_ref_len,
                      const uint64_t *d_ref_length, uint64_t ref_stride, uint32_t n_ref,
                      const void *d_qry, const uint32_t *d_qry_len, const uint64_t *d_qry_length,
                      uint64_t qry_stride, uint32_t n_qry, uint32_t hash_bytes,
                      uint32_t sketch_size, uint32_t kmer_size, double kmer_space,
                      double max_dist, double max_pvalue, uint16_t *d_numer, uint16_t *d_denom,
                      const fpm_cell_list *list, void *stream);
/* The compact grid's counts ahead of the call that computes them, e.g. before the sketches
 * exist: numer 0 and denom sketch_size in all n_qry x n_ref u16 cells, on the context's side
 * stream after the work already on `stream` (a pure write stream beside the sketch kernels).
 * The next fpm_dist_list_dev on this context whose numer / denom / n_ref / n_qry /
 * sketch_size are these takes it over: it writes no no-shared-hash counts of
 * its own, sets denom = la + lb where la + lb < sketch_size (compareSketches' min(S, la + lb)
 * at common = 0, CommandDistance.cpp:416-418) and writes its cells after the prefill.  Any
 * other dist call on the context waits for it first.  Until then only that call (or
 * fpm_ctx_synchronize) orders the grid against the prefill.  No reference counterpart: its
 * compare writes every pair (CommandDistance.cpp:365-430). */
int fpm_dist_list_prefill(fpm_ctx *ctx, uint16_t *d_numer, uint16_t *d_denom, uint32_t n_ref,
                          uint32_t n_qry, uint32_t sketch_size, void *stream);
/* host-buffer convenience: compare + finalize */
int fpm_dist(fpm_ctx *ctx, const void *ref, const uint32_t *ref_len, const uint64_t *ref_length,
             uint64_t ref_stride, uint32_t n_ref, const void *qry, const uint32_t *qry_len,
             const uint64_t *qry_length, uint64_t qry_stride, uint32_t n_qry,
             uint32_t hash_bytes, uint32_t sketch_size, uint32_t kmer_size, double kmer_space,
             double max_dist, double max_pvalue, uint32_t *out_numer, uint32_t *out_denom,
             double *out_dist, double *out_pvalue, uint8_t *out_pass);

/* ---- resident reference set -------------------------------------------------------
 * CommandDistance::run compares every query against the same reference sketch
 * (CommandDistance.cpp:191-261: the pool's CompareInput holds `const Sketch & sketchRef`
 * for all query chunks).  A refset keeps the reference rows on the device and builds their
 * bucket index ONCE; each query block then only uploads its own rows, probes the resident
 * index and runs the exact candidate compare + distance / p-value (the same results as
 * fpm_dist_dev).  sketch_size (min of the two sketches' s, :342-344) is fixed per set.
 * _create copies host rows to the device (owned); _create_dev borrows device rows, which
 * must outlive the set.  count_bytes selects u16 (2, sketch_size <= 65535) or u32 (4)
 * numer / denom cells.  fpm_refset_dist takes host query rows and host outputs (pinned
 * buffers from fpm_host_alloc copy at full PCIe rate). */
typedef struct fpm_refset fpm_refset;
int fpm_refset_create(fpm_ctx *ctx, const void *ref, const uint32_t *ref_len,
                      const uint64_t *ref_length, uint64_t ref_stride, uint32_t n_ref,
                      uint32_t hash_bytes, uint32_t sketch_size, fpm_refset **out);
int fpm_refset_create_dev(fpm_ctx *ctx, const void *d_ref, const uint32_t *d_ref_len,
                          const uint64_t *d_ref_length, uint64_t ref_stride, uint32_t n_ref,
                          uint32_t hash_bytes, uint32_t sketch_size, fpm_refset **out);
int fpm_refset_dist_dev(fpm_refset *rs, const void *d_qry, const uint32_t *d_qry_len,
                        const uint64_t *d_qry_length, uint64_t qry_stride, uint32_t n_qry,
                        uint32_t sketch_size, uint32_t count_bytes, uint32_t kmer_size,
                        double kmer_space, double max_dist, double max_pvalue, void *d_numer,
                        void *d_denom, double *d_dist, double *d_pvalue, uint8_t *d_pass,
                        void *stream);
/* The same compare, plus its transposed grid: m_* cell (r, q) at r * n_qry + q holds what
 * fpm_refset_dist_dev would give for query r of the reference set against reference q of the
 * query rows (the pair seen from the other side, CommandDistance.cpp:224-261 with the two
 * sketches exchanged).  For the sorted distinct lists of the k-mer path the candidate
 * results are scattered to both grids (compareSketches' counts are symmetric there, and so
 * are distance and p-value); otherwise (unsorted -fp lists, dense path) the transposed grid
 * is computed by the swapped call.  Multi-GPU all-vs-all dist deals unordered block pairs
 * to the ranks with this call (fpmash/shard.py: pair_block_jobs).  The query rows must not
 * be the set's own rows (that grid is its own transpose: fpm_refset_dist_dev). */
int fpm_refset_dist_mirror_dev(fpm_refset *rs, const void *d_qry, const uint32_t *d_qry_len,
                               const uint64_t *d_qry_length, uint64_t qry_stride, uint32_t n_qry,
                               uint32_t sketch_size, uint32_t count_bytes, uint32_t kmer_size,
                               double kmer_space, double max_dist, double max_pvalue,
                               void *d_numer, void *d_denom, double *d_dist, double *d_pvalue,
                               uint8_t *d_pass, void *m_numer, void *m_denom, double *m_dist,
                               double *m_pvalue, uint8_t *m_pass, void *stream);
/* The compact output (fpm_dist_list_dev) against a resident set, and with its transposed grid
 * (m_numer / m_denom cell (r, q) at r * n_qry + q, m_list its own list of cells). */
int fpm_refset_dist_list_dev(fpm_refset *rs, const void *d_qry, const uint32_t *d_qry_len,
                             const uint64_t *d_qry_length, uint64_t qry_stride, uint32_t n_qry,
                             uint32_t sketch_size, uint32_t kmer_size, double kmer_space,
                             double max_dist, double max_pvalue, uint16_t *d_numer,
                             uint16_t *d_denom, const fpm_cell_list *list, void *stream);
int fpm_refset_dist_mirror_list_dev(fpm_refset *rs, const void *d_qry, const uint32_t *d_qry_len,
                                    const uint64_t *d_qry_length, uint64_t qry_stride,
                                    uint32_t n_qry, uint32_t sketch_size, uint32_t kmer_size,
                                    double kmer_space, double max_dist, double max_pvalue,
                                    uint16_t *d_numer, uint16_t *d_denom,
                                    const fpm_cell_list *list, uint16_t *m_numer,
                                    uint16_t *m_denom, const fpm_cell_list *m_list, void *stream);
/* Rebuild the set's bucket index from its (device, borrowed) rows in place, e.g. after the
 * rows were rewritten by a new sketch run; no reallocation when the geometry is unchanged. */
int fpm_refset_reindex(fpm_refset *rs, void *stream);
int fpm_refset_dist(fpm_refset *rs, const void *qry, const uint32_t *qry_len,
                    const uint64_t *qry_length, uint64_t qry_stride, uint32_t n_qry,
                    uint32_t sketch_size, uint32_t kmer_size, double kmer_space, double max_dist,
                    double max_pvalue, uint32_t *out_numer, uint32_t *out_denom, double *out_dist,
                    double *out_pvalue, uint8_t *out_pass);
/* The compact output of one host query block (fpm_refset_dist_list_dev with host buffers):
 * out_numer / out_denom (n_qry x n_ref cells of count_bytes = 2 (u16, sketch_size <= 65535)
 * or 4 (u32), query-major, may be NULL) and the cells with numer > 0 (l_* arrays of cap
 * entries, any may be NULL).  *n_listed = the number of such cells; only the first
 * min(*n_listed, cap) are copied (the device list grows as needed). */
int fpm_refset_dist_list(fpm_refset *rs, const void *qry, const uint32_t *qry_len,
                         const uint64_t *qry_length, uint64_t qry_stride, uint32_t n_qry,
                         uint32_t sketch_size, uint32_t kmer_size, double kmer_space,
                         double max_dist, double max_pvalue, uint32_t count_bytes,
                         void *out_numer, void *out_denom, uint32_t *l_qry, uint32_t *l_ref,
                         double *l_dist, double *l_pvalue, uint8_t *l_pass, uint64_t cap,
                         uint64_t *n_listed);
void fpm_refset_free(fpm_refset *rs);

/* pinned (page-locked) host memory for staging buffers of the host-buffer calls */
int fpm_host_alloc(fpm_ctx *ctx, void **p, size_t bytes);
int fpm_host_free(fpm_ctx *ctx, void *p);

/* ---- triangle -fp ---------------------------------------------------------------
 * Replaces compareFingerprints (CommandTriangle.cpp:255-302): positional compare of
 * two lists over min(len) entries, matches = equal values at the same position (the
 * fork reads an uninitialised union half, :279; u32 values are zero-extended here).
 * distance = 1 - matches/min(len), p-value = gsl_cdf_chisq_Q(matches, 1) =
 * erfc(sqrt(matches/2)), pass = distance <= max_dist && p <= max_pvalue.
 * Host buffers, query-major output (q*n_ref + r); n_qry <= 65535 per call. */
int fpm_fp_positional_grid(fpm_ctx *ctx, const void *ref, const uint32_t *ref_len,
                           uint64_t ref_stride, uint32_t n_ref, const void *qry,
                           const uint32_t *qry_len, uint64_t qry_stride, uint32_t n_qry,
                           uint32_t hash_bytes, double max_dist, double max_pvalue,
                           uint32_t *out_numer, uint32_t *out_denom, double *out_dist,
                           double *out_pvalue, uint8_t *out_pass);

/* ---- communicator: RCCL over xGMI for the cross-GPU min-merge ------------------------
 * north_star reserves the collective for "the final min-merge only where the reference set
 * exceeds one GPU's HBM" (or one sketch is split over GPUs).  The reference has no collective:
 * one process, one pthreads pool (ThreadPool.h:13-61) feeding one MinHashHeap per genome
 * (Sketch.cpp:1354-1422).  The communicator lives on the context's device and HIP runtime
 * (librccl is dlopen'ed on first use); the caller carries the 128-byte unique id from one rank
 * to the others over any host channel (ncclGetUniqueId / ncclCommInitRank's contract). */
#define FPM_COMM_ID_BYTES 128
typedef struct fpm_comm fpm_comm;
int fpm_comm_unique_id(uint8_t id[FPM_COMM_ID_BYTES]);
/* waits until all nranks ranks have called it with the same id, up to FPM_COMM_INIT_TIMEOUT_S
 * seconds (default 120; a non-blocking RCCL set-up, aborted past the limit): then FPM_EHIP and a
 * message naming the limit, instead of blocking for ever on a peer that never joins */
int fpm_comm_create(fpm_ctx *ctx, int nranks, int rank, const uint8_t id[FPM_COMM_ID_BYTES],
                    fpm_comm **out);
void fpm_comm_destroy(fpm_comm *comm);
/* every rank's `bytes` of d_send, in rank order, into d_recv (nranks x bytes), enqueued on
 * `stream` (NULL: the context stream) */
int fpm_comm_all_gather(fpm_comm *comm, const void *d_send, void *d_recv, size_t bytes,
                        void *stream);
/* The min-merge of one sketch computed in parts (MinHashHeap.cpp:68-146: the s smallest
 * distinct of a union = the s smallest of the union of the parts' s smallest): every rank's
 * ascending bottom-s row (s hashes, d_count valid) all-gathered into library buffers and merged
 * on the device (fpm_sketch_merge_dev) into d_out / d_out_count on every rank; enqueued on
 * `stream` (NULL: the context stream). */
int fpm_sketch_min_merge_comm(fpm_comm *comm, const uint64_t *d_row, const uint32_t *d_count,
                              uint32_t s, uint64_t *d_out, uint32_t *d_out_count, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* FPMASH_H */
