/*
 * fpm_oracle.h — TEST INFRASTRUCTURE ONLY (the parity oracle and the CPU baseline).
 *
 * A plain-C restatement of fp-mash's sketch + dist hot path (Mash 2.3 fork,
 * /root/reference/mash/src/mash).  It is the checker the HIP product is
 * compared against, and the "port" CPU baseline timed by bench.py.  Only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.
 * The product (fp-mash_amd/, libfpmash.so) never links or calls it.
 *
 * Pinning: checked against the reference's own fixtures (tests/golden/, see
 * tests/golden/make_golden.py) and against the reference's hashing / MinHashHeap
 * sources compiled unmodified into oracle/_ref (oracle/Makefile).  The p-value
 * restates GSL's algorithm (GSL is not in /root/reference and not installed):
 * pinned to mash/test/ref/genomes.dist (6 significant digits) and to 50-digit
 * mpmath; bit-parity with GSL itself is unpinned.
 */
#ifndef FPM_ORACLE_H
#define FPM_ORACLE_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* MurmurHash3.cpp:255-331 */
void orc_murmur3_x64_128(const void *key, int len, uint32_t seed, uint64_t out[2]);
/* hash.cpp:12-40 (non-ARCH_32 build): h1, or its low 32 bits */
uint64_t orc_get_hash(const char *seq, int len, uint32_t seed, int use64);
/* hash.cpp:45-73: Murmur over the 8*n little-endian bytes of the values */
uint64_t orc_get_hash_fp(const uint64_t *vals, uint64_t n, uint32_t seed, int use64);

/* Sketch::Parameters subset (Sketch.h:40-113) that the hot path reads */
typedef struct {
    int kmer_size;
    uint64_t sketch_size;          /* minHashesPerWindow */
    uint32_t seed;
    int use64;
    int noncanonical;
    int preserve_case;
    unsigned char alphabet[256];   /* parameters.alphabet[] */
} orc_params;

/* setAlphabetFromString Sketch.cpp:1260-1289 (also sets use64) */
void orc_set_alphabet(orc_params *p, const char *chars);

/* MinHashHeap (MinHashHeap.cpp:68-146, multiplicityMinimum == 1, no Bloom filter) */
typedef struct orc_heap orc_heap;
orc_heap *orc_heap_new(int use64, uint64_t cardinality_max);
void orc_heap_free(orc_heap *h);
void orc_heap_try_insert(orc_heap *h, uint64_t hash);
/* HashSet::toHashList HashSet.cpp:78-118: ascending hashes (+ counts); returns count */
uint64_t orc_heap_to_list(const orc_heap *h, uint64_t *out_hashes, uint32_t *out_counts);

/* addMinHashes Sketch.cpp:664-735 (uppercases seq in place, like the reference) */
void orc_add_minhashes(orc_heap *h, char *seq, uint64_t length, const orc_params *p);

/*
 * Batch sketch (sketchSequence Sketch.cpp:1490-1517 per record for -i, or one heap
 * per group of records in stream order as sketchFile Sketch.cpp:1354-1422 does).
 * Records shorter than k are skipped (Sketch.cpp:488-492, 1373-1377).
 * group_of_rec == NULL: one sketch per record.  Output: group g's ascending
 * hashes at out_hashes[g*sketch_size ...] (u64 even for use64 == 0), its length
 * in out_count[g], counts in out_mult (nullable).  threads >= 1.
 */
int orc_sketch_batch(const orc_params *p, const char *seq, const uint64_t *rec_off,
                     uint32_t n_rec, const uint32_t *group_of_rec, uint32_t n_groups,
                     uint64_t *out_hashes, uint32_t *out_count, uint32_t *out_mult,
                     int threads);

/*
 * -fp text parsing (Sketch::initFromFingerprints Sketch.cpp:56-151, one file).
 * Splits on '\n' like std::getline, reads the ID token and then unsigned values
 * like istringstream >> uint64_t.  *lines_used is the cross-file counter
 * (LIMIT_READ_FINGERPRINT Sketch.cpp:37).  Returns the number of lines parsed.
 * Per parsed line: id span (id_off,id_len) into text; values appended to vals
 * with line_val_off[line..line+1] (line_val_off has max_lines+1 slots).
 */
uint64_t orc_fp_parse(const char *text, uint64_t text_len, uint64_t limit,
                      uint64_t *lines_used, uint64_t max_lines, uint64_t max_vals,
                      uint64_t *id_off, uint32_t *id_len, uint64_t *vals,
                      uint64_t *line_val_off);

/* CommandDistance.cpp:365-430 walk (works on sorted and unsorted lists alike) */
void orc_compare(const void *ref, uint64_t len_ref, const void *qry, uint64_t len_qry,
                 int use64, uint64_t sketch_size, uint64_t *numer, uint64_t *denom);
/* distance of CommandDistance.cpp:404-419 */
double orc_distance(uint64_t common, uint64_t denom, int kmer_size);
/* pValue CommandDistance.cpp:433-450 with gsl_cdf_binomial_Q restated */
double orc_pvalue(uint64_t x, uint64_t len_ref, uint64_t len_qry, double kmer_space,
                  uint64_t sketch_size);
/* gsl_cdf_binomial_Q(k, p, n) */
double orc_binomial_q(uint64_t k, double p, uint64_t n);

/* compareFingerprints (CommandTriangle.cpp:255-302), triangle -fp: positional matches over
 * min(len); u32 values zero-extended (the fork reads an uninitialised union half, :279).
 * distance = 1 - m/min(len); p = gsl_cdf_chisq_Q(m, 1) = erfc(sqrt(m/2)). */
void orc_positional(const void *a, uint64_t len_a, const void *b, uint64_t len_b, int use64,
                    uint64_t *matches, uint64_t *min_len, double *distance, double *pvalue);

/*
 * All-pairs dist grid, query-major / ref-minor (CommandDistance.cpp:224-261 order),
 * chunked like the reference (pairs/threads capped at 4096 per task) across
 * `threads` workers.  Sketches are rows of a dense [n][stride] array of u32 or u64.
 * Outputs (each n_qry*n_ref, index q*n_ref + r): numer, denom, distance, pvalue
 * (distance/pvalue nullable).
 */
int orc_dist_grid(const void *ref, const uint32_t *ref_len, const uint64_t *ref_length,
                  uint64_t ref_stride, uint32_t n_ref,
                  const void *qry, const uint32_t *qry_len, const uint64_t *qry_length,
                  uint64_t qry_stride, uint32_t n_qry,
                  int use64, uint64_t sketch_size, int kmer_size, double kmer_space,
                  uint32_t *out_numer, uint32_t *out_denom, double *out_dist,
                  double *out_pvalue, int threads);

#ifdef __cplusplus
}
#endif
#endif
