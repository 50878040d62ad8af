/*
 * fpm_oracle.c — TEST INFRASTRUCTURE ONLY: CPU restatement of fp-mash's
 * sketch + dist hot path, used as the parity checker and as bench.py's "port"
 * CPU baseline.  See fpm_oracle.h for the pinning statement.  Every function
 * cites the reference lines (under /root/reference/mash/src/mash) it restates.
 */
#include "fpm_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <float.h>

/* ------------------------------------------------------------------------ */
/* MurmurHash3_x64_128 — MurmurHash3.cpp:255-331 (public-domain algorithm).  */
/* ------------------------------------------------------------------------ */

static inline uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }

static inline uint64_t fmix64(uint64_t k)
{
    k ^= k >> 33;
    k *= 0xff51afd7ed558ccdULL;
    k ^= k >> 33;
    k *= 0xc4ceb9fe1a85ec53ULL;
    k ^= k >> 33;
    return k;
}

void orc_murmur3_x64_128(const void *key, int len, uint32_t seed, uint64_t out[2])
{
    const uint8_t *bytes = (const uint8_t *)key;
    const uint64_t C1 = 0x87c37b91114253d5ULL, C2 = 0x4cf5ad432745937fULL;
    uint64_t h1 = seed, h2 = seed;
    int nblk = len / 16;

    for (int b = 0; b < nblk; b++) {
        uint64_t k1, k2;
        memcpy(&k1, bytes + 16 * b, 8);   /* little-endian host, as getblock64 */
        memcpy(&k2, bytes + 16 * b + 8, 8);
        k1 *= C1; k1 = rotl64(k1, 31); k1 *= C2; h1 ^= k1;
        h1 = rotl64(h1, 27); h1 += h2; h1 = h1 * 5 + 0x52dce729;
        k2 *= C2; k2 = rotl64(k2, 33); k2 *= C1; h2 ^= k2;
        h2 = rotl64(h2, 31); h2 += h1; h2 = h2 * 5 + 0x38495ab5;
    }

    /* tail: bytes nblk*16 .. len-1; bytes 8..14 feed k2, 0..7 feed k1 */
    const uint8_t *t = bytes + 16 * nblk;
    int rem = len & 15;
    uint64_t k1 = 0, k2 = 0;
    for (int i = rem - 1; i >= 8; i--) k2 ^= (uint64_t)t[i] << (8 * (i - 8));
    if (rem > 8) { k2 *= C2; k2 = rotl64(k2, 33); k2 *= C1; h2 ^= k2; }
    for (int i = (rem < 8 ? rem : 8) - 1; i >= 0; i--) k1 ^= (uint64_t)t[i] << (8 * i);
    if (rem > 0) { k1 *= C1; k1 = rotl64(k1, 31); k1 *= C2; h1 ^= k1; }

    h1 ^= (uint64_t)(int64_t)len;
    h2 ^= (uint64_t)(int64_t)len;
    h1 += h2; h2 += h1;
    h1 = fmix64(h1); h2 = fmix64(h2);
    h1 += h2; h2 += h1;
    out[0] = h1;
    out[1] = h2;
}

/* getHash hash.cpp:12-40 */
uint64_t orc_get_hash(const char *seq, int len, uint32_t seed, int use64)
{
    uint64_t o[2];
    orc_murmur3_x64_128(seq, len, seed, o);
    return use64 ? o[0] : (uint64_t)(uint32_t)o[0];
}

/* getHashFingerPrint hash.cpp:45-73: the caller passes 8*n bytes */
uint64_t orc_get_hash_fp(const uint64_t *vals, uint64_t n, uint32_t seed, int use64)
{
    uint64_t o[2];
    orc_murmur3_x64_128(vals, (int)(n * sizeof(uint64_t)), seed, o);
    return use64 ? o[0] : (uint64_t)(uint32_t)o[0];
}

/* setAlphabetFromString Sketch.cpp:1260-1289 */
void orc_set_alphabet(orc_params *p, const char *chars)
{
    memset(p->alphabet, 0, 256);
    for (const char *c = chars; *c; c++) {
        char u = *c;
        if (!p->preserve_case && u > 96 && u < 123) u -= 32;
        p->alphabet[(unsigned char)u] = 1;
    }
    int n = 0;
    for (int i = 0; i < 256; i++) n += p->alphabet[i] ? 1 : 0;
    p->use64 = pow((double)n, (double)p->kmer_size) > pow(2.0, 32.0);
}

/* ------------------------------------------------------------------------ */
/* MinHashHeap — MinHashHeap.cpp:68-146 with HashSet (HashSet.cpp:10-76) and  */
/* HashPriorityQueue (std::priority_queue max-heap).  Keys compared as u32    */
/* when !use64 (hashLessThan hash.cpp:76-86); hashes are stored pre-masked.   */
/* ------------------------------------------------------------------------ */

struct orc_heap {
    int use64;
    uint64_t cap;          /* cardinalityMaximum */
    /* hash set: open addressing, linear probing, backward-shift delete */
    uint64_t *keys;
    uint32_t *cnt;         /* 0 == empty slot */
    uint64_t tmask;
    uint64_t size;
    /* max-heap */
    uint64_t *heap;
    uint64_t hsize;
};

static inline uint64_t slot_of(const orc_heap *h, uint64_t key)
{
    return (key * 0x9E3779B97F4A7C15ULL >> 17) & h->tmask;
}

orc_heap *orc_heap_new(int use64, uint64_t cap)
{
    orc_heap *h = (orc_heap *)calloc(1, sizeof(orc_heap));
    h->use64 = use64;
    h->cap = cap;
    uint64_t t = 16;
    while (t < 2 * (cap + 2)) t <<= 1;
    h->tmask = t - 1;
    h->keys = (uint64_t *)calloc(t, sizeof(uint64_t));
    h->cnt = (uint32_t *)calloc(t, sizeof(uint32_t));
    h->heap = (uint64_t *)malloc((cap + 2) * sizeof(uint64_t));
    return h;
}

void orc_heap_free(orc_heap *h)
{
    if (!h) return;
    free(h->keys); free(h->cnt); free(h->heap); free(h);
}

static int64_t set_find(const orc_heap *h, uint64_t key)
{
    for (uint64_t s = slot_of(h, key);; s = (s + 1) & h->tmask) {
        if (h->cnt[s] == 0) return -1;
        if (h->keys[s] == key) return (int64_t)s;
    }
}

static void set_add(orc_heap *h, uint64_t key, uint32_t c)
{
    uint64_t s = slot_of(h, key);
    while (h->cnt[s] != 0 && h->keys[s] != key) s = (s + 1) & h->tmask;
    if (h->cnt[s] == 0) { h->keys[s] = key; h->cnt[s] = c; h->size++; }
    else h->cnt[s] += c;
}

static void set_erase(orc_heap *h, uint64_t key)
{
    int64_t f = set_find(h, key);
    if (f < 0) return;
    uint64_t hole = (uint64_t)f;
    h->cnt[hole] = 0;
    h->size--;
    for (uint64_t s = (hole + 1) & h->tmask; h->cnt[s] != 0; s = (s + 1) & h->tmask) {
        uint64_t home = slot_of(h, h->keys[s]);
        /* can the entry at s move into the hole? (home not in (hole, s]) */
        uint64_t d_s = (s - home) & h->tmask, d_hole = (s - hole) & h->tmask;
        if (d_s >= d_hole) {
            h->keys[hole] = h->keys[s]; h->cnt[hole] = h->cnt[s];
            h->cnt[s] = 0; hole = s;
        }
    }
}

static void heap_push(orc_heap *h, uint64_t v)
{
    uint64_t i = h->hsize++;
    h->heap[i] = v;
    while (i > 0) {
        uint64_t p = (i - 1) / 2;
        if (h->heap[p] >= h->heap[i]) break;
        uint64_t t = h->heap[p]; h->heap[p] = h->heap[i]; h->heap[i] = t;
        i = p;
    }
}

static void heap_pop(orc_heap *h)
{
    h->heap[0] = h->heap[--h->hsize];
    uint64_t i = 0, n = h->hsize;
    for (;;) {
        uint64_t l = 2 * i + 1, r = l + 1, m = i;
        if (l < n && h->heap[l] > h->heap[m]) m = l;
        if (r < n && h->heap[r] > h->heap[m]) m = r;
        if (m == i) break;
        uint64_t t = h->heap[m]; h->heap[m] = h->heap[i]; h->heap[i] = t;
        i = m;
    }
}

void orc_heap_try_insert(orc_heap *h, uint64_t hash)
{
    if (!h->use64) hash &= 0xffffffffULL;
    if (h->size < h->cap || hash < h->heap[0]) {
        int64_t f = set_find(h, hash);
        if (f < 0) {
            set_add(h, hash, 1);       /* multiplicityMinimum == 1 branch */
            heap_push(h, hash);
        } else {
            h->cnt[f] += 1;
        }
        if (h->size > h->cap) {
            set_erase(h, h->heap[0]);
            heap_pop(h);
        }
    }
}

static int cmp_u64(const void *a, const void *b)
{
    uint64_t x = *(const uint64_t *)a, y = *(const uint64_t *)b;
    return x < y ? -1 : x > y;
}

uint64_t orc_heap_to_list(const orc_heap *h, uint64_t *out_hashes, uint32_t *out_counts)
{
    uint64_t n = 0;
    for (uint64_t s = 0; s <= h->tmask; s++)
        if (h->cnt[s]) out_hashes[n++] = h->keys[s];
    qsort(out_hashes, n, sizeof(uint64_t), cmp_u64);
    if (out_counts)
        for (uint64_t i = 0; i < n; i++) out_counts[i] = h->cnt[set_find(h, out_hashes[i])];
    return n;
}

/* ------------------------------------------------------------------------ */
/* k-mer sketching — addMinHashes Sketch.cpp:664-735, complement table and     */
/* reverseComplement Sketch.cpp:1223-1258.                                    */
/* ------------------------------------------------------------------------ */

/* complement of 'A'..'Z' (IUPAC), Sketch.cpp:1223-1250 */
static const char COMPL_AZ[26] = {
    'T', 'V', 'G', 'H', 'N', 'N', 'C', 'D', 'N', 'N', 'M', 'N', 'K',
    'N', 'N', 'N', 'N', 'Y', 'S', 'A', 'A', 'B', 'W', 'N', 'R', 'N'};

static inline char complement_of(char c)
{
    /* the reference indexes complement[c - 'A'] unchecked; only alphabet letters
     * reach a compared window, so any out-of-range byte is irrelevant */
    int i = (int)(unsigned char)c - 'A';
    return (i >= 0 && i < 26) ? COMPL_AZ[i] : 'N';
}

void orc_add_minhashes(orc_heap *h, char *seq, uint64_t length, const orc_params *p)
{
    const int k = p->kmer_size;
    if (length < (uint64_t)k) return;   /* callers never pass shorter records */

    if (!p->preserve_case)
        for (uint64_t i = 0; i < length; i++)
            if (seq[i] > 96 && seq[i] < 123) seq[i] -= 32;

    char *rev = NULL;
    if (!p->noncanonical) {
        rev = (char *)malloc(length);
        for (uint64_t i = 0; i < length; i++) rev[i] = complement_of(seq[length - i - 1]);
    }

    uint64_t j = 0;   /* first position not yet validated */
    for (uint64_t i = 0; i + k <= length; i++) {
        int bad = 0;
        for (; j < i + k; j++) {
            if (!p->alphabet[(unsigned char)seq[j]]) {
                i = j++;  /* restart past the bad byte */
                bad = 1;
                break;
            }
        }
        if (bad) continue;
        const char *fwd = seq + i;
        const char *kmer = fwd;
        if (!p->noncanonical) {
            const char *rc = rev + length - i - k;
            if (memcmp(fwd, rc, k) > 0) kmer = rc;
        }
        orc_heap_try_insert(h, orc_get_hash(kmer, k, p->seed, p->use64));
    }
    free(rev);
}

/* ------------------------------------------------------------------------ */
/* Batch sketching with a worker pool (the reference's ThreadPool fan-out,     */
/* ThreadPool.hxx:12-230; outputs are indexed so order is preserved).          */
/* ------------------------------------------------------------------------ */

typedef struct {
    const orc_params *p;
    const char *seq;
    const uint64_t *rec_off;
    uint32_t n_rec;
    const uint32_t *group_of_rec;
    uint32_t n_groups;
    const uint32_t *grp_first;   /* records of group g: grp_recs[grp_first[g]..grp_first[g+1]) */
    const uint32_t *grp_recs;
    uint64_t *out_hashes;
    uint32_t *out_count;
    uint32_t *out_mult;
    volatile uint32_t next;
    pthread_mutex_t mu;
} sk_job;

static void sketch_group(sk_job *J, uint32_t g)
{
    const orc_params *p = J->p;
    orc_heap *h = orc_heap_new(p->use64, p->sketch_size);
    uint64_t maxlen = 0;
    for (uint32_t r = J->grp_first[g]; r < J->grp_first[g + 1]; r++) {
        uint32_t rec = J->grp_recs[r];
        uint64_t l = J->rec_off[rec + 1] - J->rec_off[rec];
        if (l > maxlen) maxlen = l;
    }
    char *buf = (char *)malloc(maxlen ? maxlen : 1);
    for (uint32_t r = J->grp_first[g]; r < J->grp_first[g + 1]; r++) {
        uint32_t rec = J->grp_recs[r];
        uint64_t l = J->rec_off[rec + 1] - J->rec_off[rec];
        if (l < (uint64_t)p->kmer_size) continue;
        memcpy(buf, J->seq + J->rec_off[rec], l);
        orc_add_minhashes(h, buf, l, p);
    }
    free(buf);
    uint64_t *tmp = (uint64_t *)malloc((p->sketch_size + 2) * sizeof(uint64_t));
    uint32_t *tc = (uint32_t *)malloc((p->sketch_size + 2) * sizeof(uint32_t));
    uint64_t n = orc_heap_to_list(h, tmp, tc);
    memcpy(J->out_hashes + (uint64_t)g * p->sketch_size, tmp, n * sizeof(uint64_t));
    if (J->out_mult) memcpy(J->out_mult + (uint64_t)g * p->sketch_size, tc, n * sizeof(uint32_t));
    J->out_count[g] = (uint32_t)n;
    free(tmp); free(tc);
    orc_heap_free(h);
}

static void *sk_worker(void *arg)
{
    sk_job *J = (sk_job *)arg;
    for (;;) {
        pthread_mutex_lock(&J->mu);
        uint32_t g = J->next++;
        pthread_mutex_unlock(&J->mu);
        if (g >= J->n_groups) break;
        sketch_group(J, g);
    }
    return NULL;
}

int orc_sketch_batch(const orc_params *p, const char *seq, const uint64_t *rec_off,
                     uint32_t n_rec, const uint32_t *group_of_rec, uint32_t n_groups,
                     uint64_t *out_hashes, uint32_t *out_count, uint32_t *out_mult,
                     int threads)
{
    if (!group_of_rec) n_groups = n_rec;
    uint32_t *first = (uint32_t *)calloc(n_groups + 1, sizeof(uint32_t));
    uint32_t *recs = (uint32_t *)malloc((n_rec ? n_rec : 1) * sizeof(uint32_t));
    for (uint32_t r = 0; r < n_rec; r++) {
        uint32_t g = group_of_rec ? group_of_rec[r] : r;
        if (g >= n_groups) { free(first); free(recs); return -1; }
        first[g + 1]++;
    }
    for (uint32_t g = 0; g < n_groups; g++) first[g + 1] += first[g];
    uint32_t *fill = (uint32_t *)malloc((n_groups + 1) * sizeof(uint32_t));
    memcpy(fill, first, (n_groups + 1) * sizeof(uint32_t));
    for (uint32_t r = 0; r < n_rec; r++) {       /* stream order within a group */
        uint32_t g = group_of_rec ? group_of_rec[r] : r;
        recs[fill[g]++] = r;
    }
    free(fill);

    sk_job J;
    memset(&J, 0, sizeof(J));
    J.p = p; J.seq = seq; J.rec_off = rec_off; J.n_rec = n_rec; J.group_of_rec = group_of_rec;
    J.n_groups = n_groups; J.grp_first = first; J.grp_recs = recs;
    J.out_hashes = out_hashes; J.out_count = out_count; J.out_mult = out_mult;
    pthread_mutex_init(&J.mu, NULL);
    if (threads < 1) threads = 1;
    pthread_t *tid = (pthread_t *)malloc(sizeof(pthread_t) * threads);
    for (int t = 0; t < threads; t++) pthread_create(&tid[t], NULL, sk_worker, &J);
    for (int t = 0; t < threads; t++) pthread_join(tid[t], NULL);
    free(tid);
    pthread_mutex_destroy(&J.mu);
    free(first); free(recs);
    return 0;
}

/* ------------------------------------------------------------------------ */
/* -fp text parsing — Sketch::initFromFingerprints Sketch.cpp:82-101          */
/* (std::getline on '\n', `ss >> id`, then `while (ss >> uint64)`).            */
/* ------------------------------------------------------------------------ */

static inline int is_ws(char c)
{
    return c == ' ' || c == '\t' || c == '\n' || c == '\v' || c == '\f' || c == '\r';
}

/* istream >> unsigned long long (libstdc++ num_get semantics for the cases that
 * occur: optional sign, decimal digits, '-' negates modulo 2^64, overflow fails).
 * Returns 1 and advances *pp on success. */
static int read_u64(const char **pp, const char *end, uint64_t *out)
{
    const char *p = *pp;
    while (p < end && is_ws(*p)) p++;
    int neg = 0;
    if (p < end && (*p == '+' || *p == '-')) { neg = (*p == '-'); p++; }
    if (p >= end || *p < '0' || *p > '9') return 0;
    uint64_t v = 0;
    int ovf = 0;
    while (p < end && *p >= '0' && *p <= '9') {
        uint64_t d = (uint64_t)(*p - '0');
        if (v > (UINT64_MAX - d) / 10) ovf = 1;
        v = v * 10 + d;
        p++;
    }
    if (ovf) return 0;
    *out = neg ? (uint64_t)(0 - v) : v;
    *pp = p;
    return 1;
}

uint64_t orc_fp_parse(const char *text, uint64_t text_len, uint64_t limit,
                      uint64_t *lines_used, uint64_t max_lines, uint64_t max_vals,
                      uint64_t *id_off, uint32_t *id_len, uint64_t *vals,
                      uint64_t *line_val_off)
{
    const char *end = text + text_len;
    const char *p = text;
    uint64_t nl = 0, nv = 0;
    line_val_off[0] = 0;
    /* getline: a line exists if at least one char precedes EOF, or a '\n' is hit */
    while (p < end && *lines_used < limit && nl < max_lines) {
        const char *eol = (const char *)memchr(p, '\n', (size_t)(end - p));
        const char *le = eol ? eol : end;
        (*lines_used)++;
        const char *q = p;
        while (q < le && is_ws(*q)) q++;
        const char *ib = q;
        while (q < le && !is_ws(*q)) q++;
        id_off[nl] = (uint64_t)(ib - text);
        id_len[nl] = (uint32_t)(q - ib);
        if (q > ib) {   /* `ss >> id` succeeded; otherwise the stream is failed */
            uint64_t v;
            while (nv < max_vals && read_u64(&q, le, &v)) vals[nv++] = v;
        }
        nl++;
        line_val_off[nl] = nv;
        p = eol ? eol + 1 : end;
    }
    return nl;
}

/* ------------------------------------------------------------------------ */
/* Distance — compareSketches CommandDistance.cpp:365-430                     */
/* ------------------------------------------------------------------------ */

void orc_compare(const void *ref, uint64_t len_ref, const void *qry, uint64_t len_qry,
                 int use64, uint64_t sketch_size, uint64_t *numer, uint64_t *denom)
{
    uint64_t i = 0, j = 0, common = 0, d = 0;
    if (use64) {
        const uint64_t *a = (const uint64_t *)ref, *b = (const uint64_t *)qry;
        while (d < sketch_size && i < len_ref && j < len_qry) {
            if (a[i] < b[j]) i++;
            else if (b[j] < a[i]) j++;
            else { i++; j++; common++; }
            d++;
        }
    } else {
        const uint32_t *a = (const uint32_t *)ref, *b = (const uint32_t *)qry;
        while (d < sketch_size && i < len_ref && j < len_qry) {
            if (a[i] < b[j]) i++;
            else if (b[j] < a[i]) j++;
            else { i++; j++; common++; }
            d++;
        }
    }
    if (d < sketch_size) {
        if (i < len_ref) d += len_ref - i;
        if (j < len_qry) d += len_qry - j;
        if (d > sketch_size) d = sketch_size;
    }
    *numer = common;
    *denom = d;
}

double orc_distance(uint64_t common, uint64_t denom, int kmer_size)
{
    double jac = (double)common / (double)denom;
    if (common == denom) return 0.0;
    if (common == 0) return 1.0;
    double dist = -log(2.0 * jac / (1.0 + jac)) / (double)kmer_size;
    return dist > 1.0 ? 1.0 : dist;
}

/* --- gsl_cdf_binomial_Q restated: Q(k; p, n) = I_p(k+1, n-k) (GSL cdf/binomial.c)
 * I_x(a,b) via GSL's beta_inc_AXPY (its asymptotic branches included) / beta_cont_frac
 * (cdf/beta_inc.c; GSL is not in the reference tree: the restatement follows GSL 2.x's
 * published source, pinned to mpmath evaluations of the same formulas).  ln B(a,b)
 * is computed with a Stirling-corrected form (instead of GSL's gsl_sf_lnbeta) so
 * the large-argument cancellation stays below 1e-13 relative. */

/* ln Gamma*(x) = lnGamma(x) - [(x-1/2)ln x - x + ln(2pi)/2], x >= 10: Stirling series */
static double lngammastar_large(double x)
{
    double x2 = 1.0 / (x * x);
    /* Bernoulli terms B_{2m}/(2m(2m-1)x^(2m-1)) */
    double s = (1.0 / 12.0) - x2 * ((1.0 / 360.0) - x2 * ((1.0 / 1260.0) - x2 * ((1.0 / 1680.0)
               - x2 * ((1.0 / 1188.0) - x2 * ((691.0 / 360360.0) - x2 * (1.0 / 156.0))))));
    return s / x;
}

static double lngammastar(double x)
{
    if (x >= 10.0) return lngammastar_large(x);
    /* shift up: lnG(x) = lnG(x+n) - ln(x (x+1) ... (x+n-1)) */
    double n = ceil(10.0 - x), y = x + n, prod = 1.0;
    for (double t = x; t < y - 0.5; t += 1.0) prod *= t;
    double lg = lngammastar_large(y) + (y - 0.5) * log(y) - y - log(prod);
    return lg - ((x - 0.5) * log(x) - x);   /* the ln(2pi)/2 terms cancel */
}

static double lnbeta(double a, double b)
{
    /* ln B(a,b) = ln G*(a) + ln G*(b) - ln G*(a+b) + ln(2pi)/2
     *             + (a-1/2) ln(a/(a+b)) + (b-1/2) ln(b/(a+b)) - ... rearranged:
     * (a-1/2)ln a + (b-1/2)ln b - (a+b-1/2) ln(a+b) = -(a-1/2) log1p(b/a)
     *   - (b-1/2) log1p(a/b) ... use the exact identity below */
    double s = a + b;
    double t = -(a - 0.5) * log1p(b / a) - (b - 0.5) * log1p(a / b) - 0.5 * log(s);
    /* check: (a-.5)ln a + (b-.5)ln b - (s-.5)ln s = (a-.5)ln(a/s) + (b-.5)ln(b/s) - .5 ln s */
    return lngammastar(a) + lngammastar(b) - lngammastar(s) + 0.91893853320467274178032973640562 /* ln(2pi)/2 */ + t;
}

static double beta_cont_frac(double a, double b, double x, double epsabs)
{
    const unsigned max_iter = 512;
    const double cutoff = 2.0 * DBL_MIN;
    unsigned it = 0;
    double num = 1.0;
    double den = 1.0 - (a + b) * x / (a + 1.0);
    if (fabs(den) < cutoff) den = NAN;
    den = 1.0 / den;
    double cf = den;
    while (it < max_iter) {
        const int k = (int)it + 1;
        double coeff = k * (b - k) * x / (((a - 1.0) + 2 * k) * (a + 2 * k));
        den = 1.0 + coeff * den;
        num = 1.0 + coeff / num;
        if (fabs(den) < cutoff) den = NAN;
        if (fabs(num) < cutoff) num = NAN;
        den = 1.0 / den;
        double delta = den * num;
        cf *= delta;
        coeff = -(a + k) * (a + b + k) * x / ((a + 2 * k) * (a + 2 * k + 1.0));
        den = 1.0 + coeff * den;
        num = 1.0 + coeff / num;
        if (fabs(den) < cutoff) den = NAN;
        if (fabs(num) < cutoff) num = NAN;
        den = 1.0 / den;
        delta = den * num;
        cf *= delta;
        if (fabs(delta - 1.0) < 2.0 * DBL_EPSILON) break;
        if (cf * fabs(delta - 1.0) < epsabs) break;
        ++it;
    }
    if (it >= max_iter) return NAN;
    return cf;
}

/* Regularized incomplete gamma P(a, x) / Q(a, x) (gsl_sf_gamma_inc_P / _Q) for the small
 * shape (a < 10) of the asymptotic branches below: the series
 *   P = x^a e^-x / Gamma(a+1) * sum_n x^n / ((a+1)...(a+n))        for x < a + 1,
 * else Legendre's continued fraction for Q (modified Lentz).  Both are well conditioned
 * there: any accurate evaluation agrees with GSL's own branches to ~1e-15. */
static double lngamma_pos(double x)
{
    return lngammastar(x) + (x - 0.5) * log(x) - x + 0.91893853320467274178032973640562;
}

static double gamma_inc_P_series(double a, double x)
{
    double sum = 1.0, term = 1.0;
    for (int n = 1; n < 100000; n++) {
        term *= x / (a + n);
        sum += term;
        if (term < sum * DBL_EPSILON) break;
    }
    return exp(a * log(x) - x - lngamma_pos(a + 1.0)) * sum;
}

static double gamma_inc_Q_cf(double a, double x)
{
    const double tiny = 1e-300;
    double b = x + 1.0 - a, c = 1.0 / tiny, d = 1.0 / b, h = d;
    for (int i = 1; i < 100000; i++) {
        const double an = -(double)i * ((double)i - a);
        b += 2.0;
        d = an * d + b;
        if (fabs(d) < tiny) d = tiny;
        c = b + an / c;
        if (fabs(c) < tiny) c = tiny;
        d = 1.0 / d;
        const double del = d * c;
        h *= del;
        if (fabs(del - 1.0) < DBL_EPSILON) break;
    }
    return exp(a * log(x) - x - lngamma_pos(a)) * h;
}

static double gamma_inc_P(double a, double x)
{
    if (x <= 0.0) return 0.0;
    return x < a + 1.0 ? gamma_inc_P_series(a, x) : 1.0 - gamma_inc_Q_cf(a, x);
}

static double gamma_inc_Q(double a, double x)
{
    if (x <= 0.0) return 1.0;
    return x < a + 1.0 ? 1.0 - gamma_inc_P_series(a, x) : gamma_inc_Q_cf(a, x);
}

/* gsl_cdf_beta_P(x, a, b) = beta_inc_AXPY(1, 0, a, b, x) (GSL cdf/beta_inc.c): the two
 * asymptotic regimes of Abramowitz & Stegun 26.5.17 first (reached only when the union
 * size n passed as pValue's sketch size exceeds 1e5: a = common, b = n - common + 1), then
 * the continued fraction of the general regime */
static double beta_P(double x, double a, double b)
{
    if (x == 0.0) return 0.0;
    if (x == 1.0) return 1.0;
    if (a > 1e5 && b < 10 && x > a / (a + b)) {          /* large a, small b, x past the peak */
        const double N = a + (b - 1.0) / 2.0;
        return gamma_inc_Q(b, -N * log(x));
    }
    if (b > 1e5 && a < 10 && x < b / (a + b)) {          /* small a, large b, x before it */
        const double N = b + (a - 1.0) / 2.0;
        return gamma_inc_P(a, -N * log1p(-x));
    }
    double ln_pre = -lnbeta(a, b) + a * log(x) + b * log1p(-x);
    double pre = exp(ln_pre);
    if (x < (a + 1.0) / (a + b + 2.0)) {
        double cf = beta_cont_frac(a, b, x, 0.0);
        return pre * cf / a;
    } else {
        double epsabs = DBL_EPSILON / fabs(pre / b);
        double cf = beta_cont_frac(b, a, 1.0 - x, epsabs);
        return 1.0 - pre * cf / b;
    }
}

double orc_binomial_q(uint64_t k, double p, uint64_t n)
{
    if (k >= n) return 0.0;
    return beta_P(p, (double)k + 1.0, (double)n - (double)k);
}

/* pValue CommandDistance.cpp:433-450 */
double orc_pvalue(uint64_t x, uint64_t len_ref, uint64_t len_qry, double kmer_space,
                  uint64_t sketch_size)
{
    if (x == 0) return 1.0;
    double px = 1.0 / (1.0 + kmer_space / (double)len_ref);
    double py = 1.0 / (1.0 + kmer_space / (double)len_qry);
    double r = px * py / (px + py - px * py);
    return orc_binomial_q(x - 1, r, sketch_size);
}

/* ------------------------------------------------------------------------ */
/* Dist grid with the reference's chunking (CommandDistance.cpp:224-261)        */
/* ------------------------------------------------------------------------ */

typedef struct {
    const void *ref; const uint32_t *ref_len; const uint64_t *ref_length; uint64_t ref_stride; uint32_t n_ref;
    const void *qry; const uint32_t *qry_len; const uint64_t *qry_length; uint64_t qry_stride; uint32_t n_qry;
    int use64; uint64_t sketch_size; int kmer_size; double kmer_space;
    uint32_t *numer, *denom; double *dist, *pv;
    uint64_t chunk, n_pairs;
    uint64_t next;
    pthread_mutex_t mu;
} dg_job;

static void *dg_worker(void *arg)
{
    dg_job *J = (dg_job *)arg;
    const size_t hb = J->use64 ? 8 : 4;
    for (;;) {
        pthread_mutex_lock(&J->mu);
        uint64_t start = J->next;
        J->next += J->chunk;
        pthread_mutex_unlock(&J->mu);
        if (start >= J->n_pairs) break;
        uint64_t stop = start + J->chunk < J->n_pairs ? start + J->chunk : J->n_pairs;
        for (uint64_t idx = start; idx < stop; idx++) {
            uint64_t q = idx / J->n_ref, r = idx % J->n_ref;
            uint64_t nu, de;
            orc_compare((const char *)J->ref + r * J->ref_stride * hb, J->ref_len[r],
                        (const char *)J->qry + q * J->qry_stride * hb, J->qry_len[q],
                        J->use64, J->sketch_size, &nu, &de);
            J->numer[idx] = (uint32_t)nu;
            J->denom[idx] = (uint32_t)de;
            if (J->dist) J->dist[idx] = orc_distance(nu, de, J->kmer_size);
            if (J->pv)
                J->pv[idx] = orc_pvalue(nu, J->ref_length[r], J->qry_length[q], J->kmer_space, de);
        }
    }
    return NULL;
}

int orc_dist_grid(const void *ref, const uint32_t *ref_len, const uint64_t *ref_length,
                  uint64_t ref_stride, uint32_t n_ref,
                  const void *qry, const uint32_t *qry_len, const uint64_t *qry_length,
                  uint64_t qry_stride, uint32_t n_qry,
                  int use64, uint64_t sketch_size, int kmer_size, double kmer_space,
                  uint32_t *out_numer, uint32_t *out_denom, double *out_dist,
                  double *out_pvalue, int threads)
{
    if (threads < 1) threads = 1;
    dg_job J;
    memset(&J, 0, sizeof(J));
    J.ref = ref; J.ref_len = ref_len; J.ref_length = ref_length; J.ref_stride = ref_stride; J.n_ref = n_ref;
    J.qry = qry; J.qry_len = qry_len; J.qry_length = qry_length; J.qry_stride = qry_stride; J.n_qry = n_qry;
    J.use64 = use64; J.sketch_size = sketch_size; J.kmer_size = kmer_size; J.kmer_space = kmer_space;
    J.numer = out_numer; J.denom = out_denom; J.dist = out_dist; J.pv = out_pvalue;
    J.n_pairs = (uint64_t)n_ref * n_qry;
    uint64_t per = J.n_pairs / (uint64_t)threads;        /* pairsPerThread */
    if (per == 0) per = 1;
    if (per > 0x1000) per = 0x1000;                       /* maxPairsPerThread */
    J.chunk = per;
    if ((out_pvalue && !ref_length) || (out_pvalue && !qry_length)) return -1;
    pthread_mutex_init(&J.mu, NULL);
    pthread_t *tid = (pthread_t *)malloc(sizeof(pthread_t) * threads);
    for (int t = 0; t < threads; t++) pthread_create(&tid[t], NULL, dg_worker, &J);
    for (int t = 0; t < threads; t++) pthread_join(tid[t], NULL);
    free(tid);
    pthread_mutex_destroy(&J.mu);
    return 0;
}

/* ---- triangle -fp positional compare (CommandTriangle.cpp:255-302) ---- */
void orc_positional(const void *a, uint64_t len_a, const void *b, uint64_t len_b, int use64,
                    uint64_t *matches, uint64_t *min_len, double *distance, double *pvalue)
{
    const uint64_t m = len_a < len_b ? len_a : len_b;
    uint64_t c = 0;
    for (uint64_t i = 0; i < m; i++) {
        /* hash1.hash64 != 0 || hash2.hash64 != 0 ? compare hash64 : compare hash32 -- with
         * zero-extended u32 values both branches are "equal values" (:276-290) */
        const uint64_t x = use64 ? ((const uint64_t *)a)[i] : ((const uint32_t *)a)[i];
        const uint64_t y = use64 ? ((const uint64_t *)b)[i] : ((const uint32_t *)b)[i];
        c += x == y;
    }
    *matches = c;
    *min_len = m;
    *distance = 1.0 - ((double)c / (double)m);       /* :292, NaN when m == 0 */
    *pvalue = erfc(sqrt((double)c / 2.0));          /* gsl_cdf_chisq_Q(c, 1), :293 */
}
