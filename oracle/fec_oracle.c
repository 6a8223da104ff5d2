/*
 * fec_oracle.c — CPU restatement of the reference FEC path.  TEST INFRASTRUCTURE
 * ONLY (see fec_oracle.h): never linked into the product library.
 *
 * Every function names the reference lines whose behaviour it restates.
 */
#define _GNU_SOURCE
#include "fec_oracle.h"

#include <immintrin.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------- */
/* splitmix64, counter form                                                   */
/* ------------------------------------------------------------------------- */
static inline uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

void oracle_fill_splitmix(uint8_t* dst, uint64_t nbytes, uint64_t seed, uint64_t byte_offset) {
    for (uint64_t i = 0; i < nbytes; ++i) {
        uint64_t pos = byte_offset + i;
        uint64_t w = mix64(seed + (pos / 8 + 1) * 0x9E3779B97F4A7C15ULL);
        dst[i] = (uint8_t)(w >> (8 * (pos % 8)));
    }
}

/* ------------------------------------------------------------------------- */
/* XOR of n packets: fec_xor_simd.cpp:411-427 (scalar definition)             */
/* ------------------------------------------------------------------------- */
void oracle_xor_scalar(const uint8_t* const* pkts, size_t n, size_t packet_size, uint8_t* out) {
    /* :417-419 — nothing is written for an empty group or zero size */
    if (n == 0 || packet_size == 0) return;
    for (size_t i = 0; i < packet_size; ++i) {
        uint8_t v = pkts[0][i];
        for (size_t p = 1; p < n; ++p) v ^= pkts[p][i];
        out[i] = v;
    }
}

/* Same result computed 32 bytes at a time, as the AVX2 path (:74-204) does:
 * 128-byte main step, 32-byte step, byte tail.  (The reference's prefetch and
 * streaming-store choices do not change the bytes, so they are not restated.) */
__attribute__((target("avx2")))
void oracle_xor_avx2(const uint8_t* const* pkts, size_t n, size_t packet_size, uint8_t* out) {
    if (n == 0 || packet_size == 0) return;
    size_t i = 0;
    for (; i + 128 <= packet_size; i += 128) {
        __m256i a[4];
        for (int u = 0; u < 4; ++u) a[u] = _mm256_loadu_si256((const __m256i*)(pkts[0] + i + 32 * u));
        for (size_t p = 1; p < n; ++p)
            for (int u = 0; u < 4; ++u)
                a[u] = _mm256_xor_si256(a[u], _mm256_loadu_si256((const __m256i*)(pkts[p] + i + 32 * u)));
        for (int u = 0; u < 4; ++u) _mm256_storeu_si256((__m256i*)(out + i + 32 * u), a[u]);
    }
    for (; i + 32 <= packet_size; i += 32) {
        __m256i a = _mm256_loadu_si256((const __m256i*)(pkts[0] + i));
        for (size_t p = 1; p < n; ++p) a = _mm256_xor_si256(a, _mm256_loadu_si256((const __m256i*)(pkts[p] + i)));
        _mm256_storeu_si256((__m256i*)(out + i), a);
    }
    for (; i < packet_size; ++i) {
        uint8_t v = pkts[0][i];
        for (size_t p = 1; p < n; ++p) v ^= pkts[p][i];
        out[i] = v;
    }
}

/* fec_xor_simd.cpp:556-594.  Argument checks in the reference's order (:564-570),
 * ten packets per group (:580), repair of group g at g*packet_size (:589). */
int oracle_encode_batch_legacy(const uint8_t* slab, const uint32_t* offsets, uint32_t num_groups,
                               uint32_t packet_size, uint8_t* repair_out, int use_avx2) {
    if (slab == NULL || offsets == NULL || repair_out == NULL) return -1;
    if (num_groups == 0 || packet_size == 0) return 0;
    const uint8_t* pk[10];
    for (uint32_t g = 0; g < num_groups; ++g) {
        for (uint32_t p = 0; p < 10; ++p) pk[p] = slab + offsets[(uint64_t)g * 10 + p];
        uint8_t* dst = repair_out + (uint64_t)g * packet_size;
        if (use_avx2) oracle_xor_avx2(pk, 10, packet_size, dst);
        else oracle_xor_scalar(pk, 10, packet_size, dst);
    }
    return 0;
}

/* ------------------------------------------------------------------------- */
/* threading helper: split [0, G) into nthreads contiguous ranges             */
/* ------------------------------------------------------------------------- */
typedef void (*range_fn)(void* arg, uint64_t g0, uint64_t g1);
typedef struct { range_fn fn; void* arg; uint64_t g0, g1; } range_job;
static void* range_thread(void* p) { range_job* j = (range_job*)p; j->fn(j->arg, j->g0, j->g1); return NULL; }

static void run_ranges(range_fn fn, void* arg, uint64_t G, int nthreads) {
    if (nthreads <= 1 || G < 2) { fn(arg, 0, G); return; }
    if ((uint64_t)nthreads > G) nthreads = (int)G;
    pthread_t* th = (pthread_t*)calloc((size_t)nthreads, sizeof(pthread_t));
    range_job* jobs = (range_job*)calloc((size_t)nthreads, sizeof(range_job));
    for (int t = 0; t < nthreads; ++t) {
        jobs[t].fn = fn; jobs[t].arg = arg;
        jobs[t].g0 = G * (uint64_t)t / (uint64_t)nthreads;
        jobs[t].g1 = G * (uint64_t)(t + 1) / (uint64_t)nthreads;
        pthread_create(&th[t], NULL, range_thread, &jobs[t]);
    }
    for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
    free(th); free(jobs);
}

typedef struct { const uint8_t* data; uint32_t k, P; uint8_t* repair; } xor_contig_arg;
static void xor_contig_range(void* p, uint64_t g0, uint64_t g1) {
    xor_contig_arg* a = (xor_contig_arg*)p;
    const uint8_t* pk[256];
    for (uint64_t g = g0; g < g1; ++g) {
        for (uint32_t j = 0; j < a->k; ++j) pk[j] = a->data + (g * a->k + j) * (uint64_t)a->P;
        oracle_xor_avx2(pk, a->k, a->P, a->repair + g * a->P);
    }
}
void oracle_xor_encode_contig(const uint8_t* data, uint64_t G, uint32_t k, uint32_t P,
                              uint8_t* repair, int nthreads) {
    if (k == 0 || k > 256) return;
    xor_contig_arg a = {data, k, P, repair};
    run_ranges(xor_contig_range, &a, G, nthreads);
}

void oracle_xor_groups(oracle_xor_fn xor_fn, const uint8_t* data, uint64_t G, uint32_t k, uint32_t P,
                       uint8_t* repair) {
    const uint8_t* pk[256];
    if (xor_fn == NULL || k == 0 || k > 256) return;
    for (uint64_t g = 0; g < G; ++g) {
        for (uint32_t j = 0; j < k; ++j) pk[j] = data + (g * k + j) * (uint64_t)P;
        xor_fn(pk, k, P, repair + g * (uint64_t)P);
    }
}

/* ------------------------------------------------------------------------- */
/* GF(2^8), x^8 + x^4 + x^3 + x^2 + 1 (0x11D), generator 2                    */
/* ------------------------------------------------------------------------- */
static uint8_t gf_exp[512];
static uint8_t gf_log[256];
static uint8_t gf_mul_tab[256][256];
static pthread_once_t gf_once = PTHREAD_ONCE_INIT;

static void gf_build(void) {
    unsigned x = 1;
    for (int i = 0; i < 255; ++i) {
        gf_exp[i] = (uint8_t)x;
        gf_log[x] = (uint8_t)i;
        x <<= 1;
        if (x & 0x100) x ^= 0x11D;
    }
    for (int i = 255; i < 512; ++i) gf_exp[i] = gf_exp[i - 255];
    gf_log[0] = 0;
    for (int a = 0; a < 256; ++a)
        for (int b = 0; b < 256; ++b)
            gf_mul_tab[a][b] = (a == 0 || b == 0) ? 0 : gf_exp[gf_log[a] + gf_log[b]];
}
static inline void gf_init(void) { pthread_once(&gf_once, gf_build); }

uint8_t oracle_gf_mul(uint8_t a, uint8_t b) { gf_init(); return gf_mul_tab[a][b]; }
uint8_t oracle_gf_inv(uint8_t a) { gf_init(); return a ? gf_exp[255 - gf_log[a]] : 0; }

/* Systematic Cauchy parity matrix (SURVEY.md §8(a) "code definition"):
 *   C[i][j] = 1 / (x_i ^ y_j),  x_i = i (i < r),  y_j = r + j (j < k)
 *   step 1: divide every column j by C[0][j]        -> row 0 all ones (the XOR row)
 *   step 2: divide every row i >= 1 by its column 0 -> column 0 all ones
 * Row/column scaling keeps every square submatrix non-singular (MDS for k+r <= 256). */
int oracle_parity_matrix(uint32_t k, uint32_t r, uint8_t* M) {
    if (k == 0 || r == 0 || k + r > 256) return -1;
    gf_init();
    for (uint32_t i = 0; i < r; ++i)
        for (uint32_t j = 0; j < k; ++j)
            M[i * k + j] = oracle_gf_inv((uint8_t)(i ^ (r + j)));
    for (uint32_t j = 0; j < k; ++j) {
        uint8_t s = oracle_gf_inv(M[j]);
        for (uint32_t i = 0; i < r; ++i) M[i * k + j] = gf_mul_tab[M[i * k + j]][s];
    }
    for (uint32_t i = 1; i < r; ++i) {
        uint8_t s = oracle_gf_inv(M[i * k]);
        for (uint32_t j = 0; j < k; ++j) M[i * k + j] = gf_mul_tab[M[i * k + j]][s];
    }
    return 0;
}

typedef struct { const uint8_t* data; uint32_t k, r, P; const uint8_t* M; uint8_t* parity; } enc_arg;
static void enc_range(void* p, uint64_t g0, uint64_t g1) {
    enc_arg* a = (enc_arg*)p;
    const uint32_t k = a->k, r = a->r, P = a->P;
    for (uint64_t g = g0; g < g1; ++g) {
        const uint8_t* d = a->data + g * k * (uint64_t)P;
        uint8_t* out = a->parity + g * r * (uint64_t)P;
        memset(out, 0, (size_t)r * P);
        for (uint32_t i = 0; i < r; ++i) {
            uint8_t* o = out + (uint64_t)i * P;
            for (uint32_t j = 0; j < k; ++j) {
                const uint8_t* row = gf_mul_tab[a->M[i * k + j]];
                const uint8_t* src = d + (uint64_t)j * P;
                for (uint32_t b = 0; b < P; ++b) o[b] ^= row[src[b]];
            }
        }
    }
}

int oracle_rs_encode(const uint8_t* data, uint64_t G, uint32_t k, uint32_t r, uint32_t P,
                     uint8_t* parity, int nthreads) {
    if (k == 0 || r == 0 || k + r > 256) return -1;
    gf_init();
    uint8_t* M = (uint8_t*)malloc((size_t)k * r);
    oracle_parity_matrix(k, r, M);
    enc_arg a = {data, k, r, P, M, parity};
    run_ranges(enc_range, &a, G, nthreads);
    free(M);
    return 0;
}

/* Invert an n x n matrix over GF(2^8) by Gauss-Jordan.  Returns 0, -1 if singular. */
static int gf_invert(uint8_t* A, uint8_t* inv, uint32_t n) {
    for (uint32_t i = 0; i < n; ++i)
        for (uint32_t j = 0; j < n; ++j) inv[i * n + j] = (uint8_t)(i == j);
    for (uint32_t c = 0; c < n; ++c) {
        uint32_t piv = c;
        while (piv < n && A[piv * n + c] == 0) ++piv;
        if (piv == n) return -1;
        if (piv != c)
            for (uint32_t j = 0; j < n; ++j) {
                uint8_t t = A[c * n + j]; A[c * n + j] = A[piv * n + j]; A[piv * n + j] = t;
                t = inv[c * n + j]; inv[c * n + j] = inv[piv * n + j]; inv[piv * n + j] = t;
            }
        uint8_t s = oracle_gf_inv(A[c * n + c]);
        for (uint32_t j = 0; j < n; ++j) {
            A[c * n + j] = gf_mul_tab[A[c * n + j]][s];
            inv[c * n + j] = gf_mul_tab[inv[c * n + j]][s];
        }
        for (uint32_t i = 0; i < n; ++i) {
            if (i == c || A[i * n + c] == 0) continue;
            uint8_t f = A[i * n + c];
            for (uint32_t j = 0; j < n; ++j) {
                A[i * n + j] ^= gf_mul_tab[f][A[c * n + j]];
                inv[i * n + j] ^= gf_mul_tab[f][inv[c * n + j]];
            }
        }
    }
    return 0;
}

typedef struct {
    uint8_t* data; const uint8_t* parity; const uint64_t* masks;
    uint32_t k, r, P; const uint8_t* M; uint8_t* status; int64_t bad;
    pthread_mutex_t mu;
} dec_arg;

/* Decode by inverting the full k x k generator submatrix of the chosen survivors
 * (a different formulation from the device's syndrome form; same linear map). */
static void dec_range(void* p, uint64_t g0, uint64_t g1) {
    dec_arg* a = (dec_arg*)p;
    const uint32_t k = a->k, r = a->r, P = a->P;
    uint8_t* Gs = (uint8_t*)malloc((size_t)k * k);
    uint8_t* Inv = (uint8_t*)malloc((size_t)k * k);
    uint32_t surv[64], erased[64];
    int64_t bad = 0;
    for (uint64_t g = g0; g < g1; ++g) {
        uint64_t m = a->masks[g];
        uint32_t ne = 0, ns = 0;
        for (uint32_t j = 0; j < k; ++j) {
            if ((m >> j) & 1) erased[ne++] = j;
            else surv[ns++] = j;
        }
        if (a->status) a->status[g] = 0;
        if (ne == 0) continue;
        for (uint32_t i = 0; i < r && ns < k; ++i)
            if (!((m >> (k + i)) & 1)) surv[ns++] = k + i;
        if (ns < k) { if (a->status) a->status[g] = 1; ++bad; continue; }
        for (uint32_t s = 0; s < k; ++s)
            for (uint32_t j = 0; j < k; ++j)
                Gs[s * k + j] = surv[s] < k ? (uint8_t)(surv[s] == j) : a->M[(surv[s] - k) * k + j];
        if (gf_invert(Gs, Inv, k) != 0) { if (a->status) a->status[g] = 1; ++bad; continue; }
        uint8_t* d = a->data + g * k * (uint64_t)P;
        const uint8_t* par = a->parity + g * r * (uint64_t)P;
        for (uint32_t e = 0; e < ne; ++e) {
            uint8_t* o = d + (uint64_t)erased[e] * P;
            uint8_t* tmp = (uint8_t*)calloc(P, 1);
            for (uint32_t s = 0; s < k; ++s) {
                const uint8_t* row = gf_mul_tab[Inv[erased[e] * k + s]];
                const uint8_t* src = surv[s] < k ? d + (uint64_t)surv[s] * P : par + (uint64_t)(surv[s] - k) * P;
                for (uint32_t b = 0; b < P; ++b) tmp[b] ^= row[src[b]];
            }
            /* write after all rows read their inputs: erased shards are never survivors */
            memcpy(o, tmp, P);
            free(tmp);
        }
    }
    free(Gs); free(Inv);
    pthread_mutex_lock(&a->mu); a->bad += bad; pthread_mutex_unlock(&a->mu);
}

int64_t oracle_rs_decode(uint8_t* data, const uint8_t* parity, const uint64_t* erasure_masks,
                         uint64_t G, uint32_t k, uint32_t r, uint32_t P, uint8_t* status,
                         int nthreads) {
    if (k == 0 || r == 0 || k + r > 64) return -1;
    gf_init();
    uint8_t* M = (uint8_t*)malloc((size_t)k * r);
    oracle_parity_matrix(k, r, M);
    dec_arg a;
    a.data = data; a.parity = parity; a.masks = erasure_masks; a.k = k; a.r = r; a.P = P;
    a.M = M; a.status = status; a.bad = 0;
    pthread_mutex_init(&a.mu, NULL);
    run_ranges(dec_range, &a, G, nthreads);
    pthread_mutex_destroy(&a.mu);
    free(M);
    return a.bad;
}

/* ------------------------------------------------------------------------- */
/* Fast CPU comparator (bench.py cpu_baseline): GFNI affine multiply           */
/* ------------------------------------------------------------------------- */
/* x -> c*x is linear over GF(2): output bit i = parity(row_i & x) with row_i bit j =
 * bit i of c*2^j.  VGF2P8AFFINEQB takes row_i from byte 7-i of the 64-bit matrix. */
uint64_t oracle_gf_affine(uint8_t c) {
    gf_init();
    uint64_t A = 0;
    for (int i = 0; i < 8; ++i) {
        unsigned row = 0;
        for (int j = 0; j < 8; ++j) row |= ((unsigned)(gf_mul_tab[c][1u << j] >> i) & 1u) << j;
        A |= (uint64_t)row << (8 * (7 - i));
    }
    return A;
}

#include <cpuid.h>
int oracle_fast_isa(void) {
    unsigned a, b, c, d;
    if (!__get_cpuid_count(7, 0, &a, &b, &c, &d)) return 0;
    const int gfni = (c >> 8) & 1, avx2 = (b >> 5) & 1, avx512bw = (b >> 30) & 1, avx512f = (b >> 16) & 1;
    if (!gfni || !avx2) return 0;
    return (avx512f && avx512bw) ? 2 : 1;
}

#define FAST_MAXK 32u
#define FAST_MAXE 8u
#define FAST_TAB  512u   /* per-thread recovery-row cache entries (direct mapped) */

/* Rows for the 64-byte (AVX-512) or 32-byte (AVX2) column step of one group.
 * n_out rows; row o = sum over s < n_in of coef[o][s] * in_s.  coef 1 = plain XOR. */
typedef struct {
    uint32_t n_in, n_out;
    const uint8_t* in[FAST_MAXK > 64 ? FAST_MAXK : 64];
    uint8_t* out[FAST_MAXE];
    const uint64_t* A;     /* n_out x n_in affine matrices, row-major */
    const uint8_t* coef;   /* n_out x n_in coefficients */
} fast_job;

__attribute__((target("avx512f,avx512bw,gfni"), always_inline))
static inline void fast_rows512(const fast_job* jb, uint32_t P, const uint32_t NO) {
    for (uint32_t c = 0; c < P; c += 64) {
        const uint32_t n = P - c < 64 ? P - c : 64;
        const __mmask64 m = n == 64 ? ~0ULL : ((1ULL << n) - 1);
        __m512i acc[FAST_MAXE];
        for (uint32_t o = 0; o < NO; ++o) acc[o] = _mm512_setzero_si512();
        for (uint32_t s = 0; s < jb->n_in; ++s) {
            const __m512i x = _mm512_maskz_loadu_epi8(m, jb->in[s] + c);
            for (uint32_t o = 0; o < NO; ++o) {
                const uint32_t t = o * jb->n_in + s;
                if (jb->coef[t] == 1) acc[o] = _mm512_xor_si512(acc[o], x);
                else if (jb->coef[t] != 0)
                    acc[o] = _mm512_xor_si512(acc[o], _mm512_gf2p8affine_epi64_epi8(x, _mm512_set1_epi64((long long)jb->A[t]), 0));
            }
        }
        for (uint32_t o = 0; o < NO; ++o) _mm512_mask_storeu_epi8(jb->out[o] + c, m, acc[o]);
    }
}

__attribute__((target("avx512f,avx512bw,gfni")))
static void fast_run512(const fast_job* jb, uint32_t P) {
    switch (jb->n_out) {
        case 1: fast_rows512(jb, P, 1); break;
        case 2: fast_rows512(jb, P, 2); break;
        case 3: fast_rows512(jb, P, 3); break;
        case 4: fast_rows512(jb, P, 4); break;
        case 5: fast_rows512(jb, P, 5); break;
        case 6: fast_rows512(jb, P, 6); break;
        case 7: fast_rows512(jb, P, 7); break;
        default: fast_rows512(jb, P, 8); break;
    }
}

__attribute__((target("avx2,gfni"), always_inline))
static inline void fast_rows256(const fast_job* jb, uint32_t P, const uint32_t NO) {
    uint8_t tail[FAST_MAXE][32];
    for (uint32_t c = 0; c < P; c += 32) {
        const uint32_t n = P - c < 32 ? P - c : 32;
        __m256i acc[FAST_MAXE];
        for (uint32_t o = 0; o < NO; ++o) acc[o] = _mm256_setzero_si256();
        for (uint32_t s = 0; s < jb->n_in; ++s) {
            __m256i x;
            if (n == 32) {
                x = _mm256_loadu_si256((const __m256i*)(jb->in[s] + c));
            } else {
                uint8_t b[32] = {0};
                memcpy(b, jb->in[s] + c, n);
                x = _mm256_loadu_si256((const __m256i*)b);
            }
            for (uint32_t o = 0; o < NO; ++o) {
                const uint32_t t = o * jb->n_in + s;
                if (jb->coef[t] == 1) acc[o] = _mm256_xor_si256(acc[o], x);
                else if (jb->coef[t] != 0)
                    acc[o] = _mm256_xor_si256(acc[o], _mm256_gf2p8affine_epi64_epi8(x, _mm256_set1_epi64x((long long)jb->A[t]), 0));
            }
        }
        for (uint32_t o = 0; o < NO; ++o) {
            if (n == 32) {
                _mm256_storeu_si256((__m256i*)(jb->out[o] + c), acc[o]);
            } else {
                _mm256_storeu_si256((__m256i*)tail[o], acc[o]);
                memcpy(jb->out[o] + c, tail[o], n);
            }
        }
    }
}

__attribute__((target("avx2,gfni")))
static void fast_run256(const fast_job* jb, uint32_t P) {
    switch (jb->n_out) {
        case 1: fast_rows256(jb, P, 1); break;
        case 2: fast_rows256(jb, P, 2); break;
        case 3: fast_rows256(jb, P, 3); break;
        case 4: fast_rows256(jb, P, 4); break;
        case 5: fast_rows256(jb, P, 5); break;
        case 6: fast_rows256(jb, P, 6); break;
        case 7: fast_rows256(jb, P, 7); break;
        default: fast_rows256(jb, P, 8); break;
    }
}

static void fast_run(int isa, const fast_job* jb, uint32_t P) {
    if (isa == 2) fast_run512(jb, P);
    else fast_run256(jb, P);
}

typedef struct {
    const uint8_t* data; uint32_t k, r, P; int isa;
    const uint64_t* A; const uint8_t* coef; uint8_t* parity;
} fenc_arg;

static void fenc_range(void* p, uint64_t g0, uint64_t g1) {
    fenc_arg* a = (fenc_arg*)p;
    const uint32_t k = a->k, r = a->r, P = a->P;
    fast_job jb;
    jb.n_in = k;
    for (uint64_t g = g0; g < g1; ++g) {
        for (uint32_t j = 0; j < k; ++j) jb.in[j] = a->data + (g * k + j) * (uint64_t)P;
        for (uint32_t i0 = 0; i0 < r; i0 += FAST_MAXE) {   /* passes of up to 8 parity rows */
            jb.n_out = r - i0 < FAST_MAXE ? r - i0 : FAST_MAXE;
            for (uint32_t o = 0; o < jb.n_out; ++o) jb.out[o] = a->parity + (g * r + i0 + o) * (uint64_t)P;
            jb.A = a->A + (uint64_t)i0 * k;
            jb.coef = a->coef + (uint64_t)i0 * k;
            fast_run(a->isa, &jb, P);
        }
    }
}

int oracle_rs_encode_fast(const uint8_t* data, uint64_t G, uint32_t k, uint32_t r, uint32_t P,
                          uint8_t* parity, int nthreads) {
    const int isa = oracle_fast_isa();
    if (isa == 0 || k > 64) return oracle_rs_encode(data, G, k, r, P, parity, nthreads);
    if (k == 0 || r == 0 || k + r > 256) return -1;
    gf_init();
    uint8_t* M = (uint8_t*)malloc((size_t)k * r);
    uint64_t* A = (uint64_t*)malloc((size_t)k * r * 8);
    oracle_parity_matrix(k, r, M);
    for (uint32_t t = 0; t < k * r; ++t) A[t] = oracle_gf_affine(M[t]);
    fenc_arg a = {data, k, r, P, isa, A, M, parity};
    run_ranges(fenc_range, &a, G, nthreads);
    free(M); free(A);
    return 0;
}

/* Recovery rows of one erasure pattern (same survivor rule and inversion as dec_range). */
typedef struct {
    uint64_t mask; int valid, ok;
    uint32_t e;
    uint8_t surv[FAST_MAXK], erased[FAST_MAXE];
    uint8_t coef[FAST_MAXE * FAST_MAXK];
    uint64_t A[FAST_MAXE * FAST_MAXK];
} fast_rec;

static void fast_rec_build(fast_rec* R, uint64_t m, uint32_t k, uint32_t r, const uint8_t* M) {
    uint8_t Gs[FAST_MAXK * FAST_MAXK], Inv[FAST_MAXK * FAST_MAXK];
    uint32_t surv[64], erased[64], ns = 0, ne = 0;
    R->mask = m; R->valid = 1; R->ok = 0; R->e = 0;
    for (uint32_t j = 0; j < k; ++j) {
        if ((m >> j) & 1) erased[ne++] = j;
        else surv[ns++] = j;
    }
    for (uint32_t i = 0; i < r && ns < k; ++i)
        if (!((m >> (k + i)) & 1)) surv[ns++] = k + i;
    if (ns < k || ne > FAST_MAXE) return;
    for (uint32_t s = 0; s < k; ++s)
        for (uint32_t j = 0; j < k; ++j)
            Gs[s * k + j] = surv[s] < k ? (uint8_t)(surv[s] == j) : M[(surv[s] - k) * k + j];
    if (gf_invert(Gs, Inv, k) != 0) return;
    R->ok = 1; R->e = ne;
    for (uint32_t s = 0; s < k; ++s) R->surv[s] = (uint8_t)surv[s];
    for (uint32_t o = 0; o < ne; ++o) {
        R->erased[o] = (uint8_t)erased[o];
        for (uint32_t s = 0; s < k; ++s) {
            R->coef[o * k + s] = Inv[erased[o] * k + s];
            R->A[o * k + s] = oracle_gf_affine(Inv[erased[o] * k + s]);
        }
    }
}

typedef struct {
    uint8_t* data; const uint8_t* parity; const uint64_t* masks;
    uint32_t k, r, P; int isa; const uint8_t* M; uint8_t* status; int64_t bad;
    pthread_mutex_t mu;
} fdec_arg;

static void fdec_range(void* p, uint64_t g0, uint64_t g1) {
    fdec_arg* a = (fdec_arg*)p;
    const uint32_t k = a->k, r = a->r, P = a->P;
    const uint64_t kmask = (1ULL << k) - 1;
    fast_rec* cache = (fast_rec*)calloc(FAST_TAB, sizeof(fast_rec));
    fast_job jb;
    jb.n_in = k;
    int64_t bad = 0;
    for (uint64_t g = g0; g < g1; ++g) {
        const uint64_t m = a->masks[g];
        if (a->status) a->status[g] = 0;
        if ((m & kmask) == 0) continue;
        fast_rec* R = &cache[(m * 0x9E3779B97F4A7C15ULL) >> 55];   /* 9 bits: FAST_TAB */
        if (!R->valid || R->mask != m) fast_rec_build(R, m, k, r, a->M);
        if (!R->ok) { if (a->status) a->status[g] = 1; ++bad; continue; }
        uint8_t* d = a->data + g * k * (uint64_t)P;
        const uint8_t* par = a->parity + g * r * (uint64_t)P;
        for (uint32_t s = 0; s < k; ++s)
            jb.in[s] = R->surv[s] < k ? d + (uint64_t)R->surv[s] * P : par + (uint64_t)(R->surv[s] - k) * P;
        jb.n_out = R->e;
        for (uint32_t o = 0; o < R->e; ++o) jb.out[o] = d + (uint64_t)R->erased[o] * P;
        jb.A = R->A;
        jb.coef = R->coef;
        /* in place: erased shards are never survivors, and each column step reads all its
         * inputs before it stores */
        fast_run(a->isa, &jb, P);
    }
    free(cache);
    pthread_mutex_lock(&a->mu); a->bad += bad; pthread_mutex_unlock(&a->mu);
}

int64_t oracle_rs_decode_fast(uint8_t* data, const uint8_t* parity, const uint64_t* erasure_masks,
                              uint64_t G, uint32_t k, uint32_t r, uint32_t P, uint8_t* status,
                              int nthreads) {
    const int isa = oracle_fast_isa();
    if (isa == 0 || k > FAST_MAXK || r > FAST_MAXE)
        return oracle_rs_decode(data, parity, erasure_masks, G, k, r, P, status, nthreads);
    if (k == 0 || r == 0 || k + r > 64) return -1;
    gf_init();
    uint8_t* M = (uint8_t*)malloc((size_t)k * r);
    oracle_parity_matrix(k, r, M);
    fdec_arg a;
    a.data = data; a.parity = parity; a.masks = erasure_masks; a.k = k; a.r = r; a.P = P;
    a.isa = isa; a.M = M; a.status = status; a.bad = 0;
    pthread_mutex_init(&a.mu, NULL);
    run_ranges(fdec_range, &a, G, nthreads);
    pthread_mutex_destroy(&a.mu);
    free(M);
    return a.bad;
}

/* ------------------------------------------------------------------------- */
/* Go-path semantics                                                          */
/* ------------------------------------------------------------------------- */
/* encoder.go:113-163: maxSize over the group, zero-padded XOR (:133-143), header
 * FE C0 | groupID u64 LE | count u8 (:146-157). */
int64_t oracle_go_generate_redundancy(const uint8_t* const* pkts, const size_t* lens, size_t n,
                                      uint64_t group_id, uint8_t* out, size_t out_cap) {
    if (n == 0) return -1;
    size_t maxlen = 0;
    for (size_t p = 0; p < n; ++p) if (lens[p] > maxlen) maxlen = lens[p];
    if (maxlen == 0) return -2;
    if (out_cap < 11 + maxlen) return -3;
    out[0] = 0xFE; out[1] = 0xC0;
    for (int b = 0; b < 8; ++b) out[2 + b] = (uint8_t)(group_id >> (8 * b));
    out[10] = (uint8_t)n;
    for (size_t i = 0; i < maxlen; ++i) {
        uint8_t v = 0;
        for (size_t p = 0; p < n; ++p) if (i < lens[p]) v ^= pkts[p][i];
        out[11 + i] = v;
    }
    return (int64_t)(11 + maxlen);
}

/* decoder.go:255-287 with padTo (:62-69): out = pad(parity) ^ XOR of pad(present). */
int64_t oracle_go_recover_single(const uint8_t* const* pkts, const size_t* lens,
                                 const uint8_t* present, size_t packet_count,
                                 const uint8_t* parity_payload, size_t parity_len,
                                 size_t symbol_len, uint8_t* out) {
    int64_t missing = -1;
    for (size_t i = 0; i < packet_count; ++i) if (!present[i]) { missing = (int64_t)i; break; }
    if (missing < 0) return -1;
    for (size_t b = 0; b < symbol_len; ++b) out[b] = b < parity_len ? parity_payload[b] : 0;
    for (size_t i = 0; i < packet_count; ++i) {
        if (!present[i] || (int64_t)i == missing) continue;
        size_t L = lens[i] < symbol_len ? lens[i] : symbol_len;
        for (size_t b = 0; b < L; ++b) out[b] ^= pkts[i][b];
    }
    return missing;
}
