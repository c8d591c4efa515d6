/* CPU scan baseline — TEST/BASELINE INFRASTRUCTURE ONLY (see oracle.h).
 *
 * The timed CPU leg of bench.py's scan section (BASELINE config 3): the
 * reference's multithreaded SIMD scan driver restated for this host.
 *   - threads: thread t scans entries [t*N/T, (t+1)*N/T) of one column
 *     (multithreadedscan.cpp:227-259, scan_wrapper), pinned one per core
 *     (the reference runs under numactl --physcpubind, J/README.md:67-70);
 *   - outputs: per-thread buffers allocated and touched before timing
 *     (ResultAllocators.hpp pre_alloc_per_thread); index lists hold offsets
 *     relative to the thread's base pointer, as SIMD512 writes them
 *     (SIMD512.cpp:251-287, concatenated without offsets by join_results);
 *   - time: per-thread steady-clock time of `reps` calls, averaged over the
 *     threads (multithreadedscan.cpp run_*_scan + join_counter_values).
 * The kernels follow SIMD512.cpp's AVX-512 formulation (count :7-32, bitvector
 * :210-222, index :251-287: a 64-row predicate mask per step, popcount or an
 * 8-lane compress-store of row offsets per mask byte), for uint8 columns and for
 * the int32 widening of BASELINE config 3 (four 16-lane compares per 64 rows).
 * Without AVX-512 BW on the host a scalar loop computes the same outputs. */
#define _GNU_SOURCE
#include <immintrin.h>
#include <pthread.h>
#include <sched.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "oracle.h"

enum { K_COUNT = 0, K_BITVECTOR = 1, K_INDEX = 2 };

typedef struct {
    int kind, width, reps, cpu;
    int64_t lo, hi;
    const uint8_t *in; /* this thread's slice */
    size_t n;          /* rows in the slice (a multiple of 64 is scanned, the tail ignored) */
    uint64_t *out;     /* bitvector words or index list */
    uint64_t matches;
    double secs;
    pthread_barrier_t *bar;
    int simd;
} job_t;

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

__attribute__((target("avx512f,avx512bw"))) static inline uint64_t mask64_u8(const uint8_t *p, __m512i lo,
                                                                              __m512i hi) {
    __m512i v = _mm512_loadu_si512((const void *)p);
    return _mm512_cmpge_epu8_mask(v, lo) & _mm512_cmple_epu8_mask(v, hi);
}

__attribute__((target("avx512f,avx512bw"))) static inline uint64_t mask64_i32(const int32_t *p, __m512i lo,
                                                                               __m512i hi) {
    uint64_t m = 0;
    for (int q = 0; q < 4; q++) {
        __m512i v = _mm512_loadu_si512((const void *)(p + 16 * q));
        uint64_t k = (uint16_t)(_mm512_cmpge_epi32_mask(v, lo) & _mm512_cmple_epi32_mask(v, hi));
        m |= k << (16 * q);
    }
    return m;
}

__attribute__((target("avx512f,avx512bw"))) static uint64_t run_simd(job_t *j) {
    const size_t blocks = j->n / 64;
    const int u8 = j->width == 1;
    const __m512i lo = u8 ? _mm512_set1_epi8((char)(uint8_t)j->lo) : _mm512_set1_epi32((int32_t)j->lo);
    const __m512i hi = u8 ? _mm512_set1_epi8((char)(uint8_t)j->hi) : _mm512_set1_epi32((int32_t)j->hi);
    uint64_t total = 0;
    uint64_t *o = j->out;
    __m512i off = _mm512_set_epi64(7, 6, 5, 4, 3, 2, 1, 0);
    const __m512i step8 = _mm512_set1_epi64(8), step64 = _mm512_set1_epi64(64);
    for (size_t b = 0; b < blocks; b++) {
        const uint64_t m = u8 ? mask64_u8(j->in + 64 * b, lo, hi) : mask64_i32((const int32_t *)j->in + 64 * b, lo, hi);
        if (j->kind == K_COUNT) {
            total += (uint64_t)__builtin_popcountll(m);
        } else if (j->kind == K_BITVECTOR) {
            o[b] = m;
            total += (uint64_t)__builtin_popcountll(m); /* matches, for the caller's check */
        } else {
            if (m == 0) {
                off = _mm512_add_epi64(off, step64);
                continue;
            }
            for (int q = 0; q < 8; q++) {
                const __mmask8 part = (__mmask8)(m >> (8 * q));
                _mm512_mask_compressstoreu_epi64(o + total, part, off);
                total += (uint64_t)__builtin_popcount(part);
                off = _mm512_add_epi64(off, step8);
            }
        }
    }
    return total;
}

static uint64_t run_scalar(job_t *j) {
    const size_t rows = j->n / 64 * 64;
    uint64_t total = 0;
    for (size_t i = 0; i < rows; i++) {
        const int64_t v = j->width == 1 ? (int64_t)j->in[i] : (int64_t)((const int32_t *)j->in)[i];
        const int hit = v >= j->lo && v <= j->hi;
        if (j->kind == K_BITVECTOR) {
            if (i % 64 == 0) j->out[i / 64] = 0;
            j->out[i / 64] |= (uint64_t)hit << (i % 64);
            total += (uint64_t)hit;
        } else if (hit) {
            if (j->kind == K_INDEX) j->out[total] = i;
            total++;
        }
    }
    return total;
}

static void *worker(void *arg) {
    job_t *j = (job_t *)arg;
    if (j->cpu >= 0) {
        cpu_set_t set;
        CPU_ZERO(&set);
        CPU_SET(j->cpu, &set);
        pthread_setaffinity_np(pthread_self(), sizeof(set), &set);
    }
    /* warm-up call (touches the output pages, as pre-allocation does) */
    j->matches = j->simd ? run_simd(j) : run_scalar(j);
    pthread_barrier_wait(j->bar);
    const double t0 = now_s();
    for (int r = 0; r < j->reps; r++) j->matches = j->simd ? run_simd(j) : run_scalar(j);
    j->secs = (now_s() - t0) / j->reps;
    return NULL;
}

double oracle_cpu_scan_bench(int kind, int width, int64_t lo, int64_t hi, const void *in, size_t n, int nthreads,
                             const int *cpus, int reps, uint64_t *matches) {
    if (nthreads < 1) nthreads = 1;
    if (reps < 1) reps = 1;
    if ((width != 1 && width != 4) || kind < K_COUNT || kind > K_INDEX) return -1.0;
    const size_t per = n / (size_t)nthreads; /* num_entries_per_thread = N / T, tail ignored */
    job_t *jobs = (job_t *)calloc((size_t)nthreads, sizeof(job_t));
    pthread_t *th = (pthread_t *)calloc((size_t)nthreads, sizeof(pthread_t));
    pthread_barrier_t bar;
    pthread_barrier_init(&bar, NULL, (unsigned)nthreads);
    __builtin_cpu_init();
    const int simd = __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512bw");
    int ok = 1;
    for (int t = 0; t < nthreads; t++) {
        job_t *j = &jobs[t];
        j->kind = kind;
        j->width = width;
        j->reps = reps;
        j->cpu = cpus ? cpus[t] : -1;
        j->lo = lo;
        j->hi = hi;
        j->in = (const uint8_t *)in + (size_t)t * per * (size_t)width;
        j->n = per;
        j->bar = &bar;
        j->simd = simd;
        const size_t words = kind == K_BITVECTOR ? per / 64 : kind == K_INDEX ? per / 64 * 64 + 8 : 0;
        if (words) {
            j->out = (uint64_t *)aligned_alloc(64, ((words * 8 + 63) / 64) * 64);
            if (!j->out) ok = 0;
        }
    }
    double avg = -1.0;
    if (ok) {
        for (int t = 0; t < nthreads; t++) pthread_create(&th[t], NULL, worker, &jobs[t]);
        uint64_t total = 0;
        double sum = 0.0;
        for (int t = 0; t < nthreads; t++) {
            pthread_join(th[t], NULL);
            total += jobs[t].matches;
            sum += jobs[t].secs;
        }
        if (matches) *matches = total;
        avg = sum / nthreads;
    }
    for (int t = 0; t < nthreads; t++) free(jobs[t].out);
    pthread_barrier_destroy(&bar);
    free(jobs);
    free(th);
    return avg;
}
