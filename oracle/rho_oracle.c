/*
 * oracle/rho_oracle.c — CPU restatement of the reference's RHO radix join.
 *
 * TEST INFRASTRUCTURE ONLY (see oracle.h): the checker for tests/ and the
 * timed CPU baseline of bench.py.  Never linked into the product library.
 *
 * Follows Join-Benchmarks/lib/Joins/src/radix/radix_join.cpp:
 *   calc_num_radix_bits        :295-317      calc_num_passes          :319-329
 *   fanout/padding helpers     :331-345      bucket_chaining_join     :359-458
 *   partition_hist / _copy     :617-697      radix_cluster            :715-761
 *   serial_radix_partition     :773-841      parallel_radix_partition :851-931
 *   prj_thread                 :1067-1356    join_init_run            :1369-1638
 * The boost::lockfree task queues become arrays with atomic cursors (the queue
 * only schedules tasks; counts do not depend on it).  rdtscp cycles become
 * CLOCK_MONOTONIC seconds.
 */
#define _GNU_SOURCE
#include <pthread.h>
#include <stdatomic.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "oracle.h"

#define CACHE_LINE_SIZE 64
#define L2_CACHE_SIZE (1280 * 1024)                                  /* prj_params.h:58-60 */
#define L2_CACHE_TUPLES (L2_CACHE_SIZE / sizeof(struct row_t))       /* prj_params.h:66 */
#define SMALL_PADDING_TUPLES (3 * CACHE_LINE_SIZE / sizeof(struct row_t)) /* prj_params.h:94 */
#define HASH_BIT_MODULO(K, MASK, NBITS) (((K) & (MASK)) >> (NBITS))   /* radix_join.cpp:47 */

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

uint32_t oracle_calc_num_radix_bits(uint64_t num_r, uint64_t nthreads) {
    uint64_t max_tuples_in_cache = L2_CACHE_TUPLES / 4;
    uint64_t req = (num_r + max_tuples_in_cache - 1) / max_tuples_in_cache;
    if (req < nthreads) req = nthreads;
    uint32_t bits = 0;
    while ((1ull << bits) < req) ++bits;
    return bits;
}

uint32_t oracle_calc_num_passes(uint32_t num_radix_bits) {
    return num_radix_bits <= 13 ? 1 : 2; /* space_in_l1 = 15 - 2 */
}

static inline uint32_t fanout_pass_1(uint32_t bits, uint32_t passes) { return 1u << (bits / passes); }
static inline uint32_t fanout_pass_2(uint32_t bits, uint32_t passes) { return 1u << (bits - bits / passes); }
static inline uint32_t padding_tuples(uint32_t bits, uint32_t passes) {
    return (uint32_t)SMALL_PADDING_TUPLES * (fanout_pass_2(bits, passes) + 1);
}

/* Per-thread materialisation output: the reference's insert_output into a
 * chunked table (ChunkedTable.cpp:21-171); here one growable array per thread. */
typedef struct out_buf {
    struct output_triple_t *t;
    uint64_t n, cap;
} out_buf;

static void out_push(out_buf *o, uint32_t key, uint32_t rpay, uint32_t spay) {
    if (o->n == o->cap) {
        o->cap = o->cap ? 2 * o->cap : 1024;
        o->t = (struct output_triple_t *)realloc(o->t, o->cap * sizeof(struct output_triple_t));
    }
    o->t[o->n].key = key;
    o->t[o->n].Rpayload = rpay;
    o->t[o->n].Spayload = spay;
    o->n++;
}

/* bucket_chaining_join (:359-458): count-only branch (:428-436) and, with an
 * output buffer, the materialising branch (:437-446). */
static int64_t bucket_chaining_join(const struct row_t *R, uint64_t numR, const struct row_t *S,
                                    uint64_t numS, uint32_t num_radix_bits, out_buf *out) {
    uint32_t N = (uint32_t)numR;
    /* NEXT_POW_2 (:55-64) */
    N--; N |= N >> 1; N |= N >> 2; N |= N >> 4; N |= N >> 8; N |= N >> 16; N++;
    const uint32_t MASK = (N - 1) << num_radix_bits;
    uint32_t *next = (uint32_t *)malloc(sizeof(uint32_t) * (numR ? numR : 1));
    uint32_t *bucket = (uint32_t *)calloc(N ? N : 1, sizeof(uint32_t));
    for (uint32_t i = 0; i < numR;) {
        uint32_t idx = HASH_BIT_MODULO(R[i].key, MASK, num_radix_bits);
        next[i] = bucket[idx];
        bucket[idx] = ++i; /* positions start at 1 */
    }
    int64_t matches = 0;
    if (!out) {
        for (uint32_t i = 0; i < numS; i++) {
            uint32_t idx = HASH_BIT_MODULO(S[i].key, MASK, num_radix_bits);
            for (uint32_t hit = bucket[idx]; hit > 0; hit = next[hit - 1]) {
                if (S[i].key == R[hit - 1].key) matches++;
            }
        }
    } else {
        for (uint32_t i = 0; i < numS; i++) {
            uint32_t idx = HASH_BIT_MODULO(S[i].key, MASK, num_radix_bits);
            for (uint32_t hit = bucket[idx]; hit > 0; hit = next[hit - 1]) {
                if (S[i].key == R[hit - 1].key) {
                    matches++;
                    out_push(out, S[i].key, R[hit - 1].payload, S[i].payload);
                }
            }
        }
    }
    free(bucket);
    free(next);
    return matches;
}

/* histogram_join (:463-612), RHT's build/probe: Nhist = get_hist_size(numR)
 * (:462-467), histogram + prefix sum, R re-ordered by bucket into tmp, probe
 * scans the S key's bucket.  The non-UNROLL path is restated (the UNROLL tail at
 * :556-560 drops the "+ 1" of the bucket index; the plain loops do not). */
static int64_t histogram_join(const struct row_t *R, uint64_t numR, const struct row_t *S, uint64_t numS,
                              uint32_t num_radix_bits, out_buf *out) {
    uint32_t N = (uint32_t)numR;
    N--; N |= N >> 1; N |= N >> 2; N |= N >> 4; N |= N >> 8; N |= N >> 16; N++;
    uint32_t Nhist = N >> 2;
    if (Nhist < 4) Nhist = 4;
    const uint32_t MASK = (Nhist - 1) << num_radix_bits;
    int32_t *hist = (int32_t *)calloc(Nhist + 2, sizeof(int32_t));
    struct row_t *tmp = (struct row_t *)malloc(sizeof(struct row_t) * (numR ? numR : 1));
    for (uint32_t i = 0; i < numR; i++) ++hist[HASH_BIT_MODULO(R[i].key, MASK, num_radix_bits) + 2];
    for (uint32_t i = 2, sum = 0; i < Nhist + 2; i++) {
        sum += (uint32_t)hist[i];
        hist[i] = (int32_t)sum;
    }
    for (uint32_t i = 0; i < numR; i++) {
        const uint32_t idx = HASH_BIT_MODULO(R[i].key, MASK, num_radix_bits) + 1;
        tmp[hist[idx]] = R[i];
        hist[idx]++;
    }
    int64_t match = 0;
    for (uint32_t i = 0; i < numS; ++i) {
        const uint32_t idx = HASH_BIT_MODULO(S[i].key, MASK, num_radix_bits);
        for (int j = hist[idx], end = hist[idx + 1]; j < end; j++) {
            if (S[i].key == tmp[j].key) {
                ++match;
                if (out) out_push(out, S[i].key, tmp[j].payload, S[i].payload);
            }
        }
    }
    free(hist);
    free(tmp);
    return match;
}

static void partition_hist(const struct row_t *rel, uint32_t size, uint32_t *hist, uint32_t MASK, int32_t R) {
    for (uint32_t i = 0; i < size; ++i) ++hist[(rel[i].key & MASK) >> R];
}

static void partition_copy(const struct row_t *rel, uint32_t size, uint32_t *dst, struct row_t *tmp,
                           uint32_t MASK, int32_t R) {
    for (uint32_t i = 0; i < size; ++i) {
        uint32_t idx = (rel[i].key & MASK) >> R;
        tmp[dst[idx]] = rel[i];
        ++dst[idx];
    }
}

typedef struct task_t {
    const struct row_t *relR; uint64_t nR; struct row_t *tmpR;
    const struct row_t *relS; uint64_t nS; struct row_t *tmpS;
} task_t;

typedef struct task_array {
    task_t *t;
    _Atomic uint64_t push;
    _Atomic uint64_t pop;
    uint64_t cap;
} task_array;

static void ta_push(task_array *q, task_t t) {
    uint64_t i = atomic_fetch_add(&q->push, 1);
    if (i < q->cap) q->t[i] = t;
}
static int ta_pop(task_array *q, task_t *t) {
    uint64_t i = atomic_fetch_add(&q->pop, 1);
    uint64_t n = atomic_load(&q->push);
    if (i >= n || i >= q->cap) return 0;
    *t = q->t[i];
    return 1;
}

/* radix_cluster (:715-761): pass-2 partition of one pass-1 partition. */
static void radix_cluster(struct row_t *out, const struct row_t *in, uint64_t n, uint32_t *hist, int R, int D) {
    uint32_t M = ((1u << D) - 1) << R;
    uint32_t fanOut = 1u << D;
    uint32_t *dst = (uint32_t *)malloc(sizeof(uint32_t) * fanOut);
    partition_hist(in, (uint32_t)n, hist, M, R);
    uint32_t offset = 0;
    for (uint32_t i = 0; i < fanOut; i++) {
        dst[i] = (uint32_t)(offset + i * SMALL_PADDING_TUPLES);
        offset += hist[i];
    }
    partition_copy(in, (uint32_t)n, dst, out, M, R);
    free(dst);
}

/* serial_radix_partition (:773-841) */
static void serial_radix_partition(task_t *task, task_array *join_queue, int R, int D) {
    uint64_t offsetR = 0, offsetS = 0;
    const int fanOut = 1 << D;
    uint32_t *outputR = (uint32_t *)calloc(fanOut + 1, sizeof(uint32_t));
    uint32_t *outputS = (uint32_t *)calloc(fanOut + 1, sizeof(uint32_t));
    radix_cluster(task->tmpR, task->relR, task->nR, outputR, R, D);
    radix_cluster(task->tmpS, task->relS, task->nS, outputS, R, D);
    for (int i = 0; i < fanOut; i++) {
        if (outputR[i] > 0 && outputS[i] > 0) {
            task_t t;
            t.nR = outputR[i];
            t.relR = task->tmpR + offsetR + i * SMALL_PADDING_TUPLES;
            t.tmpR = NULL;
            offsetR += outputR[i];
            t.nS = outputS[i];
            t.relS = task->tmpS + offsetS + i * SMALL_PADDING_TUPLES;
            t.tmpS = NULL;
            offsetS += outputS[i];
            ta_push(join_queue, t);
        } else {
            offsetR += outputR[i];
            offsetS += outputS[i];
        }
    }
    free(outputR);
    free(outputS);
}

typedef struct shared_t {
    pthread_barrier_t barrier;
    uint32_t **histR, **histS;
    struct row_t *tmpR, *tmpS, *tmpR2, *tmpS2;
    uint64_t totalR, totalS;
    uint32_t bits, passes;
    int materialize;
    int rht; /* 1 = histogram_join (RHT), 0 = bucket_chaining_join (RHO) */
    task_array part_queue, join_queue;
} shared_t;

typedef struct arg_t {
    shared_t *sh;
    int tid, nthreads;
    const struct row_t *relR, *relS;
    uint64_t numR, numS;
    int64_t result;
    out_buf out;
    double t_total, t_part, t_pass1, t_pass2, t_join;
} arg_t;

/* parallel_radix_partition (:851-931) */
static void parallel_radix_partition(arg_t *a, const struct row_t *rel, uint64_t size, uint64_t total,
                                     uint32_t **hist, uint32_t *output, struct row_t *tmp, int32_t R,
                                     int32_t D, uint32_t padding) {
    const uint32_t fanOut = 1u << D;
    const uint32_t MASK = (fanOut - 1) << R;
    uint32_t *my_hist = hist[a->tid];
    uint32_t *dst = (uint32_t *)malloc(sizeof(uint32_t) * (fanOut + 1));
    partition_hist(rel, (uint32_t)size, my_hist, MASK, R);
    uint32_t sum = 0;
    for (uint32_t i = 0; i < fanOut; i++) { sum += my_hist[i]; my_hist[i] = sum; }
    pthread_barrier_wait(&a->sh->barrier);
    for (int i = 0; i < a->tid; i++)
        for (uint32_t j = 0; j < fanOut; j++) output[j] += hist[i][j];
    for (int i = a->tid; i < a->nthreads; i++)
        for (uint32_t j = 1; j < fanOut; j++) output[j] += hist[i][j - 1];
    for (uint32_t i = 0; i < fanOut; i++) {
        output[i] += i * padding;
        dst[i] = output[i];
    }
    output[fanOut] = (uint32_t)(total + fanOut * padding);
    partition_copy(rel, (uint32_t)size, dst, tmp, MASK, R);
    free(dst);
}

/* prj_thread (:1067-1356) */
static void *prj_thread(void *param) {
    arg_t *a = (arg_t *)param;
    shared_t *sh = a->sh;
    const uint32_t bits = sh->bits, passes = sh->passes;
    const int fanOut = 1 << (bits / passes);
    const int R = (int)(bits / passes);
    const int D = (int)(bits - bits / passes);
    const uint32_t num_padding = padding_tuples(bits, passes);
    uint32_t *outputR = (uint32_t *)calloc(fanOut + 1, sizeof(uint32_t));
    uint32_t *outputS = (uint32_t *)calloc(fanOut + 1, sizeof(uint32_t));
    sh->histR[a->tid] = (uint32_t *)calloc(fanOut, sizeof(uint32_t));
    sh->histS[a->tid] = (uint32_t *)calloc(fanOut, sizeof(uint32_t));

    pthread_barrier_wait(&sh->barrier);
    double t0 = now_s();
    parallel_radix_partition(a, a->relR, a->numR, sh->totalR, sh->histR, outputR, sh->tmpR, 0, R, num_padding);
    pthread_barrier_wait(&sh->barrier);
    parallel_radix_partition(a, a->relS, a->numS, sh->totalS, sh->histS, outputS, sh->tmpS, 0, R, num_padding);
    pthread_barrier_wait(&sh->barrier);
    double t1 = now_s();

    if (a->tid == 0) { /* :1174-1222 */
        for (int i = 0; i < fanOut; i++) {
            int32_t ntupR = (int32_t)(outputR[i + 1] - outputR[i] - num_padding);
            int32_t ntupS = (int32_t)(outputS[i + 1] - outputS[i] - num_padding);
            if (ntupR > 0 && ntupS > 0) {
                task_t t;
                t.nR = (uint64_t)ntupR;
                t.relR = sh->tmpR + outputR[i];
                t.tmpR = sh->tmpR2 ? sh->tmpR2 + outputR[i] : NULL;
                t.nS = (uint64_t)ntupS;
                t.relS = sh->tmpS + outputS[i];
                t.tmpS = sh->tmpS2 ? sh->tmpS2 + outputS[i] : NULL;
                ta_push(&sh->part_queue, t);
            }
        }
    }
    pthread_barrier_wait(&sh->barrier);
    task_array *join_queue = passes == 1 ? &sh->part_queue : &sh->join_queue;
    if (passes == 2) {
        task_t task;
        while (ta_pop(&sh->part_queue, &task)) serial_radix_partition(&task, &sh->join_queue, R, D);
    }
    free(outputR);
    free(outputS);
    pthread_barrier_wait(&sh->barrier);
    double t2 = now_s();
    int64_t results = 0;
    task_t task;
    while (ta_pop(join_queue, &task))
        results += (sh->rht ? histogram_join : bucket_chaining_join)(task.relR, task.nR, task.relS, task.nS, bits,
                                                                     sh->materialize ? &a->out : NULL);
    double t3 = now_s();
    a->result = results;
    a->t_total = t3 - t0;
    a->t_part = t2 - t0;
    a->t_pass1 = t1 - t0;
    a->t_pass2 = t2 - t1;
    a->t_join = t3 - t2;
    return NULL;
}

/* join_init_run (:1369-1638) with jf = bucket_chaining_join, i.e. RHO (:1640-1643).
 * With out != NULL the join materialises (config->MATERIALIZE): the per-thread
 * triples are concatenated in thread order into out (up to cap of them). */
static int64_t rho_join_impl(const struct row_t *R, uint64_t nR, const struct row_t *S, uint64_t nS, int nthreads,
                             int force_two_passes, oracle_rho_timing *timing, struct output_triple_t *out,
                             uint64_t cap, int materialize, int rht);

int64_t oracle_rho_join(const struct row_t *R, uint64_t nR, const struct row_t *S, uint64_t nS, int nthreads,
                        int force_two_passes, oracle_rho_timing *timing) {
    return rho_join_impl(R, nR, S, nS, nthreads, force_two_passes, timing, NULL, 0, 0, 0);
}

/* RHT (:1645-1648): join_init_run with histogram_join; out may be NULL (count only). */
int64_t oracle_rht_join(const struct row_t *R, uint64_t nR, const struct row_t *S, uint64_t nS, int nthreads,
                        int force_two_passes, struct output_triple_t *out, uint64_t cap) {
    return rho_join_impl(R, nR, S, nS, nthreads, force_two_passes, NULL, out, cap, out != NULL, 1);
}

int64_t oracle_rho_join_mat(const struct row_t *R, uint64_t nR, const struct row_t *S, uint64_t nS, int nthreads,
                            int force_two_passes, struct output_triple_t *out, uint64_t cap) {
    return rho_join_impl(R, nR, S, nS, nthreads, force_two_passes, NULL, out, cap, 1, 0);
}

static int64_t rho_join_impl(const struct row_t *R, uint64_t nR, const struct row_t *S, uint64_t nS, int nthreads,
                             int force_two_passes, oracle_rho_timing *timing, struct output_triple_t *out,
                             uint64_t cap, int materialize, int rht) {
    if (nthreads < 1) nthreads = 1;
    shared_t sh;
    memset(&sh, 0, sizeof(sh));
    sh.bits = oracle_calc_num_radix_bits(nR, (uint64_t)nthreads);
    sh.passes = force_two_passes ? 2 : oracle_calc_num_passes(sh.bits);
    sh.totalR = nR;
    sh.totalS = nS;
    sh.materialize = materialize;
    sh.rht = rht;
    const uint64_t fan1 = fanout_pass_1(sh.bits, sh.passes);
    const uint64_t rel_padding = (uint64_t)padding_tuples(sh.bits, sh.passes) * fan1 * sizeof(struct row_t);
    const uint64_t rsz = nR * sizeof(struct row_t) + rel_padding;
    const uint64_t ssz = nS * sizeof(struct row_t) + rel_padding;
    sh.tmpR = (struct row_t *)aligned_alloc(CACHE_LINE_SIZE, (rsz + 63) & ~63ull);
    sh.tmpS = (struct row_t *)aligned_alloc(CACHE_LINE_SIZE, (ssz + 63) & ~63ull);
    memset(sh.tmpR, 42, rsz); /* untimed, :1431-1432 */
    memset(sh.tmpS, 42, ssz);
    if (sh.passes == 2) {
        sh.tmpR2 = (struct row_t *)aligned_alloc(CACHE_LINE_SIZE, (rsz + 63) & ~63ull);
        sh.tmpS2 = (struct row_t *)aligned_alloc(CACHE_LINE_SIZE, (ssz + 63) & ~63ull);
        memset(sh.tmpR2, 42, rsz);
        memset(sh.tmpS2, 42, ssz);
    }
    sh.histR = (uint32_t **)calloc(nthreads, sizeof(uint32_t *));
    sh.histS = (uint32_t **)calloc(nthreads, sizeof(uint32_t *));
    sh.part_queue.cap = fan1 * 2;
    sh.part_queue.t = (task_t *)malloc(sizeof(task_t) * sh.part_queue.cap);
    sh.join_queue.cap = 1ull << (sh.bits + 1);
    sh.join_queue.t = (task_t *)malloc(sizeof(task_t) * sh.join_queue.cap);
    atomic_init(&sh.part_queue.push, 0); atomic_init(&sh.part_queue.pop, 0);
    atomic_init(&sh.join_queue.push, 0); atomic_init(&sh.join_queue.pop, 0);
    pthread_barrier_init(&sh.barrier, NULL, (unsigned)nthreads);

    arg_t *args = (arg_t *)calloc(nthreads, sizeof(arg_t));
    pthread_t *tid = (pthread_t *)calloc(nthreads, sizeof(pthread_t));
    const uint64_t perR = nR / nthreads, perS = nS / nthreads; /* :1457-1499 */
    for (int i = 0; i < nthreads; i++) {
        args[i].sh = &sh;
        args[i].tid = i;
        args[i].nthreads = nthreads;
        args[i].relR = R + i * perR;
        args[i].relS = S + i * perS;
        args[i].numR = (i == nthreads - 1) ? nR - i * perR : perR;
        args[i].numS = (i == nthreads - 1) ? nS - i * perS : perS;
    }
    for (int i = nthreads - 1; i >= 1; --i) pthread_create(&tid[i], NULL, prj_thread, &args[i]);
    prj_thread(&args[0]);
    int64_t result = args[0].result;
    for (int i = nthreads - 1; i >= 1; --i) {
        pthread_join(tid[i], NULL);
        result += args[i].result;
    }
    if (timing) {
        memset(timing, 0, sizeof(*timing));
        timing->radix_bits = sh.bits;
        timing->passes = sh.passes;
        timing->join_tasks = atomic_load(&(sh.passes == 1 ? &sh.part_queue : &sh.join_queue)->push);
        for (int i = 0; i < nthreads; i++) { /* max over threads, :1585-1609 */
            if (args[i].t_total > timing->s_total) timing->s_total = args[i].t_total;
            if (args[i].t_part > timing->s_partition) timing->s_partition = args[i].t_part;
            if (args[i].t_pass1 > timing->s_pass1) timing->s_pass1 = args[i].t_pass1;
            if (args[i].t_pass2 > timing->s_pass2) timing->s_pass2 = args[i].t_pass2;
            if (args[i].t_join > timing->s_join) timing->s_join = args[i].t_join;
        }
    }
    uint64_t w = 0;
    for (int i = 0; i < nthreads; i++) { /* concatenate the threads' outputs (:1554-1557) */
        for (uint64_t j = 0; j < args[i].out.n && w < cap; ++j) out[w++] = args[i].out.t[j];
        free(args[i].out.t);
    }
    for (int i = 0; i < nthreads; i++) { free(sh.histR[i]); free(sh.histS[i]); }
    free(sh.histR); free(sh.histS);
    free(sh.tmpR); free(sh.tmpS); free(sh.tmpR2); free(sh.tmpS2);
    free(sh.part_queue.t); free(sh.join_queue.t);
    pthread_barrier_destroy(&sh.barrier);
    free(args);
    free(tid);
    return result;
}

static int cmp_u32(const void *a, const void *b) {
    uint32_t x = *(const uint32_t *)a, y = *(const uint32_t *)b;
    return (x > y) - (x < y);
}

int64_t oracle_count_join_sort(const struct row_t *R, uint64_t nR, const struct row_t *S, uint64_t nS) {
    uint32_t *a = (uint32_t *)malloc(sizeof(uint32_t) * (nR ? nR : 1));
    uint32_t *b = (uint32_t *)malloc(sizeof(uint32_t) * (nS ? nS : 1));
    for (uint64_t i = 0; i < nR; i++) a[i] = R[i].key;
    for (uint64_t i = 0; i < nS; i++) b[i] = S[i].key;
    qsort(a, nR, sizeof(uint32_t), cmp_u32);
    qsort(b, nS, sizeof(uint32_t), cmp_u32);
    int64_t m = 0;
    uint64_t i = 0, j = 0;
    while (i < nR && j < nS) {
        if (a[i] < b[j]) { ++i; continue; }
        if (a[i] > b[j]) { ++j; continue; }
        uint32_t k = a[i];
        uint64_t ci = 0, cj = 0;
        while (i < nR && a[i] == k) { ++i; ++ci; }
        while (j < nS && b[j] == k) { ++j; ++cj; }
        m += (int64_t)(ci * cj);
    }
    free(a);
    free(b);
    return m;
}

void oracle_radix_partition(const struct row_t *in, uint64_t n, int nthreads, uint32_t shift, uint32_t bits,
                            struct row_t *out, uint64_t *bin_start) {
    const uint64_t F = 1ull << bits;
    const uint32_t mask = (uint32_t)(F - 1);
    if (nthreads < 1) nthreads = 1;
    uint64_t *hist = (uint64_t *)calloc((size_t)nthreads * F, sizeof(uint64_t));
    const uint64_t per = n / nthreads;
    for (int t = 0; t < nthreads; t++) {
        uint64_t b = t * per, e = (t == nthreads - 1) ? n : b + per;
        for (uint64_t i = b; i < e; i++) hist[t * F + ((in[i].key >> shift) & mask)]++;
    }
    uint64_t acc = 0;
    for (uint64_t j = 0; j < F; j++) {
        bin_start[j] = acc;
        for (int t = 0; t < nthreads; t++) {
            uint64_t c = hist[t * F + j];
            hist[t * F + j] = acc; /* start of (thread t, bin j): the :901-914 rule without padding */
            acc += c;
        }
    }
    bin_start[F] = acc;
    for (int t = 0; t < nthreads; t++) {
        uint64_t b = t * per, e = (t == nthreads - 1) ? n : b + per;
        for (uint64_t i = b; i < e; i++) out[hist[t * F + ((in[i].key >> shift) & mask)]++] = in[i];
    }
    free(hist);
}
