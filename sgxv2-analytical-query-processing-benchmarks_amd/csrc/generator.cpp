// Host-side relation and scan-column generators.
//
// Restates Join-Benchmarks/lib/AppUtilities/src/generator.cpp and genzipf.cpp so
// that relations are bit-identical to the ones the reference's native driver
// builds (App/TEEBench/native.cpp:62-101).  Keys come from glibc's rand(), which
// the reference calls through RAND_RANGE (generator.cpp:19).  glibc is a
// third-party dependency not vendored in the reference; its published TYPE_3
// additive-feedback algorithm (random_r.c: degree 31, separation 3, state
// seeded by the 16807 LCG, 310 outputs discarded) is restated below and
// checked against the system libc's rand() in tests/test_generator.py.
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <memory>
#include <random>
#include <thread>
#include <vector>

#include "sgxamd/generator.h"

namespace {

// glibc random_r.c TYPE_3 state: r[i] = r[i-31] + r[i-3] (mod 2^32), output r >> 1.
struct GlibcRand {
    int32_t state[31];
    int f = 3;  // fptr = &state[SEP_3]
    int r = 0;  // rptr = &state[0]

    void seed(unsigned int s) {
        int32_t word = static_cast<int32_t>(s == 0 ? 1u : s);  // srandom_r: seed 0 -> 1
        state[0] = word;
        for (int i = 1; i < 31; ++i) {
            // Schrage's method for 16807 * word mod (2^31 - 1), as in srandom_r.
            long hi = word / 127773;
            long lo = word % 127773;
            long w = 16807 * lo - 2836 * hi;
            if (w < 0) w += 2147483647;
            word = static_cast<int32_t>(w);
            state[i] = word;
        }
        f = 3;
        r = 0;
        for (int k = 0; k < 310; ++k) next();  // kc = 10 * rand_deg discards
    }

    inline int32_t next() {
        uint32_t val = static_cast<uint32_t>(state[f]) + static_cast<uint32_t>(state[r]);
        state[f] = static_cast<int32_t>(val);
        f = (f == 30) ? 0 : f + 1;
        r = (r == 30) ? 0 : r + 1;
        return static_cast<int32_t>(val >> 1);
    }
};

GlibcRand g_rand;
bool g_seeded = false;

inline void check_seed() {
    // generator.cpp:83-91 seeds from time(NULL) when unseeded; a library must be
    // reproducible, so an unseeded generator behaves as glibc's default seed 1.
    if (!g_seeded) {
        g_rand.seed(1);
        g_seeded = true;
    }
}

// RAND_RANGE(N) = (double)rand() / ((double)RAND_MAX + 1) * (N)   (generator.cpp:19)
inline double rand_range(double n) {
    return static_cast<double>(g_rand.next()) / (2147483647.0 + 1.0) * n;
}

// knuth_shuffle (generator.cpp:100-109): i = n-1 .. 1, j = RAND_RANGE(i), swap keys.
// The random stream does not depend on the data, so indexes are drawn a few
// steps ahead and their tuples prefetched; the swap order is unchanged.
void knuth_shuffle(row_t *t, uint64_t n) {
    if (n < 2) return;
    constexpr int LA = 32;
    int64_t ring[LA];
    uint64_t next_i = n - 1;  // next i whose j is drawn
    int head = 0, filled = 0;
    auto draw = [&]() {
        int64_t j = static_cast<int64_t>(rand_range(static_cast<double>(next_i)));
        __builtin_prefetch(&t[j], 1, 0);
        ring[(head + filled) % LA] = j;
        ++filled;
        --next_i;
    };
    while (filled < LA && next_i > 0) draw();
    for (uint64_t i = n - 1; i > 0; --i) {
        int64_t j = ring[head];
        head = (head + 1) % LA;
        --filled;
        if (next_i > 0) draw();
        type_key tmp = t[i].key;
        t[i].key = t[j].key;
        t[j].key = tmp;
    }
}

// random_unique_gen (generator.cpp:143-153): keys 1..n then shuffle.
void random_unique_gen(row_t *t, uint64_t n, uint64_t payload_base) {
    for (uint64_t i = 0; i < n; ++i) {
        t[i].key = static_cast<type_key>(i + 1);
        t[i].payload = static_cast<type_value>(payload_base + i);
    }
    knuth_shuffle(t, n);
}

// random_unique_gen_maxid (generator.cpp:156-169): integer jump = maxid / n.
void random_unique_gen_maxid(row_t *t, uint64_t n, uint32_t maxid, uint64_t payload_base) {
    double jump = static_cast<double>(maxid / n);
    double id = maxid == 0 ? 0 : 1;
    for (uint32_t i = 0; i < n; ++i) {
        t[i].key = static_cast<uint32_t>(id);
        t[i].payload = static_cast<type_value>(payload_base + i);
        id += jump;
    }
    knuth_shuffle(t, n);
}

}  // namespace

extern "C" {

void mi355_gen_seed(unsigned int seed) {  // seed_generator, generator.cpp:75-80
    g_rand.seed(seed);
    g_seeded = true;
}

int mi355_gen_rand(void) {
    check_seed();
    return g_rand.next();
}

int mi355_gen_pk(row_t *out, uint64_t n) {  // create_relation_pk, generator.cpp:352-377
    if (!out && n) return -1;
    check_seed();
    random_unique_gen(out, n, 0);
    return 0;
}

int mi355_gen_fk(row_t *out, uint64_t n, int64_t maxid) {  // create_relation_fk, :474-512
    if ((!out && n) || maxid <= 0) return -1;
    check_seed();
    const uint64_t m = static_cast<uint64_t>(maxid);
    const uint64_t iters = n / m;
    for (uint64_t i = 0; i < iters; ++i) random_unique_gen(out + m * i, m, m * i);
    const uint64_t rem = n % m;
    if (rem > 0) random_unique_gen(out + m * iters, rem, m * iters);
    return 0;
}

int mi355_gen_fk_sel(row_t *out, uint64_t n, int64_t maxid) {  // create_relation_fk_sel, :515-553
    if (!out && n) return -1;
    check_seed();
    const uint64_t m = static_cast<uint64_t>(maxid);
    const uint64_t iters = maxid != 0 ? n / m : 0;
    const uint32_t maxid32 = static_cast<uint32_t>(maxid);  // random_unique_gen_maxid takes uint32_t
    for (uint64_t i = 0; i < iters; ++i) random_unique_gen_maxid(out + m * i, m, maxid32, m * i);
    const uint64_t rem = maxid != 0 ? n % m : n;
    if (rem > 0) random_unique_gen_maxid(out + m * iters, rem, maxid32, m * iters);
    return 0;
}

// gen_zipf (genzipf.cpp:87-144) with gen_alphabet (:34-49) and gen_zipf_lut (:57-81).
//
// The two mt19937_64 streams (the alphabet shuffle and the uniform draws) are
// sequential by nature and independent of each other, so they run on two threads
// while the others compute the LUT terms.  The reference's bisection (:118-136)
// returns the smallest index whose LUT entry is >= r (lower bound).  A guide table
// g[b] = lower_bound(b / K) for K = 2^k buckets brackets every search:
// b = floor(r * K) is exact in double arithmetic (K is a power of two), and
// g[b] <= lower_bound(r) <= g[b + 1] because b/K <= r < (b+1)/K, so the bracketed
// search returns exactly the reference's position with a few cache-resident steps
// instead of ~28 dependent misses over a 2 GiB LUT (BASELINE config 5: 96 s -> ~8 s).
int mi355_gen_zipf(row_t *out, uint64_t n, uint32_t alphabet_size, double theta, uint64_t seed,
                   int nthreads) {
    if ((!out && n) || alphabet_size == 0) return -1;
    if (nthreads < 1) nthreads = 1;

    // uninitialised buffers: value-initialising 3 GiB costs seconds at config 5
    std::unique_ptr<uint32_t[]> alphabet(new uint32_t[alphabet_size]);
    std::unique_ptr<double[]> rs(new double[n]);
    std::thread shuffler([&]() {
        for (uint32_t i = 0; i < alphabet_size; ++i) alphabet[i] = i + 1;  // no 0 in the alphabet
        std::mt19937_64 gen{seed};
        std::shuffle(alphabet.get(), alphabet.get() + alphabet_size, gen);
    });
    std::thread drawer([&]() {
        std::mt19937_64 gen{seed};
        std::uniform_real_distribution<double> dist{0.0, 1.0};
        for (uint64_t i = 0; i < n; ++i) rs[i] = dist(gen);
    });

    auto parallel_for = [nthreads](uint64_t total, auto &&fn) {
        if (nthreads == 1 || total < 4096) {
            fn(uint64_t{0}, total);
            return;
        }
        std::vector<std::thread> th;
        const uint64_t chunk = (total + nthreads - 1) / nthreads;
        for (int t = 0; t < nthreads; ++t) {
            const uint64_t b = t * chunk, e = std::min<uint64_t>(total, b + chunk);
            if (b < e) th.emplace_back(fn, b, e);
        }
        for (auto &x : th) x.join();
    };

    // lut[i-1] = (sum_{k<=i} 1/k^theta) / (sum_{k<=N} 1/k^theta): the terms are
    // computed in parallel, both sums stay sequential (bit-exact with the reference).
    std::unique_ptr<double[]> lut(new double[alphabet_size]);
    parallel_for(alphabet_size, [&](uint64_t b, uint64_t e) {
        for (uint64_t i = b; i < e; ++i) lut[i] = 1.0 / pow(static_cast<unsigned int>(i + 1), theta);
    });
    double scaling = 0.0;
    for (uint32_t i = 0; i < alphabet_size; ++i) scaling += lut[i];
    double sum = 0.0;
    for (uint32_t i = 0; i < alphabet_size; ++i) {
        sum += lut[i];
        lut[i] = sum / scaling;
    }

    const double *L = lut.get();
    const uint32_t last = alphabet_size - 1;
    // the reference's position for r: 0 if lut[0] >= r, else the bisection's `right`
    // (never past `last`, even if rounding left lut[last] below r)
    auto lower = [L, last](double r, uint32_t lo, uint32_t hi) -> uint32_t {
        while (lo < hi) {  // smallest i in [lo, hi] with L[i] >= r, hi if none
            const uint32_t m = lo + (hi - lo) / 2;
            if (L[m] < r) lo = m + 1; else hi = m;
        }
        return std::min(lo, last);
    };
    constexpr int kGuideBits = 22;
    constexpr uint32_t K = 1u << kGuideBits;
    std::vector<uint32_t> guide(K + 1);
    parallel_for(K, [&](uint64_t b, uint64_t e) {
        for (uint64_t i = b; i < e; ++i) guide[i] = lower(std::ldexp(static_cast<double>(i), -kGuideBits), 0, last);
    });
    guide[K] = last;

    shuffler.join();
    drawer.join();
    // searches run 16 at a time in lock step, so their cache misses overlap
    constexpr int kLanes = 16;
    parallel_for(n, [&](uint64_t b, uint64_t e) {
        for (uint64_t i = b; i < e; i += kLanes) {
            const int cnt = static_cast<int>(std::min<uint64_t>(kLanes, e - i));
            double r[kLanes];
            uint32_t lo[kLanes], hi[kLanes];
            for (int j = 0; j < cnt; ++j) {
                r[j] = rs[i + j];
                const uint32_t g = static_cast<uint32_t>(std::ldexp(r[j], kGuideBits));  // floor(r * K)
                lo[j] = guide[g];
                hi[j] = guide[g + 1];
            }
            for (bool active = true; active;) {
                active = false;
                for (int j = 0; j < cnt; ++j) {
                    if (lo[j] < hi[j]) {
                        const uint32_t m = lo[j] + (hi[j] - lo[j]) / 2;
                        if (L[m] < r[j]) lo[j] = m + 1; else hi[j] = m;
                        active = true;
                    }
                }
            }
            for (int j = 0; j < cnt; ++j) {
                out[i + j].key = alphabet[std::min(lo[j], last)];
                out[i + j].payload = static_cast<type_value>(i + j);
            }
        }
    });
    return 0;
}

int mi355_gen_scan_u8(uint8_t *out, size_t n) {  // Allocator.hpp:94-110 (uint8: i % 256)
    if (!out && n) return -1;
    for (size_t i = 0; i < n; ++i) out[i] = static_cast<uint8_t>(i & 255);
    return 0;
}

int mi355_gen_scan_i32(int32_t *out, size_t n) {
    if (!out && n) return -1;
    for (size_t i = 0; i < n; ++i) out[i] = static_cast<int32_t>(i & 255);
    return 0;
}

}  // extern "C"
