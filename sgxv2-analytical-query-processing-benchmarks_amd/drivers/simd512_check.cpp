// simd512_check — a reference-style caller of the SIMD512:: scans, compiled against the
// header-only adapter sgxamd/SIMD512_mi355.hpp (the drop-in for
// Scan-Micro-Benchmarks/shared_libraries/SimdScan/include/SIMD512.hpp:39-105) and run on the
// MI355X.  It calls every adapter function the way the reference's drivers and Catch2 tests
// do (multithreadedscan.cpp:48-55,97-106, testsimdscan.cpp), with a 64-byte aligned
// CacheAlignedVector (SIMD512.hpp:20-27), and dumps every result so that
// tests/test_scan_gpu.py can compare them with the oracle.
//
//   simd512_check <dir>
// reads   <dir>/col_u8.bin  (u8 column), index_u64.bin (explicit index vectors),
//         dict8.bin / codes16.bin + dict16.bin / codes32.bin + dict32.bin (dictionary scans),
//         preds.txt (one "lo hi" pair per line: u8 predicates; the dictionary scans use them
//         as value predicates), self_alloc.txt (initial sizes of the self-allocating vector)
// writes  <dir>/out/p<k>_<function>.bin and <dir>/out/results.txt ("key value" lines).
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <new>
#include <string>
#include <vector>

#include "sgxamd/SIMD512_mi355.hpp"

template <typename T>
struct AlignedAllocator {  // SIMD512.hpp:12-25: 64-byte aligned storage
    using value_type = T;
    AlignedAllocator() = default;
    template <typename U>
    AlignedAllocator(const AlignedAllocator<U> &) {}
    T *allocate(size_t n) { return static_cast<T *>(::operator new(n * sizeof(T), std::align_val_t(64))); }
    void deallocate(T *p, size_t) { ::operator delete(p, std::align_val_t(64)); }
    template <typename U>
    bool operator==(const AlignedAllocator<U> &) const { return true; }
    template <typename U>
    bool operator!=(const AlignedAllocator<U> &) const { return false; }
};
template <typename T>
using CacheAlignedVector = std::vector<T, AlignedAllocator<T>>;

template <typename T>
static CacheAlignedVector<T> read_file(const std::string &path) {
    std::ifstream f(path, std::ios::binary | std::ios::ate);
    if (!f) {
        std::fprintf(stderr, "cannot read %s\n", path.c_str());
        std::exit(2);
    }
    const size_t bytes = (size_t)f.tellg();
    CacheAlignedVector<T> v(bytes / sizeof(T));
    f.seekg(0);
    f.read(reinterpret_cast<char *>(v.data()), (std::streamsize)bytes);
    return v;
}

template <typename T>
static void write_file(const std::string &path, const T *p, size_t n) {
    std::ofstream f(path, std::ios::binary);
    f.write(reinterpret_cast<const char *>(p), (std::streamsize)(n * sizeof(T)));
}

int main(int argc, char **argv) {
    if (argc < 2) {
        std::fprintf(stderr, "usage: simd512_check <dir>\n");
        return 2;
    }
    const std::string dir = argv[1], out = dir + "/out/";
    const auto col = read_file<uint8_t>(dir + "/col_u8.bin");
    const auto index = read_file<uint64_t>(dir + "/index_u64.bin");
    const auto dict8 = read_file<int64_t>(dir + "/dict8.bin");
    const auto codes16 = read_file<uint16_t>(dir + "/codes16.bin");
    const auto dict16 = read_file<int64_t>(dir + "/dict16.bin");
    const auto codes32 = read_file<uint32_t>(dir + "/codes32.bin");
    const auto dict32 = read_file<int64_t>(dir + "/dict32.bin");
    std::vector<std::pair<int, int>> preds;
    {
        std::ifstream f(dir + "/preds.txt");
        int lo, hi;
        while (f >> lo >> hi) preds.push_back({lo, hi});
    }
    std::vector<size_t> initial_sizes;
    {
        std::ifstream f(dir + "/self_alloc.txt");
        size_t s;
        while (f >> s) initial_sizes.push_back(s);
    }
    const size_t n = col.size();
    const void *in = col.data();  // the reference passes reinterpret_cast<__m512i *>(data)
    std::FILE *res = std::fopen((out + "results.txt").c_str(), "w");
    for (size_t k = 0; k < preds.size(); ++k) {
        const auto lo = (SIMD512::pred_t)preds[k].first, hi = (SIMD512::pred_t)preds[k].second;
        const std::string p = out + "p" + std::to_string(k) + "_";
        std::fprintf(res, "p%zu_count %zu\n", k, SIMD512::count(lo, hi, in, n));
        std::fprintf(res, "p%zu_sum %zu\n", k, SIMD512::sum(lo, hi, in, n));

        CacheAlignedVector<uint64_t> bv(n / 64);  // __mmask64 per 64 rows
        SIMD512::bitvector_scan(lo, hi, in, n, bv.data());
        write_file(p + "bitvector.bin", bv.data(), bv.size());

        CacheAlignedVector<size_t> ix(n);  // the caller sizes it (multithreadedscan.cpp:97-106)
        SIMD512::implicit_index_scan(lo, hi, in, n, ix.data());
        write_file(p + "implicit.bin", ix.data(), ix.size());

        CacheAlignedVector<size_t> ex(n);
        SIMD512::explicit_index_scan(lo, hi, index.data(), in, n, ex.data());
        write_file(p + "explicit.bin", ex.data(), ex.size());

        CacheAlignedVector<uint32_t> vals(n);
        const size_t nv = SIMD512::scan(lo, hi, in, n, vals.data());
        std::fprintf(res, "p%zu_scan %zu\n", k, nv);
        write_file(p + "scan.bin", vals.data(), nv);

        for (size_t j = 0; j < initial_sizes.size(); ++j) {
            for (int cut = 0; cut < 2; ++cut) {
                CacheAlignedVector<size_t> sa(initial_sizes[j], 7);
                SIMD512::implicit_index_scan_self_alloc(lo, hi, in, n, sa, cut != 0);
                std::fprintf(res, "p%zu_self_alloc_%zu_%d %zu\n", k, j, cut, sa.size());
                if (cut) write_file(p + "self_alloc_" + std::to_string(j) + ".bin", sa.data(), sa.size());
            }
        }

        CacheAlignedVector<int64_t> d8, d16, d32;
        SIMD512::dict_scan_8bit_64bit(preds[k].first, preds[k].second, dict8.data(), in, n, d8, true);
        SIMD512::dict_scan_16bit_64bit(preds[k].first, preds[k].second, dict16.data(), codes16.data(),
                                       codes16.size(), d16);
        SIMD512::dict_scan_32bit_64bit(preds[k].first, preds[k].second, dict32.data(), dict32.size(),
                                       codes32.data(), codes32.size(), d32);
        write_file(p + "dict8.bin", d8.data(), d8.size());
        write_file(p + "dict16.bin", d16.data(), d16.size());
        write_file(p + "dict32.bin", d32.data(), d32.size());
    }
    std::fclose(res);
    std::printf("simd512_check: %zu predicates over %zu rows done\n", preds.size(), n);
    return 0;
}
