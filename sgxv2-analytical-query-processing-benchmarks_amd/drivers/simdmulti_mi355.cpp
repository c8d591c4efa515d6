// simdmulti_mi355 — the reference's SimdScanMulti driver
// (Scan-Micro-Benchmarks/microbenchmarks/SimdScanMulti/App/App.cpp) on the MI355X: the same
// gflags-style flags (App/flags.hpp:8-40), the same configuration spectrum (types.hpp:140-190:
// modes x threads x entries x selectivities), the same predicate mapping
// (types.hpp:125,134: lo = 0, hi = (uint8_t)round(sel / 100 * 255)), the same uint8 column
// (Allocator.hpp:94-110: data[i] = i % 256, max_entries * reruns of it) and the same CSV rows
// (PerfEventBlock: the BenchmarkParameters in alphabetical order, then timeMicroSec and
// cpuCycles), so results/plot.py:20-24,73-74 reads the output unchanged.
//
// What maps how:
//   * the column lives in HBM (generated there, mi355_gen_scan_u8_dev); every scan is one
//     device-wide call of the C-ABI (sgxamd/scan.h) over the rerun's `entries` rows.  The
//     reference splits a rerun into numThreads contiguous slices (multithreadedscan.cpp:227-236)
//     because one CPU core cannot saturate memory; the GPU parallelises inside the call, so
//     numThreads is kept as a configuration axis (and CSV column) but does not split the call.
//   * cpuCycles = the host-clock time of the num_runs timed calls of every rerun (the
//     reference's rdtscpWrapper around the same loop, multithreadedscan.cpp:50-55, 97-106),
//     converted at the reference build's 2.9 GHz (plot.py:10); deviceMicroSec = the same
//     calls' kernel time from HIP events; timeMicroSec = the whole block's wall time.
//   * modes: bitvector -> mi355_scan_bitvector_u8; noIndex -> mi355_scan_index_u8 (the
//     self-allocating index scan with pre_alloc'd output, ResultAllocators.hpp:7-18); scalar
//     (ScalarScan.hpp:8-18, the same output) -> the same GPU index scan; dict ->
//     mi355_dict_scan_8bit_64bit over a 256-entry dictionary dict[i] = i (Allocator.hpp:111-115).
//   * --enclave / --preload / --numa: there is no enclave and no NUMA on the device; only "f"
//     is accepted.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "sgxamd/generator.h"
#include "sgxamd/rho.h"
#include "sgxamd/scan.h"

namespace {

struct Flags {
    std::string enclave = "f", preload = "f", mode = "noIndex,bitvector", unique_data = "t", numa = "f";
    uint64_t num_reruns = 0, num_warmup_runs = 0, num_runs = 1, min_threads = 1, max_threads = 1;
    uint64_t min_entries = 1 << 12, max_entries = 1 << 26, min_entries_exp = 0, max_entries_exp = 0;
    uint64_t max_selectivity = 10, min_selectivity = 10, step_selectivity = 1;
    bool join = false, debug = false, pre_alloc = true;
};

[[noreturn]] void die(const std::string &msg) {
    std::fprintf(stderr, "simdmulti_mi355: %s\n", msg.c_str());
    std::exit(1);
}

bool parse_bool(const std::string &v) { return v == "1" || v == "t" || v == "true" || v == "yes"; }

// gflags syntax: --name=value, --name value, --flag / --noflag for booleans
Flags parse(int argc, char **argv) {
    Flags f;
    std::map<std::string, std::string *> strs{{"enclave", &f.enclave},     {"preload", &f.preload},
                                               {"mode", &f.mode},           {"unique_data", &f.unique_data},
                                               {"numa", &f.numa}};
    std::map<std::string, uint64_t *> nums{
        {"num_reruns", &f.num_reruns},           {"num_warmup_runs", &f.num_warmup_runs},
        {"num_runs", &f.num_runs},               {"min_threads", &f.min_threads},
        {"max_threads", &f.max_threads},         {"min_entries", &f.min_entries},
        {"max_entries", &f.max_entries},         {"min_entries_exp", &f.min_entries_exp},
        {"max_entries_exp", &f.max_entries_exp}, {"max_selectivity", &f.max_selectivity},
        {"min_selectivity", &f.min_selectivity}, {"step_selectivity", &f.step_selectivity}};
    std::map<std::string, bool *> bools{{"join", &f.join}, {"debug", &f.debug}, {"pre_alloc", &f.pre_alloc}};
    for (int i = 1; i < argc; ++i) {
        std::string a = argv[i];
        if (a == "--help" || a == "-h") {
            std::printf("simdmulti_mi355 --mode=noIndex,bitvector,dict,scalar --min_entries_exp=N --max_entries_exp=N\n"
                        "  --min_selectivity=S --max_selectivity=S --step_selectivity=S --num_runs=K --num_reruns=R\n"
                        "  --num_warmup_runs=W --unique_data=t|f|b --min_threads=T --max_threads=T [--debug]\n");
            std::exit(0);
        }
        if (a.rfind("--", 0) != 0) die("unexpected argument " + a);
        a = a.substr(2);
        std::string name = a, val;
        const size_t eq = a.find('=');
        bool has_val = eq != std::string::npos;
        if (has_val) {
            name = a.substr(0, eq);
            val = a.substr(eq + 1);
        }
        if (bools.count(name)) {
            *bools[name] = has_val ? parse_bool(val) : true;
            continue;
        }
        if (name.rfind("no", 0) == 0 && bools.count(name.substr(2)) && !has_val) {
            *bools[name.substr(2)] = false;
            continue;
        }
        if (!has_val) {
            if (i + 1 >= argc) die("--" + name + " needs a value");
            val = argv[++i];
        }
        if (strs.count(name)) *strs[name] = val;
        else if (nums.count(name)) *nums[name] = std::strtoull(val.c_str(), nullptr, 10);
        else die("unknown flag --" + name);
    }
    if (f.min_entries % 64 != 0) die("--min_entries must be a multiple of 64 (flags.hpp ValidateNumEntries)");
    for (auto *t : {&f.enclave, &f.preload, &f.numa})
        if (*t != "f") die("--enclave / --preload / --numa: only 'f' exists on the MI355X (no enclave, no NUMA)");
    return f;
}

enum class Mode { bitvector = 0, noIndex = 1, dict = 2, scalar = 3 };
const char *kModeNames[] = {"bitvector", "noindex", "dict", "scalar"};  // types.hpp:19

std::vector<Mode> parse_modes(const std::string &v) {  // flags.hpp parse_modes
    std::vector<Mode> out;
    size_t start = 0;
    while (start <= v.size()) {
        size_t c = v.find(',', start);
        if (c == std::string::npos) c = v.size();
        const std::string s = v.substr(start, c - start);
        if (s == "noIndex") out.push_back(Mode::noIndex);
        else if (s == "bitvector") out.push_back(Mode::bitvector);
        else if (s == "dict") out.push_back(Mode::dict);
        else if (s == "scalar") out.push_back(Mode::scalar);
        else die("Illegal value for --mode: " + s);
        start = c + 1;
    }
    return out;
}

std::vector<bool> trinary(const std::string &v) {  // types.cpp convert_trinary
    if (v == "t") return {true};
    if (v == "f") return {false};
    if (v == "b") return {false, true};
    die("trinary flag must be t, f or b");
}

std::vector<uint64_t> span(uint64_t lo, uint64_t hi, uint64_t step, bool exp) {  // ParameterSpan::to_vector
    if (hi < lo) die("Max must be bigger than min!");
    if (step == 0) die("Step must be > 0!");
    std::vector<uint64_t> v;
    for (uint64_t x = lo; x <= hi; x = exp ? x << step : x + step) {
        v.push_back(x);
        if (exp && x == 0) break;
    }
    return v;
}

#define HIPCHECK(c)                                                                  \
    do {                                                                             \
        hipError_t e_ = (c);                                                         \
        if (e_ != hipSuccess) die(std::string(#c) + ": " + hipGetErrorString(e_)); \
    } while (0)

void check(int rc, const char *what) {
    if (rc != MI355_OK) die(std::string(what) + " failed: " + mi355_last_error());
}

double device_ms_of_last_call() {
    const char *names[64];
    double ms[64];
    const int n = mi355_timing_get(names, ms, 64);
    double t = 0;
    for (int i = 0; i < n && i < 64; ++i) t += ms[i];
    return t;
}

}  // namespace

int main(int argc, char **argv) {
    const Flags F = parse(argc, argv);
    const auto modes = parse_modes(F.mode);
    const uint64_t emin = F.min_entries_exp ? (1ull << F.min_entries_exp) : F.min_entries;
    const uint64_t emax = F.max_entries_exp ? (1ull << F.max_entries_exp) : F.max_entries;
    const auto entries = span(emin, emax, 1, true);
    const auto threads = span(F.min_threads, F.max_threads, 1, true);
    if ((F.max_selectivity - F.min_selectivity) % F.step_selectivity != 0) die("Min + n * step does not reach max!");
    const auto sels = span(F.min_selectivity, F.max_selectivity, F.step_selectivity, false);
    if (F.join) die("--join (merging per-thread index lists) has no per-thread lists on the MI355X");
    if (mi355_device_count() == 0) die("no gfx950 device visible");

    // the column: max_entries * reruns of i % 256 (App.cpp: num_total_entries), in HBM
    const uint64_t total = emax * (F.num_reruns > 0 ? F.num_reruns : 1);
    uint8_t *data = nullptr;
    HIPCHECK(hipMalloc(&data, total));
    check(mi355_gen_scan_u8_dev(data, total, 0, 0, nullptr), "gen_scan_u8_dev");
    int64_t *dict = nullptr;
    {
        std::vector<int64_t> h(256);
        for (int i = 0; i < 256; ++i) h[i] = i;
        HIPCHECK(hipMalloc(&dict, 256 * sizeof(int64_t)));
        HIPCHECK(hipMemcpy(dict, h.data(), 256 * sizeof(int64_t), hipMemcpyHostToDevice));
    }
    // pre-allocated outputs for the largest rerun (ResultAllocators.hpp:7-18 pre_alloc_per_thread)
    void *out = nullptr;
    HIPCHECK(hipMalloc(&out, emax * sizeof(uint64_t)));
    mi355_timing_enable(1);

    const std::vector<std::string> cols = {"dataLoading", "datasizeKiB", "enclaveMode", "entries",
                                           "numRuns",     "numThreads",  "numa",        "reruns",
                                           "selectivity", "unique",      "warmup",      "writeMode",
                                           "timeMicroSec", "cpuCycles",  "deviceMicroSec", "matches",
                                           "inputGiBps",  "scale"};
    bool header = true;
    for (Mode mode : modes)
        for (bool unique : trinary(F.unique_data))
            for (uint64_t nthreads : threads)
                for (uint64_t ent : entries)
                    for (uint64_t sel : sels) {
                        const uint64_t reruns = F.num_reruns == 0 ? emax / ent : F.num_reruns;
                        const uint64_t warm = unique ? 0 : F.num_warmup_runs;
                        const uint64_t runs = unique ? 1 : F.num_runs;
                        const uint8_t lo = 0;
                        const uint8_t hi = (uint8_t)std::round((double)sel / 100.0 * 255.0);  // types.hpp:125,134
                        if (ent * reruns > total) die("entries * reruns exceed the allocated column");
                        const auto t0 = std::chrono::steady_clock::now();
                        double host_us = 0, dev_us = 0;
                        uint64_t matches = 0;
                        for (uint64_t r = 0; r < reruns; ++r) {
                            const uint8_t *col = data + ent * r;  // scan_wrapper's run_offset
                            auto one = [&]() {
                                uint64_t k = 0;
                                switch (mode) {
                                    case Mode::bitvector:
                                        check(mi355_scan_bitvector_u8(lo, hi, col, ent, (uint64_t *)out),
                                              "bitvector_scan");
                                        break;
                                    case Mode::noIndex:
                                    case Mode::scalar:
                                        check(mi355_scan_index_u8(lo, hi, col, ent, (uint64_t *)out, ent, &k),
                                              "implicit_index_scan_self_alloc");
                                        break;
                                    case Mode::dict:
                                        check(mi355_dict_scan_8bit_64bit(lo, hi, dict, col, ent, (int64_t *)out, ent,
                                                                         &k),
                                              "dict_scan_8bit_64bit");
                                        break;
                                }
                                return k;
                            };
                            for (uint64_t w = 0; w < warm; ++w) one();
                            const auto a = std::chrono::steady_clock::now();
                            for (uint64_t k = 0; k < runs; ++k) {
                                matches = one();
                                dev_us += device_ms_of_last_call() * 1000.0;
                            }
                            host_us += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - a)
                                           .count();
                        }
                        if (mode == Mode::bitvector)  // the bitvector call returns no count (untimed)
                            check(mi355_scan_count_u8(lo, hi, data + ent * (reruns - 1), ent, &matches), "count");
                        const double wall_us =
                            std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
                        const uint64_t cycles = (uint64_t)(host_us * 2900.0);  // plot.py:10, 2.9 GHz
                        const double gibps = dev_us > 0 ? (double)ent * runs * reruns / (dev_us * 1e-6) / (1ull << 30)
                                                        : 0.0;
                        char sel_s[32], t_s[32], d_s[32], g_s[32];
                        std::snprintf(sel_s, sizeof sel_s, "%f", sel / 100.0);
                        std::snprintf(t_s, sizeof t_s, "%f", wall_us);
                        std::snprintf(d_s, sizeof d_s, "%f", dev_us);
                        std::snprintf(g_s, sizeof g_s, "%f", gibps);
                        const std::vector<std::string> vals = {
                            "noPreload", std::to_string(ent / 1024), "native", std::to_string(ent),
                            std::to_string(runs), std::to_string(nthreads), "no", std::to_string(reruns), sel_s,
                            std::to_string(unique ? 1 : 0), std::to_string(warm), kModeNames[(int)mode], t_s,
                            std::to_string(cycles), d_s, std::to_string(matches), g_s,
                            std::to_string(ent * reruns * runs)};
                        // PerfEventBlock's layout: ", "-separated, each column right-aligned to its width
                        std::string hl, vl;
                        for (size_t c = 0; c < cols.size(); ++c) {
                            const size_t w = std::max(cols[c].size(), vals[c].size());
                            char buf[128];
                            std::snprintf(buf, sizeof buf, "%*s%s", (int)w, cols[c].c_str(), c + 1 < cols.size() ? ", " : "");
                            hl += buf;
                            std::snprintf(buf, sizeof buf, "%*s%s", (int)w, vals[c].c_str(), c + 1 < cols.size() ? ", " : "");
                            vl += buf;
                        }
                        if (header) std::printf("%s\n", hl.c_str());
                        std::printf("%s\n", vl.c_str());
                        std::fflush(stdout);
                        header = false;
                        if (F.debug)
                            std::fprintf(stderr, "mode=%s entries=%lu sel=%lu [%u, %u] matches=%lu\n",
                                         kModeNames[(int)mode], (unsigned long)ent, (unsigned long)sel, lo, hi,
                                         (unsigned long)matches);
                    }
    (void)hipFree(data);
    (void)hipFree(dict);
    (void)hipFree(out);
    return 0;
}
