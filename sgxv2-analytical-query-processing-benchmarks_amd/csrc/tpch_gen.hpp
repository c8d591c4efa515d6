// Synthetic TPC-H column values, one pure function per column of (seed, row):
// the host generator (tpch_io.cpp) and the device generator (tpch_kernels.hip)
// call the same functions, so both produce identical tables.
//
// Distributions follow the TPC-H specification (v3, clause 4.2.3) for the
// columns the reference's queries read (TpcHTypes.hpp:53-87); values are encoded
// the way the reference's CSV loader encodes dbgen text (TpcHCommons.cpp:141-183,
// 347-353, 625-665): unmatched strings become 0, and "REG AIR" — which the
// loader looks for as "AIR REG" — becomes 0 too.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace sgxamd {
namespace tpch {

constexpr uint64_t kDay = 86400;
constexpr uint32_t kStartDay = 8035;     // 1992-01-01, days since 1970-01-01
constexpr uint32_t kEndDay = 10591;      // 1998-12-31
constexpr uint32_t kCurrentDay = 9298;   // 1995-06-17 (returnflag cut-off)
constexpr uint32_t kOrderDayHi = kEndDay - 151;

// rows per unit of scale_milli (SF1 = 1000)
constexpr uint64_t kCustPerMilli = 150, kOrdPerMilli = 1500, kPartPerMilli = 200;
constexpr uint64_t kNations = 25;

enum Col : uint32_t {
    kCMkt = 1, kCNation, kPBrand, kPSize, kPContainer, kOCust, kODate, kLCount, kLPart, kLQty,
    kLShip, kLCommit, kLReceipt, kLFlag, kLInstruct, kLMode
};

__host__ __device__ inline uint64_t mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
__host__ __device__ inline uint64_t draw(uint64_t seed, uint32_t col, uint64_t row) {
    return mix64(seed ^ mix64(((uint64_t)col << 56) ^ row));
}
// uniform integer in [lo, hi]
__host__ __device__ inline uint64_t uni(uint64_t seed, uint32_t col, uint64_t row, uint64_t lo, uint64_t hi) {
    return lo + draw(seed, col, row) % (hi - lo + 1);
}

__host__ __device__ inline uint64_t n_customer(uint32_t sm) { return kCustPerMilli * sm; }
__host__ __device__ inline uint64_t n_orders(uint32_t sm) { return kOrdPerMilli * sm; }
__host__ __device__ inline uint64_t n_part(uint32_t sm) { return kPartPerMilli * sm; }

// ---- customer (clause 4.2.3: C_MKTSEGMENT random of 5, C_NATIONKEY random [0, 24])
__host__ __device__ inline uint8_t c_mktsegment(uint64_t seed, uint64_t i) {
    // AUTOMOBILE, BUILDING, FURNITURE, MACHINERY, HOUSEHOLD
    return uni(seed, kCMkt, i, 0, 4) == 1 ? 1 : 0;
}
__host__ __device__ inline uint32_t c_nationkey(uint64_t seed, uint64_t i) {
    return (uint32_t)uni(seed, kCNation, i, 0, kNations - 1);
}

// ---- part (P_BRAND = Brand#MN, M,N in [1,5]; P_SIZE in [1,50]; P_CONTAINER = S1 S2)
__host__ __device__ inline uint8_t p_brand(uint64_t seed, uint64_t i) {
    const uint64_t mn = uni(seed, kPBrand, i, 0, 24);  // M = mn / 5 + 1, N = mn % 5 + 1
    const uint32_t code = (uint32_t)((mn / 5 + 1) * 10 + (mn % 5 + 1));
    return code == 12 ? 1 : code == 23 ? 2 : code == 34 ? 3 : 0;
}
__host__ __device__ inline uint32_t p_size(uint64_t seed, uint64_t i) { return (uint32_t)uni(seed, kPSize, i, 1, 50); }
__host__ __device__ inline uint8_t p_container(uint64_t seed, uint64_t i) {
    // S1 in {SM, LG, MED, JUMBO, WRAP}, S2 in {CASE, BOX, BAG, JAR, PKG, PACK, CAN, DRUM}
    const uint32_t v = (uint32_t)uni(seed, kPContainer, i, 0, 39);
    const uint32_t s1 = v / 8, s2 = v % 8;
    // reference codes (TpcHTypes.hpp:27-38): SM CASE..PKG 1-4, MED BAG/BOX/PKG/PACK 5-8, LG CASE/BOX/PACK/PKG 9-12
    if (s1 == 0) return s2 == 0 ? 1 : s2 == 1 ? 2 : s2 == 5 ? 3 : s2 == 4 ? 4 : 0;
    if (s1 == 2) return s2 == 2 ? 5 : s2 == 1 ? 6 : s2 == 4 ? 7 : s2 == 5 ? 8 : 0;
    if (s1 == 1) return s2 == 0 ? 9 : s2 == 1 ? 10 : s2 == 5 ? 11 : s2 == 4 ? 12 : 0;
    return 0;
}

// ---- orders (sparse O_ORDERKEY: 8 of every 32 keys; O_CUSTKEY never a multiple of 3;
//      O_ORDERDATE uniform in [STARTDATE, ENDDATE - 151 days])
__host__ __device__ inline uint32_t o_orderkey(uint64_t i) { return (uint32_t)((i / 8) * 32 + (i % 8) + 1); }
__host__ __device__ inline uint32_t o_custkey(uint64_t seed, uint64_t i, uint64_t ncust) {
    const uint64_t eligible = ncust - ncust / 3;
    const uint64_t r = uni(seed, kOCust, i, 0, eligible - 1);
    return (uint32_t)((r / 2) * 3 + (r % 2) + 1);
}
__host__ __device__ inline uint32_t o_orderday(uint64_t seed, uint64_t i) {
    return (uint32_t)uni(seed, kODate, i, kStartDay, kOrderDayHi);
}
// lineitems of order i: uniform [1, 7]
__host__ __device__ inline uint32_t o_lines(uint64_t seed, uint64_t i) { return (uint32_t)uni(seed, kLCount, i, 1, 7); }

// ---- lineitem row r belonging to order o (clause 4.2.3 date rules)
struct Line {
    uint64_t shipdate, commitdate, receiptdate;
    uint32_t partkey;
    float quantity;
    uint8_t shipmode, shipinstruct;
    char returnflag;
};
__host__ __device__ inline Line make_line(uint64_t seed, uint64_t r, uint32_t orderday, uint64_t npart) {
    Line L;
    const uint32_t ship = orderday + (uint32_t)uni(seed, kLShip, r, 1, 121);
    const uint32_t commit = orderday + (uint32_t)uni(seed, kLCommit, r, 30, 90);
    const uint32_t receipt = ship + (uint32_t)uni(seed, kLReceipt, r, 1, 30);
    L.shipdate = ship * kDay;
    L.commitdate = commit * kDay;
    L.receiptdate = receipt * kDay;
    L.partkey = (uint32_t)uni(seed, kLPart, r, 1, npart);
    L.quantity = (float)uni(seed, kLQty, r, 1, 50);
    // REG AIR, AIR, RAIL, SHIP, TRUCK, MAIL, FOB -> reference codes (REG AIR unmatched)
    const uint32_t m = (uint32_t)uni(seed, kLMode, r, 0, 6);
    L.shipmode = m == 1 ? 3 : m == 3 ? 2 : m == 5 ? 1 : 0;
    // DELIVER IN PERSON, COLLECT COD, NONE, TAKE BACK RETURN
    L.shipinstruct = uni(seed, kLInstruct, r, 0, 3) == 0 ? 1 : 0;
    L.returnflag = receipt <= kCurrentDay ? (uni(seed, kLFlag, r, 0, 1) ? 'R' : 'A') : 'N';
    return L;
}

}  // namespace tpch
}  // namespace sgxamd
