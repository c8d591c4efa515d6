// sgxamd/tpch.hpp — C++-linkage drop-ins for the reference's TPC-H callers.
//
// Same declarations (and mangled symbols) as the reference:
//   void tpch_q3 (result_t*, const CustomerTable*, const OrdersTable*, const LineItemTable*, const char*, joinconfig_t*)
//   void tpch_q10(result_t*, const CustomerTable*, const OrdersTable*, const LineItemTable*, const NationTable*,
//                 const char*, joinconfig_t*)
//   void tpch_q12(result_t*, const LineItemTable*, const OrdersTable*, const char*, joinconfig_t*)
//   void tpch_q19(result_t*, const LineItemTable*, const PartTable*, const char*, joinconfig_t*)
//       Join-Benchmarks/lib/TPCH-Queries/include/tpch.hpp:7-21 (tpch.cpp:36-309)
// and the table loaders of App/TpcH/TpcHCommons.hpp:26-65, reading
// getPath(scale, tbl) = $SGXAMD_TPCH_DATA (default "../data") + "/scale%03d/" + tbl.
//
// `algorithm` is "RHO" or "RHT" (the radix joins this library replaces); the
// queries run on the current MI355X (sgxamd/tpch.h) and print the reference's
// log lines (tpch.cpp, time_print.cpp:18-35).  result->totalresults is the last
// join's cardinality as in the reference; Q19 also carries its materialised join
// (result_type 1, chunked_table_t; release with mi355_free_chunked_table).
#pragma once

#include <cstdint>
#include <string>

#include "sgxamd/data_types.h"
#include "sgxamd/tpch.h"

void tpch_q3(result_t *result, const struct CustomerTable *c, const struct OrdersTable *o,
             const struct LineItemTable *l, const char *algorithm, struct joinconfig_t *config);
void tpch_q10(result_t *result, const CustomerTable *c, const OrdersTable *o, const LineItemTable *l,
              const NationTable *n, const char *algorithm, joinconfig_t *config);
void tpch_q12(result_t *result, const LineItemTable *l, const OrdersTable *o, const char *algorithm,
              joinconfig_t *config);
void tpch_q19(result_t *result, const LineItemTable *l, const PartTable *p, const char *algorithm,
              joinconfig_t *config);

std::string getPath(int scale, const std::string &tbl);
int load_lineitems_from_binary(LineItemTable *l_table, uint8_t query, uint8_t scale);
int load_lineitem_from_csv(LineItemTable *l_table, uint8_t scale);
void free_lineitem(LineItemTable *l_table);
int load_orders_from_binary(OrdersTable *o_table, uint8_t query, uint8_t scale);
int load_orders_from_csv(OrdersTable *o_table, uint8_t scale);
void free_orders(OrdersTable *o_table);
int load_customers_from_binary(CustomerTable *c_table, uint8_t query, uint8_t scale);
int load_customer_from_csv(CustomerTable *c_table, uint8_t scale);
void free_customer(CustomerTable *c_table);
int load_parts_from_binary(PartTable *p, uint8_t query, uint8_t scale);
int load_part_from_csv(PartTable *p, uint8_t scale);
void free_part(PartTable *p);
int load_nations_from_binary(NationTable *n_table, uint8_t query, uint8_t scale);
int load_nation_from_csv(NationTable *n, uint8_t scale);
void free_nation(NationTable *n);
