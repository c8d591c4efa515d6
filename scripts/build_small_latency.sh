#!/bin/bash
# Builds scripts/small_latency_c (C-ABI small-join host-overhead probe) against the in-tree library.
set -e
cd "$(dirname "$0")/.."
PKG=sgxv2-analytical-query-processing-benchmarks_amd
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O2 -std=c++17 -Iinclude scripts/small_latency_c.cpp \
  -L"$PKG" -lsgxamd -Wl,-rpath,'$ORIGIN/../'"$PKG" -o scripts/small_latency_c
