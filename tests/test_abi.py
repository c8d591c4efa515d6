"""The C-ABI library loads on a CPU-only host and exports every symbol the
headers in include/sgxamd declare (no compute calls here)."""
import ctypes as C
import os
import re
import subprocess

from conftest import PKG, ROOT

INCLUDE = os.path.join(ROOT, "include", "sgxamd")
LIB = os.path.join(PKG, "libsgxamd.so")

# C++-linkage drop-ins of sgxamd/joins.hpp with the reference's mangled names
# (radix_join.h:29-30, joins.cpp:55).
CXX_SYMBOLS = {
    "RHO": "_Z3RHOPK7table_tS1_PK12joinconfig_t",
    "run_join": "_Z8run_joinP8result_tPK7table_tS3_PKcPK12joinconfig_t",
    # TPC-H callers, tpch.hpp:7-21, and a loader, TpcHCommons.hpp:33
    "tpch_q3": "_Z7tpch_q3P8result_tPK13CustomerTablePK11OrdersTablePK13LineItemTablePKcP12joinconfig_t",
    "tpch_q10": "_Z8tpch_q10P8result_tPK13CustomerTablePK11OrdersTablePK13LineItemTablePK11NationTablePKcP12joinconfig_t",
    "tpch_q12": "_Z8tpch_q12P8result_tPK13LineItemTablePK11OrdersTablePKcP12joinconfig_t",
    "tpch_q19": "_Z8tpch_q19P8result_tPK13LineItemTablePK9PartTablePKcP12joinconfig_t",
    "load_lineitems_from_binary": "_Z26load_lineitems_from_binaryP13LineItemTablehh",
}


def declared_c_functions():
    names = set()
    for h in ("rho.h", "scan.h", "generator.h", "tpch.h", "multi.h"):
        text = open(os.path.join(INCLUDE, h)).read()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        names |= set(re.findall(r"\b(mi355_\w+)\s*\(", text))
    return sorted(names)


def exported():
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True, check=True).stdout
    return {line.split()[-1] for line in out.splitlines() if " T " in line}


def test_library_loads_without_gpu(sgx):
    assert os.path.exists(LIB)
    assert sgx.version().startswith("sgxamd-mi355")
    # counting devices must not fail on a CPU-only host
    assert sgx.device_count() >= 0


def test_every_declared_c_symbol_is_exported(sgx):
    decl = declared_c_functions()
    assert len(decl) >= 28
    exp = exported()
    missing = [d for d in decl if d not in exp]
    assert not missing, missing
    # and the ctypes binding covers exactly the declared set
    assert set(sgx.SIGNATURES) == set(decl)


def test_cxx_dropins_exported():
    exp = exported()
    for name, mangled in CXX_SYMBOLS.items():
        assert mangled in exp, name


def test_struct_layouts_match_reference(sgx):
    # data-types.h:44-54, 107-114, 162-176 (x86-64)
    assert C.sizeof(sgx.row_t) == 8
    assert C.sizeof(sgx.table_t) == 24
    assert C.sizeof(sgx.result_t) == 48
    assert sgx.result_t.throughput.offset == 16
    assert sgx.result_t.result.offset == 32
    assert C.sizeof(sgx.joinconfig_t) == 48
    assert sgx.joinconfig_t.MATERIALIZE.offset == 32


def test_static_asserts_compile_as_c_and_cxx(tmp_path):
    src = tmp_path / "t.c"
    src.write_text('#include "sgxamd/data_types.h"\n#include "sgxamd/rho.h"\n#include "sgxamd/scan.h"\n'
                   '#include "sgxamd/generator.h"\n#include "sgxamd/multi.h"\nint main(void){return 0;}\n')
    subprocess.run(["gcc", "-std=c11", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(tmp_path / "a")],
                   check=True)
    cpp = tmp_path / "t.cpp"
    # instantiate every adapter template the way a reference caller would (compile only)
    cpp.write_text('#include <vector>\n#include "sgxamd/joins.hpp"\n#include "sgxamd/SIMD512_mi355.hpp"\n'
                   'void use(const void *in, const int64_t *d, std::vector<int64_t> &v, std::vector<size_t> &ix) {\n'
                   '  SIMD512::dict_scan_8bit_64bit(0, 1, d, in, 64, v, true);\n'
                   '  SIMD512::dict_scan_16bit_64bit(0, 1, d, in, 64, v);\n'
                   '  SIMD512::dict_scan_32bit_64bit(0, 1, d, 99, in, 64, v);\n'
                   '  SIMD512::implicit_index_scan_self_alloc(0, 1, in, 64, ix, true);\n'
                   '  (void)SIMD512::sum(0, 1, in, 64); (void)SIMD512::count(0, 1, in, 64);\n}\n'
                   'int main(){return 0;}\n')
    subprocess.run(["g++", "-std=c++17", "-c", "-I", os.path.join(ROOT, "include"), str(cpp), "-o",
                    str(tmp_path / "b.o")], check=True)


def test_compute_without_gpu_fails_loudly(sgx):
    """No silent CPU fallback: on a CPU-only host compute calls return NO_DEVICE."""
    if sgx.device_count() > 0:
        return
    import numpy as np

    col = np.arange(1024, dtype=np.int32)
    try:
        sgx.scan_count(0, 10, col, len(col))
    except sgx.Mi355Error as e:
        assert e.code == sgx.MI355_ERR_NO_DEVICE
    else:
        raise AssertionError("scan ran without a GPU")
    R = np.zeros(16, dtype=np.uint64)
    try:
        sgx.rho_join(R, 16, R, 16)
    except sgx.Mi355Error as e:
        assert e.code == sgx.MI355_ERR_NO_DEVICE
    else:
        raise AssertionError("join ran without a GPU")
    try:
        sgx.rho_join_multi(R, 16, R, 16, 4, transport="rehearsal")
    except sgx.Mi355Error as e:
        assert e.code == sgx.MI355_ERR_NO_DEVICE
    else:
        raise AssertionError("multi-GPU join ran without a GPU")


def test_multi_rejects_bad_world(sgx):
    import numpy as np

    R = np.zeros(16, dtype=np.uint64)
    for g in (0, 3, 6, 512):
        try:
            sgx.rho_join_multi(R, 16, R, 16, g)
        except sgx.Mi355Error as e:
            assert e.code == sgx.MI355_ERR_INVALID
        else:
            raise AssertionError(g)


def test_stats_structs_match_ctypes(sgx, tmp_path):
    """The ctypes mirrors of mi355_rho_stats / mi355_multi_stats (python/sgxamd) have the C
    headers' size and field offsets: a C program compiled against include/ prints them."""
    structs = {"mi355_rho_stats": sgx.rho_stats, "mi355_multi_stats": sgx.multi_stats}
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "sgxamd/rho.h"', '#include "sgxamd/multi.h"',
             "int main(void) {"]
    for cname, py in structs.items():
        lines.append(f'printf("{cname} size %zu\\n", sizeof({cname}));')
        for f, _ in py._fields_:
            lines.append(f'printf("{cname} {f} %zu\\n", offsetof({cname}, {f}));')
    lines.append("return 0; }")
    src = tmp_path / "stats_layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "stats_layout"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split("\n")
    got = {tuple(line.split()[:2]): int(line.split()[2]) for line in out if line}
    for cname, py in structs.items():
        assert got[(cname, "size")] == C.sizeof(py), cname
        for f, _ in py._fields_:
            assert got[(cname, f)] == getattr(py, f).offset, (cname, f)
