#!/usr/bin/env python3
"""Generate the typed SOS reduction / scan / broadcast entry points.

SOS stamps its reductions out of m4 type tables (bindings/shmem_bind_c.m4:93-180)
through SHMEM_DEF_TO_ALL / SHMEM_DEF_REDUCE (src/collectives_c.c4:221-292).  This
generator holds the same tables -- including SOS's mapping of uint8/16/32/64 onto the
SIGNED INT8..INT64 internal types (shmem_bind_c.m4:113-116, :136-139, :162-165), which
makes their min/max compare signed -- and writes:

  include/shmem_reductions.h      198 prototypes + C11 _Generic macros
                                  (mpp/shmem.h4:952-991) + C++ overloads (:249-296)
  include/shmemx_scans.h          52 shmemx_<T>_sum_{inscan,exscan} prototypes + generics
                                  (mpp/shmemx_c_func.h4:78-86, mpp/shmemx.h4:71-133)
  sos_amd/csrc/reductions_gen.cpp the definitions (strong pshmem_*, weak shmem_*
                                  aliases as SOS's profiling interface,
                                  src/collectives_c.c4:36-166), plus the 24 typed team
                                  broadcasts shmem_<T>_broadcast (SHMEM_BIND_C_RMA,
                                  src/collectives_c.c4:402-429) and the 52 scans
                                  (src/collectives_c.c4:294-340)

Run: python sos_amd/csrc/gen_bindings.py   (build() runs it; output is committed).
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# (stype, C type, internal datatype) -- bindings/shmem_bind_c.m4
COLL_INTS = [("short", "short", "SHORT"), ("int", "int", "INT"), ("long", "long", "LONG"),
             ("longlong", "long long", "LONG_LONG")]
AND_OR_XOR = [
    ("uchar", "unsigned char", "UCHAR"), ("short", "short", "SHORT"),
    ("ushort", "unsigned short", "USHORT"), ("int", "int", "INT"), ("uint", "unsigned int", "UINT"),
    ("long", "long", "LONG"), ("ulong", "unsigned long", "ULONG"),
    ("longlong", "long long", "LONG_LONG"), ("ulonglong", "unsigned long long", "ULONG_LONG"),
    ("int8", "int8_t", "INT8"), ("int16", "int16_t", "INT16"), ("int32", "int32_t", "INT32"),
    ("int64", "int64_t", "INT64"),
    ("uint8", "uint8_t", "INT8"), ("uint16", "uint16_t", "INT16"),    # signed ITYPE (SOS quirk)
    ("uint32", "uint32_t", "INT32"), ("uint64", "uint64_t", "INT64"),  # signed ITYPE (SOS quirk)
    ("size", "size_t", "SIZE_T")]
MIN_MAX = [
    ("char", "char", "CHAR"), ("schar", "signed char", "SCHAR"), ("short", "short", "SHORT"),
    ("int", "int", "INT"), ("long", "long", "LONG"), ("longlong", "long long", "LONG_LONG"),
    ("ptrdiff", "ptrdiff_t", "PTRDIFF_T"), ("uchar", "unsigned char", "UCHAR"),
    ("ushort", "unsigned short", "USHORT"), ("uint", "unsigned int", "UINT"),
    ("ulong", "unsigned long", "ULONG"), ("ulonglong", "unsigned long long", "ULONG_LONG"),
    ("int8", "int8_t", "INT8"), ("int16", "int16_t", "INT16"), ("int32", "int32_t", "INT32"),
    ("int64", "int64_t", "INT64"),
    ("uint8", "uint8_t", "INT8"), ("uint16", "uint16_t", "INT16"),
    ("uint32", "uint32_t", "INT32"), ("uint64", "uint64_t", "INT64"),
    ("size", "size_t", "SIZE_T"), ("float", "float", "FLOAT"), ("double", "double", "DOUBLE"),
    ("longdouble", "long double", "LONG_DOUBLE")]
SUM_PROD = MIN_MAX + [("complexd", "double _Complex", "DOUBLE_COMPLEX"),
                      ("complexf", "float _Complex", "FLOAT_COMPLEX")]
# bindings/shmem_bind_c.m4:10-34 (broadcast element types; bytes only, no ITYPE)
RMA = [("float", "float"), ("double", "double"), ("longdouble", "long double"), ("char", "char"),
       ("schar", "signed char"), ("short", "short"), ("int", "int"), ("long", "long"),
       ("longlong", "long long"), ("uchar", "unsigned char"), ("ushort", "unsigned short"),
       ("uint", "unsigned int"), ("ulong", "unsigned long"), ("ulonglong", "unsigned long long"),
       ("int8", "int8_t"), ("int16", "int16_t"), ("int32", "int32_t"), ("int64", "int64_t"),
       ("uint8", "uint8_t"), ("uint16", "uint16_t"), ("uint32", "uint32_t"), ("uint64", "uint64_t"),
       ("size", "size_t"), ("ptrdiff", "ptrdiff_t")]
# bindings/shmem_bind_c11.m4:13-28 (generic selector: base types only)
GENERIC_RMA = RMA[:14]
FLOATS = [("float", "float", "FLOAT"), ("double", "double", "DOUBLE"),
          ("longdouble", "long double", "LONG_DOUBLE")]
CMPLX = [("complexf", "float _Complex", "FLOAT_COMPLEX"),
         ("complexd", "double _Complex", "DOUBLE_COMPLEX")]

OPS = {"and": "BAND", "or": "BOR", "xor": "BXOR", "min": "MIN", "max": "MAX", "sum": "SUM",
       "prod": "PROD"}

# src/collectives_c.c4:270-292
TO_ALL = ([(t, o) for o in ("and", "or", "xor") for t in COLL_INTS]
          + [(t, "min") for t in COLL_INTS] + [(t, "min") for t in FLOATS]
          + [(t, "max") for t in COLL_INTS] + [(t, "max") for t in FLOATS]
          + [(t, "sum") for t in COLL_INTS] + [(t, "sum") for t in FLOATS] + [(t, "sum") for t in CMPLX]
          + [(t, "prod") for t in COLL_INTS] + [(t, "prod") for t in FLOATS] + [(t, "prod") for t in CMPLX])
REDUCE = ([(t, o) for o in ("and", "or", "xor") for t in AND_OR_XOR]
          + [(t, o) for o in ("sum", "prod") for t in SUM_PROD]
          + [(t, o) for o in ("min", "max") for t in MIN_MAX])

REDUCE_TABLE = {"and": AND_OR_XOR, "or": AND_OR_XOR, "xor": AND_OR_XOR, "min": MIN_MAX,
                "max": MIN_MAX, "sum": SUM_PROD, "prod": SUM_PROD}

# Generic (C11 _Generic / C++ overload) selector tables: base C types only
# (bindings/shmem_bind_c11.m4:69-112, bindings/shmem_bind_cxx.m4:63-107).  The
# fixed-width "extras" SOS appends at configure time are aliases of these base types
# on x86-64 glibc (int8_t = signed char, int64_t = long, size_t = unsigned long, ...),
# so none is distinct here.
_BASE_UNSIGNED = [("uchar", "unsigned char"), ("ushort", "unsigned short"),
                  ("uint", "unsigned int"), ("ulong", "unsigned long"),
                  ("ulonglong", "unsigned long long")]
_BASE_MIN_MAX = [("char", "char"), ("schar", "signed char"), ("short", "short"), ("int", "int"),
                 ("long", "long"), ("longlong", "long long")] + _BASE_UNSIGNED + [
                 ("float", "float"), ("double", "double"), ("longdouble", "long double")]
GENERIC_TABLE = {"and": _BASE_UNSIGNED, "or": _BASE_UNSIGNED, "xor": _BASE_UNSIGNED,
                 "min": _BASE_MIN_MAX, "max": _BASE_MIN_MAX,
                 "sum": _BASE_MIN_MAX + [("complexd", "double _Complex"),
                                         ("complexf", "float _Complex")]}
GENERIC_TABLE["prod"] = GENERIC_TABLE["sum"]


def to_all_sig(prefix, st, ct, op):
    return (f"void {prefix}shmem_{st}_{op}_to_all({ct} *target, const {ct} *source, int nreduce, "
            f"int PE_start, int logPE_stride, int PE_size, {ct} *pWrk, long *pSync)")


def reduce_sig(prefix, st, ct, op):
    return (f"int {prefix}shmem_{st}_{op}_reduce(shmem_team_t team, {ct} *dest, const {ct} *source, "
            f"size_t nreduce)")


def bcast_sig(prefix, st, ct):
    return (f"int {prefix}shmem_{st}_broadcast(shmem_team_t team, {ct} *dest, const {ct} *source, "
            f"size_t nelems, int PE_root)")


def scan_sig(prefix, st, ct, kind):
    return (f"int {prefix}shmemx_{st}_sum_{kind}(shmem_team_t team, {ct} *dest, const {ct} *source, "
            f"size_t nelems)")


SCANS = [(t, k) for k in ("exscan", "inscan") for t in SUM_PROD]


def c11_generic(name, arms, argidx=1):
    out = [f"#define {name}(...) \\",
           f"    _Generic(SHMEM_C11_TYPE_EVAL_PTR(SHMEM_C11_ARG{argidx}(__VA_ARGS__)), \\",
           ", \\\n".join(arms) + " \\", "    )(__VA_ARGS__)"]
    return out


def scan_header():
    out = ["/* shmemx_scans.h -- GENERATED by sos_amd/csrc/gen_bindings.py; do not edit.",
           " *",
           " * SOS's team prefix-sum extensions shmemx_<T>_sum_{inscan,exscan}",
           " * (mpp/shmemx_c_func.h4:78-86) with their C++ overloads and C11 generic",
           " * selectors (mpp/shmemx.h4:71-133). */",
           "#ifndef SHMEMX_SCANS_H", "#define SHMEMX_SCANS_H", "",
           "#ifdef __cplusplus", 'extern "C" {', "#endif", ""]
    for (st, ct, it), k in SCANS:
        out.append(f"SHMEM_FUNCTION_ATTRIBUTES {scan_sig('', st, ct, k)};")
    for (st, ct, it), k in SCANS:
        out.append(f"{scan_sig('p', st, ct, k)};")
    out += ["", "#ifdef __cplusplus", "}  /* extern \"C\" */", "#endif", ""]
    out.append("#if defined(__cplusplus)")
    for k in ("exscan", "inscan"):
        for st, ct in GENERIC_TABLE["sum"]:
            out.append(f"static inline int shmemx_sum_{k}(shmem_team_t team, {ct} *dest, "
                       f"const {ct} *source, size_t nelems) {{ return shmemx_{st}_sum_{k}(team, "
                       f"dest, source, nelems); }}")
    out.append("#elif defined(__STDC_VERSION__) && __STDC_VERSION__ >= 201112L")
    out.append("#ifndef SHMEM_C11_TYPE_EVAL_PTR")
    out.append("#define SHMEM_C11_TYPE_EVAL_PTR(arg) &*(arg)")
    out.append("#define SHMEM_C11_ARG1(first, ...) SHMEM_C11_ARG1_HELPER(__VA_ARGS__, sentinel)")
    out.append("#define SHMEM_C11_ARG1_HELPER(second, ...) second")
    out.append("#endif")
    for k in ("exscan", "inscan"):
        out += c11_generic(f"shmemx_sum_{k}",
                           [f"        {ct}*: shmemx_{st}_sum_{k}" for st, ct in GENERIC_TABLE["sum"]])
    out.append("#endif")
    out += ["", "#endif /* SHMEMX_SCANS_H */", ""]
    return "\n".join(out)


def header():
    out = ["/* shmem_reductions.h -- GENERATED by sos_amd/csrc/gen_bindings.py; do not edit.",
           " *",
           " * The SOS reduction family: 44 active-set *_to_all and 154 team *_reduce entry",
           " * points with SOS's signatures (mpp/shmem_c_func.h4:413-438, :688-702), the 24",
           " * typed team broadcasts (:673-676), the C11 generic selectors (mpp/shmem.h4:",
           " * 934-939, :952-991) and C++ overloads (:228-233, :249-296). */",
           "#ifndef SHMEM_REDUCTIONS_H", "#define SHMEM_REDUCTIONS_H", "",
           "#ifdef __cplusplus", 'extern "C" {', "#endif", ""]
    out.append("/* active-set reductions (deprecated in OpenSHMEM 1.5, kept by SOS) */")
    for (st, ct, it), op in TO_ALL:
        out.append(f"SHMEM_FUNCTION_ATTRIBUTES {to_all_sig('', st, ct, op)};")
    out.append("")
    out.append("/* team reductions */")
    for (st, ct, it), op in REDUCE:
        out.append(f"SHMEM_FUNCTION_ATTRIBUTES {reduce_sig('', st, ct, op)};")
    out.append("")
    out.append("/* typed team broadcasts (mpp/shmem_c_func.h4:673-676) */")
    for st, ct in RMA:
        out.append(f"SHMEM_FUNCTION_ATTRIBUTES {bcast_sig('', st, ct)};")
    out.append("")
    out.append("/* profiling interface: pshmem_* are the implementations, shmem_* weak aliases */")
    for (st, ct, it), op in TO_ALL:
        out.append(f"{to_all_sig('p', st, ct, op)};")
    for (st, ct, it), op in REDUCE:
        out.append(f"{reduce_sig('p', st, ct, op)};")
    for st, ct in RMA:
        out.append(f"{bcast_sig('p', st, ct)};")
    out += ["", "#ifdef __cplusplus", "}  /* extern \"C\" */", "#endif", ""]
    # C++ overloads
    out.append("#if defined(__cplusplus)")
    for op in ("and", "or", "xor", "min", "max", "sum", "prod"):
        for st, ct in GENERIC_TABLE[op]:
            out.append(f"static inline int shmem_{op}_reduce(shmem_team_t team, {ct} *dest, "
                       f"const {ct} *source, size_t nreduce) {{ return shmem_{st}_{op}_reduce(team, "
                       f"dest, source, nreduce); }}")
    for st, ct in GENERIC_RMA:
        out.append(f"static inline int shmem_broadcast(shmem_team_t team, {ct} *dest, const {ct} *source, "
                   f"size_t nelems, int PE_root) {{ return shmem_{st}_broadcast(team, dest, source, "
                   f"nelems, PE_root); }}")
    # C11 generics
    out.append("#elif defined(__STDC_VERSION__) && __STDC_VERSION__ >= 201112L")
    out.append("#define SHMEM_C11_TYPE_EVAL_PTR(arg) &*(arg)")
    out.append("#define SHMEM_C11_ARG1(first, ...) SHMEM_C11_ARG1_HELPER(__VA_ARGS__, sentinel)")
    out.append("#define SHMEM_C11_ARG1_HELPER(second, ...) second")
    for op in ("and", "or", "xor", "min", "max", "sum", "prod"):
        arms = [f"        {ct}*: shmem_{st}_{op}_reduce" for st, ct in GENERIC_TABLE[op]]
        out.append(f"#define shmem_{op}_reduce(...) \\")
        out.append("    _Generic(SHMEM_C11_TYPE_EVAL_PTR(SHMEM_C11_ARG1(__VA_ARGS__)), \\")
        out.append(", \\\n".join(arms) + " \\")
        out.append("    )(__VA_ARGS__)")
    out += c11_generic("shmem_broadcast", [f"        {ct}*: shmem_{st}_broadcast" for st, ct in GENERIC_RMA])
    out.append("#endif")
    out += ["", "#endif /* SHMEM_REDUCTIONS_H */", ""]
    return "\n".join(out)


def source():
    out = ["// reductions_gen.cpp -- GENERATED by sos_amd/csrc/gen_bindings.py; do not edit.",
           "//",
           "// The 198 typed SOS reduction entry points.  Each is SHMEM_DEF_TO_ALL or",
           "// SHMEM_DEF_REDUCE (src/collectives_c.c4:221-269): argument checks, then the",
           "// dispatcher with the (op, internal datatype) pair of bindings/shmem_bind_c.m4.",
           '#include "shmem.h"', '#include "shmemx.h"', '#include "sosx.h"',
           '#include "api_internal.h"', "",
           'extern "C" {', ""]
    for (st, ct, it), op in TO_ALL:
        name = f"shmem_{st}_{op}_to_all"
        out.append(f"{to_all_sig('p', st, ct, op)}")
        out.append("{")
        out.append(f"    sos_api_to_all(target, source, nreduce, sizeof({ct}), PE_start, logPE_stride, "
                   f"PE_size, pWrk, pSync, SOSX_OP_{OPS[op]}, SOSX_DT_{it}, \"{name}\");")
        out.append("}")
        out.append(f"{to_all_sig('', st, ct, op)} __attribute__((weak, alias(\"p{name}\")));")
        out.append("")
    for (st, ct, it), op in REDUCE:
        name = f"shmem_{st}_{op}_reduce"
        out.append(f"{reduce_sig('p', st, ct, op)}")
        out.append("{")
        out.append(f"    return sos_api_reduce(team, dest, source, nreduce, sizeof({ct}), "
                   f"SOSX_OP_{OPS[op]}, SOSX_DT_{it}, \"{name}\");")
        out.append("}")
        out.append(f"{reduce_sig('', st, ct, op)} __attribute__((weak, alias(\"p{name}\")));")
        out.append("")
    for st, ct in RMA:
        name = f"shmem_{st}_broadcast"
        out.append(f"{bcast_sig('p', st, ct)}")
        out.append("{")
        out.append(f"    return sos_api_broadcast(team, dest, source, nelems, sizeof({ct}), PE_root, "
                   f"\"{name}\");")
        out.append("}")
        out.append(f"{bcast_sig('', st, ct)} __attribute__((weak, alias(\"p{name}\")));")
        out.append("")
    for (st, ct, it), k in SCANS:
        name = f"shmemx_{st}_sum_{k}"
        out.append(f"{scan_sig('p', st, ct, k)}")
        out.append("{")
        out.append(f"    return sos_api_scan(team, dest, source, nelems, sizeof({ct}), SOSX_OP_SUM, "
                   f"SOSX_DT_{it}, {1 if k == 'exscan' else 0}, \"{name}\");")
        out.append("}")
        out.append(f"{scan_sig('', st, ct, k)} __attribute__((weak, alias(\"p{name}\")));")
        out.append("")
    out += ['}  // extern "C"', ""]
    return "\n".join(out)


def symbols():
    """All generated public names (used by the ABI test)."""
    return ([f"shmem_{st}_{op}_to_all" for (st, ct, it), op in TO_ALL]
            + [f"shmem_{st}_{op}_reduce" for (st, ct, it), op in REDUCE]
            + [f"shmem_{st}_broadcast" for st, ct in RMA]
            + [f"shmemx_{st}_sum_{k}" for (st, ct, it), k in SCANS])


def main():
    assert len(TO_ALL) == 44 and len(REDUCE) == 154, (len(TO_ALL), len(REDUCE))
    assert len(RMA) == 24 and len(SCANS) == 52, (len(RMA), len(SCANS))
    targets = {os.path.join(ROOT, "include", "shmem_reductions.h"): header(),
               os.path.join(ROOT, "include", "shmemx_scans.h"): scan_header(),
               os.path.join(ROOT, "sos_amd", "csrc", "reductions_gen.cpp"): source()}
    check = "--check" in sys.argv
    stale = False
    for path, text in targets.items():
        old = open(path).read() if os.path.exists(path) else None
        if old != text:
            stale = True
            if not check:
                with open(path, "w") as fh:
                    fh.write(text)
    if check and stale:
        print("generated bindings are stale", file=sys.stderr)
        return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
