"""CPU: the oracle's and the product's datatype/op tables diffed mechanically against the
reference's own source TEXT (src/shmem_internal_op.h, src/transport.h,
src/transport_none.h).  Nothing of the reference is compiled or executed: the header is
read as text, its tables are extracted with regular expressions, and the C types it
names are measured by gcc in a program this test writes itself.

What this pins: the seven op macro bodies, the 26-case
reduce_local dispatch (datatype -> op class -> C type), the 154 FUNC_OP_CREATE
instances it calls, and both enums -- for the oracle (oracle/sos_oracle.c) and for the
product's device table (sos_amd/csrc/dtypes.h, include/sosx.h).  It does not pin
arithmetic results; those rest on the oracle (known answers in test_oracle_kat.py).

Skipped where /root/reference is absent (the GPU box)."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference/src"
OP_H = os.path.join(REF, "shmem_internal_op.h")

pytestmark = pytest.mark.skipif(not os.path.exists(OP_H), reason="reference checkout not present")

OPS = ["BAND", "BOR", "BXOR", "MIN", "MAX", "SUM", "PROD"]
OP_FUNC = {"and": "BAND", "or": "BOR", "xor": "BXOR", "min": "MIN", "max": "MAX", "sum": "SUM",
           "prod": "PROD"}


def _text(path):
    return open(path).read()


def _strip_comments(t):
    return re.sub(r"/\*.*?\*/", "", t, flags=re.S)


def _norm(s):
    return re.sub(r"\s+", "", s)


def _enum(path, name):
    body = re.search(r"enum\s+" + name + r"\s*\{(.*?)\}", _strip_comments(_text(path)), re.S).group(1)
    return [e.strip() for e in body.split(",") if e.strip()]


def ref_ops():
    return [e.replace("SHM_INTERNAL_", "") for e in _enum(os.path.join(REF, "transport_none.h"), "shm_internal_op_t")]


def ref_dtypes():
    return [e.replace("SHM_INTERNAL_", "") for e in _enum(os.path.join(REF, "transport.h"), "shm_internal_datatype_t")]


def ref_op_macros():
    """{'max': '((a)>(b)?(a):(b))', ...} from `#define shmem_internal_<op>_op(a, b) body`."""
    out = {}
    for m in re.finditer(r"#define\s+shmem_internal_(\w+)_op\(a,\s*b\)\s*(.+)", _text(OP_H)):
        out[m.group(1)] = _norm(m.group(2))
    return out


def ref_func_ops():
    """{(type_name, c_type, op, calc_macro)} of every FUNC_OP_CREATE instance."""
    inst = set()
    for m in re.finditer(r"^FUNC_OP_CREATE\((\w+),\s*([\w ]+?),\s*(\w+),\s*(\w+)\)", _text(OP_H), re.M):
        inst.add((m.group(1), " ".join(m.group(2).split()), m.group(3), m.group(4)))
    return inst


def ref_class_ops():
    """{'FP': {'MIN', ...}, ...}: the ops each REDUCE_LOCAL_DTYPE_CASE_<class> macro accepts."""
    t = _text(OP_H)
    out = {}
    for m in re.finditer(r"#define REDUCE_LOCAL_DTYPE_CASE_(\w+)\(dtype, dtype_name, c_type\)(.*?)\bbreak;\s*\n\n",
                         t, re.S):
        out[m.group(1)] = set(re.findall(r"case SHM_INTERNAL_(\w+):", m.group(2)))
    return out


def ref_dispatch():
    """[(dtype, class, dtype_name, c_type)] of shmem_internal_reduce_local's switch."""
    body = _text(OP_H).split("shmem_internal_reduce_local(")[1]
    rows = []
    for m in re.finditer(r"REDUCE_LOCAL_DTYPE_CASE_(\w+)\(SHM_INTERNAL_(\w+),\s*(\w+),\s*([\w ]+?)\);", body):
        rows.append((m.group(2), m.group(1), m.group(3), " ".join(m.group(4).split())))
    return rows


def test_reference_tables_parse():
    """The extraction itself: sizes the rest of the file relies on."""
    assert ref_ops() == OPS
    assert len(ref_dtypes()) == 28
    assert set(ref_op_macros()) == set(OP_FUNC)
    assert len(ref_func_ops()) == 154    # 18 INT x 7 + 6 FP x 4 + 2 CPLX x 2
    assert set(ref_class_ops()) == {"FP", "CPLX", "INT", "AND_OR_XOR"}
    assert len(ref_dispatch()) == 26


def test_reference_dispatch_is_self_consistent():
    """Every function a dispatch case calls is one FUNC_OP_CREATE makes, with the same C
    type and the op's own calc macro (guards the extraction, not the reference)."""
    funcs = {(tn, op): (ct, calc) for tn, ct, op, calc in ref_func_ops()}
    classes = ref_class_ops()
    for dt, cls, name, ctype in ref_dispatch():
        for op in classes[cls]:
            fop = {v: k for k, v in OP_FUNC.items()}[op]
            assert (name, fop) in funcs, (dt, op)
            ct, calc = funcs[(name, fop)]
            assert ct == ctype and calc == f"shmem_internal_{fop}_op", (dt, op, ct, calc)


# -- the oracle (oracle/sos_oracle.c) ---------------------------------------------------

ORACLE = os.path.join(ROOT, "oracle", "sos_oracle.c")


def oracle_enum(first):
    t = _strip_comments(_text(ORACLE))
    body = re.search(r"enum\s*\{\s*(" + first + r".*?)\}", t, re.S).group(1)
    names = [e.split("=")[0].strip() for e in body.split(",") if e.strip()]
    return [n for n in names if n != "D_COUNT"]


def test_oracle_enums_match_reference():
    assert [n[2:] for n in oracle_enum("O_BAND")] == ref_ops()
    assert [n[2:] for n in oracle_enum("D_SIGNED_BYTE")] == ref_dtypes()


def test_oracle_op_macros_match_reference():
    ora = {}
    for m in re.finditer(r"#define O_(\w+)F\(a, b\)\s*(.+)", _text(ORACLE)):
        ora[m.group(1).lower()] = _norm(m.group(2))
    assert ora == ref_op_macros()


def test_oracle_dispatch_matches_reference():
    """Same datatype -> op class -> C type rows as shmem_internal_reduce_local; the
    oracle's class macros accept the same op sets."""
    t = _text(ORACLE)
    body = t.split("int oracle_reduce_local(")[1].split("\n}\n")[0]
    ora = {m.group(1): (m.group(2), " ".join(m.group(3).split()))
           for m in re.finditer(r"case D_(\w+):\s*O_CASE_(\w+)\(([\w ]+?)\);", body)}
    ref = {dt: (cls, ctype) for dt, cls, _, ctype in ref_dispatch()}
    assert ora == ref
    classes = ref_class_ops()
    for cls in ("FP", "CPLX", "INT"):
        mac = re.search(r"#define O_CASE_" + cls + r"\(ctype\)(.*?)\n(?:#|\n)", t, re.S).group(1)
        got = set(re.findall(r"case O_(\w+):", mac))
        assert got == classes[cls], cls


# -- the product (include/sosx.h, sos_amd/csrc/dtypes.h) -----------------------------------

def product_defines(prefix):
    t = _text(os.path.join(ROOT, "include", "sosx.h"))
    return {m.group(1): int(m.group(2)) for m in re.finditer(r"#define " + prefix + r"(\w+)\s+(\d+)", t)}


def test_product_enums_match_reference():
    ops = product_defines("SOSX_OP_")
    assert [k for k, _ in sorted(ops.items(), key=lambda kv: kv[1])] == ref_ops()
    dts = {k: v for k, v in product_defines("SOSX_DT_").items() if k != "COUNT"}
    assert [k for k, _ in sorted(dts.items(), key=lambda kv: kv[1])] == ref_dtypes()


def _measure_ctypes(ctypes_, tmp_path):
    """sizeof, signedness and floatness of each C type, measured by gcc -std=gnu11 on
    this host (x86-64 LP64, the reference's target)."""
    src = ["#include <stdio.h>", "#include <stddef.h>", "#include <stdint.h>", "int main(void){"]
    for i, ct in enumerate(ctypes_):
        if "_Complex" in ct:
            src.append(f'printf("{i} %zu 0 2\\n", sizeof({ct}));')
        else:
            src.append(f'printf("{i} %zu %d %d\\n", sizeof({ct}), (int)(({ct})-1 < ({ct})0), '
                       f'(int)(({ct})0.5 != ({ct})0));')
    src.append("return 0;}")
    c = tmp_path / "m.c"
    c.write_text("\n".join(src) + "\n")
    exe = tmp_path / "m"
    subprocess.run(["gcc", "-std=gnu11", str(c), "-o", str(exe)], check=True)
    out = {}
    for ln in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split("\n"):
        if ln:
            i, size, signed, fl = map(int, ln.split())
            out[ctypes_[i]] = (size, signed, fl)
    return out


def test_product_device_table_matches_reference_ctypes(tmp_path):
    """dtypes.h's storage kind and op class for every datatype equal what the reference's
    C type is on x86-64: the width, signed compare, fp/complex -- and long double the
    80-bit x87 kind in a 16-byte slot.  Datatypes the reference's switch lacks are
    K_INVALID."""
    t = _text(os.path.join(ROOT, "sos_amd", "csrc", "dtypes.h"))
    tab = {m.group(1): (m.group(2), m.group(3), int(m.group(4)))
           for m in re.finditer(r"/\*\s*(\w+)[^*]*\*/\s*\{(K_\w+),\s*(C_\w+),\s*(\d+)\}", t)}
    assert list(tab) == ref_dtypes()
    rows = {dt: (cls, ctype) for dt, cls, _, ctype in ref_dispatch()}
    meas = _measure_ctypes(sorted({c for _, c in rows.values()}), tmp_path)
    for dt in ref_dtypes():
        kind, cls, size = tab[dt]
        if dt not in rows:
            assert (kind, cls, size) == ("K_INVALID", "C_NONE", 0), dt
            continue
        rcls, ctype = rows[dt]
        assert cls == "C_" + rcls, dt
        msize, signed, fl = meas[ctype]
        assert size == msize, dt
        if fl == 2:
            want = {8: "K_C32", 16: "K_C64"}[msize]
        elif fl:
            want = {4: "K_F32", 8: "K_F64", 16: "K_LDBL"}[msize]
        else:
            want = f"K_{'S' if signed else 'U'}{8 * msize}"
        assert kind == want, (dt, ctype, kind, want)


def test_product_accepts_exactly_the_reference_pairs():
    """sosx_check_op (the product's argument check, before any device work) accepts a
    (datatype, op) pair iff the reference's switch has a case for it; otherwise it
    answers as the reference raises: invalid data type vs unsupported reduction."""
    from sos_amd import _lib
    L = _lib.lib()
    rows = {dt: cls for dt, cls, _, _ in ref_dispatch()}
    classes = ref_class_ops()
    for d, dt in enumerate(ref_dtypes()):
        for o, op in enumerate(ref_ops()):
            rc = L.sosx_check_op(o, d)
            if dt not in rows:
                assert rc == -1, (dt, op, rc)          # RAISE_ERROR_MSG("invalid data type")
            elif op in classes[rows[dt]]:
                assert rc == 0, (dt, op, rc)
            else:
                assert rc == -2, (dt, op, rc)          # RAISE_ERROR_STR("unsupported reduction")


# -- the generated API's type tables (sos_amd/csrc/gen_bindings.py) -------------------------

M4 = "/root/reference/bindings/shmem_bind_c.m4"


def m4_table(name):
    """Rows of `define(`<name>', ...)` in bindings/shmem_bind_c.m4: (stype, C type[, ITYPE])."""
    t = _text(M4)
    body = t.split("define(`" + name + "'")[1].split("')dnl")[0]
    rows = []
    for m in re.finditer(r"\$1\((\w+),\s*([\w ]+?)\s*(?:,\s*`SHM_INTERNAL_(\w+)'.*?)?\)", body):
        rows.append((m.group(1), " ".join(m.group(2).split())) + ((m.group(3),) if m.group(3) else ()))
    return rows


@pytest.mark.skipif(not os.path.exists(M4), reason="reference bindings not present")
def test_generated_api_type_tables_match_m4():
    """gen_bindings.py's tables -- which stamp the 198 reductions, 52 scans and 24
    broadcasts -- equal the reference's m4 tables row for row, in order, including the
    uint8..uint64 -> signed INT8..INT64 internal types."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "sos_amd", "csrc"))
    import gen_bindings as G
    pairs = {"SHMEM_BIND_C_COLL_INTS": G.COLL_INTS, "SHMEM_BIND_C_COLL_AND_OR_XOR": G.AND_OR_XOR,
             "SHMEM_BIND_C_COLL_MIN_MAX": G.MIN_MAX, "SHMEM_BIND_C_COLL_SUM_PROD": G.SUM_PROD,
             "SHMEM_BIND_C_COLL_FLOATS": G.FLOATS, "SHMEM_BIND_C_COLL_CMPLX": G.CMPLX,
             "SHMEM_BIND_C_RMA": G.RMA}
    for name, ours in pairs.items():
        ref = m4_table(name)
        assert ref, name
        assert [tuple(r) for r in ours] == ref, name
