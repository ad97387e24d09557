"""CPU: the C-ABI library loads, exports every function include/*.h declares, the
generated bindings are current, and SOS programs compile against include/shmem.h."""
import os
import re
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
INC = os.path.join(ROOT, "include")
LIB = os.path.join(ROOT, "sos_amd", "libsos_amd.so")
REF_PI = "/root/reference/examples/pi_reduce.c"


def declared_functions():
    names = set()
    for h in ("shmem.h", "shmemx.h", "sosx.h", "shmem_reductions.h", "shmemx_scans.h"):
        text = open(os.path.join(INC, h)).read()
        text = text.split("#if defined(__cplusplus)\nstatic inline")[0]  # skip inline overloads
        for m in re.finditer(r"^\s*(?:SHMEM_FUNCTION_ATTRIBUTES\s+)?(?:const\s+)?[\w ]+?\**\s*\b(\w+)\(",
                             text, re.M):
            name = m.group(1)
            if name.startswith(("shmem", "pshmem", "sosx")) and not name.startswith("SHMEM"):
                names.add(name)
    return names


def exported_symbols():
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True,
                         check=True).stdout
    return {ln.split()[-1] for ln in out.splitlines() if len(ln.split()) == 3}


def test_library_loads_and_exports_everything():
    from sos_amd import _lib
    _lib.lib()
    declared = declared_functions()
    assert len(declared) > 550  # 274 typed shmem_* + their pshmem_* + runtime + sosx
    missing = sorted(declared - exported_symbols())
    assert not missing, missing


def test_typed_collective_symbols():
    # 198 reductions (44 to_all + 154 reduce), 24 typed broadcasts, 52 sum scans
    sys.path.insert(0, os.path.join(ROOT, "sos_amd", "csrc"))
    import gen_bindings
    names = gen_bindings.symbols()
    assert len(names) == 274 and len(set(names)) == 274
    assert sum(n.endswith("_broadcast") for n in names) == 24
    assert sum(n.endswith(("_inscan", "_exscan")) for n in names) == 52
    exp = exported_symbols()
    assert all(n in exp and "p" + n in exp for n in names)
    # SOS quirks carried over: uint8..64 reduce with the SIGNED internal type
    src = open(os.path.join(ROOT, "sos_amd", "csrc", "reductions_gen.cpp")).read()
    assert 'SOSX_OP_MAX, SOSX_DT_INT32, "shmem_uint32_max_reduce"' in src
    assert 'SOSX_OP_MIN, SOSX_DT_INT8, "shmem_uint8_min_reduce"' in src
    assert 'SOSX_OP_MAX, SOSX_DT_UCHAR, "shmem_uchar_max_reduce"' in src


def test_generated_bindings_current():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "sos_amd", "csrc", "gen_bindings.py"),
                        "--check"])
    assert r.returncode == 0


def test_constants_match_sos():
    text = open(os.path.join(INC, "shmem.h")).read()
    for name, val in (("SHMEM_REDUCE_SYNC_SIZE", 35), ("SHMEM_BCAST_SYNC_SIZE", 1),
                      ("SHMEM_BARRIER_SYNC_SIZE", 16), ("SHMEM_COLLECT_SYNC_SIZE", 18),
                      ("SHMEM_SYNC_SIZE", 35), ("SHMEM_REDUCE_MIN_WRKDATA_SIZE", 1),
                      ("SHMEM_SYNC_VALUE", 0)):
        assert re.search(rf"#define {name} {val}\b", text), name


def _compile(src, lang, tmp_path, extra=()):
    exe = str(tmp_path / "a.out")
    cc = "gcc" if lang == "c" else "g++"
    std = ["-std=gnu11"] if lang == "c" else ["-std=c++17"]
    cmd = [cc, *std, "-Wall", "-I", INC, "-I/opt/rocm/include", "-D__HIP_PLATFORM_AMD__", src, "-o",
           exe, "-L", os.path.dirname(LIB), "-lsos_amd", f"-Wl,-rpath,{os.path.dirname(LIB)}",
           "-L/opt/rocm/lib", "-lamdhip64", *extra]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    return exe


@pytest.mark.skipif(not os.path.exists(REF_PI), reason="reference checkout not present")
def test_reference_pi_reduce_compiles_unchanged(tmp_path):
    """examples/pi_reduce.c (shmem_sum_reduce C11 generic on long long) builds as-is."""
    _compile(REF_PI, "c", tmp_path)


def test_own_examples_compile(tmp_path):
    for f in ("pi_reduce_amd.c", "reduce_types.c"):
        _compile(os.path.join(ROOT, "examples", f), "c", tmp_path)


def test_cxx_overloads_compile(tmp_path):
    src = tmp_path / "t.cpp"
    src.write_text('#include <shmem.h>\nint main(){ shmem_init(); static long long a, b; '
                   'static double d[4], e[4]; static unsigned u[3], v[3];\n'
                   'shmem_sum_reduce(SHMEM_TEAM_WORLD, &a, &b, 1); shmem_max_reduce(SHMEM_TEAM_WORLD, d, e, 4);\n'
                   'shmem_xor_reduce(SHMEM_TEAM_WORLD, u, v, 3); shmem_finalize(); return 0; }\n')
    _compile(str(src), "cxx", tmp_path)


def test_bcast_scan_generics_compile(tmp_path):
    body = ('static long long a[4], b[4]; static double d[4], e[4]; static int i4[4], j4[4];\n'
            'static long ps[SHMEM_BCAST_SYNC_SIZE];\n'
            'shmem_broadcast(SHMEM_TEAM_WORLD, a, b, 4, 0); shmem_broadcast(SHMEM_TEAM_WORLD, d, e, 4, 0);\n'
            'shmem_broadcastmem(SHMEM_TEAM_WORLD, i4, j4, sizeof i4, 0);\n'
            'shmem_broadcast64(a, b, 4, 0, 0, 0, shmem_n_pes(), ps);\n'
            'shmem_broadcast32(i4, j4, 4, 0, 0, 0, shmem_n_pes(), ps);\n'
            'shmemx_sum_inscan(SHMEM_TEAM_WORLD, d, e, 4); shmemx_sum_exscan(SHMEM_TEAM_WORLD, i4, j4, 4);\n')
    for lang, ext, hdr in (("c", "c", "#include <shmem.h>\n#include <shmemx.h>\n"),
                           ("cxx", "cpp", "#include <shmem.h>\n#include <shmemx.h>\n")):
        src = tmp_path / f"t.{ext}"
        src.write_text(hdr + "int main(void){ shmem_init();\n" + body + "shmem_finalize(); return 0; }\n")
        _compile(str(src), lang, tmp_path)


def test_plan_abi_rejects_bad_args():
    from sos_amd import shmem as S
    L = S.lib()
    assert L.sosx_plan_encode(2, 0, 0, 10, 4, 0, 0, None, 0) < 0       # P = 0
    assert L.sosx_plan_encode(2, 4, 4, 10, 4, 0, 0, None, 0) < 0       # me out of range
    assert L.sosx_plan_encode(9, 4, 0, 10, 4, 0, 0, None, 0) < 0       # bad algorithm
    assert L.sosx_plan_encode(2, 4, 0, 0, 4, 0, 0, None, 0) == 3       # count 0: no rounds


def test_combine_status_codes_without_gpu():
    """Argument/type validation happens before any device work."""
    from sos_amd import _lib
    L = _lib.lib()
    assert L.sosx_check_op(5, 23) == 0
    assert L.sosx_check_op(0, 23) == -2     # and on float: FP class
    assert L.sosx_check_op(3, 26) == -2     # min on complex
    assert L.sosx_check_op(5, 0) == -1      # SIGNED_BYTE is not reducible
    assert L.sosx_check_op(5, 25) == 0      # long double is valid in SOS ...
    assert L.sosx_combine(5, 25, None, None, 0, None) == 0   # ... (count 0: nothing to do)
    assert L.sosx_dtype_size(27) == 16 and L.sosx_dtype_size(25) == 16


@pytest.mark.parametrize("order", ["lib_then_torch", "torch_then_lib"])
def test_one_hip_runtime_per_process(order):
    """libsos_amd.so and torch share ONE HIP runtime whatever the import order (two copies
    made the process abort at exit: "double free or corruption")."""
    first, second = (("from sos_amd import _lib; _lib.lib()", "import torch")
                     if order == "lib_then_torch" else
                     ("import torch", "from sos_amd import _lib; _lib.lib()"))
    code = (f"import sys; sys.path.insert(0, {ROOT!r})\n{first}\n{second}\n"
            "from sos_amd import _lib\n"
            "dup = {k: v for k, v in _lib.loaded_runtimes().items() if len(v) > 1}\n"
            "assert not dup, dup\nprint('one runtime')\n")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "one runtime" in r.stdout


def test_team_handle_is_sos_type(tmp_path):
    """shmem_team_t is SOS's `struct shmem_impl_team_t *` (mpp/shmem-def.h.in:94-96) and
    SHMEM_TEAM_INVALID is NULL (:110): a C++ library built against SOS's typedef (the
    first TU below restates it, as code compiled against SOS's shmem.h sees it), with a
    function overloaded on the handle type, links with user code built against this
    include/shmem.h -- the mangled names agree -- and C rejects a pointer of another type."""
    lib_tu = tmp_path / "sos_side.cpp"
    lib_tu.write_text(
        "typedef struct shmem_impl_team_t { int dummy; } * shmem_team_t;\n"
        "int team_tag(shmem_team_t t) { return t ? 1 : 2; }\n"
        "int team_tag(void *p) { return p ? 3 : 4; }\n")
    user_tu = tmp_path / "user.cpp"
    user_tu.write_text(
        "#include <shmem.h>\n#include <stdio.h>\n"
        "int team_tag(shmem_team_t t);\nint team_tag(void *p);\n"
        "int main(void){ shmem_team_t t = SHMEM_TEAM_INVALID; int x = 0;\n"
        "  printf(\"%d %d %d\\n\", team_tag(t), team_tag((void *)&x), t == NULL); return 0; }\n")
    exe = str(tmp_path / "a.out")
    r = subprocess.run(["g++", "-std=c++17", "-Wall", "-I", INC, str(lib_tu), str(user_tu), "-o", exe],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    out = subprocess.run([exe], capture_output=True, text=True, check=True).stdout.split()
    assert out == ["2", "3", "1"], out
    bad = tmp_path / "bad.c"
    bad.write_text("#include <shmem.h>\nint main(void){ int x; shmem_team_t t = &x; return t != 0; }\n")
    r = subprocess.run(["gcc", "-std=gnu11", "-Werror=incompatible-pointer-types", "-I", INC,
                        "-c", str(bad), "-o", str(tmp_path / "bad.o")], capture_output=True, text=True)
    assert r.returncode != 0 and "incompatible" in r.stderr, r.stderr


def _hip_define(name):
    text = open("/opt/rocm/include/hip/hip_runtime_api.h").read()
    m = re.search(rf"#define {name} (0x[0-9a-fA-F]+|\d+)", text)
    assert m, name
    return int(m.group(1), 0)


def test_p2p_mapping_flags():
    """The p2p transport's cross-process mappings, against the HIP
    headers: the pair-counter segment is hipHostRegister'ed Mapped and fine-grained (not
    hipExtHostRegisterCoarseGrained, not the uncached/IO variants), and a peer's heap is
    opened with hipIpcMemLazyEnablePeerAccess (peer access to another GPU)."""
    import ctypes
    from sos_amd import _lib
    L = _lib.lib()
    reg, ipc = ctypes.c_uint(0xFFFF), ctypes.c_uint(0xFFFF)
    L.sosx_p2p_flags(ctypes.byref(reg), ctypes.byref(ipc))
    assert reg.value & _hip_define("hipHostRegisterMapped")
    for bad in ("hipExtHostRegisterCoarseGrained", "hipHostRegisterIoMemory", "hipExtHostRegisterUncached"):
        assert not reg.value & _hip_define(bad), bad
    assert ipc.value == _hip_define("hipIpcMemLazyEnablePeerAccess")


def test_small_fold_rejects_bad_args():
    """sosx_small_fold validates before any device work (CPU)."""
    import ctypes
    from sos_amd import _lib
    L = _lib.lib()
    one = (ctypes.c_void_p * 1)(1)
    flags = 1
    nb = ctypes.byref(ctypes.c_int(-1))
    assert L.sosx_small_fold(5, 23, None, one, None, 3, 1, flags, 1, nb, None) == -3       # p2 not pow2
    assert L.sosx_small_fold(5, 23, None, one, None, 1, (1 << 20) + 1, flags, 1, nb, None) == -3
    assert L.sosx_small_fold(5, 23, None, one, None, 1, 1, None, 1, nb, None) == -3        # no flags
    assert L.sosx_small_fold(5, 23, None, one, None, 1, 1, flags, 1, None, None) == -3     # no nblocks
    assert L.sosx_small_fold(0, 23, None, one, None, 1, 1, flags, 1, nb, None) == -2       # and on float
    assert L.sosx_small_fold(5, 0, None, one, None, 1, 1, flags, 1, nb, None) == -1        # SIGNED_BYTE
    assert L.sosx_small_fold(5, 23, None, one, None, 1, 0, flags, 1, nb, None) == 0        # count 0


def test_small_ring_rejects_bad_args():
    """sosx_small_ring validates before any device work (CPU)."""
    import ctypes
    from sos_amd import _lib
    L = _lib.lib()
    ins = (ctypes.c_void_p * 9)(*([1] * 9))
    nb = ctypes.c_int(-1)
    assert L.sosx_small_ring(5, 23, None, ins, 1, 1, 1, 1, ctypes.byref(nb), None) == -3        # np < 2
    assert L.sosx_small_ring(5, 23, None, ins, 9, 1, 1, 1, ctypes.byref(nb), None) == -3        # np > 8
    assert L.sosx_small_ring(5, 23, None, ins, 2, (1 << 20) + 1, 1, 1, ctypes.byref(nb), None) == -3
    assert L.sosx_small_ring(5, 23, None, ins, 2, 1, None, 1, ctypes.byref(nb), None) == -3      # no flags
    assert L.sosx_small_ring(0, 24, None, ins, 2, 1, 1, 1, ctypes.byref(nb), None) == -2         # and on double
    assert L.sosx_small_ring(5, 23, None, ins, 2, 0, 1, 1, ctypes.byref(nb), None) == 0 and nb.value == 0


def test_small_device_bytes_setter():
    """sosx_set_small_device_bytes returns the previous limit (host state only, CPU)."""
    from sos_amd import _lib
    L = _lib.lib()
    prev = L.sosx_set_small_device_bytes(12345)
    assert L.sosx_set_small_device_bytes(0) == 12345
    assert L.sosx_set_small_device_bytes(prev) == 0
    assert L.sosx_small_path_device_calls() == 0


def test_small_stage_rejects_bad_args():
    """sosx_small_stage validates before any device work (CPU)."""
    import ctypes
    from sos_amd import _lib
    L = _lib.lib()
    w = (ctypes.c_void_p * 65)(*([8] * 65))
    v = (ctypes.c_uint64 * 65)()
    assert L.sosx_small_stage(None, 16, 4, w, v, 1, None) == -3                  # no dst
    assert L.sosx_small_stage(16, None, 4, w, v, 1, None) == -3                  # no src
    assert L.sosx_small_stage(16, 16, (1 << 20) + 1, w, v, 1, None) == -3        # too large
    assert L.sosx_small_stage(16, 16, 4, w, v, 0, None) == -3                    # no posts
    assert L.sosx_small_stage(16, 16, 4, w, v, 65, None) == -3                   # > SOSX_MAX_FOLD
    assert L.sosx_small_stage(16, 16, 4, None, v, 1, None) == -3
    assert L.sosx_small_stage(16, 16, 4, w, None, 1, None) == -3
    z = (ctypes.c_void_p * 2)(8, None)
    assert L.sosx_small_stage(16, 16, 4, z, v, 2, None) == -3                    # a null word
