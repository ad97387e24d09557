"""CPU: tools/oshrun + the TCP bootstrap of shmem_init() (rank discovery, PE 0's
broadcast, all-gather), and oshrun's abort propagation (PMI_Abort semantics)."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OSHRUN = os.path.join(ROOT, "tools", "oshrun")

PROBE = r"""
import ctypes, sys
L = ctypes.CDLL(sys.argv[1])
r, s, tok = ctypes.c_int(), ctypes.c_int(), ctypes.c_ulonglong()
ranks = (ctypes.c_int * 64)()
rc = L.sosx_bootstrap_probe(ctypes.byref(r), ctypes.byref(s), ranks, 64, ctypes.byref(tok))
assert rc == 0, rc
assert list(ranks[:s.value]) == list(range(s.value)), list(ranks[:s.value])
assert tok.value == 0x5EED0000 + s.value
print("PE", r.value, "of", s.value, "ok")
"""


def test_oshrun_bootstrap_exchange(tmp_path):
    script = tmp_path / "probe.py"
    script.write_text(PROBE)
    lib = os.path.join(ROOT, "sos_amd", "libsos_amd.so")
    for np_ in (1, 3, 8):
        r = subprocess.run([sys.executable, OSHRUN, "-np", str(np_), "--timeout", "60",
                            sys.executable, str(script), lib], capture_output=True, text=True,
                           timeout=120)
        assert r.returncode == 0, r.stderr
        assert sorted(r.stdout.split("\n")[:-1]) == sorted(f"PE {i} of {np_} ok" for i in range(np_))


def test_oshrun_abort_propagates(tmp_path):
    script = tmp_path / "abort.py"
    script.write_text("import os, sys, time\n"
                      "if os.environ['SHMEM_PE'] == '1': sys.exit(3)\n"
                      "time.sleep(30)\n")
    r = subprocess.run([sys.executable, OSHRUN, "-np", "4", sys.executable, str(script)],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 3
