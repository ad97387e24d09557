"""CPU: the N > 1 bench's transport switching (sos_amd/team_bench.py) against a fake
library: each measured transport selects the library transport and, for p2p, the
signalling mode; an unavailable one reports False; reset restores rccl + host mode."""
from sos_amd import team_bench as TB


class _Lib:
    def __init__(self, transports_ok, stream_ok):
        self.calls = []
        self.transports_ok, self.stream_ok = transports_ok, stream_ok

    def shmemx_set_transport(self, tid):
        self.calls.append(("transport", tid))
        return 0 if tid in self.transports_ok else -1

    def sosx_set_rccl_allgather(self, on):
        self.calls.append(("allgather", on))
        return 0

    def sosx_set_rccl_allreduce(self, mode):
        self.calls.append(("allreduce", mode))
        return 0

    def sosx_set_p2p_signal_mode(self, mode):
        self.calls.append(("signal", mode))
        return -1 if (mode == 1 and not self.stream_ok) else 0


class _Wrap:
    def __init__(self, lib):
        self._lib = lib

    def lib(self):
        return self._lib


def test_use_transport_selects_transport_and_signal_mode():
    lib = _Lib({0, 1}, stream_ok=True)
    S = L = _Wrap(lib)
    assert TB.T_NAMES == ("rccl", "rccl_ag", "p2p", "p2p_host", "rccl_ar")
    assert [TB.use_transport(S, L, t) for t in TB.T_NAMES] == [True] * 5
    assert lib.calls == [("transport", 0), ("allgather", 0), ("allreduce", 0),
                         ("transport", 0), ("allgather", 1), ("allreduce", 0),
                         ("transport", 1), ("allgather", 0), ("allreduce", 0), ("signal", 1),
                         ("transport", 1), ("allgather", 0), ("allreduce", 0), ("signal", 0),
                         ("transport", 0), ("allgather", 0), ("allreduce", 2)]
    lib.calls.clear()
    TB.reset_transport(S, L)
    assert lib.calls == [("transport", 0), ("allgather", 0), ("allreduce", 0), ("signal", 1)]


def test_unavailable_transports_report_false():
    lib = _Lib({1}, stream_ok=False)   # RCCL down, stream signalling unavailable
    S = L = _Wrap(lib)
    assert [TB.use_transport(S, L, t) for t in TB.T_NAMES] == [False, False, False, True, False]


class _Dist:
    """gloo stand-in for one rank: all_reduce(MIN) leaves the tensor as it is."""
    class ReduceOp:
        MIN = "min"

    def all_reduce(self, t, op=None):
        assert op == "min"


def _run_preflight(monkeypatch, stdout, rc=0, timeout=False):
    import subprocess
    import torch

    class FakePopen:
        def __init__(self, cmd, cwd=None, env=None, stdout=None, stderr=None):
            assert cmd[-3:] == ["-m", "sos_amd.team_bench", "--preflight"]
            assert env["MASTER_PORT"] == str(29500 + TB.PREFLIGHT_PORT_OFFSET)
            assert env["SHMEMX_P2P_TIMEOUT"] == "20"
            stdout.write(out_text)
            stdout.flush()
            self.returncode = None
            self.killed = False

        def poll(self):
            if not timeout:
                self.returncode = rc
            return self.returncode

        def kill(self):
            self.killed = True
            self.returncode = -9

        def wait(self):
            return self.returncode

    out_text = stdout
    monkeypatch.setattr(subprocess, "Popen", FakePopen)
    monkeypatch.setattr(TB, "PREFLIGHT_LIMIT_S", 0.5)
    monkeypatch.setenv("MASTER_PORT", "29500")
    monkeypatch.delenv("SOSX_BENCH_PREFLIGHT", raising=False)
    return TB.preflight(torch, _Dist(), 0, 2)


def test_preflight_all_clean(monkeypatch):
    out = "".join(f'{{"t": "{t}", "ok": true}}\n' for t in TB.T_NAMES)
    pre = _run_preflight(monkeypatch, out)
    assert pre["ran"] and all(pre["ok"].values()) and pre["why"] == "ok"


def test_preflight_child_died_mid_way(monkeypatch):
    """The child ended (a p2p wait's _exit) after reporting rccl/rccl_ag: the transport it
    died in and every one it never reached count as failed."""
    out = 'noise\n{"t": "rccl", "ok": true}\n{"t": "rccl_ag", "ok": true}\n'
    pre = _run_preflight(monkeypatch, out, rc=1)
    assert pre["ok"] == {"rccl": True, "rccl_ag": True, "p2p": False, "p2p_host": False,
                         "rccl_ar": False}
    assert pre["why"] == "child rc=1"


def test_preflight_mismatch_and_timeout(monkeypatch):
    out = ('{"t": "rccl", "ok": true}\n{"t": "rccl_ag", "ok": false, "mismatches": 3}\n'
           '{"t": "p2p", "ok": true}\n')
    pre = _run_preflight(monkeypatch, out, timeout=True)
    assert pre["ok"] == {"rccl": True, "rccl_ag": False, "p2p": True, "p2p_host": False,
                         "rccl_ar": False}
    assert pre["why"] == "child killed after 0 s"


def test_preflight_disabled_transports_are_skipped():
    lib = _Lib({0, 1}, stream_ok=True)
    S = L = _Wrap(lib)
    TB.DISABLED.update({"p2p", "rccl_ag"})
    try:
        assert [TB.use_transport(S, L, t) for t in TB.T_NAMES] == [True, False, False, True, True]
    finally:
        TB.DISABLED.clear()


def test_preflight_off(monkeypatch):
    import torch
    monkeypatch.setenv("SOSX_BENCH_PREFLIGHT", "0")
    pre = TB.preflight(torch, _Dist(), 0, 2)
    assert not pre["ran"] and all(pre["ok"].values())
