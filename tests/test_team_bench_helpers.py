"""CPU: the N > 1 bench's helpers (tools/team_bench.py) against fakes: transport
switching (each measured transport selects the library transport and, for p2p, the
signalling mode; an unavailable one reports False; reset restores rccl + stream mode),
the preflight job's verdicts, and which transport `value` may come from."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import team_bench as TB  # noqa: E402


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
            assert cmd[-1] == "--preflight" and cmd[-2].endswith(os.path.join("tools", "team_bench.py"))
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


def _res(t_step, mismatches, available=True):
    return {"t_step": t_step, "mismatches": mismatches, "available": available}


def test_value_never_from_rccl_allreduce():
    """rccl_ar is RCCL's own ncclAllReduce: even clean and fastest it never gives `value`."""
    results = {"rccl": _res(3.0, 0), "rccl_ag": _res(2.9, 0), "p2p": _res(2.5, 0),
               "p2p_host": _res(2.7, 0), "rccl_ar": _res(1.0, 0)}
    assert TB.select_primary(results) == ("p2p", None)
    results["p2p"] = _res(2.5, 4)          # a failed check is never `value` either
    assert TB.select_primary(results) == ("p2p_host", None)
    assert "rccl_ar" not in TB.VALUE_T


def test_value_null_when_every_check_fails():
    results = {"rccl": _res(3.0, 1), "rccl_ag": _res(2.9, 7), "p2p": {"available": False},
               "p2p_host": {"available": False}, "rccl_ar": _res(1.0, 0)}
    primary, why = TB.select_primary(results)
    assert primary is None and "rccl 1" in why and "rccl_ag 7" in why
    primary, why = TB.select_primary({"rccl_ar": _res(1.0, 0), "p2p": {"available": False}})
    assert primary is None and "available" in why


def test_workload_names_what_ran():
    assert "ncclAllGather" in TB.workload_text("rccl_ag", "float", "sum", 8, 2)
    assert "host-signalled" in TB.workload_text("p2p_host", "float", "sum", 8, 2)
    assert "no valid measurement" in TB.workload_text(None, "float", "sum", 8, 2)


def test_workload_names_the_device_map():
    """config.workload / parallelism come from the distinct GPUs the ranks reported: the
    8-GPU node's line says 1 PE per MI355X, a one-GPU rehearsal says the GPU is shared."""
    one_per = TB.workload_text("rccl", "float", "sum", 8, 8, 8)
    assert "8 PEs on 8 GPUs (1 per MI355X)" in one_per
    shared = TB.workload_text("p2p", "float", "sum", 8, 8, 1)
    assert "8 PEs on 1 GPU (shared" in shared and "1 per MI355X" not in shared
    assert TB.parallelism_text(8, 8) == "pe8" and TB.parallelism_text(8, 1) == "pe8_on_1gpu"
    assert "4 PEs on 2 GPUs (shared" in TB.workload_text("p2p", "float", "sum", 8, 4, 2)


def test_headline_fields_n2():
    """The N > 1 line's rate fields at N = 2 with a 2-rank RCCL communicator (what the
    stand-in's ncclCommCount reports): value = both PEs' payload per step, algbw_GiBs =
    one PE's vector per step, the definition stated in the line."""
    f = TB.headline_fields(2, 1 << 20, 4, 0.001, [2, 2])
    assert f["n_gpus"] == 2 and f["rccl_comm_ranks"] == [2, 2]
    assert abs(f["value"] - 2 * 4 * (1 << 20) / 0.001 / TB.GiB) < 1e-3
    assert abs(f["algbw_GiBs"] * 2 - f["value"]) < 1e-2
    assert "1->8 scaling curve plots this" in f["value_definition"]
    none = TB.headline_fields(2, 8, 4, None, [-1, -1])
    assert none["value"] is None and none["algbw_GiBs"] is None and none["rccl_comm_ranks"] == [-1, -1]


def test_xgmi_fractions_null_when_ranks_share_a_gpu():
    """N = 2 ranks on one device: no xGMI link carries the bytes, so the line carries no
    link roofline (bound "shared-gpu", fractions null) however fast the step was -- round
    5's line printed frac_one_link 7.4 there.  With one GPU per rank the fractions are
    the link rates' (and a real step cannot exceed 7 links)."""
    wire = 2 * (2 - 1) / 2 * (128 << 20) * 4
    fast = 1e-5  # far faster than any link: only a shared device can do that
    f = TB.xgmi_fields(wire, fast, world=2, ngpus=1)
    assert f["frac_one_link"] is None and f["frac_7_links"] is None and f["busbw_GBs"] > 0
    assert TB.team_bound(2, 1) == "shared-gpu" and TB.team_bound(8, 8) == "xgmi"
    g = TB.xgmi_fields(wire, 0.01, world=2, ngpus=2)
    assert abs(g["frac_one_link"] - wire / 0.01 / 1e9 / TB.XGMI_LINK_GBS) < 1e-3
    assert 0 < g["frac_7_links"] < g["frac_one_link"] <= 1
