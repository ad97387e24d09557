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
    assert TB.T_NAMES == ("rccl", "rccl_ag", "p2p", "p2p_host")
    assert [TB.use_transport(S, L, t) for t in TB.T_NAMES] == [True, True, True, True]
    assert lib.calls == [("transport", 0), ("allgather", 0),
                         ("transport", 0), ("allgather", 1),
                         ("transport", 1), ("allgather", 0), ("signal", 1),
                         ("transport", 1), ("allgather", 0), ("signal", 0)]
    lib.calls.clear()
    TB.reset_transport(S, L)
    assert lib.calls == [("transport", 0), ("allgather", 0), ("signal", 1)]


def test_unavailable_transports_report_false():
    lib = _Lib({1}, stream_ok=False)   # RCCL down, stream signalling unavailable
    S = L = _Wrap(lib)
    assert [TB.use_transport(S, L, t) for t in TB.T_NAMES] == [False, False, False, True]
