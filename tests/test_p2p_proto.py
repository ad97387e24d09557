"""CPU: the p2p transport's pairing protocol, both signalling modes, under ThreadSanitizer.

tests/p2p_proto_harness.cpp runs the product's own protocol code (sosp2p::exec_host and
sosp2p::exec_stream, sos_amd/csrc/p2p_proto.h, the functions p2p.cpp calls) with the
product's plans (plan.cpp) on CPU threads: one host thread and one ordered worker ("stream") per
PE, P = 2..12, every reduction schedule, both scans, broadcasts from the first and last
PE, in and out of place, misaligned operands, each result checked.  Built with
-fsanitize=thread, a clean run means every byte a PE reads from a peer is ordered after
the peer's writes, and every overwrite after the peers' reads, by the protocol's
counters alone.  The negative control drops the drain before a
round's receives are marked consumed and must be reported.

The same runs check the consumer half of the memory-visibility rule:
the backend classifies waits and launches itself, and every launch that reads a peer's
bytes must follow an acquire issued after the wait for the peer's post.  The negative
control drops the protocol's acquires and must be caught.
"""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "tests", "build")


def _build(name, *defs):
    os.makedirs(OUT, exist_ok=True)
    exe = os.path.join(OUT, name)
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fsanitize=thread", "-pthread", *defs,
           "-I" + os.path.join(ROOT, "include"), "-I" + os.path.join(ROOT, "sos_amd", "csrc"),
           os.path.join(ROOT, "tests", "p2p_proto_harness.cpp"),
           os.path.join(ROOT, "sos_amd", "csrc", "plan.cpp"), "-o", exe]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    return exe


@pytest.fixture(scope="module")
def harness():
    return _build("p2p_proto_harness_tsan")


def test_host_protocol_race_free(harness):
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1 exitcode=66")
    r = subprocess.run([harness, "1"], capture_output=True, text=True, timeout=900, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "ThreadSanitizer" not in r.stderr, r.stderr[-4000:]
    assert "calls OK" in r.stdout and int(r.stdout.split(":")[1].split()[0]) > 8000, r.stdout
    assert "peer reads, each after an acquire" in r.stdout, r.stdout


def test_broken_protocol_is_caught():
    exe = _build("p2p_proto_harness_broken", "-DBROKEN_DRAIN")
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1 exitcode=66")
    r = subprocess.run([exe, "1"], capture_output=True, text=True, timeout=900, env=env)
    assert r.returncode != 0
    assert "ThreadSanitizer: data race" in r.stderr or "wrong result" in r.stderr, r.stderr[-3000:]


def test_missing_acquire_is_caught():
    exe = _build("p2p_proto_harness_noacq", "-DBROKEN_ACQUIRE")
    r = subprocess.run([exe, "1"], capture_output=True, text=True, timeout=900)
    assert r.returncode != 0
    assert "peer read without an acquire" in r.stderr, r.stderr[-3000:]
