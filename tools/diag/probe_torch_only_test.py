"""Diagnostic pytest module: torch only (exit-time crash hunt)."""
import torch


def test_torch_only():
    t = torch.ones(1000, device="cuda")
    assert float(t.sum()) == 1000.0
