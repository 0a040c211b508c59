"""The bf16 gradient hand-over between fused backwards (vitmi/modules.py: _handover /
_take_lp) on the CPU, with the device cast replaced by torch's: a copy is used only by the
tensor object it was attached to and only while that tensor is unmodified.  Round 2 keyed
the copies by data_ptr(), so an unrelated gradient that the caching allocator later placed
at the same address silently received a stale copy; these cases pin the replacement."""
import torch

from vitmi import modules

BF = torch.bfloat16


def _patch(monkeypatch):
    casts = []

    def cast(t, dst=None):
        casts.append(t)
        return t.to(BF)
    monkeypatch.setattr(modules.ops, "cast_bf16", cast)
    return casts


def test_same_object_unmodified_uses_the_copy(monkeypatch):
    casts = _patch(monkeypatch)
    g = torch.randn(6, 4)
    lp = torch.full((6, 4), 7.0, dtype=BF)          # deliberately not g's values
    modules._handover(g, lp)
    got = modules._take_lp(g.view(6, 4), BF, g)
    assert got.data_ptr() == lp.data_ptr() and not casts
    # taken once: a second consumer casts
    again = modules._take_lp(g, BF)
    assert torch.equal(again, g.to(BF)) and len(casts) == 1


def test_in_place_update_invalidates_the_copy(monkeypatch):
    casts = _patch(monkeypatch)
    g = torch.randn(6, 4)
    modules._handover(g, g.to(BF))
    g.add_(1.0)                                      # e.g. autograd accumulating in place
    got = modules._take_lp(g, BF)
    assert torch.equal(got, g.to(BF)) and len(casts) == 1


def test_other_tensor_at_same_address_never_sees_the_copy(monkeypatch):
    casts = _patch(monkeypatch)
    g = torch.randn(6, 4)
    modules._handover(g, torch.zeros(6, 4, dtype=BF))
    alias = g.view(6, 4)                             # same storage and data_ptr, other object
    assert alias.data_ptr() == g.data_ptr()
    got = modules._take_lp(alias, BF)
    assert torch.equal(got, g.to(BF)) and len(casts) == 1


def test_fp32_is_passthrough(monkeypatch):
    casts = _patch(monkeypatch)
    g = torch.randn(3, 3)
    assert modules._take_lp(g, torch.float32) is g and not casts
