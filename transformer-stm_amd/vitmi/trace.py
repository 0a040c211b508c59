"""ROCTx ranges around the training step's phases (SURVEY.md §5 profiling; the reference's
counterpart is the TensorBoard callback, models/CvT(Par).py:472,476).

``enable()`` binds the ROCm marker library through the C ABI (vitmi_trace_enable); then
``with trace.range("forward"): ...`` shows up as a region in ``rocprofv3 --marker-trace``.
Disabled (the default) a range costs one Python branch."""
from __future__ import annotations

from contextlib import contextmanager

from ._lib import check, lib

_on = False


def enable(on: bool = True) -> None:
    global _on
    check(lib().vitmi_trace_enable(int(on)), "trace_enable")
    _on = bool(on)


def enabled() -> bool:
    return _on


@contextmanager
def range(name: str):  # noqa: A001  (roctx vocabulary)
    if not _on:
        yield
        return
    lib().vitmi_trace_push(name.encode())
    try:
        yield
    finally:
        lib().vitmi_trace_pop()
