"""Fork/join guard for HIP-graph capture.

HIP's stream capture handles one level of fork/join: streams forked from the capture's
origin stream (``side.wait_stream(origin)``) and joined back into it
(``origin.wait_stream(side)``).  A stream forked from a forked stream, or a wait between
two forked streams, made ``hipStreamEndCapture`` segfault on this image
(``tools/micro/nested_fork_probe.py``; DESIGN.md §7b, the reverted detector/descriptor
split).  ``guard(origin)`` wraps a capture: every cross-stream wait issued from Python
(``Stream.wait_stream`` / ``Stream.wait_event`` with an event recorded through
``Event.record``) must have the origin stream on one side, otherwise it raises before the
capture can reach the crash.  Waits that autograd issues in C++ during a captured backward
mirror the forward's (Python) fork structure, so checking the forward's is sufficient.
"""
from __future__ import annotations

import contextlib
import threading


class NestedForkError(RuntimeError):
    pass


class ForkJoinChecker:
    """The rule itself, on any stream objects that compare with ==."""

    def __init__(self, origin):
        self.origin = origin
        self.waits = []  # (waiter, waited) in order, for tests and diagnostics

    def check(self, waiter, waited):
        self.waits.append((waiter, waited))
        if waiter == waited or waiter == self.origin or waited == self.origin:
            return
        raise NestedForkError(
            "graph capture: a wait between two side streams (%r waits on %r); only forks from "
            "and joins into the capture's origin stream are allowed (hipStreamEndCapture "
            "crashes on nested fork topologies)" % (waiter, waited))


_ACTIVE = threading.local()


@contextlib.contextmanager
def guard(origin, stream_cls=None, event_cls=None):
    """Inside: every Stream.wait_event / wait_stream is checked against the fork/join rule
    with ``origin`` the capture's stream.  stream_cls / event_cls default to torch.cuda's
    (the CPU test passes stubs with the same methods)."""
    if stream_cls is None or event_cls is None:
        import torch
        stream_cls = stream_cls or torch.cuda.Stream
        event_cls = event_cls or torch.cuda.Event
    checker = ForkJoinChecker(origin)
    prev = getattr(_ACTIVE, "checker", None)
    _ACTIVE.checker = checker
    orig_record, orig_wait_event = event_cls.record, stream_cls.wait_event

    def record(ev, stream=None):
        if stream is None:
            import torch
            stream = torch.cuda.current_stream()
        ev._hreg_stream = stream
        return orig_record(ev, stream)

    def wait_event(st, ev):
        src = getattr(ev, "_hreg_stream", None)
        c = getattr(_ACTIVE, "checker", None)
        if src is not None and c is not None:
            c.check(st, src)
        return orig_wait_event(st, ev)

    event_cls.record, stream_cls.wait_event = record, wait_event
    try:
        yield checker
    finally:
        event_cls.record, stream_cls.wait_event = orig_record, orig_wait_event
        _ACTIVE.checker = prev


def capture_origin():
    """The origin stream of the guarded capture in progress on this thread, or None."""
    c = getattr(_ACTIVE, "checker", None)
    return None if c is None else c.origin


@contextlib.contextmanager
def graph(g, pool=None, capture_error_mode="global"):
    """``torch.cuda.graph(g, pool)`` with the fork/join guard on its capture stream.  (r4: an
    explicit hipGraphUpload after each capture made the driver's --steps 20 line 2.5 % slower,
    6853 / 6823 / 6998 vs 7041 / 7034 / 7071 pairs/s on one box, and was removed.)
    capture_error_mode "thread_local": other threads' HIP calls stay legal during the capture --
    the RCCL process group's watchdog thread queries its work events at any time, and in the
    default global mode that query fails the capture and the watchdog terminates the process
    ("operation not permitted when stream is capturing", r5's 1-rank RCCL test)."""
    import torch
    with torch.cuda.graph(g, pool=pool, capture_error_mode=capture_error_mode):
        with guard(torch.cuda.current_stream()):
            yield
