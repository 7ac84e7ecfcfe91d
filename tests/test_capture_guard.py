"""The fork/join guard of graph captures (pcd_reg_hregnet_amd/capture.py; VERDICT r3 weak
item 7): forks from and joins into the capture's origin stream pass, a wait between two side
streams (a stream forked from a forked stream) raises before hipStreamEndCapture could crash.
CPU only: stub streams / events with torch.cuda's method shapes."""
import pytest

from pcd_reg_hregnet_amd import capture


class StubStream:
    def __init__(self, name):
        self.name = name
        self.log = []

    def __eq__(self, o):
        return isinstance(o, StubStream) and o.name == self.name

    def __hash__(self):
        return hash(self.name)

    def __repr__(self):
        return self.name

    def wait_event(self, ev):
        self.log.append(ev)

    def record_event(self):
        ev = StubEvent()
        ev.record(self)
        return ev

    def wait_stream(self, other):  # torch.cuda.Stream.wait_stream's shape
        self.wait_event(other.record_event())


class StubEvent:
    def record(self, stream=None):
        self.stream = stream


def _guard(origin):
    return capture.guard(origin, stream_cls=StubStream, event_cls=StubEvent)


def test_fork_and_join_on_origin_pass():
    o, a, b = StubStream("origin"), StubStream("a"), StubStream("b")
    with _guard(o) as chk:
        a.wait_stream(o)      # fork
        b.wait_stream(o)      # fork
        o.wait_stream(a)      # join
        o.wait_stream(b)      # join
        a.wait_stream(o)      # re-fork after a join (train_graph's queued running updates)
        ev = StubEvent()
        ev.record(a)
        o.wait_event(ev)      # join through an explicit event
    assert len(chk.waits) == 6
    # the patch is undone on exit: no check outside the capture
    a.wait_stream(b)


@pytest.mark.parametrize("case", ["nested", "side_to_side_event"])
def test_nested_fork_raises(case):
    o, a, b = StubStream("origin"), StubStream("a"), StubStream("b")
    with _guard(o):
        a.wait_stream(o)
        with pytest.raises(capture.NestedForkError):
            if case == "nested":
                b.wait_stream(a)  # b forked from the forked stream a
            else:
                ev = StubEvent()
                ev.record(b)
                a.wait_event(ev)


def test_checker_rule():
    chk = capture.ForkJoinChecker("o")
    chk.check("x", "o")
    chk.check("o", "x")
    chk.check("x", "x")
    with pytest.raises(capture.NestedForkError):
        chk.check("x", "y")


def test_capture_origin_exposed_inside_guard_only():
    """engine._fork_begin forks only from the capture's origin (capture_origin) and never
    inside a capture without a caller-owned side stream."""
    o = StubStream("origin")
    assert capture.capture_origin() is None
    with _guard(o):
        assert capture.capture_origin() == o
        with _guard(StubStream("inner")):
            assert capture.capture_origin() == StubStream("inner")
        assert capture.capture_origin() == o
    assert capture.capture_origin() is None
