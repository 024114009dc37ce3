"""Host-side logic of the ordered lanes (no GPU): which lane runs which
epoch / group across calls (the tickets dv_lanes_order expects: lane l's
m-th execution is ticket m * L + l), and which error a failed call raises."""
import threading

import pytest

import dvcc
from dvcc import _lib as L
from dvcc.engine import CCEngine


class _Lane:
    def __init__(self, ix, log):
        self.ix, self.log = ix, log


def _owner(nl):
    eng = CCEngine.__new__(CCEngine)
    eng._ctx = None
    log = []
    eng._order = [_Lane(i, log) for i in range(nl)]
    eng._order_next = 0
    return eng, log


def test_run_ordered_lane_assignment_continues_across_calls():
    eng, log = _owner(4)
    lock = threading.Lock()
    seen, base = [], [0]

    def call(ctx, i):
        with lock:
            seen.append((ctx.ix, base[0] + i))  # (the epoch's place in the whole sequence)
        return (ctx.ix, i)
    out = eng.run_ordered(6, call)  # epochs 0..5 -> lanes 0,1,2,3,0,1
    assert out == [(0, 0), (1, 1), (2, 2), (3, 3), (0, 4), (1, 5)]
    base[0] = 6
    out = eng.run_ordered(3, call)  # the next call starts at lane 2
    assert out == [(2, 0), (3, 1), (0, 2)]
    # every epoch k ran on lane k % 4, and every lane ran its epochs in order
    assert all(x == k % 4 for x, k in seen)
    for ln in range(4):
        mine = [k for (x, k) in seen if x == ln]
        assert mine == sorted(mine)
    assert eng._order_next == 1


def test_run_ordered_raises_the_failing_epochs_error_first():
    eng, _ = _owner(2)

    def call(ctx, i):
        if i == 2:
            raise dvcc.DvccError(L.DV_ERR_KEY_NOT_FOUND, "probe")
        if i > 2:
            raise dvcc.DvccError(L.DV_ERR_STATE, "order ended")
        return i
    with pytest.raises(dvcc.DvccError) as ei:
        eng.run_ordered(5, call)
    assert ei.value.code == L.DV_ERR_KEY_NOT_FOUND
