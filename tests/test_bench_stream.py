"""bench.py's frame streaming (CPU): with split calls (finish lagging 1 .. n-1 frames behind begin)
every frame is begun, finished and retired exactly once, in frame order per context, a context
never holds two frames, and a frame is finished before it is retired (the C-ABI returns
SM_ERR_STATE otherwise)."""
import pytest

torch = pytest.importorskip("torch")
import bench  # noqa: E402


class FakeCtx:
    def __init__(self, k, log):
        self.k, self.log, self.frame, self.state, self.next = k, log, None, "idle", 0

    def match_begin(self, D, params):
        assert self.state == "idle", "begin on a context that still holds a frame"
        self.state = "begun"
        self.log.append(("begin", self.k))

    def match_finish(self):
        assert self.state == "begun", "finish without begin"
        self.state = "finished"
        self.log.append(("finish", self.k))

    def match_async(self, D, params):
        self.match_begin(D, params)
        self.match_finish()


@pytest.mark.parametrize("n", [1, 2, 3, 4])
@pytest.mark.parametrize("steps", [0, 1, 2, 3, 7, 12])
@pytest.mark.parametrize("split", [True, False])
@pytest.mark.parametrize("lag", [1, 2, 3])
def test_stream_frames_order(n, steps, split, lag):
    log = []
    ctxs = [FakeCtx(k, log) for k in range(n)]

    def retire(c):
        assert c.state == "finished", "retire before finish"
        c.state = "idle"
        log.append(("retire", c.k))

    bench.stream_frames(ctxs, steps, 64, None, retire, split=split, lag=lag)
    assert all(c.state == "idle" for c in ctxs)
    for what in ("begin", "finish", "retire"):
        seq = [k for w, k in log if w == what]
        assert seq == [i % n for i in range(steps)], what  # every frame once, in frame order
    if split and n > 1 and steps > 1:
        # frame i+1's tree is enqueued before frame i's filter
        assert log.index(("begin", 1)) < log.index(("finish", 0))
