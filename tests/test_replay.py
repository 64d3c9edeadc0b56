"""pm_amd.replay's collective stand-in (ReplayDist) on the CPU: it hands each
collective its recorded result in call order, checks the rank's own
contribution against the recording, and refuses a call sequence that differs
from the recorded one. (The recording itself and the rank frames run on the
GPU: tests/test_gpu_fullscale.py.)"""
import pytest

torch = pytest.importorskip("torch")


def _recording(world=2):
    from pm_amd.replay import Recording
    rec = Recording(world)
    rows = torch.arange(world * 3 * 6, dtype=torch.float32).reshape(world * 3, 6)
    ins = [torch.tensor([r + 1, 10 * r], dtype=torch.int64) for r in range(world)]
    red = torch.stack(ins).sum(0)
    tags = [torch.tensor([5 * r, 5 * r + 1, -7], dtype=torch.int32) for r in range(world)]   # -7: padding
    rec.plan_sizes = [2, 2] if world == 2 else [2] * world
    rec.ops = [("counts", [3] * world), ("rows", (rows, 3)), ("reduce", ("sum", ins, red)),
               ("tags", (tags, torch.cat(tags)))]
    return rec, rows, ins, red, tags


def test_replay_hands_back_recorded_results():
    from pm_amd.replay import ReplayDist
    rec, rows, ins, red, tags = _recording()
    for r in range(2):
        d = ReplayDist(rec, r)
        ns = [torch.zeros(1, dtype=torch.int64) for _ in range(2)]
        d.all_gather(ns, torch.tensor([3]))
        assert [int(x) for x in ns] == [3, 3]
        out = torch.empty_like(rows)
        w = d.all_gather_into_tensor(out, rows[r * 3:(r + 1) * 3].clone(), async_op=True)
        assert w.wait() and torch.equal(out, rows)
        buf = ins[r].clone()
        d.all_reduce(buf, op=d.ReduceOp.SUM)
        assert torch.equal(buf, red)
        everyone = torch.empty(6, dtype=torch.int32)
        mine = tags[r].clone()
        mine[2] = 99   # the padding past the rank's load is not compared
        d.all_gather_into_tensor(everyone, mine)
        assert torch.equal(everyone, torch.cat(tags))
        img = torch.full((2, 2), r + 1, dtype=torch.int32)
        d.reduce(img, dst=0, op=d.ReduceOp.SUM)
        assert d.done() and torch.equal(d.image, img)


def test_replay_refuses_a_different_contribution_or_order():
    from pm_amd.replay import ReplayDist
    rec, rows, ins, red, tags = _recording()
    d = ReplayDist(rec, 1)
    with pytest.raises(AssertionError):
        d.all_gather([torch.zeros(1, dtype=torch.int64)] * 2, torch.tensor([4]))   # wrong count
    d = ReplayDist(rec, 0)
    with pytest.raises(AssertionError):
        d.all_reduce(ins[0].clone(), op=d.ReduceOp.SUM)   # counts were recorded first
    d = ReplayDist(rec, 0)
    d.all_gather([torch.zeros(1, dtype=torch.int64)] * 2, torch.tensor([3]))
    bad = rows[0:3].clone()
    bad[1, 2] += 1
    with pytest.raises(AssertionError):
        d.all_gather_into_tensor(torch.empty_like(rows), bad)   # different photon rows
    assert not d.done()
