"""CPU tests of the facade's host logic (no GPU calls): the reference retrain procedures
of MF / NCF, the RQ2 stage timers, the maxinf on-disk influence vector, and the solver
choice."""
import os

import numpy as np
import pytest

from influence import experiments
from influence.genericNeuralNet import rq2_timing
from influence.matrix_factorization import MF
from influence.NCF import NCF


class StubTrainer(object):
    """Records the calls a retrain makes (the real trainer is torch on the GPU)."""

    class Opt(object):
        def __init__(self, log):
            self.log = log

        def reset(self):
            self.log.append(("reset",))

    def __init__(self):
        self.log = []
        self.opt = StubTrainer.Opt(self.log)

    def step(self, users, items, labels):
        self.log.append(("step", np.asarray(users).copy(), np.asarray(items).copy(), np.asarray(labels).copy()))

    def full_batch(self, users, items, labels, n):
        self.log.append(("full", len(users), n))


def _bare(cls, batch_size):
    m = cls.__new__(cls)          # no GPU context: only host-side methods are exercised
    m.batch_size = batch_size
    m._tr = StubTrainer()
    return m


def _feed(n):
    return {"users": np.arange(n, dtype=np.int64), "items": np.arange(n, dtype=np.int64) % 5,
            "labels": np.arange(n, dtype=np.float32)}


@pytest.mark.parametrize("cls,resets", [(MF, True), (NCF, False)])
def test_retrain_is_reference_minibatch(cls, resets):
    """MF.retrain (mf:69-76): reset_optimizer_op, then num_steps steps on next_batch(batch_size)
    of a fresh DataSet of the feed rows; NCF.retrain (NCF.py:68-72): the same without the reset."""
    m = _bare(cls, 4)
    np.random.seed(0)
    m.retrain(5, _feed(10))
    log = m._tr.log
    if resets:
        assert log[0] == ("reset",)
        log = log[1:]
    assert [e[0] for e in log] == ["step"] * 5
    sizes = [e[1].size for e in log]
    assert sizes[:3] == [4, 4, 2]                     # sequential batches, short last one (dataset.py:49-70)
    assert np.array_equal(log[0][1], np.arange(4)) and np.array_equal(log[1][1], np.arange(4, 8))
    assert np.array_equal(log[0][3], np.arange(4, dtype=np.float64))
    # then the epoch wrap: batches of a global-np.random permutation of the rows (dataset.py:60-66)
    np.random.seed(0)
    perm = np.arange(10)
    np.random.shuffle(perm)
    assert np.array_equal(np.concatenate([log[3][1], log[4][1]]), perm[:8])


def test_full_batch_retrain_stays_available():
    m = _bare(MF, 4)
    m.retrain_full_batch(7, _feed(10))
    assert m._tr.log == [("full", 10, 7)]


def test_rq2_stage_timers():
    """The three prints of mf:224-250 from the library's phase sums (ms, count)."""
    lines = []
    phases = {"prepare": (0.0, 0), "solve": (2.0, 1), "score": (5.0, 1), "topk": (0.5, 1), "chunks": (1.0, 1)}
    t = rq2_timing(phases, 1234, 0.25, log=lines.append)
    for key in ("inverse_hvp_s", "multiply_s", "total_s", "wall_s", "n"):
        assert key in t
    assert t["inverse_hvp_s"] == pytest.approx(3.0e-3) and t["multiply_s"] == pytest.approx(5.5e-3)
    assert t["total_s"] == pytest.approx(8.5e-3) and t["n"] == 1234
    assert lines[0].startswith("Inverse HVP took ")
    assert lines[1].startswith("Multiplying by 1234 train examples took ")
    assert lines[2].startswith("Total time is ")


class StubModel(object):
    """get_influence_batch of one query with a known influence vector."""

    def __init__(self, tmpdir, infl, rel):
        self.train_dir = str(tmpdir)
        self.model_name = "stub_MF"
        self.infl = np.asarray(infl, np.float64)
        self.rel = np.asarray(rel, np.int64)

    def get_influence_batch(self, test_indices, K=1, full=True, return_x=True):
        from oracle import fia_oracle as fo
        pos = fo.topk(self.infl, K)
        pad = K - pos.size
        return {"offsets": np.array([0, self.infl.size]), "rel_idx": self.rel, "influence": self.infl,
                "topk_pos": np.concatenate([pos, -np.ones(pad, np.int64)])[None],
                "topk_idx": np.concatenate([self.rel[pos], -np.ones(pad, np.int64)])[None],
                "topk_val": np.concatenate([self.infl[pos], np.full(pad, np.nan)])[None]}


def test_maxinf_writes_total_y_diffs(tmp_path):
    """experiments.py:43: the full predicted vector of a maxinf query goes to
    <train_dir>/<model_name>-[<t>]-_total_y_diffs.npy before the top-K is taken."""
    infl = np.array([0.1, -0.7, 0.3, 0.7, -0.2])
    m = StubModel(tmp_path, infl, [10, 11, 12, 13, 14])
    vals, pos, rows = experiments.maxinf(m, 42, num_to_remove=2)
    path = os.path.join(str(tmp_path), "stub_MF-[42]-_total_y_diffs.npy")
    assert path == experiments.total_y_diffs_path(m, 42)
    assert os.path.exists(path)
    assert np.array_equal(np.load(path, allow_pickle=False), infl)
    assert list(pos) == [1, 3] and list(rows) == [11, 13] and list(vals) == [-0.7, 0.7]   # tie: lower position first
    assert np.array_equal(m.train_indices_of_test_case, [10, 11, 12, 13, 14])


def test_lissa_is_refused_not_ignored():
    """gnn:503-508 would run LiSSA; this build has only the exact solve and says so."""
    m = _bare(MF, 4)
    with pytest.raises(NotImplementedError):
        m.get_influence_on_test_loss([0], np.arange(3), approx_type="lissa")
    with pytest.raises(ValueError):
        m.get_influence_on_test_loss([0], np.arange(3), approx_type="newton")


def test_profiled_call_keeps_caller_profiling_state():
    """get_influence_on_test_loss times its own call (RQ2 timers) through
    Context.profiled_call: the caller's phase mask is restored and the sums it had
    accumulated but not read are still returned by its next profile_read."""
    from influence import _lib

    class FakeLib:
        def __init__(self):
            self.mask, self.pending = 0, [0.0] * _lib.FIA_NUM_PHASES

        def fia_set_profiling(self, h, mask):
            self.mask = mask
            return 0

        def run(self, ms):                      # a library call: records the enabled phases
            for p in range(_lib.FIA_NUM_PHASES):
                if self.mask >> p & 1:
                    self.pending[p] += ms

        def fia_profile_read(self, h, ms, cnt):
            for p in range(_lib.FIA_NUM_PHASES):
                ms[p], cnt[p] = self.pending[p], int(self.pending[p] > 0)
            self.pending = [0.0] * _lib.FIA_NUM_PHASES
            return 0

    ctx = object.__new__(_lib.Context)
    ctx.lib, ctx.h, ctx._mask, ctx._carry = FakeLib(), None, 0, None
    ctx.set_profiling(True, phases=("score",))
    ctx.lib.run(2.0)                            # the caller's own measurement, not yet read
    res, mine = ctx.profiled_call(lambda: ctx.lib.run(5.0) or "r")
    assert res == "r"
    assert mine["score"][0] == 5.0 and mine["solve"][0] == 5.0     # every phase during the call
    assert ctx._mask == 1 << _lib.PHASES.index("score")             # caller's mask restored
    ctx.lib.run(1.0)
    after = ctx.profile_read()
    assert after["score"][0] == 3.0 and after["solve"][0] == 0.0    # 2 (before) + 1 (after)
