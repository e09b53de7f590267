"""Gradient-producer bookkeeping of the fused optimizer (ops/optim.py FusedAdam.register_producer), on CPU tensors:
which flat-gradient ranges may be overwritten by a producer, the float4 ranges and partial slots handed to the fused
update, the static-decision rules (alignment, slot limit, env switch).  The GPU side is tests/test_gpu_extras.py::
test_mlp_grad_producers_match_accumulating_path."""
import torch

from masters_thesis_amd.ops import optim as O


def _opt(shapes, monkeypatch):
    params = [torch.nn.Parameter(torch.zeros(*s)) for s in shapes]
    flat = O.FlatParameters(params)
    opt = O.FusedAdam(flat, lr=1e-3)
    # pretend the single-launch HIP path is available (the bookkeeping is host-side only)
    opt.hip = True
    opt.single_launch = True
    opt._nparts = 16
    opt.ext_parts = torch.zeros(opt.MAX_PRODUCERS * opt._nparts)
    monkeypatch.setenv("MTA_OPTIM_PRODUCERS", "1")
    return opt, params


def test_register_ranges_and_slots(monkeypatch):
    opt, params = _opt([(8, 4), (3,), (4, 4)], monkeypatch)  # flat offsets 0, 32, 36 (float4-aligned starts)
    f = opt.flat
    offs = f.offsets
    a = opt.register_producer(params[0].grad)
    assert a is not None and a.numel() == 16 and a.data_ptr() == opt.ext_parts.data_ptr()
    # a 3-float bias is not float4-granular: refused (accumulates as usual)
    assert opt.register_producer(params[1].grad) is None
    # every parameter starts on a float4 boundary (the 3-float bias is followed by a zero gap): the third is a producer
    assert offs == [0, 32, 36] and f.padded % 4 == 0
    assert opt.register_producer(params[2].grad) is not None
    # a range that does not start on a float4 boundary is refused
    assert opt.register_producer(f.grad[33:37]) is None
    assert sorted(opt._plan.values()) == [(0, 8, 0), (9, 13, 1)]


def test_double_registration_falls_back_to_accumulation(monkeypatch):
    """a weight whose gradient GEMM runs twice before one step() (a weight used twice, two backward
    calls) must not be overwritten by the second producer: the second registration returns None (accumulate), the
    range leaves this step's covered plan (the update re-reads it for the norm and zeroes it), its slot is freed,
    and the next step covers it again."""
    opt, params = _opt([(8, 4), (4, 4), (4,)], monkeypatch)
    assert opt.register_producer(params[0].grad) is not None
    assert opt.register_producer(params[1].grad) is not None
    assert opt.register_producer(params[0].grad) is None  # second producer of the same range: accumulate
    assert opt.register_producer(params[0].grad) is None  # and any further one this step
    assert sorted(opt._plan.values()) == [(8, 12, 1)]
    # an overlapping sub-range of a covered range is a double producer too
    assert opt.register_producer(opt.flat.grad[32:36]) is None and opt._plan == {}
    # the freed slots are reused by a new range
    assert opt.register_producer(params[2].grad) is not None
    assert sorted(v[2] for v in opt._plan.values()) == [0]
    # next step: everything starts fresh
    opt._plan, opt._dropped = {}, set()
    assert opt.register_producer(params[0].grad) is not None


def test_slot_limit_and_switch(monkeypatch):
    opt, params = _opt([(4,)] * 12, monkeypatch)
    got = [opt.register_producer(p.grad) for p in params]
    assert sum(g is not None for g in got) == opt.MAX_PRODUCERS
    assert all(g is None for g in got[opt.MAX_PRODUCERS:])
    slots = sorted(v[2] for v in opt._plan.values())
    assert slots == list(range(opt.MAX_PRODUCERS))
    opt._plan = {}
    monkeypatch.setenv("MTA_OPTIM_PRODUCERS", "0")
    assert opt.register_producer(params[0].grad) is None


def test_foreign_gradient_refused(monkeypatch):
    opt, _ = _opt([(8,)], monkeypatch)
    other = torch.zeros(64)
    assert opt.register_producer(other[:8]) is None


def test_active_optimizer_hook(monkeypatch):
    opt, params = _opt([(8,)], monkeypatch)
    O.set_producer_optimizer(None)
    assert O.register_grad_producer(params[0].grad) is None
    O.set_producer_optimizer(opt)
    try:
        assert O.register_grad_producer(params[0].grad) is not None
    finally:
        O.set_producer_optimizer(None)


def test_step_hands_packed_partials_after_double_registration(monkeypatch):
    """after A (slot 0), B (slot 1) and a second registration of A, only B is covered, in slot 1.
    The kernel sums every partial it is handed, so step() must pass slots [0, 1] with A's stale slot 0 zeroed (not
    slot 0 alone, which would drop B's partials and add A's stale ones to the clip norm)."""
    opt, params = _opt([(8, 4), (4, 4)], monkeypatch)
    pa = opt.register_producer(params[0].grad)
    pb = opt.register_producer(params[1].grad)
    pa.fill_(7.0)  # A's first producer wrote its partials
    pb.fill_(1.0)  # B's producer wrote its partials
    assert opt.register_producer(params[0].grad) is None  # A again: accumulates, its range leaves the plan
    seen = {}

    class _C:
        def adam_fused(self, *a):
            seen["cov_s"], seen["cov_e"], seen["ext"], seen["ext_only"] = a[-4], a[-3], a[-2], a[-1]

    monkeypatch.setattr(O, "lib", lambda *a, **k: _C())
    opt.partials = torch.zeros(4)
    opt.ticket = torch.zeros(1, dtype=torch.int64)
    opt.step(max_norm=5.0)
    assert seen["cov_s"] == [8] and seen["cov_e"] == [12]
    ext = seen["ext"]
    assert ext.numel() == 2 * opt._nparts
    assert float(ext.sum()) == float(opt._nparts)  # B's partials only; A's stale slot zeroed
    assert seen["ext_only"] is False


def test_step_takes_the_norm_from_allreduce_partials(monkeypatch):
    """world > 1: the xGMI all-reduce's partials of the reduced gradient are the clip norm's only
    source (ext_only), and the producers' ranges are still handed over so the update leaves them unzeroed."""
    opt, params = _opt([(8, 4), (4, 4)], monkeypatch)
    assert opt.register_producer(params[0].grad) is not None
    seen = {}

    class _C:
        def adam_fused(self, *a):
            seen["cov_s"], seen["cov_e"], seen["ext"], seen["ext_only"] = a[-4], a[-3], a[-2], a[-1]

    monkeypatch.setattr(O, "lib", lambda *a, **k: _C())
    opt.partials = torch.zeros(4)
    opt.ticket = torch.zeros(1, dtype=torch.int64)
    sq = torch.ones(256)
    opt.step(max_norm=5.0, zero_grad=True, ext_norm=sq)
    assert seen["ext"] is sq and seen["ext_only"] is True
    assert seen["cov_s"] == [0] and seen["cov_e"] == [8]
    assert opt.grads_zeroed and opt._plan == {}
