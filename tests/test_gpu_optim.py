"""The fused optimizer tail of round 6 (csrc/optim.hip) against the single-purpose launches it
replaced and plain torch: one slab-reduction launch for several slabs (wide and narrow), the
gradient assembly with its finite check and statistics row, both Adam groups in one launch, and the
optimizer commit inside the weight repack. Reference: the two optimizers of /root/reference
train.py:36-37 (torch.optim.Adam, L2 weight decay) and their step at train.py:101-105."""
import pytest
import torch

from macbf_gnn_amd.ops import native

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _rand(*shape, seed=0):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(*shape, generator=g).to(DEV)


def test_reduce_multi_equals_reduce_rows_and_torch():
    """Wide slabs: bitwise the per-slab reduce_rows sums (same fixed order); the narrow loss-partial
    slab (12 columns x 4,096 rows, 64 row slices) and every slab within fp32 rounding of a float64
    torch sum."""
    jobs = [(_rand(256, 28896, seed=1), 28896), (_rand(256, 10368, seed=2), 10368), (_rand(4096, 12, seed=3), 12),
            (_rand(40, 8, seed=4), 8)]
    outs = [torch.zeros(c, device=DEV) for _, c in jobs]
    native.reduce_multi([(p, o, False) for (p, _), o in zip(jobs, outs)])
    torch.cuda.synchronize()
    for (p, c), o in zip(jobs, outs):
        ref = torch.zeros(c, device=DEV)
        native.reduce_rows(p, ref)
        torch.cuda.synchronize()
        assert torch.equal(o, ref), c
        want = p.double().sum(0).float()
        torch.testing.assert_close(o, want, rtol=1e-5, atol=1e-4 * p.shape[0] ** 0.5)


def test_reduce_multi_accumulates():
    p, o = _rand(64, 32, seed=5), _rand(32, seed=6)
    ref = o.clone() + p.double().sum(0).float()
    native.reduce_multi([(p, o, True)])
    torch.cuda.synchronize()
    torch.testing.assert_close(o, ref, rtol=1e-5, atol=1e-5)


def test_adam_multi_is_bitwise_two_adam_launches():
    n = 51141
    ranges = [(0, 30000), (30000, n)]
    base = [_rand(n, seed=s) for s in (7, 8)] + [_rand(n, seed=9).abs()]
    grad = _rand(n, seed=10)
    outs = []
    for fused in (False, True):
        p, m, v = (t.clone() for t in base)
        steps = torch.tensor([3, 5], dtype=torch.int32, device=DEV)
        ok = torch.ones(1, dtype=torch.int32, device=DEV)
        if fused:
            native.adam_multi(p, grad, m, v, [(a, b, steps[i:i + 1]) for i, (a, b) in enumerate(ranges)],
                              1e-3, 0.9, 0.999, 1e-8, 1e-2, ok=ok)
        else:
            for i, (a, b) in enumerate(ranges):
                native.adam(p, grad, m, v, a, b, 1e-3, 0.9, 0.999, 1e-8, 1e-2, 1, ok=ok, step_dev=steps[i:i + 1])
        torch.cuda.synchronize()
        outs.append((p, m, v))
    for x, y in zip(*outs):
        assert torch.equal(x, y)
    # a cleared guard flag leaves everything untouched
    p, m, v = (t.clone() for t in base)
    native.adam_multi(p, grad, m, v, [(0, n, torch.zeros(1, dtype=torch.int32, device=DEV))], 1e-3, 0.9, 0.999, 1e-8,
                      0.0, ok=torch.zeros(1, dtype=torch.int32, device=DEV))
    torch.cuda.synchronize()
    assert torch.equal(p, base[0]) and torch.equal(m, base[1]) and torch.equal(v, base[2])


@pytest.mark.parametrize("ok_in,fp16", [(1, False), (0, False), (1, True), (0, True)])
def test_commit_in_pack_gather_equals_step_commit(ok_in, fp16):
    """The optimizer commit run by the weight-repack launch == the step_commit kernel: step counts
    of the masked groups, skip count, fp16 loss scale / good-step count, the statistics row's two
    fields, the re-armed flag."""
    res = []
    for via_pack in (False, True):
        ok = torch.full((1,), ok_in, dtype=torch.int32, device=DEV)
        steps = torch.tensor([4, 9], dtype=torch.int32, device=DEV)
        skipped = torch.tensor([2], dtype=torch.int32, device=DEV)
        gscale = torch.tensor([1024.0], device=DEV) if fp16 else None
        good = torch.tensor([999], dtype=torch.int32, device=DEV) if fp16 else None
        row = torch.zeros(18, device=DEV)
        kw = dict(gscale=gscale, good=good, growth=1000, stats_row=row)
        if via_pack:
            src = _rand(100, seed=11)
            idx16 = torch.arange(64, dtype=torch.int32, device=DEV)
            idx32 = torch.arange(32, dtype=torch.int32, device=DEV)
            out16 = torch.empty(64, dtype=torch.bfloat16, device=DEV)
            out32 = torch.empty(32, device=DEV)
            native.pack_gather(src, idx16, out16, idx32, out32, commit=native.step_commit_args(ok, steps, 0b10, skipped,
                                                                                               **kw))
            torch.cuda.synchronize()
            assert torch.equal(out32, src[:32]) and torch.equal(out16, src[:64].bfloat16())
        else:
            native.step_commit(ok, steps, 0b10, skipped, **kw)
        torch.cuda.synchronize()
        res.append([ok, steps, skipped, row] + ([gscale, good] if fp16 else []))
    for x, y in zip(*res):
        assert torch.equal(x, y)
    assert int(res[1][0]) == 1                                   # re-armed


def test_grad_assemble_check_and_stats_row():
    """grad_assemble with ok: clears it on a non-finite assembled element only; with stats: the row
    stats_pack writes."""
    n = 5000
    red = _rand(3 * n, seed=12)
    ptr = torch.arange(0, 3 * n + 1, 3, dtype=torch.int32, device=DEV)
    src = torch.arange(3 * n, dtype=torch.int32, device=DEV)
    sums, counts, local = _rand(10, seed=13), _rand(3, seed=14), _rand(3, seed=15)
    for poison in (False, True):
        r = red.clone()
        if poison:
            r[4711] = float("inf")
        grad = torch.empty(n, device=DEV)
        ok = torch.ones(1, dtype=torch.int32, device=DEV)
        row, ref_row = torch.zeros(18, device=DEV), torch.zeros(18, device=DEV)
        native.grad_assemble(r, ptr, src, grad, scale=0.5, ok=ok, stats=(sums, counts, local, row))
        native.stats_pack(sums, counts, local, ref_row)
        g0 = torch.empty(n, device=DEV)
        native.grad_assemble(r, ptr, src, g0, scale=0.5)
        torch.cuda.synchronize()
        assert torch.equal(grad, g0)
        assert int(ok) == (0 if poison else 1)
        assert torch.equal(row, ref_row)
