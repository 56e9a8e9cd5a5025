"""Host logic of the batched tables (efl.lib.coalesce_runs): which entries of a batch merge into one
run, and how long runs are cut. CPU tensors stand in for device buffers (only addresses matter)."""
import torch

from efl.lib import coalesce_runs


def _views(n_slices, n, dtype):
    buf = torch.empty(n_slices * n, dtype=dtype)
    return [buf[i * n:(i + 1) * n] for i in range(n_slices)], buf


def test_slices_of_one_table_are_one_run():
    xs, xb = _views(64, 1000, torch.float32)
    ms, mb = _views(64, 1000, torch.int64)
    es, eb = _views(64, 1000, torch.int64)
    runs = coalesce_runs(xs, ms, es, chunk=1 << 40)
    assert runs == [(xb.data_ptr(), mb.data_ptr(), eb.data_ptr(), 64000)]


def test_chunking_and_order():
    xs, xb = _views(10, 1000, torch.float32)
    ms, mb = _views(10, 1000, torch.int64)
    es, eb = _views(10, 1000, torch.int64)
    runs = coalesce_runs(xs, ms, es, chunk=4096)
    assert [r[3] for r in runs] == [4096, 4096, 1808]
    assert runs[1] == (xb.data_ptr() + 4096 * 4, mb.data_ptr() + 4096 * 8, eb.data_ptr() + 4096 * 8, 4096)


def test_breaks_where_any_stream_breaks():
    xs, _ = _views(6, 100, torch.float32)
    ms, _ = _views(6, 100, torch.int64)
    es = [torch.empty(100, dtype=torch.int64) for _ in range(6)]   # not adjacent to each other
    es[1] = torch.empty(100, dtype=torch.int64)
    runs = coalesce_runs(xs, ms, es)
    assert sum(r[3] for r in runs) == 600
    # every run is a real continuation in all three streams
    for p0, p1, p2, n in runs:
        assert n % 100 == 0


def test_out_of_order_and_reversed_slices_do_not_merge():
    xs, _ = _views(4, 50, torch.float32)
    ms, _ = _views(4, 50, torch.int64)
    es, _ = _views(4, 50, torch.int64)
    rev = coalesce_runs(xs[::-1], ms[::-1], es[::-1])
    assert [r[3] for r in rev] == [50, 50, 50, 50]
    mixed = coalesce_runs([xs[0], xs[1], xs[3]], [ms[0], ms[1], ms[3]], [es[0], es[1], es[3]])
    assert [r[3] for r in mixed] == [100, 50]


def test_empty_entries_are_dropped():
    xs, _ = _views(3, 10, torch.float32)
    ms, _ = _views(3, 10, torch.int64)
    es, _ = _views(3, 10, torch.int64)
    e = torch.empty(0)
    runs = coalesce_runs([xs[0], e, xs[1], xs[2]], [ms[0], e.long(), ms[1], ms[2]], [es[0], e.long(), es[1], es[2]])
    assert [r[3] for r in runs] == [30]
    assert coalesce_runs([e], [e.long()], [e.long()]) == []


def test_batch_tables_reject_strided_and_mismatched_entries():
    """BatchTables checks its entries on the host before any device table exists: a strided view
    or streams of different sizes are refused (the kernels read numel() contiguous elements)."""
    import pytest
    from efl import errors
    from efl.lib import BatchTables
    x = torch.empty(10, 4)
    m = torch.empty(10, 4, dtype=torch.int64)
    with pytest.raises(errors.InvalidArgumentError, match="not contiguous"):
        BatchTables([x[:, ::2]], [m[:, ::2].contiguous()], [m[:, ::2].contiguous()])
    with pytest.raises(errors.InvalidArgumentError, match="different sizes"):
        BatchTables([x], [m[:5]], [m])
    with pytest.raises(errors.InvalidArgumentError, match="as many"):
        BatchTables([x, x], [m], [m])
