"""CompactBuffer's ring layout (mgx/compact.py, ring=True) on the CPU: the row arithmetic only -- every
rollout's observations 1..T land in its own block, its observation 0 and history rows are the previous
rollouts' last rows (the ones the gather's wrap-around walk reaches), and carry_over() moves nothing.  The
gather kernel itself is checked on the GPU (tests/test_compact.py::test_carry_over_and_minibatch_gather)."""
import pytest

torch = pytest.importorskip("torch")


class _Eng:                                   # the attributes CompactBuffer reads from an MgxEngine
    def __init__(self, n, n_stack):
        self.n, self.n_stack, self.device = n, n_stack, torch.device("cpu")


@pytest.mark.parametrize("T,k", [(20, 4), (8, 4), (3, 4), (2, 4), (1, 4), (5, 1), (16, 8)])
def test_ring_rows(T, k):
    from mgx.compact import CompactBuffer
    buf = CompactBuffer(_Eng(6, k), T, ring=True)
    H = k - 1
    assert buf.blocks == 1 + -(-(H + 1) // T) and buf.R == buf.blocks * T
    assert buf.rows.shape[0] == buf.R
    seq = {}                                   # global observation index -> physical row
    for c in range(3 * buf.blocks + 2):
        if c:
            buf.carry_over()
        b = buf.block
        assert b == c % buf.blocks
        assert [buf.row(t) for t in range(1, T + 1)] == list(range(b * T, b * T + T))   # this rollout's block
        assert buf.dones.data_ptr() == buf.starts[b * T].data_ptr()
        for t in range(0, T + 1):
            g = c * T + t                      # observation 0 of rollout c = observation T of rollout c - 1
            if g in seq:
                assert seq[g] == buf.row(t), (c, t)
            seq[g] = buf.row(t)
        # the H history rows before observation 0 are the previous rollouts' rows, still unwritten by this one
        if c:
            hist = [(buf.row(0) - j) % buf.R for j in range(H + 1)]
            assert not set(hist) & set(range(b * T, b * T + T))
            assert all(hist[j] == seq[c * T - j] for j in range(H + 1) if c * T - j in seq)
        tt = torch.arange(T + 1)
        assert torch.equal(buf.index(tt, 2), torch.tensor([buf.row(int(t)) * 6 + 2 for t in tt]))


def test_copy_layout_rows_unchanged():
    from mgx.compact import CompactBuffer
    buf = CompactBuffer(_Eng(4, 4), 8)
    assert buf.R == 8 + 3 + 1 and [buf.row(t) for t in range(9)] == list(range(3, 12))
    buf.carry_over()
    assert buf.row(0) == 3 and buf.block == 0
