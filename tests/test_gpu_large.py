"""GPU: maximum sizes -- more than 2^31 rows on one MI355X.

288 GB of HBM holds billions of particles per GPU, so every row index, tile
index, segment start and byte offset on the path must be 64-bit.  The oracle
cannot run at this size in seconds, so the check is by size-independent
properties that together pin the result exactly:
  * per-destination counts equal an independent bincount of the bins;
  * each destination segment holds only rows of that destination (the
    payload of row i is i), in strictly increasing row order;
so every segment is exactly the stable selection data[dest == d]
(redist.py:195-198) -- the same statement the oracle makes at small sizes.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

mgr = pytest.importorskip("mpi_grid_redistribute_amd")
from mpi_grid_redistribute_amd import GridPartitioner  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")


def _fill(n, pos, data, chunk=1 << 28):
    """pos[i] = hash(i) mod 2^24 / 2^24 (exact in f32, in the box),
    data[i] = i mod 2^32 (4-byte rows)."""
    for a in range(0, n, chunk):
        b = min(n, a + chunk)
        i = torch.arange(a, b, dtype=torch.int64, device="cuda")
        h = (i * 2654435761) & 0xFFFFFF
        pos[a:b, 0] = h.to(torch.float32) * (1.0 / (1 << 24))
        data[a:b] = i.to(torch.int32)   # wraps mod 2^32 (two's complement)


@pytest.mark.parametrize("topo", [[8], [3]])
def test_partition_beyond_int32_rows(topo):
    n = (1 << 31) + 4097                    # ragged last tile
    nb = topo[0]
    pos = torch.empty((n, 1), dtype=torch.float32, device="cuda")
    data = torch.empty(n, dtype=torch.int32, device="cuda")
    _fill(n, pos, data)
    P = GridPartitioner(topo, [1.0])
    out, counts = P.partition_device(data.view(torch.uint8), 4, pos)
    torch.cuda.synchronize()
    # in-box f32 positions with an f64 box wrap to themselves (S9): unchanged
    bins = torch.empty(n, dtype=torch.uint8, device="cuda")
    for a in range(0, n, 1 << 28):
        b = min(n, a + (1 << 28))
        # trunc((x / 1.0) * nb) in f64, as numpy computes it (x is exact in f64)
        bins[a:b] = (pos[a:b, 0].to(torch.float64) * nb).floor().to(torch.uint8)
    exp_counts = torch.bincount(bins, minlength=nb)
    got_counts = counts.cpu()
    assert torch.equal(got_counts, exp_counts.cpu()), (got_counts, exp_counts)
    assert int(got_counts.sum()) == n
    rows = out[: n * 4].view(torch.int32)
    start = 0
    for d in range(nb):
        c = int(got_counts[d])
        idx = rows[start:start + c].to(torch.int64) & 0xFFFFFFFF
        if c:
            # payload i mod 2^32 -> row index: rows >= 2^32 do not exist (n < 2^32)
            assert bool((bins[idx] == d).all()), f"destination {d}: foreign rows"
            assert bool((idx[1:] > idx[:-1]).all()), f"destination {d}: order not stable"
        start += c
        del idx
    # the last rows (above 2^31) landed: their payload shows up
    tail = (n - 1) & 0xFFFFFFFF
    d_last = int(bins[n - 1])
    seg0 = int(got_counts[:d_last].sum())
    assert int(rows[seg0 + int(got_counts[d_last]) - 1].to(torch.int64) & 0xFFFFFFFF) == tail
