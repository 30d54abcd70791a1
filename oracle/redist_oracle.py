"""CPU oracle (NumPy restatement) of the reference redistribution path.

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import this module, and only as the
checker / the timed CPU baseline.  The product package
(``mpi_grid_redistribute_amd``) never imports anything under ``oracle/``.

This is a fresh restatement of the algorithm in
``dkorytov/mpi_grid_redistribute`` ``redist.py`` (md5 3012918...), written
against the semantics table SURVEY.md §0 (S1-S14).  Every function cites the
reference lines it restates.  Arithmetic is deliberately done with the same
NumPy operations (``%`` = ``np.remainder``, true division, ``astype(int64)``) so
that the float semantics match numpy 2.2.6 bit for bit (S1, S2, S9, S10).

Pinning: ``tests/golden/*.npz`` were produced by running the reference itself
(``tests/golden/make_golden.py``, fake communicator); ``tests/test_oracle.py``
checks this module and the C restatement (``oracle/mgr_oracle.c``) against them.

Divergences from the reference that the oracle encodes on purpose (the
product mirrors them, DESIGN.md §Boundary lists them):
  * an empty rank does not raise ``ValueError`` (S5): it contributes nothing
    and still receives (the reference crashes at ``redist.py:158``);
  * the module wrapper implements the intended behaviour (S13).
"""
from __future__ import annotations

import numpy as np

INT64_MIN = np.iinfo(np.int64).min


# ----------------------------------------------------------------- geometry
class Geometry:
    """Host plan of ``MPIGridRedistributor.__init__`` (redist.py:16-61)."""

    def __init__(self, grid_topology, box_length, size, rank=0):
        # redist.py:40  np.array(grid_topology, dtype=np.int)  (truncating cast)
        self.grid_topology = np.array(grid_topology).astype(np.int64)
        self.size = int(size)
        self.rank = int(rank)
        # redist.py:43-44
        ranks_required = int(np.prod(self.grid_topology))
        assert ranks_required <= self.size
        self.dim = len(self.grid_topology)
        # redist.py:46 keeps the caller's dtype (int box -> int64, S11a)
        self.box_length = np.array(box_length)
        assert self.dim == len(self.box_length)
        # redist.py:49-51
        self.cell_length = np.zeros(self.dim)
        for d in range(self.dim):
            self.cell_length[d] = self.box_length[d] / self.grid_topology[d]
        # redist.py:53-58 row-major offsets, last axis fastest (S4)
        self.cell_index_offset = np.zeros(self.dim, dtype=np.int64)
        off = 1
        for j in range(self.dim - 1, -1, -1):
            self.cell_index_offset[j] = off
            off *= int(self.grid_topology[j])
        # redist.py:60-61
        self.rank_cell_index = indexes_from_cell_number(self, np.array([self.rank]))[0]
        self.rank_cell_limits = cell_limits_from_indexes(self, np.array([self.rank_cell_index]))[0]


def periodic_wrap(values, box):
    """``_periodic_wrapping`` (redist.py:328-329): ((x % L) + L) % L with numpy
    floor-remainder semantics; float or integer alike (S1, S3)."""
    return ((values % box) + box) % box


def cell_indexes_from_position(geo: Geometry, position, periodic=True):
    """``get_cell_indexes_from_position`` (redist.py:63-71).

    Mutates ``position`` in place when periodic (S1), then bins from the
    written-back value (S2, S9): trunc((t / L) * n) with x86 INT64_MIN for
    NaN/out-of-range (S10)."""
    idx = np.zeros((len(position), geo.dim), dtype=np.int64)
    for d in range(geo.dim):
        if periodic:
            position[:, d] = periodic_wrap(position[:, d], geo.box_length[d])
        with np.errstate(invalid="ignore"):
            idx[:, d] = (position[:, d] / geo.box_length[d] * geo.grid_topology[d]).astype(np.int64)
    return idx


def cell_number_from_indexes(geo: Geometry, indexes, periodic=True, check_range=True):
    """``get_cell_number_from_indexes`` (redist.py:73-85).

    Non-periodic branch keeps the reference's ``&`` (redist.py:80): the range
    check can never select anything, so nothing is set to -1."""
    indexes = np.asarray(indexes)
    cell = np.zeros(len(indexes), dtype=np.int64)
    if not periodic:
        for d in range(geo.dim):
            cell += geo.cell_index_offset[d] * indexes[:, d]
        if check_range:
            for d in range(geo.dim):
                outside = (indexes[:, d] < 0) & (indexes[:, d] >= geo.grid_topology[d])
                cell[outside] = -1
    else:
        for d in range(geo.dim):
            cell += geo.cell_index_offset[d] * periodic_wrap(indexes[:, d], geo.grid_topology[d])
    return cell


def cell_number_from_position(geo: Geometry, position, periodic=True):
    """``get_cell_number_from_position`` (redist.py:87-90).  ``periodic`` is not
    forwarded to the index stage (redist.py:90), so indexes always wrap (S3)."""
    return cell_number_from_indexes(geo, cell_indexes_from_position(geo, position, periodic))


def indexes_from_cell_number(geo: Geometry, cell_numbers):
    """``get_indexes_from_cell_number`` (redist.py:92-97): true division then
    truncating assignment into an int array."""
    cell_numbers = np.asarray(cell_numbers)
    out = np.zeros((len(cell_numbers), geo.dim), dtype=int)
    for d in range(geo.dim):
        out[:, d] = cell_numbers / geo.cell_index_offset[d]
        cell_numbers = cell_numbers % geo.cell_index_offset[d]
    return out


def cell_limits_from_indexes(geo: Geometry, cell_indexes):
    """``get_cell_limits_from_indexes`` (redist.py:99-113)."""
    cell_indexes = np.asarray(cell_indexes)
    lim = np.zeros((len(cell_indexes), geo.dim, 2))
    for d in range(geo.dim):
        lim[:, d, 0] = cell_indexes[:, d] * geo.cell_length[d]
        lim[:, d, 1] = (cell_indexes[:, d] + 1) * geo.cell_length[d]
    return lim


# ----------------------------------------------------------- split/exchange
def stable_split(data, rank_to_send, size):
    """The send-buffer build of ``redistribute_by_cell_number``
    (redist.py:195-198): one boolean mask pass per destination, original order
    kept, ids outside [0, size) dropped (S6).  Reference cost: O(N * size)."""
    return [data[rank_to_send == i] for i in range(size)]


def alltoall_concat(send_lists):
    """``np.concatenate(comm.alltoall(send_buff))`` (redist.py:199) for all
    ranks at once: rank r receives [src0->r, src1->r, ...] (S7)."""
    size = len(send_lists)
    return [np.concatenate([send_lists[s][r] for s in range(size)]) for r in range(size)]


def stable_partition(data, dest, nbins):
    """Single-array form of the split: concat_d data[dest == d] plus the
    nbins+1 segment offsets (the 1-GPU Cfg2 output).  Uses a
    stable argsort, which orders identically to the mask passes."""
    dest = np.asarray(dest)
    keep = (dest >= 0) & (dest < nbins)
    order = np.argsort(np.where(keep, dest, nbins), kind="stable")
    order = order[: int(keep.sum())]
    counts = np.bincount(dest[keep].astype(np.int64), minlength=nbins)
    offsets = np.zeros(nbins + 1, dtype=np.int64)
    np.cumsum(counts, out=offsets[1:])
    return data[order], offsets


def redistribute_by_position_all_ranks(grid_topology, box_length, size, data_list, pos_list,
                                       periodic=True):
    """``redistribute_by_position`` without overload (redist.py:115-162),
    executed for every rank.  Mutates each ``pos_list[r]`` in place (S1).
    Returns the per-rank outputs (S7 order)."""
    sends = []
    for r in range(size):
        geo = Geometry(grid_topology, box_length, size, r)
        dest = cell_number_from_position(geo, pos_list[r], periodic=periodic)
        if len(dest):  # redist.py:158-159 (vacuous after S3); empty: see header
            assert dest.min() >= 0 and dest.max() < size
        sends.append(stable_split(data_list[r], dest, size))
    return alltoall_concat(sends)


def redistribute_by_cell_number_all_ranks(size, data_list, ids_list):
    """``redistribute_by_cell_number`` (redist.py:169-200) for every rank."""
    return alltoall_concat([stable_split(d, i, size) for d, i in zip(data_list, ids_list)])


def redistribute_fields_by_position_all_ranks(grid_topology, box_length, size, fields_list,
                                              pos_list, periodic=True):
    """SoA redistribution -- several arrays sharing axis 0 -- by the
    reference's own multi-field pattern (redist.py:157-164): ONE binning of
    the positions per rank (:157, wrapping ``pos_list[r]`` in place, S1), then
    every field split with that same ``rank_to_send`` (:160 for ``data``,
    :164 for ``position``; :195-198) and exchanged (:199).  A field that IS
    ``pos_list[r]`` moves its wrapped values.  Returns per-rank lists of the
    fields' outputs (S7 order)."""
    nf = len(fields_list[0]) if fields_list else 0
    sends = [[] for _ in range(nf)]
    for r in range(size):
        geo = Geometry(grid_topology, box_length, size, r)
        dest = cell_number_from_position(geo, pos_list[r], periodic=periodic)
        for i in range(nf):
            sends[i].append(stable_split(fields_list[r][i], dest, size))
    per_field = [alltoall_concat(sends[i]) for i in range(nf)]
    return [[per_field[i][r] for i in range(nf)] for r in range(size)]


def redistribute_fields_by_cell_number_all_ranks(size, fields_list, ids_list):
    """``redistribute_by_cell_number`` (redist.py:169-200) of every field of a
    SoA payload with the same ids, for every rank: per-rank lists."""
    nf = len(fields_list[0]) if fields_list else 0
    per_field = [redistribute_by_cell_number_all_ranks(size, [f[i] for f in fields_list], ids_list)
                 for i in range(nf)]
    return [[per_field[i][r] for i in range(nf)] for r in range(size)]


# ------------------------------------------------------- position helpers
def stack_position(columns):
    """``stack_position`` (redist.py:311-312): d columns of N -> (N, d),
    ``np.vstack(columns).T``."""
    return np.vstack(columns).T


def unstack_position(position, dim):
    """Intended behaviour of ``unstack_position`` (redist.py:314-318), whose
    text is broken (``for d in self.dim``, ``reusult``): the dim columns."""
    return [position[:, d] for d in range(dim)]


def mpi_grid_redistribute_all_ranks(data_list, pos_list, grid_topology, box_lengths, size,
                                    overload_lengths=None, periodic=True):
    """Intended behaviour of the module function ``mpi_grid_redistribute``
    (redist.py:11-13): a redistributor per rank, then
    ``redistribute_by_position(data, pos, overload_lengths, periodic)``
    (the reference calls a misspelled method and raises, S13)."""
    if overload_lengths is None:
        return redistribute_by_position_all_ranks(grid_topology, box_lengths, size, data_list,
                                                  pos_list, periodic=periodic)
    return redistribute_by_position_overload_all_ranks(grid_topology, box_lengths, size,
                                                       data_list, pos_list, overload_lengths,
                                                       periodic=periodic)


# ------------------------------------------------------- overload / halo
def _send_rows(field_local, pos_local, field_ov, pos_ov, d, thr, right, keep):
    """One side of ``exchange_overload_by_position``'s selection
    (redist.py:271-287): rows of the local field and of the overload buffer
    whose coordinate d is > thr (right) or < thr (left), local first."""
    if not keep:  # _prepare_data_to_send(..., False) (redist.py:320-326)
        return field_local[:0]
    if right:
        a, b = field_local[pos_local[:, d] > thr], field_ov[pos_ov[:, d] > thr]
    else:
        a, b = field_local[pos_local[:, d] < thr], field_ov[pos_ov[:, d] < thr]
    return np.concatenate([a, b], axis=0)


def exchange_overload_all_ranks(grid_topology, box_length, size, data_list, pos_list,
                                overload_lengths, periodic=True):
    """``exchange_overload_by_position`` (redist.py:202-309) executed for every
    rank at once.  Per dimension d, for the data and then the position field
    (:264): rank r sends the rows beyond its right threshold to its right
    neighbour a and receives from its left neighbour b (:289-295), then sends
    the rows below its left threshold to b and receives from a (:298-303);
    the overload buffer grows as concat(buffer, from_a, from_b) (:305-306).
    Kept quirks: no periodic shift of positions; with periodic=False the
    left send uses the RIGHT neighbour's flag (:287); the selection of the
    buffer uses the positions received in earlier dimensions only.
    Returns the per-rank overload data (not the positions, :309)."""
    geos = [Geometry(grid_topology, box_length, size, r) for r in range(size)]
    dim = geos[0].dim
    assert len(overload_lengths) == dim
    ov = [[data_list[r][:0], np.zeros((0, dim), dtype=pos_list[r].dtype)] for r in range(size)]
    for d in range(dim):
        nb = []
        for r in range(size):
            g = geos[r]
            ea = np.zeros(dim, dtype=np.int64)
            ea[d] = 1
            ia, ib = g.rank_cell_index + ea, g.rank_cell_index - ea
            a = cell_number_from_indexes(g, np.array([ia]))[0]
            b = cell_number_from_indexes(g, np.array([ib]))[0]
            if periodic:
                keep_a = keep_b = True
            else:
                keep_a = cell_number_from_indexes(g, np.array([ia]), periodic=False)[0] == a
                keep_b = keep_a  # redist.py:287 passes the right neighbour's flag
            nb.append((int(a), int(b), keep_a, keep_b))
        for fi, fields in ((0, data_list), (1, pos_list)):
            to_a, to_b = [], []
            for r in range(size):
                g = geos[r]
                hi = g.rank_cell_limits[d, 1] - overload_lengths[d]
                lo = g.rank_cell_limits[d, 0] + overload_lengths[d]
                _, _, keep_a, keep_b = nb[r]
                to_a.append(_send_rows(fields[r], pos_list[r], ov[r][fi], ov[r][1], d, hi, True,
                                       keep_a))
                to_b.append(_send_rows(fields[r], pos_list[r], ov[r][fi], ov[r][1], d, lo, False,
                                       keep_b))
            new = []
            for r in range(size):
                a, b = nb[r][0], nb[r][1]
                # my left neighbour b sent its to_a to me (its right neighbour)
                from_b = to_a[b]
                from_a = to_b[a]
                new.append(np.concatenate([ov[r][fi], from_a, from_b]))
            for r in range(size):
                ov[r][fi] = new[r]
    return [ov[r][0] for r in range(size)]


def redistribute_by_position_overload_all_ranks(grid_topology, box_length, size, data_list,
                                                pos_list, overload_lengths, periodic=True):
    """``redistribute_by_position`` with ``overload_lengths`` (redist.py:157-166):
    bin with ``periodic`` (:157), redistribute data and positions with the same
    destinations, exchange the overload (periodic=True: the flag is not
    forwarded from :165), and return concat(local, overload) per rank."""
    dest = []
    for r in range(size):
        geo = Geometry(grid_topology, box_length, size, r)
        dest.append(cell_number_from_position(geo, pos_list[r], periodic=periodic))
    local = redistribute_by_cell_number_all_ranks(size, data_list, dest)
    local_pos = redistribute_by_cell_number_all_ranks(size, pos_list, dest)
    ovd = exchange_overload_all_ranks(grid_topology, box_length, size, local, local_pos,
                                      overload_lengths)
    return [np.concatenate((local[r], ovd[r]), axis=0) for r in range(size)]


# --------------------------------------------------- fine cells (f4, Cfg5)
def fine_cell_ids(grid_topology, fine_cells, box_length, position):
    """Fine cell of every row inside its rank's cell:
    the reference's binning (redist.py:63-71) over the global fine grid
    topology * fine, without a position wrap (the rows were wrapped by the
    redistribution), the integer index wrap that get_cell_number_from_position
    always applies (:90, S3), then k % fine per dimension, numbered row-major
    over fine (last axis fastest)."""
    topo = np.array(grid_topology).astype(np.int64)
    fine = np.array(fine_cells).astype(np.int64)
    glob = topo * fine
    geo = Geometry(glob, box_length, int(np.prod(glob)))
    with np.errstate(invalid="ignore"):
        idx = cell_indexes_from_position(geo, position.copy(), periodic=False)
    k = periodic_wrap(idx, glob) % fine
    off = np.ones(len(fine), dtype=np.int64)
    for j in range(len(fine) - 2, -1, -1):
        off[j] = off[j + 1] * fine[j + 1]
    return (k * off).sum(axis=1)


def fine_cell_sort(data, fine_id, nfine):
    """Stable sort of a rank's rows by fine cell: data[argsort(fine_id,
    kind='stable')] plus the nfine+1 cell offsets."""
    return stable_partition(data, fine_id, nfine)


# --------------------------------------------------------- synthetic inputs
_M64 = (1 << 64) - 1


def splitmix64(x):
    """splitmix64 finaliser on uint64 numpy arrays (SURVEY §8d generator)."""
    x = (np.asarray(x, dtype=np.uint64) + np.uint64(0x9E3779B97F4A7C15))
    x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return x ^ (x >> np.uint64(31))


def synth_uniform(seed, gid_start, n, dim=3, box=1.0):
    """u = (splitmix64(seed ^ (3*gid + d)) >> 11) * 2^-53, times L per dim.
    Same stream as the device generator ``mgr_synth_uniform``."""
    gid = np.arange(gid_start, gid_start + n, dtype=np.uint64)
    box = np.broadcast_to(np.asarray(box, dtype=np.float64), (dim,))
    pos = np.empty((n, dim), dtype=np.float64)
    with np.errstate(over="ignore"):
        for d in range(dim):
            h = splitmix64(np.uint64(seed) ^ (np.uint64(3) * gid + np.uint64(d)))
            pos[:, d] = (h >> np.uint64(11)).astype(np.float64) * (2.0 ** -53) * box[d]
    return pos
