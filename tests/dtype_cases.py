"""Seeded position/box inputs of every dtype pair (test infrastructure):
shared by the CPU oracle cross-check and the GPU parity tests."""
import numpy as np

ALL_DTYPES = [np.float16, np.float32, np.float64, np.int8, np.int16, np.int32, np.int64,
              np.uint8, np.uint16, np.uint32, np.uint64, np.bool_]


def dtype_case(dt, boxdt, n):
    """Positions of dtype dt against a box of dtype boxdt on topology
    [3, 5, 2]: in-box and out-of-box values (-3L..4L), integer extremes for
    narrow integers, odd values above 2^63 for uint64."""
    rng = np.random.default_rng(sum(map(ord, np.dtype(dt).str + np.dtype(boxdt).str)))
    topo = [3, 5, 2]
    kb = np.dtype(boxdt).kind
    box = (np.array([True, True, True]) if kb == "b" else
           np.array([14, 6, 100]).astype(boxdt) if kb in "iu" else
           np.array([0.7, 6.5, 3.0]).astype(boxdt))
    b64 = box.astype(np.float64)
    raw = rng.uniform(-3, 4, (n, 3)) * b64
    raw[::13] = rng.uniform(0, 1, (len(raw[::13]), 3)) * b64
    if np.dtype(dt).kind in "iu":
        info = np.iinfo(dt)
        raw = np.clip(np.floor(raw * (8 if b64.min() < 10 else 1)), info.min, info.max)
        if info.bits < 64:
            raw[::101] = rng.integers(info.min, info.max, (len(raw[::101]), 3))
    with np.errstate(all="ignore"):
        pos = raw.astype(dt)
        if np.dtype(dt) == np.uint64:
            pos[::97] = rng.integers(0, 2 ** 63, (len(pos[::97]), 3), dtype=np.uint64) * 2 + 1
    return topo, box, pos
