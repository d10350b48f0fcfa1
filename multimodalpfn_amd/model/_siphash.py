"""Row-vectorised SipHash-2-4 with the all-zero key.

CPython 3.10 hashes ``bytes`` with SipHash-2-4 keyed by the interpreter's hash
secret, which ``PYTHONHASHSEED=0`` sets to zero.  The reference fingerprint
feature is ``hash(row.tobytes())`` (``model/preprocessing.py:476-479``), so its
values are reproducible only under ``PYTHONHASHSEED=0``.  This module computes
exactly those values for every row of a table at once (numpy ``uint64`` lanes),
independent of the running interpreter's hash seed.
"""

from __future__ import annotations

import numpy as np

_U = np.uint64


def _rotl(x: np.ndarray, r: int) -> np.ndarray:
    return (x << _U(r)) | (x >> _U(64 - r))


def _round(v0, v1, v2, v3):
    v0 = v0 + v1
    v1 = _rotl(v1, 13) ^ v0
    v0 = _rotl(v0, 32)
    v2 = v2 + v3
    v3 = _rotl(v3, 16) ^ v2
    v0 = v0 + v3
    v3 = _rotl(v3, 21) ^ v0
    v2 = v2 + v1
    v1 = _rotl(v1, 17) ^ v2
    v2 = _rotl(v2, 32)
    return v0, v1, v2, v3


_NATIVE = None


def _native():
    """The library's ``mmpfn_siphash24_rows`` (host code, one pass over the bytes), or None where the
    library cannot be loaded (host preprocessing also runs in CPU-only processes, e.g. ``fit``)."""
    global _NATIVE
    if _NATIVE is None:
        try:
            from multimodalpfn_amd import _lib

            _NATIVE = _lib.load_library().mmpfn_siphash24_rows
        except (OSError, RuntimeError, AttributeError):
            _NATIVE = False
    return _NATIVE or None


def siphash24_rows(rows: np.ndarray) -> np.ndarray:
    """Python ``hash(row.tobytes())`` (zero secret) of each row of a 2-D array, as int64."""
    rows = np.ascontiguousarray(rows)
    fn = _native()
    if fn is not None:
        n = rows.shape[0]
        out = np.empty(n, np.int64)
        if n:
            nb = rows.nbytes // n
            if fn(rows.ctypes.data, n, nb, out.ctypes.data) != 0:
                raise ValueError("mmpfn_siphash24_rows: bad arguments")
        return out
    return siphash24_rows_numpy(rows)


def siphash24_rows_numpy(rows: np.ndarray) -> np.ndarray:
    """The same hash in numpy ``uint64`` lanes (reference restatement; the fallback)."""
    rows = np.ascontiguousarray(rows)
    n = rows.shape[0]
    raw = rows.reshape(n, -1).view(np.uint8) if rows.size else np.zeros((n, 0), np.uint8)
    nb = raw.shape[1]
    n_words = nb // 8
    with np.errstate(over="ignore"):
        words = np.ascontiguousarray(raw[:, : n_words * 8]).view("<u8")
        v0 = np.full(n, 0x736F6D6570736575, _U)
        v1 = np.full(n, 0x646F72616E646F6D, _U)
        v2 = np.full(n, 0x6C7967656E657261, _U)
        v3 = np.full(n, 0x7465646279746573, _U)
        for j in range(n_words):
            m = words[:, j]
            v3 = v3 ^ m
            v0, v1, v2, v3 = _round(v0, v1, v2, v3)
            v0, v1, v2, v3 = _round(v0, v1, v2, v3)
            v0 = v0 ^ m
        last = np.full(n, (nb & 0xFF) << 56, _U)
        for k in range(nb - n_words * 8):  # tail bytes, little endian
            last = last | (raw[:, n_words * 8 + k].astype(_U) << _U(8 * k))
        v3 = v3 ^ last
        v0, v1, v2, v3 = _round(v0, v1, v2, v3)
        v0, v1, v2, v3 = _round(v0, v1, v2, v3)
        v0 = v0 ^ last
        v2 = v2 ^ _U(0xFF)
        for _ in range(4):
            v0, v1, v2, v3 = _round(v0, v1, v2, v3)
        h = (v0 ^ v1 ^ v2 ^ v3).view(np.int64)
    if nb == 0:
        h = np.zeros(n, np.int64)  # hash(b"") == 0
    return np.where(h == -1, np.int64(-2), h)  # CPython reserves -1
