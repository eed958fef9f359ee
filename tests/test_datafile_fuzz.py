"""Randomised checks of the data-file boundary (main.cu:29-67's text format; gpad_datafile_read /
gpad_datafile_write, csrc/gpad_io.cpp), CPU only: random sizes in the three layouts and awkward
float32 values (subnormals, extremes, -0, values that need all 9 significant digits) write and read
back bit for bit; truncated or corrupted files give an error code, never a crash or a partial
result."""
from __future__ import annotations

import os

import numpy as np
import pytest

from gpad_mpc import _lib, datafile


def _vals(rng, k):
    """float32 values incl. the hard cases of a decimal round trip."""
    pool = np.array([0.0, -0.0, 1.0, -1.0, 1e-45, -1e-45, 1.17549435e-38, 3.4028235e38, -3.4028235e38,
                     0.1, 1.0 / 3.0, 16777217.0, 2.0 ** -126, 123456.789], np.float32)
    x = rng.normal(0, 1, k).astype(np.float32) * np.float32(10.0) ** rng.integers(-30, 30, k).astype(np.float32)
    pick = rng.random(k) < 0.2
    x[pick] = pool[rng.integers(0, len(pool), int(pick.sum()))]
    bits = rng.integers(0, 2 ** 32, k, dtype=np.uint64).astype(np.uint32).view(np.float32)
    raw = (rng.random(k) < 0.1) & np.isfinite(bits)
    x[raw] = bits[raw]
    return np.nan_to_num(x, nan=0.5, posinf=1e30, neginf=-1e30).astype(np.float32)


def _random_data(rng, layout):
    n_u, N = int(rng.integers(1, 7)), int(rng.integers(1, 9))
    m = int(rng.integers(1, 40)) if layout != _lib.FILE_FLAT else 4 * n_u * N + int(rng.integers(0, 2 * N + 1))
    n, k = n_u * N, int(rng.integers(1, 30))
    rows = N if layout == _lib.FILE_FLAT else n
    return datafile.GpadData(n_u=n_u, N=N, m=m, L=float(_vals(rng, 1)[0] or 1.0),
                             M_G=_vals(rng, rows * m).reshape(rows, m), g_P=_vals(rng, n),
                             G_L=_vals(rng, rows * m).reshape(m, rows), p_D=_vals(rng, m),
                             theta=_vals(rng, k), beta=_vals(rng, k))


@pytest.mark.parametrize("layout", [_lib.FILE_ROWMAJOR, _lib.FILE_FLIPPED, _lib.FILE_FLAT])
def test_datafile_random_roundtrip_bitexact(tmp_path, layout):
    rng = np.random.default_rng(7 + layout)
    for i in range(40):
        d = _random_data(rng, layout)
        p = str(tmp_path / f"f{i}.txt")
        datafile.write(p, d, layout)
        r = datafile.read(p, layout)
        assert (r.n_u, r.N, r.m, r.num_iterations) == (d.n_u, d.N, d.m, d.num_iterations)
        assert np.float32(r.L).view(np.uint32) == np.float32(d.L).view(np.uint32)
        for k in ("M_G", "g_P", "G_L", "p_D", "theta", "beta"):
            a, b = getattr(r, k), getattr(d, k)
            assert a.shape == b.shape, k
            assert np.array_equal(a.view(np.uint32), b.view(np.uint32)), (i, k)  # bits, -0 included


def test_datafile_corruptions_fail_cleanly(tmp_path):
    rng = np.random.default_rng(11)
    d = _random_data(rng, _lib.FILE_ROWMAJOR)
    good = str(tmp_path / "good.txt")
    datafile.write(good, d, _lib.FILE_ROWMAJOR)
    text = open(good).read()
    ok = err = 0
    for i in range(300):
        kind = i % 4
        if kind == 0:    # truncated anywhere
            bad = text[: int(rng.integers(0, len(text)))]
        elif kind == 1:  # a token replaced by garbage
            toks = text.split()
            j = int(rng.integers(0, len(toks)))
            toks[j] = str(rng.choice(["x", "--", "1e", "nan(", "0x", "", "1.0.0", "+-3"]))
            bad = " ".join(toks)
        elif kind == 2:  # a header field made negative / huge
            toks = text.split()
            j = int(rng.integers(0, 4))
            toks[j] = str(rng.choice(["-1", "0", "2147483647", "99999999999"]))
            bad = " ".join(toks)
        else:            # random bytes spliced in
            k = int(rng.integers(0, len(text)))
            bad = text[:k] + "".join(chr(int(c)) for c in rng.integers(33, 127, 5)) + text[k:]
        p = str(tmp_path / f"bad{i}.txt")
        with open(p, "w") as fh:
            fh.write(bad)
        try:
            r = datafile.read(p, _lib.FILE_ROWMAJOR)
        except _lib.GpadError:
            err += 1
            continue
        ok += 1  # still a well-formed file (e.g. a spliced digit): sizes must be self-consistent
        assert r.M_G.shape == (r.n_u * r.N, r.m) and r.theta.shape == r.beta.shape
        os.remove(p)
    assert err > 150, (ok, err)
