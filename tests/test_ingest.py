"""f2 ingest on the CPU: the MRC2014 and .thu I/O of thunder_amd.io, and the
numpy restatement of the image preprocessing (oracle/preprocess.py) pinned by
known answers (the reference holds no preprocessed fixtures: parity
unpinned).  The device path is tests/test_gpu_ingest.py."""
import struct

import numpy as np
import pytest

from oracle import preprocess as opp
from thunder_amd import io


@pytest.mark.parametrize("dtype", [np.float32, np.int16, np.float16, np.uint16, np.int8])
def test_mrc_round_trip(tmp_path, dtype):
    rng = np.random.default_rng(1)
    a = (rng.standard_normal((5, 24, 32)) * 40).astype(dtype)
    p = tmp_path / "s.mrcs"
    io.write_mrc(p, a, pixel_size=1.32)
    h, d = io.read_mrc(p)
    assert (h.nx, h.ny, h.nz) == (32, 24, 5)
    assert h.mode == {np.float32: 2, np.int16: 1, np.float16: 12, np.uint16: 6, np.int8: 0}[dtype]
    assert abs(h.pixel_size - 1.32) < 1e-6
    assert np.array_equal(np.asarray(d), a)
    raw = p.read_bytes()
    assert len(raw) == 1024 + a.nbytes and raw[208:212] == b"MAP "


def test_mrc_big_endian_and_extended_header(tmp_path):
    """A big-endian file (machine stamp 0x11 0x11) with an extended header of
    NSYMBT bytes: the data start after it and are byte-swapped on read."""
    rng = np.random.default_rng(2)
    a = rng.standard_normal((3, 8, 8)).astype(np.float32)
    h = io.MrcHeader(8, 8, 3, 2, cella=(8.0, 8.0, 3.0), nsymbt=96, byteorder=">")
    p = tmp_path / "be.mrc"
    p.write_bytes(h.pack() + bytes(96) + a.astype(">f4").tobytes())
    h2, d = io.read_mrc(p, mmap=False)
    assert h2.byteorder == ">" and h2.nsymbt == 96 and h2.mode == 2
    assert np.array_equal(d.astype(np.float32), a)
    # NX / MODE are the first words, per the spec
    assert struct.unpack(">4i", p.read_bytes()[:16]) == (8, 8, 3, 2)


def test_thu_round_trip_and_ctf_attrs(tmp_path):
    rng = np.random.default_rng(3)
    n = 7
    ctf = np.stack([np.full(n, 300e3), rng.uniform(1e4, 3e4, n), rng.uniform(1e4, 3e4, n),
                    rng.uniform(0, np.pi, n), np.full(n, 2.7e7), np.full(n, 0.1), np.zeros(n)], 1)
    q = rng.standard_normal((n, 4))
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    t = io.thu_table(n, [f"{i + 1:06d}@stack.mrcs" for i in range(n)], ctf, q,
                     rng.standard_normal((n, 2)), group=np.arange(n) % 3)
    p = tmp_path / "p.thu"
    io.write_thu(p, t)
    lines = p.read_text().splitlines()
    assert len(lines) == n and all(len(ln.split()) == 27 for ln in lines)
    r = io.read_thu(p)
    assert r["particlePath"] == t["particlePath"]
    for name in io.THU_COLUMNS:
        if name not in ("particlePath", "micrographPath"):
            assert np.allclose(r[name], t[name], rtol=0, atol=5e-9 * max(1.0, np.abs(t[name]).max()))
    a = io.thu_ctf_attrs(r, 1.32)
    assert a.shape == (n, 8) and np.allclose(a[:, 0], 1.32) and np.allclose(a[:, 2], ctf[:, 1])


def test_thu_rejects_short_rows(tmp_path):
    p = tmp_path / "bad.thu"
    p.write_text("1 2 3\n")
    with pytest.raises(ValueError):
        io.read_thu(p)


def test_load_images_from_stacks(tmp_path):
    rng = np.random.default_rng(4)
    a = rng.standard_normal((4, 16, 16)).astype(np.float32)
    b = rng.standard_normal((1, 16, 16)).astype(np.float32)
    io.write_mrc(tmp_path / "a.mrcs", a)
    io.write_mrc(tmp_path / "b.mrc", b)
    t = io.thu_table(3, ["000003@a.mrcs", "b.mrc", "1@a.mrcs"])
    imgs = io.load_images(t, str(tmp_path))
    assert np.array_equal(imgs[0], a[2]) and np.array_equal(imgs[1], b[0])
    assert np.array_equal(imgs[2], a[0])


def test_preprocess_restatement_known_answers():
    """Background N(7, 3^2) outside the mask radius, a bright disc inside:
    after substractBgImg the background has mean 0 and sample sd 1 (so
    statImg's bgStddev(0) is 1), the stored image is the centred one rolled
    by N/2, the soft mask is 1 inside r, 0 past r + 6 and 1/2 half-way, and
    the forward transform is numpy's unnormalised rfft2."""
    N, r = 64, 20.0
    rng = np.random.default_rng(5)
    c = (rng.standard_normal((N, N)) * 3 + 7).astype(np.float32)
    yy, xx = np.mgrid[:N, :N] - N // 2
    c[np.hypot(xx, yy) < 10] += 50
    img = opp.load(c)
    assert img[0, 0] == c[N // 2, N // 2]
    out, st = opp.stats_and_normalise(img, r)
    i, j = opp.rl_coords(N)
    bg = i.astype(float) ** 2 + j.astype(float) ** 2 > r * r
    assert abs(out[bg].astype(np.float64).mean()) < 1e-6
    assert abs(st[2] - 1.0) < 1e-6 and abs(st[0] - 7) < 0.2 and abs(st[1] - 3) < 0.1
    keep = opp.soft_mask_keep(N, r)
    u = np.hypot(i, j)
    assert np.all(keep[u < r] == 1) and np.all(keep[u > r + 6] == 0)
    half = np.isclose(u, r + 3)
    assert half.any() and np.allclose(keep[half], 0.5, atol=1e-6)
    ft, oft = opp.finish(out, r, 1.0)
    assert np.allclose(oft, np.fft.rfft2(out.astype(np.float64)))
    # re-masking an image supported inside r changes nothing
    inner = np.where(u < r, out, 0).astype(np.float64)
    assert np.allclose(opp.remask(np.fft.rfft2(inner), N, r), np.fft.rfft2(inner), atol=1e-9)
