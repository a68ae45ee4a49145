"""Particle-stack I/O for the ingest row (f2): MRC2014 image stacks and
THUNDER's .thu particle table.

MRC2014 is written from the format's public specification (a 1024-byte
header of 56 little-endian 4-byte words + ten 80-byte labels, an optional
extended header of NSYMBT bytes, then NX x NY x NZ voxels, X fastest; modes 0
int8, 1 int16, 2 float32, 6 uint16, 12 float16).  The reader memory-maps the
data block, so a 100k-particle stack is never loaded whole.

The .thu table is one particle per line, 27 whitespace-separated columns in
the order of include/Database.h:22-290 (THU_VOLTAGE .. THU_SCORE): the CTF
attributes (CTFAttr, include/Database.h:302), the particle and micrograph
paths, coordinates, group / class ids, the quaternion, k1..k3, the
translation and its spreads, the defocus factor and its spread, the score.
A particle path "n@stack.mrcs" is slice n (1-based) of that stack, a bare
path a single image (Optimiser::initImg, src/Optimiser.cpp:4638-4660).
"""
import os
import struct

import numpy as np

MRC_MODES = {0: np.int8, 1: np.int16, 2: np.float32, 6: np.uint16, 12: np.float16}
_MODE_OF = {np.dtype(v): k for k, v in MRC_MODES.items()}

THU_COLUMNS = ("voltage", "defocusU", "defocusV", "defocusTheta", "Cs", "amplitudeContrast",
               "phaseShift", "particlePath", "micrographPath", "coordinateX", "coordinateY",
               "groupID", "classID", "quat0", "quat1", "quat2", "quat3", "k1", "k2", "k3",
               "transX", "transY", "stdTransX", "stdTransY", "defocusFactor",
               "stdDefocusFactor", "score")
_THU_INT = ("groupID", "classID")
_THU_STR = ("particlePath", "micrographPath")


class MrcHeader:
    """The fields of the 1024-byte MRC2014 header this module uses."""

    def __init__(self, nx, ny, nz, mode, cella=(0.0, 0.0, 0.0), nsymbt=0, origin=(0.0, 0.0, 0.0),
                 dmin=0.0, dmax=0.0, dmean=0.0, rms=0.0, ispg=0, byteorder="<", exttyp=b"\0\0\0\0",
                 nversion=20140, labels=()):
        self.nx, self.ny, self.nz, self.mode = int(nx), int(ny), int(nz), int(mode)
        self.cella, self.nsymbt, self.origin = tuple(cella), int(nsymbt), tuple(origin)
        self.dmin, self.dmax, self.dmean, self.rms = dmin, dmax, dmean, rms
        self.ispg, self.byteorder, self.exttyp, self.nversion = ispg, byteorder, exttyp, nversion
        self.labels = tuple(labels)

    @property
    def dtype(self):
        if self.mode not in MRC_MODES:
            raise ValueError(f"MRC mode {self.mode} is not an image mode this reader handles")
        return np.dtype(MRC_MODES[self.mode]).newbyteorder(self.byteorder)

    @property
    def pixel_size(self):
        return self.cella[0] / self.nx if self.nx else 0.0

    def pack(self):
        e = self.byteorder
        w = struct.pack(e + "10i", self.nx, self.ny, self.nz, self.mode, 0, 0, 0,
                        self.nx, self.ny, self.nz)
        w += struct.pack(e + "6f", *self.cella, 90.0, 90.0, 90.0)
        w += struct.pack(e + "3i", 1, 2, 3)
        w += struct.pack(e + "3f", self.dmin, self.dmax, self.dmean)
        w += struct.pack(e + "2i", self.ispg, self.nsymbt)
        extra = bytearray(100)
        extra[8:12] = self.exttyp
        extra[12:16] = struct.pack(e + "i", self.nversion)
        w += bytes(extra)
        w += struct.pack(e + "3f", *self.origin)
        w += b"MAP "
        w += b"DA\x00\x00" if e == "<" else b"\x11\x11\x00\x00"
        w += struct.pack(e + "f", self.rms)
        labels = [lb.encode()[:80].ljust(80) for lb in self.labels[:10]]
        w += struct.pack(e + "i", len(labels))
        w += b"".join(labels).ljust(800, b"\0")
        assert len(w) == 1024
        return w

    @classmethod
    def unpack(cls, buf):
        if len(buf) < 1024:
            raise ValueError("MRC header shorter than 1024 bytes")
        # byte order: the machine stamp (word 54), else the plausibility of MODE
        stamp = buf[212:214]
        e = ">" if stamp == b"\x11\x11" else "<"
        if stamp not in (b"DA", b"DD", b"\x11\x11", b"D\x00") and \
                struct.unpack("<i", buf[12:16])[0] not in MRC_MODES:
            e = ">"
        nx, ny, nz, mode = struct.unpack(e + "4i", buf[0:16])
        cella = struct.unpack(e + "3f", buf[40:52])
        dmin, dmax, dmean = struct.unpack(e + "3f", buf[76:88])
        ispg, nsymbt = struct.unpack(e + "2i", buf[88:96])
        exttyp = bytes(buf[104:108])
        nversion = struct.unpack(e + "i", buf[108:112])[0]
        origin = struct.unpack(e + "3f", buf[196:208])
        rms = struct.unpack(e + "f", buf[216:220])[0]
        nl = max(0, min(10, struct.unpack(e + "i", buf[220:224])[0]))
        labels = [bytes(buf[224 + 80 * k:304 + 80 * k]).rstrip(b" \0").decode(errors="replace")
                  for k in range(nl)]
        if nx <= 0 or ny <= 0 or nz <= 0:
            raise ValueError(f"MRC header: bad dimensions {nx} x {ny} x {nz}")
        return cls(nx, ny, nz, mode, cella, nsymbt, origin, dmin, dmax, dmean, rms, ispg, e,
                   exttyp, nversion, labels)


def read_mrc(path, mmap=True):
    """(header, data [nz, ny, nx]) -- data memory-mapped (read-only) by default."""
    with open(path, "rb") as f:
        h = MrcHeader.unpack(f.read(1024))
    off = 1024 + h.nsymbt
    shape = (h.nz, h.ny, h.nx)
    need = off + int(np.prod(shape)) * h.dtype.itemsize
    if os.path.getsize(path) < need:
        raise ValueError(f"{path}: {os.path.getsize(path)} bytes, the header needs {need}")
    if mmap:
        data = np.memmap(path, dtype=h.dtype, mode="r", offset=off, shape=shape)
    else:
        data = np.fromfile(path, dtype=h.dtype, count=int(np.prod(shape)), offset=off).reshape(shape)
    return h, data


def write_mrc(path, data, pixel_size=1.0, labels=("thunder_amd",)):
    """data [nz, ny, nx] (or [ny, nx]) of a supported dtype, X fastest."""
    a = np.asarray(data)
    if a.ndim == 2:
        a = a[None]
    if a.dtype not in _MODE_OF:
        a = a.astype(np.float32)
    nz, ny, nx = a.shape
    af = a.astype(np.float64)
    h = MrcHeader(nx, ny, nz, _MODE_OF[a.dtype], (nx * pixel_size, ny * pixel_size, nz * pixel_size),
                  dmin=float(af.min()), dmax=float(af.max()), dmean=float(af.mean()),
                  rms=float(af.std()), labels=labels)
    with open(path, "wb") as f:
        f.write(h.pack())
        f.write(np.ascontiguousarray(a, dtype=a.dtype.newbyteorder("<")).tobytes())
    return h


def read_thu(path):
    """The .thu table as a dict of columns (numpy arrays; the paths as lists)."""
    rows = []
    with open(path) as f:
        for ln, line in enumerate(f, 1):
            w = line.split()
            if not w:
                continue
            if len(w) != len(THU_COLUMNS):
                raise ValueError(f"{path}:{ln}: {len(w)} columns, expected {len(THU_COLUMNS)}")
            rows.append(w)
    out = {}
    for k, name in enumerate(THU_COLUMNS):
        col = [r[k] for r in rows]
        if name in _THU_STR:
            out[name] = col
        elif name in _THU_INT:
            out[name] = np.array([int(v) for v in col], np.int64)
        else:
            out[name] = np.array([float(v) for v in col], np.float64)
    return out


def write_thu(path, table):
    """Write a table (dict of columns, as read_thu returns) with the reference's
    column formats (%18.9f for reals, %6d for ids, %s for paths)."""
    n = len(table["particlePath"])
    with open(path, "w") as f:
        for i in range(n):
            parts = []
            for name in THU_COLUMNS:
                v = table[name][i]
                if name in _THU_STR:
                    parts.append(str(v))
                elif name in _THU_INT:
                    parts.append("%6d" % int(v))
                else:
                    parts.append("%18.9f" % float(v))
            f.write(" ".join(parts) + "\n")


def thu_table(n, particle_paths, ctf_attrs=None, quat=None, trans=None, group=None):
    """A .thu table for n particles; ctf_attrs [n, >=7] {voltage (V), defocusU,
    defocusV (A), defocusTheta (rad), Cs (A), amplitude contrast, phase shift}."""
    t = {name: np.zeros(n, np.int64 if name in _THU_INT else np.float64) for name in THU_COLUMNS
         if name not in _THU_STR}
    t["particlePath"] = list(particle_paths)
    t["micrographPath"] = ["mic.mrc"] * n
    if ctf_attrs is not None:
        for k, name in enumerate(THU_COLUMNS[:7]):
            t[name] = np.asarray(ctf_attrs, np.float64)[:, k]
    t["quat0"][:] = 1.0
    if quat is not None:
        for k in range(4):
            t[f"quat{k}"] = np.asarray(quat, np.float64)[:, k]
    if trans is not None:
        t["transX"], t["transY"] = (np.asarray(trans, np.float64)[:, k] for k in range(2))
    t["defocusFactor"][:] = 1.0
    if group is not None:
        t["groupID"] = np.asarray(group, np.int64)
    return t


def thu_ctf_attrs(table, pixel_size):
    """[n, 8] float32 rows {pixelSize, voltage, dU, dV, theta, Cs, ampC,
    phaseShift} -- the attribute layout of thx_ctf -- from a .thu table."""
    n = len(table["particlePath"])
    a = np.zeros((n, 8), np.float32)
    a[:, 0] = pixel_size
    for k, name in enumerate(THU_COLUMNS[:7]):
        a[:, 1 + k] = table[name]
    return a


def load_images(table, prefix=""):
    """The particles of a .thu table as one [n, N, N] float32 array, centred
    as stored (the device preprocessing takes them centred); stacks are
    memory-mapped and each read once."""
    paths = table["particlePath"]
    cache = {}
    out = None
    for i, p in enumerate(paths):
        if "@" in p:
            s, fn = p.split("@", 1)
            slc = int(s) - 1
        else:
            slc, fn = 0, p
        fn = os.path.join(prefix, fn)
        if fn not in cache:
            cache[fn] = read_mrc(fn)
        h, d = cache[fn]
        if not 0 <= slc < h.nz:
            raise ValueError(f"{p}: slice {slc + 1} of {h.nz}")
        if out is None:
            out = np.empty((len(paths), h.ny, h.nx), np.float32)
        if (h.ny, h.nx) != out.shape[1:]:
            raise ValueError(f"{p}: {h.nx} x {h.ny} images, expected {out.shape[2]} x {out.shape[1]}")
        out[i] = d[slc]
    return out
