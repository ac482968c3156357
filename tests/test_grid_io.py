"""CPU: the persistent log-odds grid (dmf_grid_save / dmf_grid_load, csrc/dmf_io.hip;
SURVEY.md §5 checkpoint / resume).  Host-only code: round trip of grid, geometry and fusion
parameters; header-only reads; the file's layout (magic, little-endian header, x-major
int16 grid, CRC-32 = zlib.crc32 of every byte before it); torn, corrupted and foreign files
are rejected; a too-small buffer reports DMF_ERR_CAPACITY."""
import struct
import zlib

import numpy as np
import pytest

from dmf_amd import _lib


def _grid(dims, seed=0):
    return np.random.default_rng(seed).integers(-2000, 3512, size=dims).astype(np.int16)


@pytest.mark.parametrize("dims", [(1, 1, 1), (5, 3, 7), (64, 33, 17)])
def test_round_trip(tmp_path, dims):
    g = _grid(dims)
    bounds = (-0.5, 0.5, -0.25, 0.75, 0.0, 1.0 / 3)
    prm = _lib.default_fuse_params(dmin_mm=200, dmax_mm=1000)
    path = tmp_path / "grid.dmf"
    _lib.grid_save(path, g, dims, bounds, prm)
    g2, b2, p2 = _lib.grid_load(path)
    assert g2.shape == dims and np.array_equal(g2, g)
    assert b2 == bounds
    assert (p2.dmin_mm, p2.dmax_mm, p2.l_hit, p2.l_miss, p2.l_min, p2.l_max) == (200, 1000, 847, -405, -2000, 3511)
    raw = path.read_bytes()
    n = int(np.prod(dims))
    assert len(raw) == 104 + 2 * n + 4 and raw[:8] == b"DMFGRID1"
    assert struct.unpack_from("<III", raw, 8) == (1, 104, dims[0])
    assert struct.unpack_from("<6d", raw, 32) == bounds
    assert np.array_equal(np.frombuffer(raw, "<i2", count=n, offset=104), g.reshape(-1))
    assert struct.unpack_from("<I", raw, 104 + 2 * n)[0] == zlib.crc32(raw[:104 + 2 * n])


def test_rejects_bad_files(tmp_path):
    g = _grid((6, 5, 4), 1)
    path = tmp_path / "g.dmf"
    _lib.grid_save(path, g, g.shape, (0, 1, 0, 1, 0, 1))
    raw = bytearray(path.read_bytes())
    L = _lib.load()
    h = _lib.dmf_grid_header()
    buf = np.empty(g.size, np.int16)

    def load(data, cap=g.size):
        p = tmp_path / "x.dmf"
        p.write_bytes(bytes(data))
        import ctypes as C
        return L.dmf_grid_load(str(p).encode(), C.addressof(h), buf.ctypes.data, cap)
    assert load(raw) == _lib.DMF_OK and np.array_equal(buf.reshape(g.shape), g)
    bad = bytearray(raw)
    bad[104 + 7] ^= 0x40  # one grid bit
    assert load(bad) == _lib.DMF_ERR_INVALID
    assert load(raw[:-3]) == _lib.DMF_ERR_INVALID  # torn
    assert load(raw + b"\0") == _lib.DMF_ERR_INVALID  # trailing bytes
    bad = bytearray(raw)
    bad[0:8] = b"NOTAGRID"
    assert load(bad) == _lib.DMF_ERR_INVALID
    bad = bytearray(raw)
    bad[8] = 2  # version
    assert load(bad) == _lib.DMF_ERR_INVALID
    assert load(raw, cap=g.size - 1) == _lib.DMF_ERR_CAPACITY
    with pytest.raises(ValueError):
        _lib.grid_save(path, g, (6, 5, 5), (0, 1, 0, 1, 0, 1))


def test_huge_dims_rejected_before_allocation(tmp_path):
    """a corrupted header naming 2^20 x 2^20 x 2^20 cells is rejected from the
    file's size in the header-only read (DMF_ERR_INVALID), before grid_load sizes a buffer."""
    import struct
    g = _grid((4, 4, 4), 2)
    path = tmp_path / "g.dmf"
    _lib.grid_save(path, g, g.shape, (0, 1, 0, 1, 0, 1))
    raw = bytearray(path.read_bytes())
    struct.pack_into("<iii", raw, 16, 1 << 20, 1 << 20, 1 << 20)
    bad = tmp_path / "huge.dmf"
    bad.write_bytes(bytes(raw))
    with pytest.raises(_lib.DmfError) as e:
        _lib.grid_load(bad)
    assert e.value.status == _lib.DMF_ERR_INVALID


def _save_under_fsize_limit(path, limit):
    """Child process: dmf_grid_save of a 5x4x3 grid with RLIMIT_FSIZE = limit bytes (writes past
    it fail with EFBIG, SIGXFSZ ignored); prints the DmfError status or 'ok'."""
    import subprocess
    import sys
    code = f"""
import resource, signal, sys
sys.path[:0] = {sys.path!r}
import numpy as np
from dmf_amd import _lib
signal.signal(signal.SIGXFSZ, signal.SIG_IGN)
resource.setrlimit(resource.RLIMIT_FSIZE, ({limit}, {limit}))
g = (np.arange(60, dtype=np.int16) * 7).reshape(5, 4, 3)
try:
    _lib.grid_save({str(path)!r}, g, g.shape, (0, 1, 0, 1, 0, 1))
    print("ok")
except _lib.DmfError as e:
    print("err", e.status)
"""
    return subprocess.run([sys.executable, "-c", code], stdout=subprocess.PIPE, text=True, timeout=120).stdout.strip()


def test_save_replaces_atomically(tmp_path):
    """dmf_grid_save writes a unique temporary beside path (mkstemp), syncs it,
    renames it over path and syncs the directory: a save that fails mid-write (here: a file
    size limit) leaves the previous file intact and no temporary behind."""
    g = _grid((5, 4, 3), 3)
    path = tmp_path / "g.dmf"
    _lib.grid_save(path, g, g.shape, (0, 1, 0, 1, 0, 1))
    before = path.read_bytes()
    assert sorted(p.name for p in tmp_path.iterdir()) == ["g.dmf"]
    assert _save_under_fsize_limit(path, 64) == f"err {_lib.DMF_ERR_INVALID}"
    assert path.read_bytes() == before
    assert sorted(p.name for p in tmp_path.iterdir()) == ["g.dmf"]  # the temporary is gone
    g2, _, _ = _lib.grid_load(path)
    assert np.array_equal(g2, g)


def test_concurrent_saves_never_tear(tmp_path):
    """Two writers of one path use their own temporaries: the file is always one whole grid."""
    from concurrent.futures import ThreadPoolExecutor
    path = tmp_path / "g.dmf"
    grids = [_grid((40, 30, 20), s) for s in (1, 2)]

    def save(k):
        for _ in range(20):
            _lib.grid_save(path, grids[k], grids[k].shape, (0, 1, 0, 1, 0, 1))
    with ThreadPoolExecutor(2) as ex:
        list(ex.map(save, (0, 1)))
    g, _, _ = _lib.grid_load(path)
    assert any(np.array_equal(g, x) for x in grids)
    assert sorted(p.name for p in tmp_path.iterdir()) == ["g.dmf"]


def test_saved_file_mode(tmp_path):
    """the mkstemp temporary (created 0600) gets the mode a plain fopen would give
    (0666 less the umask) for a new file, and keeps the mode of a file it replaces."""
    import os
    import stat
    g = _grid((4, 3, 2), 5)
    old = os.umask(0o022)
    try:
        path = tmp_path / "new.dmf"
        _lib.grid_save(path, g, g.shape, (0, 1, 0, 1, 0, 1))
        assert stat.S_IMODE(os.stat(path).st_mode) == 0o644
        os.umask(0o077)
        path2 = tmp_path / "new2.dmf"
        _lib.grid_save(path2, g, g.shape, (0, 1, 0, 1, 0, 1))
        assert stat.S_IMODE(os.stat(path2).st_mode) == 0o600
        os.chmod(path, 0o640)
        _lib.grid_save(path, g, g.shape, (0, 1, 0, 1, 0, 1))
        assert stat.S_IMODE(os.stat(path).st_mode) == 0o640
    finally:
        os.umask(old)
