"""The HDF5 reader (csrc/h5read.cpp, which replaces h5py in
dataset/modelNetData.py:43-47 and dataset/shapeNetData.py:176-181) under
AddressSanitizer + UBSan (`make asan`, tests/asan/h5check.cpp), fed the
fixture files truncated at many points, with corrupted bytes, and with
8-byte fields overwritten by out-of-range offsets / sizes.  Every run must end
in a clean read or a clean error (exit 0 / 1): no sanitizer report, no signal.
CPU only."""
import os
import shutil
import subprocess

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
H5 = os.path.join(REPO, "tests", "golden", "h5")
BIN = os.path.join(REPO, "build", "asan", "h5check")
FILES = {"modelnet_gzip.h5": ["data", "label"], "modelnet_contig.h5": ["data", "label"],
         "shapenet_latest.h5": ["data", "label", "pid"], "many_members.h5": ["data"]}
ENV = dict(os.environ, ASAN_OPTIONS="exitcode=99:detect_leaks=0:abort_on_error=0",
           UBSAN_OPTIONS="halt_on_error=1:exitcode=98")


@pytest.fixture(scope="module")
def h5check():
    if shutil.which("g++") is None:
        pytest.skip("no host C++ compiler")
    subprocess.run(["make", "-C", REPO, "asan"], check=True, capture_output=True)
    return BIN


def _run(binary, path, name, keep1=0):
    r = subprocess.run([binary, path, name, str(keep1)], capture_output=True, text=True, env=ENV,
                       timeout=60)
    report = r.stderr
    assert r.returncode in (0, 1) and "Sanitizer" not in report and "runtime error" not in report, \
        f"{os.path.basename(path)}:{name} rc={r.returncode}\n{report[-2000:]}"
    return r.returncode, r.stdout


def test_asan_reads_the_valid_fixtures(h5check):
    for f, names in FILES.items():
        for n in names:
            rc, out = _run(h5check, os.path.join(H5, f), n)
            assert rc == 0 and out.startswith("ok"), (f, n, out)
            rc, _ = _run(h5check, os.path.join(H5, f), n, keep1=5)
            assert rc == 0


@pytest.mark.parametrize("fname", sorted(FILES))
def test_asan_truncated_files(h5check, tmp_path, fname):
    raw = open(os.path.join(H5, fname), "rb").read()
    cuts = sorted(set(list(range(0, min(len(raw), 1024), 37)) +
                      [int(x) for x in np.linspace(1024, len(raw) - 1, 24)]))
    for cut in cuts:
        p = tmp_path / "t.h5"
        p.write_bytes(raw[:cut])
        for n in FILES[fname]:
            _run(h5check, str(p), n)


@pytest.mark.parametrize("fname", sorted(FILES))
def test_asan_corrupted_bytes_and_offsets(h5check, tmp_path, fname):
    """Random byte flips (mostly in the metadata at the front), and aligned
    8-byte fields overwritten with huge or just-out-of-range values (object
    header / B-tree / heap / chunk addresses, dims, sizes)."""
    raw = np.frombuffer(open(os.path.join(H5, fname), "rb").read(), np.uint8)
    rng = np.random.default_rng(len(raw))
    meta = min(len(raw), 4096)
    bad_vals = [2 ** 64 - 1, 2 ** 63, 2 ** 40, len(raw), len(raw) + 1, len(raw) - 1, 2 ** 31]
    for k in range(60):
        b = raw.copy()
        if k % 2 == 0:
            for _ in range(1 + k % 5):
                pos = int(rng.integers(0, meta)) if rng.random() < 0.85 else int(rng.integers(0, len(raw)))
                b[pos] ^= np.uint8(1 << int(rng.integers(0, 8)))
        else:
            pos = int(rng.integers(0, max(1, meta - 8) // 8)) * 8
            b[pos:pos + 8] = np.frombuffer(np.uint64(bad_vals[k % len(bad_vals)]).tobytes(), np.uint8)
        p = tmp_path / "c.h5"
        p.write_bytes(b.tobytes())
        for n in FILES[fname]:
            _run(h5check, str(p), n)
