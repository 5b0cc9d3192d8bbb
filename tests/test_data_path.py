"""Data path on the CPU: the HDF5-free reader against files
written by the real HDF5 library (tests/golden/h5/make_h5_fixtures.py: h5py
3.3 / libhdf5 1.10.6; gzip-chunked as PointNet writes ModelNet40, contiguous,
shuffle + partial edge chunks, v0 and v3 superblocks, a 40-member group), and
the dataset mirrors' split / slicing / item format / jitter against the
reference's logic (dataset/modelNetData.py, dataset/shapeNetData.py)."""
import os

import numpy as np
import pytest

from adversarial_learning_on_pointclouds_amd import dataset as D

H5 = os.path.join(os.path.dirname(__file__), "golden", "h5")
EXP = np.load(os.path.join(H5, "expected.npz"))


@pytest.mark.parametrize("key", sorted(EXP.files))
def test_reader_matches_hdf5_library(key):
    fn, name = key.split("/")
    path = os.path.join(H5, fn + ".h5")
    e = EXP[key]
    shape, code = D.h5_info(path, name)
    assert shape == e.shape
    kind = {"f": (D.H5_F32 if e.itemsize == 4 else D.H5_F64)}.get(e.dtype.kind)
    if kind is None:
        kind = (D.H5_INT if e.dtype.kind == "i" else D.H5_UINT) | (e.itemsize << 4)
    assert code == kind
    got = D.read_h5(path, name)
    assert got.dtype == (np.float32 if e.dtype.kind == "f" else np.int64)
    assert np.array_equal(got, e.astype(got.dtype))


def test_reader_first_points_slice():
    """data[:, 0:npts, :] (modelNetData.py:46) and pid[:, 0:npts] (shapeNetData.py:180)."""
    d = D.read_h5(os.path.join(H5, "modelnet_gzip.h5"), "data", keep1=17)
    assert np.array_equal(d, EXP["modelnet_gzip/data"][:, :17, :])
    pid = D.read_h5(os.path.join(H5, "shapenet_latest.h5"), "pid", keep1=33)
    assert np.array_equal(pid, EXP["shapenet_latest/pid"][:, :33].astype(np.int64))
    d = D.read_h5(os.path.join(H5, "many_members.h5"), "data", keep1=100)  # > dims[1]: all
    assert np.array_equal(d, EXP["many_members/data"].astype(np.float32))


def test_reader_errors_are_loud(tmp_path):
    with pytest.raises(RuntimeError, match="no object"):
        D.read_h5(os.path.join(H5, "modelnet_gzip.h5"), "pid")
    bad = tmp_path / "x.h5"
    bad.write_bytes(b"not an hdf5 file" * 8)
    with pytest.raises(RuntimeError, match="not an HDF5 file"):
        D.read_h5(str(bad), "data")
    with pytest.raises(RuntimeError, match="cannot open"):
        D.read_h5(str(tmp_path / "missing.h5"), "data")


def _list(tmp_path, names):
    p = tmp_path / "files.txt"
    p.write_text("".join(os.path.join(H5, n) + "\n" for n in names))
    return str(p)


def test_modelnet_split_and_items(tmp_path):
    lst = _list(tmp_path, ["modelnet_gzip.h5", "modelnet_contig.h5"])
    all_d = np.concatenate([EXP["modelnet_gzip/data"][:, :32], EXP["modelnet_contig/data"][:, :32]])
    all_l = np.squeeze(np.concatenate([EXP["modelnet_gzip/label"], EXP["modelnet_contig/label"]]))
    gt_rows = np.array([6, 0, 3])
    gt = D.ModelNetDatasetGT(lst, gt_rows, npoints=32, data_augmentation=False)
    ng = D.ModelNetDataset_noGT(lst, gt_rows, npoints=32, data_augmentation=False)
    assert len(gt) == 3 and len(ng) == 5
    p, c = gt[1]
    assert p.dtype == np.float32 and c.dtype == np.int64
    assert np.array_equal(p, all_d[0]) and c == all_l[0]
    assert np.array_equal(ng[0], all_d[1]) and np.array_equal(ng[4], all_d[7])
    full = D.ModelNetDatasetGT(lst, None, npoints=32, data_augmentation=False)
    assert len(full) == 8


def test_modelnet_jitter_matches_reference_formula(tmp_path):
    lst = _list(tmp_path, ["modelnet_gzip.h5"])
    ds = D.ModelNetDatasetGT(lst, None, npoints=64, data_augmentation=True)
    np.random.seed(7)
    p, _ = ds[2]
    np.random.seed(7)  # modelNetData.py:88-90, f64 then float32 (:76)
    ref = (np.clip(0.01 * np.random.randn(64, 3), -0.05, 0.05) + EXP["modelnet_gzip/data"][2]).astype(np.float32)
    assert np.array_equal(p, ref)
    assert np.abs(p - EXP["modelnet_gzip/data"][2]).max() <= 0.05 + 1e-7


def test_shapenet_items(tmp_path):
    lst = _list(tmp_path, ["shapenet_latest.h5"])
    gt = D.ShapeNetDatasetGT(np.array([4, 1]), lst, num_classes=16, num_pts=40)
    ng = D.ShapeNetDataset_noGT(np.array([4, 1]), lst, num_classes=16, num_pts=40)
    p, oh, seg = gt[0]
    assert np.array_equal(p, EXP["shapenet_latest/data"][4, :40])
    assert oh.shape == (1, 16) and oh.dtype == np.float32
    assert oh[0].argmax() == EXP["shapenet_latest/label"][4, 0] and oh.sum() == 1
    assert np.array_equal(seg, EXP["shapenet_latest/pid"][4, :40].astype(np.int64))
    assert len(ng) == 5
    p, oh = ng[2]
    assert np.array_equal(p, EXP["shapenet_latest/data"][3, :40])
