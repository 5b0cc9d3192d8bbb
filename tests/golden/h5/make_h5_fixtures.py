"""Write small HDF5 fixtures in the ModelNet40 / ShapeNet-part layout with the
real HDF5 library (h5py 3.3 / libhdf5 1.10.6 of the image's /opt/conda Python,
which the build's own Python lacks), for the HDF5-free reader (csrc/h5read.cpp).

    /opt/conda/bin/python3.9 tests/golden/h5/make_h5_fixtures.py

Layouts follow what the reference's loaders read (dataset/modelNetData.py:43-47,
dataset/shapeNetData.py:176-181): 'data' [n, npts, 3] float32, 'label' [n, 1],
'pid' [n, npts] (ShapeNet).  PointNet's own HDF5 writer stores them gzip-chunked
(compression='gzip', compression_opts=4), so the fixtures cover that, plain
contiguous storage, the shuffle filter, partial edge chunks, both superblock
generations (libver 'earliest' = v0 superblock / v1 object headers / symbol-table
groups; 'latest' = v3 superblock / v2 object headers / link messages), and a
group with enough members for several symbol-table nodes.  The expected arrays
go to expected.npz next to the files.
"""
import os
import sys

sys.path.insert(0, "/opt/conda/lib/python3.9/site-packages")
import h5py  # noqa: E402
import numpy as np  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    rng = np.random.default_rng(2024)
    exp = {}

    # 1: PointNet-style ModelNet file: gzip-4 chunked, v0 superblock
    d = rng.uniform(-1, 1, (5, 64, 3)).astype(np.float32)
    lab = rng.integers(0, 40, (5, 1)).astype(np.uint8)
    with h5py.File(os.path.join(HERE, "modelnet_gzip.h5"), "w", libver="earliest") as f:
        f.create_dataset("data", data=d, compression="gzip", compression_opts=4)
        f.create_dataset("label", data=lab, compression="gzip", compression_opts=4)
    exp["modelnet_gzip/data"], exp["modelnet_gzip/label"] = d, lab

    # 2: contiguous storage, int32 labels
    d = rng.uniform(-1, 1, (3, 40, 3)).astype(np.float32)
    lab = rng.integers(0, 40, (3, 1)).astype(np.int32)
    with h5py.File(os.path.join(HERE, "modelnet_contig.h5"), "w", libver="earliest") as f:
        f.create_dataset("data", data=d)
        f.create_dataset("label", data=lab)
    exp["modelnet_contig/data"], exp["modelnet_contig/label"] = d, lab

    # 3: ShapeNet-part file, latest format, shuffle + gzip, partial edge chunks
    d = rng.uniform(-1, 1, (7, 50, 3)).astype(np.float32)
    lab = rng.integers(0, 16, (7, 1)).astype(np.uint8)
    pid = rng.integers(0, 50, (7, 50)).astype(np.uint8)
    with h5py.File(os.path.join(HERE, "shapenet_latest.h5"), "w", libver="latest") as f:
        f.create_dataset("data", data=d, chunks=(2, 16, 3), shuffle=True, compression="gzip")
        f.create_dataset("label", data=lab)
        f.create_dataset("pid", data=pid, chunks=(3, 20), compression="gzip", compression_opts=9)
    exp["shapenet_latest/data"], exp["shapenet_latest/label"] = d, lab
    exp["shapenet_latest/pid"] = pid

    # 4: a root group with 40 members (several symbol-table nodes), float64 and
    #    int16 / int64 types, the dataset of interest in the middle
    with h5py.File(os.path.join(HERE, "many_members.h5"), "w", libver="earliest") as f:
        for i in range(40):
            f.create_dataset(f"extra{i:02d}", data=np.full((2,), i, np.int16))
        d = rng.normal(0, 1, (4, 10, 3))
        f.create_dataset("data", data=d)  # float64
        lab = rng.integers(-5, 40, (4, 1)).astype(np.int64)
        f.create_dataset("label", data=lab, chunks=(1, 1), compression="gzip")
    exp["many_members/data"], exp["many_members/label"] = d, lab
    exp["many_members/extra17"] = np.full((2,), 17, np.int16)

    np.savez_compressed(os.path.join(HERE, "expected.npz"), **exp)
    for fn in sorted(os.listdir(HERE)):
        print(fn, os.path.getsize(os.path.join(HERE, fn)))


if __name__ == "__main__":
    main()
