"""Data path: the reference's HDF5 datasets without h5py, and a
device-resident batch loader.

* ``read_h5`` reads one dataset of an HDF5 file through the library's own
  reader (``pcadv_h5_read``, csrc/h5read.cpp; h5py is not in this image).
* ``ModelNetDatasetGT`` / ``ModelNetDataset_noGT`` (dataset/modelNetData.py:
  14-168) and ``ShapeNetDatasetGT`` / ``ShapeNetDataset_noGT``
  (dataset/shapeNetData.py:97-294) keep the reference's constructor arguments,
  GT / no-GT split (the no-GT set is the complement of ``sample_list``,
  ``np.setdiff1d``), first-``npoints`` slicing and item format, so they drop
  into ``torch.utils.data.DataLoader`` unchanged.  ModelNet items are jittered
  on the host exactly as the reference does (f64 numpy draws) when
  ``data_augmentation`` is on.
* ``DeviceCloudLoader`` is the MI355X path: the whole split is uploaded to HBM
  once and every batch is one ``pcadv_gather_clouds`` launch (gather by a
  shuffled index, jitter from device Philox draws, labels / part ids alongside)
  - no per-step host work or PCIe copy, and capturable into the step's graph.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch
import torch.utils.data as data

from . import _lib
from ._lib import GatherJob, check, stream_ptr

H5_F32, H5_F64, H5_INT, H5_UINT = 1, 2, 3, 4


def h5_info(path, name):
    """(shape, stored type code) of dataset ``name`` in the HDF5 file ``path``."""
    lib = _lib.load()
    rank, dims, dt = ctypes.c_int(), (ctypes.c_int64 * 8)(), ctypes.c_int()
    check(lib.pcadv_h5_info(str(path).encode(), name.encode(), ctypes.byref(rank), dims,
                            ctypes.byref(dt)), "pcadv_h5_info")
    return tuple(int(dims[i]) for i in range(rank.value)), int(dt.value)


def read_h5(path, name, keep1=0, dtype=None):
    """f[name][:] (or f[name][:, 0:keep1, ...]) as float32 (float datasets) or
    int64 (integer datasets), or the requested ``dtype`` of those two."""
    lib = _lib.load()
    shape, code = h5_info(path, name)
    shape = list(shape)
    if len(shape) >= 2 and 0 < keep1 < shape[1]:
        shape[1] = keep1
    if dtype is None:
        dtype = np.float32 if code in (H5_F32, H5_F64) else np.int64
    dtype = np.dtype(dtype)
    if dtype not in (np.dtype(np.float32), np.dtype(np.int64)):
        raise TypeError("read_h5 returns float32 or int64")
    out = np.empty(shape, dtype)
    check(lib.pcadv_h5_read(str(path).encode(), name.encode(),
                            0 if dtype == np.float32 else 1, int(keep1),
                            out.ctypes.data_as(ctypes.c_void_p), out.nbytes), "pcadv_h5_read")
    return out


def _files(list_filename):
    return [line.rstrip() for line in open(list_filename)]


def jitter_point_cloud(data, sigma=0.01, clip=0.05, rng=np.random):
    """dataset/modelNetData.py:80-91: per-point Gaussian jitter, clipped (f64)."""
    N, C = data.shape
    assert clip > 0
    jittered = np.clip(sigma * rng.randn(N, C), -1 * clip, clip)
    jittered += data
    return jittered


class ModelNetDatasetGT(data.Dataset):
    """dataset/modelNetData.py:14-103: the labelled ModelNet40 clouds (rows
    ``sample_list`` of the concatenated files, all rows when it is None)."""

    def __init__(self, root_list, sample_list, npoints=1024, data_augmentation=True):
        self.sample_list = sample_list
        self.npoints = npoints
        self.data_augmentation = data_augmentation
        self.data_files = _files(root_list)
        data_, labels = [], []
        for fn in self.data_files:  # :43-47: data[:, 0:num_points, :], label
            data_.append(read_h5(fn, "data", keep1=npoints))
            labels.append(read_h5(fn, "label"))
        total_data = np.concatenate(data_, 0).astype(np.float32)
        total_labels = np.squeeze(np.concatenate(labels, 0)).astype(np.int32)
        if isinstance(sample_list, np.ndarray):
            self.select_data = total_data[sample_list, :, :]
            self.select_labels = total_labels[sample_list]
        else:
            self.select_data = total_data.copy()
            self.select_labels = total_labels.copy()

    def __getitem__(self, index):
        ptc, cls = self.select_data[index], self.select_labels[index]
        if self.data_augmentation:
            ptc = jitter_point_cloud(ptc)
        return ptc.astype(np.float32), cls.astype(np.int64)

    def __len__(self):
        return self.select_data.shape[0]


def _nogt_rows(n, gt_sample_list):
    nogt = np.setdiff1d(np.arange(n), gt_sample_list)
    assert len(np.setdiff1d(nogt, gt_sample_list)) == len(nogt), "Intersection!"
    assert len(np.setdiff1d(gt_sample_list, nogt)) == len(gt_sample_list), "Intersection!"
    return nogt


class ModelNetDataset_noGT(data.Dataset):
    """dataset/modelNetData.py:106-168: the unlabelled complement of
    ``sample_list`` (items are point arrays only)."""

    def __init__(self, root_list, sample_list, npoints=1024, data_augmentation=True):
        self.sample_list = sample_list
        self.npoints = npoints
        self.data_augmentation = data_augmentation
        self.data_files = _files(root_list)
        total = np.concatenate([read_h5(fn, "data", keep1=npoints) for fn in self.data_files],
                               0).astype(np.float32)
        self.select_data = total[_nogt_rows(total.shape[0], sample_list), :, :]

    def __getitem__(self, index):
        ptc = self.select_data[index]
        if self.data_augmentation:
            ptc = jitter_point_cloud(ptc)
        return ptc.astype(np.float32)

    def __len__(self):
        return self.select_data.shape[0]


def one_hot(label, num_classes):
    """dataset/shapeNetData.py:92-95."""
    oh = np.zeros((1, num_classes), dtype=np.float32)
    oh[0, label] = 1
    return oh


class ShapeNetDatasetGT(data.Dataset):
    """dataset/shapeNetData.py:97-201: points, one-hot object class (1, 16) and
    per-point part ids (no augmentation)."""

    def __init__(self, sample_list, root_list, num_classes, num_pts=2048):
        self.sample_list = sample_list
        self.num_classes = num_classes
        self.npts = num_pts
        self.data_files = _files(root_list)
        pts = np.concatenate([read_h5(fn, "data", keep1=num_pts) for fn in self.data_files], 0)
        lab = np.concatenate([read_h5(fn, "label") for fn in self.data_files], 0)
        seg = np.concatenate([read_h5(fn, "pid", keep1=num_pts) for fn in self.data_files], 0)
        pts, lab, seg = pts.astype(np.float32), lab.astype(np.int64), seg.astype(np.int64)
        if isinstance(sample_list, np.ndarray):
            self.select_data = pts[sample_list, :, :]
            self.select_labels = lab[sample_list]
            self.select_segs = seg[sample_list, :]
        else:
            self.select_data, self.select_labels, self.select_segs = pts.copy(), lab.copy(), seg.copy()

    def __getitem__(self, index):
        return (self.select_data[index], one_hot(self.select_labels[index], self.num_classes),
                self.select_segs[index])

    def __len__(self):
        return self.select_data.shape[0]


class ShapeNetDataset_noGT(data.Dataset):
    """dataset/shapeNetData.py:204-294: the complement of ``sample_list``
    (points and one-hot class)."""

    def __init__(self, sample_list, root_list, num_classes, num_pts=2048):
        self.sample_list = sample_list
        self.num_classes = num_classes
        self.npts = num_pts
        self.data_files = _files(root_list)
        pts = np.concatenate([read_h5(fn, "data", keep1=num_pts) for fn in self.data_files], 0)
        lab = np.concatenate([read_h5(fn, "label") for fn in self.data_files], 0)
        rows = _nogt_rows(pts.shape[0], sample_list)
        self.select_data = pts.astype(np.float32)[rows, :, :]
        self.select_labels = lab.astype(np.int64)[rows]

    def __getitem__(self, index):
        return self.select_data[index], one_hot(self.select_labels[index], self.num_classes)

    def __len__(self):
        return self.select_data.shape[0]


def _dp_rank_world(rank, world_size):
    """(rank, world) of a loader: as given, else the initialised default
    torch.distributed group's, else (0, 1)."""
    import torch.distributed as dist
    if world_size is None:
        world_size = dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1
    if rank is None:
        rank = dist.get_rank() if world_size > 1 else 0
    rank, world_size = int(rank), int(world_size)
    if world_size < 1 or not 0 <= rank < world_size:
        raise ValueError(f"rank {rank} of world size {world_size}")
    return rank, world_size


def _broadcast_int(v):
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        raise RuntimeError("a data-parallel DeviceCloudLoader without a seed needs an initialised "
                           "process group (to share rank 0's seed); pass seed= on every rank")
    t = torch.tensor([int(v)], dtype=torch.int64)
    if dist.get_backend() == "nccl":
        t = t.cuda()
    dist.broadcast(t, src=0)
    return int(t.item())


def shard_order(order, B, rank, world):
    """Rank `rank`'s rows of each whole global batch of an epoch order: the
    global batches are order[k W B : (k + 1) W B] and this rank takes their
    rows [rank B, rank B + B), concatenated in batch order (a ragged tail of
    fewer than W B clouds is dropped).  Works on any 1-D tensor (host or
    device)."""
    Bg = B * world
    nb = order.numel() // Bg
    return order[:nb * Bg].reshape(nb, world, B)[:, rank].reshape(-1).contiguous()


class DeviceCloudLoader:
    """A DataLoader over one of the datasets above whose whole split lives in
    HBM (ModelNet40 train: 9 840 x 1 024 x 3 f32 = 121 MB of the 288 GB).

    Iterating yields batches shaped like ``torch.utils.data.DataLoader(dataset,
    batch_size, shuffle)`` would: (pts, labels) for ModelNetDatasetGT, pts for
    ModelNetDataset_noGT, (pts, cls_onehot, seg) / (pts, cls_onehot) for the
    ShapeNet sets - all on the device, each batch one pcadv_gather_clouds
    launch (jitter from device Philox draws when the dataset augments).
    ``noise``: optional callable(b, npts) -> f64 standard normals (host numpy),
    for parity runs against the reference's jitter.

    ``seed`` keys the shuffle and the jitter draws; None (the default) takes
    one from torch's default generator, so two loaders built alike draw
    independent jitter as the reference's np.random does.  The dataset kind is
    mixed into the Philox key too: a GT and a no-GT loader given the same
    seed still draw different fields.

    Data parallelism (``world_size`` > 1, ``rank``; default: the initialised
    torch.distributed group's, else one process): ``batch_size`` is the
    per-rank batch B.  Every rank draws the same epoch permutation (the seed
    is rank 0's, broadcast when it is not given) and takes rows
    [rank B, rank B + B) of each global batch of world_size x B clouds
    (shard_order), jittered with the Philox draws of those global rows; so
    the ranks' batches are exactly the slices of a one-process loader of
    batch world_size x B with the same seed.  A ragged last global batch is
    dropped (drop_last is forced on): unequal shards would not average to the
    global batch's mean losses."""

    _KIND_TAG = {"modelnet_gt": 1, "modelnet_nogt": 2, "shapenet_gt": 3, "shapenet_nogt": 4}

    def __init__(self, dataset, batch_size, shuffle=True, seed=None, device="cuda", drop_last=False,
                 sigma=0.01, clip=0.05, rank=None, world_size=None):
        self.lib = _lib.load()
        self.rank, self.world = _dp_rank_world(rank, world_size)
        if self.world > 1:
            drop_last = True
        self.ds, self.B, self.shuffle, self.drop_last = dataset, int(batch_size), shuffle, drop_last
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise ValueError("DeviceCloudLoader keeps the split in HBM: a HIP device is required")
        if self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        self.pts = torch.from_numpy(np.ascontiguousarray(dataset.select_data, np.float32)).to(self.device)
        self.n, self.npts = int(self.pts.shape[0]), int(self.pts.shape[1])
        lab = getattr(dataset, "select_labels", None)
        self.labels = None if lab is None else torch.from_numpy(
            np.ascontiguousarray(lab.reshape(self.n, -1), np.int64)).to(self.device)
        seg = getattr(dataset, "select_segs", None)
        self.segs = None if seg is None else torch.from_numpy(
            np.ascontiguousarray(seg, np.int64)).to(self.device)
        self.kind = ("modelnet_gt" if isinstance(dataset, ModelNetDatasetGT) else
                     "modelnet_nogt" if isinstance(dataset, ModelNetDataset_noGT) else
                     "shapenet_gt" if isinstance(dataset, ShapeNetDatasetGT) else
                     "shapenet_nogt" if isinstance(dataset, ShapeNetDataset_noGT) else None)
        if self.kind is None:
            raise TypeError(f"unsupported dataset {type(dataset).__name__}")
        self.sigma = float(sigma) if getattr(dataset, "data_augmentation", False) else 0.0
        self.clip = float(clip)
        if seed is None:
            seed = int(torch.randint(0, 2 ** 62, (1,)).item())
            if self.world > 1:  # one permutation and one jitter field for every rank
                seed = _broadcast_int(seed)
        self.seed = (int(seed) ^ (self._KIND_TAG[self.kind] << 58)) & 0xFFFFFFFFFFFFFFFF
        self.gen = torch.Generator(device=self.device)
        self.gen.manual_seed(int(seed))
        self.step = torch.zeros(1, device=self.device, dtype=torch.int32)
        self.noise = None

    def __len__(self):
        Bg = self.B * self.world  # the global batch
        return self.n // Bg if self.drop_last else (self.n + Bg - 1) // Bg

    @property
    def order_len(self):
        """Length of epoch_order(): the split, or this rank's shard of the
        whole global batches."""
        return self.n if self.world == 1 else len(self) * self.B

    def gather(self, idx, noise=None, out=None, _checked=False, out_lab=None):
        """One batch for the device index tensor ``idx`` (int64, each in
        [0, len(dataset)): checked here, one host read; the epoch order of
        __iter__ is in range by construction and skips it).  ``out`` /
        ``out_lab``: tensors to write the points (b, npts, 3) / labels (b, width)
        into (a captured graph's static inputs)."""
        b = int(idx.numel())
        if idx.dtype != torch.int64 or idx.device != self.device or not idx.is_contiguous():
            raise ValueError("idx: contiguous int64 on the loader's device")
        if b and not _checked:
            lo, hi = torch.aminmax(idx)
            if int(lo) < 0 or int(hi) >= self.n:
                raise IndexError(f"gather: index out of range [0, {self.n}) "
                                 f"(min {int(lo)}, max {int(hi)})")
        pts = out if out is not None else torch.empty(b, self.npts, 3, device=self.device)
        lw = 0 if self.labels is None else int(self.labels.shape[1])
        lab = None
        if self.labels is not None:
            lab = out_lab if out_lab is not None else torch.empty(b, lw, device=self.device,
                                                                  dtype=torch.int64)
            if tuple(lab.shape) != (b, lw) or lab.dtype != torch.int64 or not lab.is_contiguous():
                raise ValueError(f"out_lab: expected contiguous int64 ({b}, {lw})")
        seg = None if self.segs is None else torch.empty(b, self.npts, device=self.device,
                                                         dtype=torch.int64)
        nz = None
        if noise is not None and self.sigma > 0:
            nz = torch.as_tensor(noise, dtype=torch.float64).to(self.device).contiguous()
            if tuple(nz.shape) != (b, self.npts, 3):
                raise ValueError(f"noise: expected ({b}, {self.npts}, 3)")
        P = lambda t: None if t is None else ctypes.c_void_p(t.data_ptr())  # noqa: E731
        check(self.lib.pcadv_gather_clouds(P(self.pts), self.n, self.npts, self.npts, P(idx), b,
                                           P(self.labels), lw, P(self.segs), self.sigma, self.clip,
                                           P(nz), self.seed, P(self.step), P(pts), P(lab), P(seg),
                                           self.rank * self.B, stream_ptr()), "pcadv_gather_clouds")
        self.step += 1
        return self._pack(pts, lab, seg)

    def _pack(self, pts, lab, seg):
        if self.kind == "modelnet_gt":
            return pts, lab[:, 0]
        if self.kind == "modelnet_nogt":
            return pts
        oh = torch.zeros(pts.shape[0], 1, self.ds.num_classes, device=self.device)
        oh.scatter_(2, lab[:, :1].unsqueeze(1), 1.0)
        return (pts, oh, seg) if self.kind == "shapenet_gt" else (pts, oh)

    def epoch_order(self):
        """One epoch's order of the split: a fresh permutation from the loader's
        generator when shuffling (what __iter__ draws at the start of an epoch);
        under data parallelism this rank's shard of it (shard_order)."""
        if self.shuffle:
            order = torch.randperm(self.n, device=self.device, generator=self.gen)
        else:
            order = torch.arange(self.n, device=self.device)
        if self.world > 1:
            order = shard_order(order, self.B, self.rank, self.world)
        return order

    def index_batches(self):
        """The index slices of one epoch, in the order __iter__ gathers them."""
        order = self.epoch_order()
        for k in range(len(self)):
            yield order[k * self.B:(k + 1) * self.B]

    def gather_at(self, order, cursor, out, out_lab=None, out_seg=None):
        """Batch *cursor (device int32) of the epoch order `order` (int64, on the
        device) into `out` / `out_lab` (/ `out_seg`, the part ids of a ShapeNet
        split): the graph-replayed form of gather (no host copy per batch).
        The step counter is NOT advanced here: the caller advances it and the
        cursor (pcadv_iter_epilogue)."""
        j = self._gather_job(order, cursor, out, out_lab, out_seg)
        check(self.lib.pcadv_gather_clouds_at(j.src, j.n_src, j.npts, j.src_npts, j.order,
                                              j.cursor, j.B, j.src_lab, j.lab_width, j.src_seg,
                                              j.sigma, j.clip, j.seed, j.step, j.out, j.out_lab,
                                              j.out_seg, j.rng_row0, stream_ptr()),
              "pcadv_gather_clouds_at")

    def _gather_job(self, order, cursor, out, out_lab=None, out_seg=None):
        """The checked arguments of one gather_at as a pcadv_gather_job."""
        lw = 0 if self.labels is None else int(self.labels.shape[1])
        if out_lab is None and self.labels is not None:
            raise ValueError("gather_at: out_lab required for a labelled split")
        if (out_seg is None) != (self.segs is None):
            raise ValueError("gather_at: out_seg goes with (and only with) a part-labelled split")
        B = self.B

        def need(t, name, shape, dtype):
            if (t.device != self.device or t.dtype != dtype or tuple(t.shape) != shape
                    or not t.is_contiguous()):
                raise ValueError(f"gather_at: {name} must be contiguous {dtype} {shape} on "
                                 f"{self.device} (got {t.dtype} {tuple(t.shape)} on {t.device})")
        need(out, "out", (B, self.npts, 3), torch.float32)
        if self.labels is not None:
            need(out_lab, "out_lab", (B, lw), torch.int64)
        if out_seg is not None:
            need(out_seg, "out_seg", (B, self.npts), torch.int64)
        need(order, "order", (self.order_len,), torch.int64)
        need(cursor, "cursor", (1,), torch.int32)
        P = lambda t: None if t is None else t.data_ptr()  # noqa: E731
        return GatherJob(src=P(self.pts), n_src=self.n, npts=self.npts, src_npts=self.npts,
                         order=P(order), cursor=P(cursor), B=self.B, src_lab=P(self.labels),
                         lab_width=lw, src_seg=P(self.segs), sigma=self.sigma, clip=self.clip,
                         seed=self.seed, step=P(self.step), out=P(out), out_lab=P(out_lab),
                         out_seg=P(out_seg), rng_row0=self.rank * self.B)

    def __iter__(self):
        for idx in self.index_batches():
            yield self.gather(idx.contiguous(), _checked=True)


def gather_at_multi(items):
    """Several loaders' gather_at in ONE launch (pcadv_gather_clouds_multi):
    items = [(loader, order, cursor, out, out_lab, out_seg), ...] (out_lab /
    out_seg None where the split has none), at most 4; each batch is bitwise
    what loader.gather_at would write.  The graph-replayed iteration's GT and
    no-GT batches (trainer._GraphedIteration)."""
    if not 1 <= len(items) <= 4:
        raise ValueError(f"gather_at_multi: {len(items)} loaders (1..4)")
    jobs = (GatherJob * len(items))(*[ld._gather_job(*rest) for ld, *rest in items])
    lib = items[0][0].lib
    check(lib.pcadv_gather_clouds_multi(jobs, len(items), stream_ptr()),
          "pcadv_gather_clouds_multi")
