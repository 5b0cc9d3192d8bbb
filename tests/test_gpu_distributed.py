"""The split adversarial step behind the overlapped data-parallel all-reduce
(pcadv_adv_args.part): part 1 (everything before the feature backward) then
part 2 (the feature backward) must equal the whole step bitwise, and the
bucketed all-reduce must give the same replicas as the single all-reduce.

The multi-rank case runs two gloo ranks on the one GPU of the box (RCCL needs
one device per rank); the gloo all-reduce of device tensors is the same
arithmetic on the same buckets as RCCL's.
"""
import os
import socket

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

B, N = 8, 256


def _models(dev):
    import adversarial_learning_on_pointclouds_amd as pc
    torch.manual_seed(0)
    return pc.PointNetCls(k=40).to(dev), pc.DeepConvDiscNet(40, 1).to(dev)


def _batch(dev, seed, b=B):
    g = torch.Generator().manual_seed(seed)
    pg = (torch.rand(b, N, 3, generator=g) * 2 - 1).to(dev)
    pn = (torch.rand(b, N, 3, generator=g) * 2 - 1).to(dev)
    lab = torch.randint(0, 40, (b,), generator=g).to(dev)
    return pg, lab, pn


def test_parts_equal_whole_step():
    from adversarial_learning_on_pointclouds_amd.step import AdvTrainStep
    dev = torch.device("cuda:0")
    outs = []
    for split in (False, True):
        m, d = _models(dev)
        st = AdvTrainStep(m, d, B, N, seed=7, device=dev)
        for k in range(3):
            pg, lab, pn = _batch(dev, 10 + k)
            if split:
                st(pg, lab, pn, apply_adam=False, part=1)
                st(pg, lab, pn, apply_adam=True, part=2)
            else:
                st(pg, lab, pn)
        torch.cuda.synchronize()
        outs.append((st.grad_flat.clone(), st.g_param.clone(), st.d_param.clone(),
                     st.losses.clone()))
    for a, b in zip(*outs):
        assert torch.equal(a, b)


def test_split_adam_equals_whole_adam():
    """adam(part=1) then adam(part=2) (the early bucket's parameters updated
    beside the late all-reduce) equals adam() bitwise, over three steps."""
    from adversarial_learning_on_pointclouds_amd.step import AdvTrainStep
    dev = torch.device("cuda:0")
    outs = []
    for split in (False, True):
        m, d = _models(dev)
        st = AdvTrainStep(m, d, B, N, seed=7, device=dev)
        for k in range(3):
            st.grads(*_batch(dev, 20 + k))
            if split:
                st.adam(part=1)
                st.adam(part=2)
            else:
                st.adam()
        torch.cuda.synchronize()
        outs.append((st.g_param.clone(), st.g_m.clone(), st.g_v.clone(), st.d_param.clone(),
                     st.d_m.clone(), st.d_v.clone()))
    for a, b in zip(*outs):
        assert torch.equal(a, b)
    with pytest.raises(RuntimeError):
        st.adam(part=3)


def test_part_graphs_equal_whole_graph():
    from adversarial_learning_on_pointclouds_amd.step import AdvTrainStep
    dev = torch.device("cuda:0")
    pg, lab, pn = _batch(dev, 3)
    res = []
    for split in (False, True):
        m, d = _models(dev)
        st = AdvTrainStep(m, d, B, N, seed=7, device=dev)
        if split:
            g1 = st.capture_on(pg, lab, pn, apply_adam=False, part=1)
            g2 = st.capture_on(pg, lab, pn, apply_adam=True, part=2)
            for _ in range(2):
                g1.replay()
                g2.replay()
        else:
            g = st.capture_on(pg, lab, pn)
            for _ in range(2):
                g.replay()
        torch.cuda.synchronize()
        res.append((st.g_param.clone(), st.d_param.clone(), st.losses.clone()))
    for a, b in zip(*res):
        assert torch.equal(a, b)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, port, out_dir):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=2)
    try:
        from adversarial_learning_on_pointclouds_amd.distributed import DataParallelAdvStep
        from adversarial_learning_on_pointclouds_amd.step import AdvTrainStep
        dev = torch.device("cuda:0")
        torch.cuda.set_device(dev)
        for overlap in (False, True):
            m, d = _models(dev)
            st = AdvTrainStep(m, d, B, N, seed=7 + rank, device=dev)
            dp = DataParallelAdvStep(st, overlap=overlap)
            graph = dp.capture(*_batch(dev, 40 + rank))
            for k in range(2):
                dp(*_batch(dev, 20 + 2 * k + rank))   # eager
                graph.replay()                        # captured halves around the all-reduce
            torch.cuda.synchronize()
            np.save(os.path.join(out_dir, f"g{rank}_{int(overlap)}.npy"), st.g_param.cpu().numpy())
            np.save(os.path.join(out_dir, f"d{rank}_{int(overlap)}.npy"), st.d_param.cpu().numpy())
    finally:
        dist.destroy_process_group()


def test_bucketed_allreduce_matches_single(tmp_path):
    import torch.multiprocessing as mp
    mp.spawn(_worker, args=(_free_port(), str(tmp_path)), nprocs=2, join=True)
    for name in ("g", "d"):
        ref = np.load(tmp_path / f"{name}0_0.npy")
        for rank in (0, 1):
            for ov in (0, 1):
                got = np.load(tmp_path / f"{name}{rank}_{ov}.npy")
                assert np.array_equal(got, ref), (name, rank, ov)
