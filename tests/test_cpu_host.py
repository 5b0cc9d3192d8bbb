"""CPU-side checks: the C-ABI library loads and exports every symbol of
include/pcadv.h (no compute), layouts agree, drop-in modules keep the
reference's state_dict, host-side validation refuses bad inputs."""
import os
import re

import numpy as np
import pytest
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _header_symbols():
    src = open(os.path.join(REPO, "include", "pcadv.h")).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[\w]+\**\s+\**(pcadv_\w+)\s*\(", src, re.M)))


def test_library_exports_header_symbols():
    from adversarial_learning_on_pointclouds_amd import _lib
    lib = _lib.load()
    syms = _header_symbols()
    assert len(syms) >= 12
    for s in syms:
        assert hasattr(lib, s), s
        assert s in _lib.SIGNATURES, s
    assert sorted(_lib.SIGNATURES) == syms  # nothing bound that the header does not declare
    assert lib.pcadv_abi_version() == _lib.ABI_VERSION == 10


def test_layout_matches_header_enums():
    from adversarial_learning_on_pointclouds_amd import _lib
    src = open(os.path.join(REPO, "include", "pcadv.h")).read()
    enums = {k: int(v) for k, v in re.findall(r"(PCADV_[GD]_\w+) = (\d+)", src)}
    assert enums["PCADV_G_NUMEL"] == _lib.G_NUMEL and enums["PCADV_D_NUMEL"] == _lib.D_NUMEL
    from oracle import pointnet_np as onp
    for spec, layout, prefix in ((onp.cls_spec(40), _lib.G_LAYOUT, "G"),
                                 (onp.disc_spec(40, 1), _lib.D_LAYOUT, "D")):
        off = 0
        for name, shape in spec:
            assert layout[name] == off, name
            assert off % 4 == 0  # float4 alignment of every tensor
            off += int(np.prod(shape))


def test_state_dict_matches_reference_spec():
    import adversarial_learning_on_pointclouds_amd as pc
    from oracle import pointnet_np as onp
    sd = pc.PointNetCls(k=40).state_dict()
    assert [(k, tuple(v.shape)) for k, v in sd.items()] == [(k, s) for k, s in onp.cls_spec(40)]
    sd = pc.DeepConvDiscNet(40, 1).state_dict()
    assert [(k, tuple(v.shape)) for k, v in sd.items()] == [(k, s) for k, s in onp.disc_spec(40, 1)]


def test_workspace_sizes():
    from adversarial_learning_on_pointclouds_amd import _lib
    lib = _lib.load()
    # x3 (C*N*128 f32) is the only per-point activation the step keeps
    assert lib.pcadv_adv_step_workspace_bytes(32, 1024) > 64 * 1024 * 128 * 4
    # the two-kernel forward keeps its screening state in registers: no scratch
    assert lib.pcadv_feat_fwd_workspace_bytes(64, 1024) == 256
    # segmentation engine: point-axis slabs of the weight gradient (32 x O x K),
    # per-128-point-tile top-2 keys of conv6 + max, CE partials
    # 64 output tiles -> 12 slabs of the point axis (~768 workgroups); 16 clouds x 3
    nz = 8  # 64 tiles x 8 slabs: the 512 workgroups of one dispatch round
    assert lib.pcadv_gemm_wgrad_workspace_bytes(32768, 2048, 512, 0) == (nz * 2048 * (512 + 1) + 2048) * 4 + 512
    nz = 16 * 2
    assert lib.pcadv_gemm_wgrad_workspace_bytes(32768, 256, 960, 2048) == (nz * 256 * (960 + 1) + 16 * 256) * 4 + 512
    assert lib.pcadv_gemm_wgrad_workspace_bytes(300, 64, 3, 7) == 0  # rows % rows_per_group
    assert lib.pcadv_conv_max_x3_workspace_bytes(16, 2048, 2048) == 16 * 16 * 2048 * 8 + 256
    assert lib.pcadv_row_ce_workspace_bytes(32768) == 128 * 4 + 256
    assert lib.pcadv_feat_bwd_workspace_bytes(64, 1024) == 64 * 8 * 12736 * 4


def test_ops_refuse_cpu_tensors():
    from adversarial_learning_on_pointclouds_amd import ops
    with pytest.raises(ValueError):
        ops.linear_fwd(torch.zeros(4, 8), torch.zeros(3, 8), torch.zeros(3))


def test_make_D_label_and_pool():
    from adversarial_learning_on_pointclouds_amd.utils import make_D_label
    from adversarial_learning_on_pointclouds_amd.image_pool import ImagePool
    x = torch.zeros(1000, 1)
    hi = make_D_label(x, 1, "cpu", random=True)
    lo = make_D_label(x, 0, "cpu", random=True)
    assert hi.min() >= 0.7 and hi.max() <= 1.05 and lo.min() >= 0 and lo.max() <= 0.305
    assert torch.equal(make_D_label(x, 1, "cpu"), torch.ones(1000, 1))
    assert ImagePool(0).query(x) is x


def test_error_message_roundtrip():
    from adversarial_learning_on_pointclouds_amd import _lib
    lib = _lib.load()
    rc = lib.pcadv_linear_fwd(None, None, None, None, 0, 0, 0, 0, None, None, 0, 0.0, 0, None)
    assert rc == -1
    assert b"bad shape" in lib.pcadv_last_error()


def test_gather_multi_and_epilogue_refuse_bad_arguments():
    """ABI 7's batched gather and iteration epilogue validate on the host before
    any launch (no GPU needed): job counts outside 1..4, a job without its
    source, counters beyond 64, a ring without its counter."""
    import ctypes
    from adversarial_learning_on_pointclouds_amd import _lib
    lib = _lib.load()
    jobs = (_lib.GatherJob * 5)()
    for n in (0, 5):
        assert lib.pcadv_gather_clouds_multi(jobs, n, None) == -1
        assert b"jobs" in lib.pcadv_last_error()
    assert lib.pcadv_gather_clouds_multi(jobs, 1, None) == -1  # src / order / cursor missing
    assert b"bad arguments" in lib.pcadv_last_error()
    x = ctypes.c_int(0)
    assert lib.pcadv_iter_epilogue(ctypes.byref(x), 65, None, 0, None, 0, None, None) == -1
    assert b"counters" in lib.pcadv_last_error()
    f = ctypes.c_float(0)
    assert lib.pcadv_iter_epilogue(None, 0, ctypes.byref(f), 4, ctypes.byref(f), 8, None, None) == -1
    assert b"loss ring" in lib.pcadv_last_error()


def test_image_pool_history_vs_reference_g10():
    """ImagePool(3) over six queries on a seeded Python RNG returns what the
    reference's utils/image_pool.py:26-55 returned (fixture g10)."""
    import random
    from golden_util import load
    from adversarial_learning_on_pointclouds_amd.image_pool import ImagePool
    fx = load("g10_host_helpers.npz")
    pool = ImagePool(int(fx["pool_size"]))
    random.seed(int(fx["random_seed"]))
    for q, want in zip(fx["queries"], fx["pool_out"]):
        got = pool.query(torch.from_numpy(q))
        assert got.requires_grad
        assert np.array_equal(got.detach().numpy(), want)
    assert pool.num_imgs == 3


def test_image_pool_plan_equals_per_sample_history():
    """ImagePool's planned query (one gather, one scatter) returns and keeps
    what the per-sample loop of utils/image_pool.py:26-55 would, including a
    slot swapped more than once within one batch (pool of 2, batches of 7)."""
    import random
    from adversarial_learning_on_pointclouds_amd.image_pool import ImagePool

    def loop_query(bank, filled, size, batch):  # the reference's order of draws
        out = batch.clone()
        for i in range(batch.shape[0]):
            if filled < size:
                bank[filled] = batch[i]
                filled += 1
            elif random.random() > 0.5:
                slot = random.randrange(size)
                out[i] = bank[slot].clone()
                bank[slot] = batch[i]
        return out, filled

    gen = torch.Generator().manual_seed(3)
    for size, bsz in ((2, 7), (5, 3), (4, 4)):
        pool = ImagePool(size)
        bank, filled = torch.zeros(size, 6), 0
        random.seed(size * 10 + bsz)
        state = random.getstate()
        for _ in range(8):
            batch = torch.randn(bsz, 6, generator=gen)
            random.setstate(state)
            want, filled = loop_query(bank, filled, size, batch)
            random.setstate(state)
            got = pool.query(batch)
            state = random.getstate()
            assert torch.equal(got.detach(), want) and got.requires_grad
            assert torch.equal(pool._bank[:filled], bank[:filled]) and pool.num_imgs == filled


def test_init_weights_xavier_vs_reference_g10():
    """init_weights(DeepConvDiscNet, 'xavier') on a seeded torch RNG gives the
    reference's weights (utils/model_utils.py:27-58, fixture g10)."""
    from golden_util import check_tensor
    from golden_util import load
    import adversarial_learning_on_pointclouds_amd as pc
    from adversarial_learning_on_pointclouds_amd.model_utils import init_weights
    fx = load("g10_host_helpers.npz")
    torch.manual_seed(int(fx["torch_seed"]))
    md = pc.DeepConvDiscNet(40, 1)
    init_weights(md, "xavier", init_gain=1.0, verbose=False)
    for name, p in md.named_parameters():
        check_tensor(fx, "xavier." + name, p.detach().numpy(), tol=0.0)
    with pytest.raises(NotImplementedError):
        init_weights(pc.DeepConvDiscNet(40, 1), "bogus", verbose=False)


def test_image_pool_checks_sample_shape():
    """ImagePool(k > 0) keeps its history in one preallocated tensor: while the
    history is empty a new sample shape or dtype reallocates it; once it holds
    samples, a mismatching batch raises a clear error instead of failing
    inside copy_ or silently casting."""
    import torch
    from adversarial_learning_on_pointclouds_amd.image_pool import ImagePool
    pool = ImagePool(3)
    out = pool.query(torch.zeros(0, 40))       # empty batch: nothing stored
    assert out.shape == (0, 40) and pool.num_imgs == 0
    pool.query(torch.ones(2, 7, dtype=torch.float64))  # re-sized while empty
    assert pool.num_imgs == 2
    with pytest.raises(ValueError, match="ImagePool"):
        pool.query(torch.ones(2, 40))
    with pytest.raises(ValueError, match="ImagePool"):
        pool.query(torch.ones(2, 7, dtype=torch.float32))


def test_shard_order_slices_global_batches():
    """DeviceCloudLoader's data-parallel sharding (dataset.shard_order): rank r
    of W takes rows [r B, r B + B) of every whole global batch of W B clouds of
    the shared epoch order; the ranks' shards tile the whole batches exactly
    once and the ragged tail is dropped."""
    import torch
    from adversarial_learning_on_pointclouds_amd.dataset import shard_order
    order = torch.randperm(23, generator=torch.Generator().manual_seed(0))
    B, W = 3, 2
    shards = [shard_order(order, B, r, W) for r in range(W)]
    assert all(s.numel() == 3 * B for s in shards)  # 23 // 6 = 3 global batches
    for k in range(3):
        glob = order[k * B * W:(k + 1) * B * W]
        assert torch.equal(torch.cat([s[k * B:(k + 1) * B] for s in shards]), glob)
    assert torch.equal(shard_order(order, B, 0, 1), order[:21])


def _c_layout(struct, fields, tmp_path):
    """sizeof and offsetof of a C struct of include/pcadv.h, from gcc."""
    import shutil
    import subprocess
    if shutil.which("gcc") is None or not os.path.isdir("/opt/rocm/include"):
        pytest.skip("gcc or the ROCm headers are absent")
    body = "".join(f'  printf("%zu\\n", offsetof({struct}, {f}));\n' for f in fields)
    src = tmp_path / "layout.c"
    src.write_text(f'#include <stdio.h>\n#include "pcadv.h"\nint main(void) {{\n'
                   f'  printf("%zu\\n", sizeof({struct}));\n{body}  return 0;\n}}\n')
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-D__HIP_PLATFORM_AMD__", "-I", os.path.join(REPO, "include"),
                    "-I", "/opt/rocm/include", str(src), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split()
    return int(out[0]), [int(v) for v in out[1:]]


@pytest.mark.parametrize("name", ["AdvArgs", "GatherJob", "PwWgradJob", "PwLayer"])
def test_ctypes_structs_match_the_c_layout(name, tmp_path):
    """The ctypes mirrors of pcadv_adv_args / pcadv_gather_job (the structs
    the trainer fills) have the C structs' size and field offsets."""
    from adversarial_learning_on_pointclouds_amd import _lib
    py = getattr(_lib, name)
    c = {"AdvArgs": "pcadv_adv_args", "GatherJob": "pcadv_gather_job",
         "PwWgradJob": "pcadv_pw_wgrad_job", "PwLayer": "pcadv_pw_layer"}[name]
    fields = [f for f, _ in py._fields_]
    size, offs = _c_layout(c, fields, tmp_path)
    assert ctypes_sizeof(py) == size
    assert [getattr(py, f).offset for f in fields] == offs


def ctypes_sizeof(t):
    import ctypes
    return ctypes.sizeof(t)


def test_load_refuses_another_abi(tmp_path, monkeypatch):
    """a library of another ABI (a stale build, an old PCADV_LIB) is
    refused at load instead of binding shifted arguments."""
    import subprocess
    from adversarial_learning_on_pointclouds_amd import _lib
    src = tmp_path / "old.c"
    src.write_text("int pcadv_abi_version(void) { return 5; }\n")
    so = tmp_path / "libold.so"
    subprocess.run(["gcc", "-shared", "-fPIC", "-o", str(so), str(src)], check=True)
    monkeypatch.setattr(_lib, "LIB_PATH", str(so))
    monkeypatch.setattr(_lib, "_lib", None)
    with pytest.raises(_lib.PcadvError, match="ABI 5"):
        _lib.load()
