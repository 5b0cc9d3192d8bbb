"""One data-parallel form of the adversarial iteration on a one-rank RCCL
group, replayed K times for a kernel trace (bench.py --config dp1 alternates
the forms; a trace needs one): plain | dp4 | dp1g | dp2 | dp2g (see bench.bench_dp1).

    rocprofv3 --kernel-trace ... -- python tools/dp_trace.py dp4 [K]
"""
import os
import sys

os.environ.setdefault("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "0")
import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as tdist  # noqa: E402

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402


def main():
    form = sys.argv[1]
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", str(bench._free_port()))
    tdist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    from adversarial_learning_on_pointclouds_amd.step import AdvTrainStep
    from adversarial_learning_on_pointclouds_amd.distributed import DataParallelAdvStep
    model, model_D = bench.make_models(dev, seed=0)
    B, N = bench.B, bench.N
    step = AdvTrainStep(model, model_D, B, N, seed=1234, device=dev)
    runner = DataParallelAdvStep(step, overlap=True)
    flat = DataParallelAdvStep(step, broadcast_params=False, overlap=False)
    rng = np.random.default_rng(1000)
    p = (torch.from_numpy(rng.uniform(-1, 1, (B, N, 3)).astype(np.float32)).to(dev),
         torch.from_numpy(rng.integers(0, 40, B)).to(dev),
         torch.from_numpy(rng.uniform(-1, 1, (B, N, 3)).astype(np.float32)).to(dev))
    g = {"plain": lambda: step.capture_on(*p), "dp4": lambda: runner.capture(*p),
         "dp1g": lambda: runner.capture_single(*p), "dp2": lambda: flat.capture(*p),
         "dp2g": lambda: flat.capture_single(*p)}[form]()
    for _ in range(K):
        g.replay()
    torch.cuda.synchronize()
    print(f"{form}: {K} iterations done", flush=True)
    tdist.destroy_process_group()


if __name__ == "__main__":
    main()
