"""Where the driver's 20-step bench regions lose time against 200-step ones
(VERDICT r05 item 1).  Builds the bench's adversarial step graphs exactly as
`bench.py` does (same models, seeds, resident pool, DEBUG_CLR_GRAPH_PACKET_CAPTURE=0),
then times, in one process:

  A  the driver's sequence: 5 warm-up replays, three 20-step regions;
  B  host enqueue time of 20 replays (perf_counter after the replay loop,
     before the synchronize) against the region time;
  C  twelve more 20-step regions back to back (does the region converge?);
  D  three 200-step regions;
  E  20-step regions after 1 / 10 / 100 ms of host idle (clock ramp-down);
  F  one 20-step region timed with HIP events around each replay.

Prints one JSON object.  Usage: python tools/driver_gap.py [out.json]
"""
import json
import os
import sys
import time

os.environ.setdefault("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "0")
import numpy as np  # noqa: E402
import torch  # noqa: E402

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402


def region(graphs, steps, k0=0):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(steps):
        graphs[(k0 + k) % len(graphs)].replay()
    t_enq = time.perf_counter() - t0
    torch.cuda.synchronize()
    return time.perf_counter() - t0, t_enq


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else None
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    from adversarial_learning_on_pointclouds_amd.step import AdvTrainStep
    model, model_D = bench.make_models(dev, seed=0)
    B, N = bench.B, bench.N
    step = AdvTrainStep(model, model_D, B, N, seed=1234, device=dev, precision="fp32")
    pool = []
    for k in range(bench.POOL):
        rng = np.random.default_rng(1000 + k * 64)
        pool.append((torch.from_numpy(rng.uniform(-1, 1, (B, N, 3)).astype(np.float32)).to(dev),
                     torch.from_numpy(rng.integers(0, 40, B)).to(dev),
                     torch.from_numpy(rng.uniform(-1, 1, (B, N, 3)).astype(np.float32)).to(dev)))
    graphs = [step.capture_on(*p) for p in pool]
    res = {}
    for k in range(5):
        graphs[k % len(graphs)].replay()
    res["A_driver_regions_ms"] = [round(region(graphs, 20)[0] * 1e3, 4) for _ in range(3)]
    b = [region(graphs, 20) for _ in range(3)]
    res["B_region_ms"] = [round(t * 1e3, 4) for t, _ in b]
    res["B_enqueue_ms"] = [round(e * 1e3, 4) for _, e in b]
    res["C_regions20_ms"] = [round(region(graphs, 20)[0] * 1e3, 4) for _ in range(12)]
    res["D_regions200_ms"] = [round(region(graphs, 200)[0] * 1e3, 3) for _ in range(3)]
    e = {}
    for idle in (0.001, 0.01, 0.1):
        ts = []
        for _ in range(3):
            time.sleep(idle)
            ts.append(round(region(graphs, 20)[0] * 1e3, 4))
        e[f"{idle * 1e3:g}ms"] = ts
    res["E_after_idle_ms"] = e
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(21)]
    torch.cuda.synchronize()
    ev[0].record()
    for k in range(20):
        graphs[k % len(graphs)].replay()
        ev[k + 1].record()
    torch.cuda.synchronize()
    res["F_per_replay_us"] = [round(ev[k].elapsed_time(ev[k + 1]) * 1e3, 1) for k in range(20)]
    # G: the same per-replay events after a long warm stretch (steady state)
    for k in range(400):
        graphs[k % len(graphs)].replay()
    ev[0].record()
    for k in range(20):
        graphs[k % len(graphs)].replay()
        ev[k + 1].record()
    torch.cuda.synchronize()
    res["G_per_replay_warm_us"] = [round(ev[k].elapsed_time(ev[k + 1]) * 1e3, 1) for k in range(20)]
    s = json.dumps(res, indent=1)
    print(s, flush=True)
    if out:
        with open(out, "w") as f:
            f.write(s + "\n")


if __name__ == "__main__":
    main()
