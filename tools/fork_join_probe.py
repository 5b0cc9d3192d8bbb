"""What a fork / join costs inside a replayed HIP graph (VERDICT r05 item 3:
re-measure round 2's 5-11 us per edge under the current dispatch mode,
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0).  Chains of small kernels (one 256-thread
workgroup each, ~2 us) captured as

    serial : A -> B1 -> B2 -> ... -> C                (one stream)
    forked : A -> (B1 -> ... on s1 || B2 -> ... on s2) -> C

with the same kernels; per-replay time by HIP events over 400 replays.
Writes one JSON line.  python tools/fork_join_probe.py [depth]
"""
import json
import os
import sys

os.environ.setdefault("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "0")
import torch  # noqa: E402


def main():
    depth = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    dev = torch.device("cuda:0")
    x = [torch.zeros(256, device=dev) for _ in range(4)]
    s0 = torch.cuda.Stream()
    s1 = torch.cuda.Stream()

    def k(t):
        t.add_(1.0)

    def serial():
        k(x[0])
        for _ in range(depth):
            k(x[1])
        for _ in range(depth):
            k(x[2])
        k(x[3])

    def forked():
        k(x[0])
        cur = torch.cuda.current_stream()
        s1.wait_stream(cur)
        for _ in range(depth):
            k(x[1])
        with torch.cuda.stream(s1):
            for _ in range(depth):
                k(x[2])
        cur.wait_stream(s1)
        k(x[3])

    def chain_only():  # A -> B1 x depth -> C (one branch's length)
        k(x[0])
        for _ in range(depth):
            k(x[1])
        k(x[3])

    res = {}
    for name, body in (("serial", serial), ("forked", forked), ("one_branch", chain_only)):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(s0):
            body()
            torch.cuda.synchronize()
            with torch.cuda.graph(g, stream=s0):
                body()
        torch.cuda.synchronize()
        for _ in range(50):
            g.replay()
        torch.cuda.synchronize()
        times = []
        for _ in range(3):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(400):
                g.replay()
            e1.record()
            torch.cuda.synchronize()
            times.append(e0.elapsed_time(e1) * 1e3 / 400)
        res[name] = round(sorted(times)[1], 2)
    kernels = {"serial": 2 + 2 * depth, "forked": 2 + 2 * depth, "one_branch": 2 + depth}
    out = {"probe": "fork/join edges in a replayed HIP graph", "depth": depth,
           "us_per_replay": res, "kernels": kernels,
           "us_per_kernel_serial": round(res["serial"] / kernels["serial"], 2),
           "fork_join_cost_us": round(res["forked"] - res["one_branch"], 2),
           "runtime": {"DEBUG_CLR_GRAPH_PACKET_CAPTURE": os.environ.get("DEBUG_CLR_GRAPH_PACKET_CAPTURE")}}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
