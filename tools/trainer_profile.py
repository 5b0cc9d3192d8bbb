"""Host-side profile of trainer.run_training over DeviceCloudLoaders (the
bench's --config trainer workload): cProfile of one run of K iterations, top
functions by own time, and the host issue time vs the wall time.

    python tools/trainer_profile.py [K] [use_graph 0/1]
"""
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    use_graph = bool(int(sys.argv[2])) if len(sys.argv) > 2 else True
    import argparse
    a = argparse.Namespace(warmup=20, steps=K, repeats=1)
    # reuse bench_trainer's run() through a small shim
    import logging
    import tempfile
    import torch
    from adversarial_learning_on_pointclouds_amd import dataset as D
    from adversarial_learning_on_pointclouds_amd import trainer
    from adversarial_learning_on_pointclouds_amd.image_pool import ImagePool
    dev = torch.device("cuda", 0)
    gt_ds, ng_ds = bench._synthetic_modelnet(1024, 4096)
    log = logging.getLogger("tp")
    log.addHandler(logging.NullHandler())
    log.propagate = False

    def run(iters):
        model, model_D = bench.make_models(dev, seed=0)
        opt = torch.optim.Adam(model.parameters(), lr=1e-4)
        opt_D = torch.optim.Adam(model_D.parameters(), lr=1e-4)
        gt = D.DeviceCloudLoader(gt_ds, 32, seed=1, drop_last=True)
        ng = D.DeviceCloudLoader(ng_ds, 32, seed=2, drop_last=True)
        ns = argparse.Namespace(device="cuda", total_iterations=iters, iter_save_epoch=10 ** 9,
                                iter_test_epoch=10 ** 9, exp_dir=tempfile.mkdtemp(), tensorboard=False,
                                lambda_cls=1.0, lambda_adv=0.001, batch_size=32,
                                use_graph=use_graph, log_every=1)
        trainer.run_training(gt, ng, enumerate(gt), enumerate(ng), [next(iter(gt))], model, model_D,
                             torch.nn.BCEWithLogitsLoss(), torch.nn.CrossEntropyLoss(), opt, opt_D,
                             ImagePool(0), ImagePool(0), log, log, None, ns)
        torch.cuda.synchronize()

    run(20)
    pr = cProfile.Profile()
    t0 = time.perf_counter()
    pr.enable()
    run(K)
    pr.disable()
    print(f"wall {time.perf_counter() - t0:.4f}s for {K} iterations (+ setup)")
    pstats.Stats(pr).sort_stats("tottime").print_stats(25)


if __name__ == "__main__":
    main()
