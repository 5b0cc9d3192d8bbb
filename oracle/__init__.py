"""CPU oracle for the PointNet adversarial train step — TEST INFRASTRUCTURE ONLY.

This package is a from-scratch numpy (fp32) restatement of the reference's hot
path (YiruS/Adversarial_Learning_on_PointClouds: ``models/pointnet.py``,
``models/discriminator.py``, ``utils/trainer.py:run_training``, ``utils/utils.py``,
``torch.optim.Adam``).  It is the *checker*: only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import it.
The product path (``adversarial_learning_on_pointclouds_amd``) never imports it
and fails loudly when its HIP library is missing.

Parity pinning: the restatement is pinned against golden vectors captured from
the reference itself (imported from /root/reference in the build container by
``tests/golden/make_golden.py``); see ``tests/test_oracle_golden.py``.
"""
