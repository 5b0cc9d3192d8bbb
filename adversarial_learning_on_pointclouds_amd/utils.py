"""GAN glue with the interface of utils/utils.py:9-31 (make_logger, make_D_label)."""
from __future__ import annotations

import logging
import os
import sys

import torch


def make_logger(filename, args):
    """A root logger at INFO that writes bare messages both to
    <args.exp_dir>/<filename> and to stdout, and records `args` first
    (interface of utils/utils.py:9-20)."""
    root = logging.getLogger()
    plain = logging.Formatter()
    for handler in (logging.FileHandler(os.path.join(args.exp_dir, filename)),
                    logging.StreamHandler(sys.stdout)):
        handler.setFormatter(plain)
        root.addHandler(handler)
    root.setLevel(logging.INFO)
    root.info(args)
    return root


_SOFT_RANGE = {0: (0.0, 0.305), 1: (0.7, 1.05)}


def make_D_label(input, value, device, random=False):
    """Discriminator targets shaped like `input` (utils/utils.py:22-31): the
    constant `value`, or with random=True soft labels U(0.7, 1.05) for 1 and
    U(0, 0.305) for 0.  Drawn directly on `device` (the reference draws on the
    host and copies)."""
    shape = input.data.size()
    if not random:
        return torch.full(shape, float(value), device=device)
    lo, hi = _SOFT_RANGE[value]
    return torch.empty(shape, device=device).uniform_(lo, hi)
