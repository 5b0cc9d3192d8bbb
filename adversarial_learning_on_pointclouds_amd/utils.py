"""GAN glue of utils/utils.py:9-31 (make_logger, make_D_label)."""
from __future__ import annotations

import logging
import os
import sys

import torch


def make_logger(filename, args):
    """utils/utils.py:9-20 (root logger, file + stdout handlers)."""
    logger = logging.getLogger()
    file_log_handler = logging.FileHandler(os.path.join(args.exp_dir, filename))
    logger.addHandler(file_log_handler)
    stderr_log_handler = logging.StreamHandler(sys.stdout)
    logger.addHandler(stderr_log_handler)
    logger.setLevel("INFO")
    formatter = logging.Formatter()
    file_log_handler.setFormatter(formatter)
    stderr_log_handler.setFormatter(formatter)
    logger.info(args)
    return logger


def make_D_label(input, value, device, random=False):
    """utils/utils.py:22-31: hard labels, or U(0.7,1.05) for value 1 and
    U(0,0.305) for value 0 when random.  Drawn directly on `device` (the
    reference draws on the host and copies)."""
    if random:
        if value == 0:
            lower, upper = 0, 0.305
        elif value == 1:
            lower, upper = 0.7, 1.05
        return torch.empty(input.data.size(), device=device).uniform_(lower, upper)
    return torch.full(input.data.size(), float(value), device=device)
