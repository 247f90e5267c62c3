"""Measured GEMM solution table for the library GEMMs (hipBLASLt / rocBLAS through PyTorch).

The hand-written kernels cover the fused hot ops; plain projections (ViT's QKV / proj / MLP
GEMMs, classifier heads) stay library GEMMs.  hipBLASLt's heuristic pick for a shape is not
always its fastest solution, so PyTorch's TunableOp benchmarks the candidates once and the
winners are kept in ``rocket_amd/tuning/gemm_mi355x.csv`` (measured on MI355X with this image's
ROCm / hipBLASLt; the validators in the file make other stacks ignore it).  ViT-B/16 bs128:
37.1 -> 33.0 ms per training step.

* default on a HIP device: TunableOp enabled, table read, NO tuning (unlisted shapes use the
  library heuristic, so no first-use benchmarking stalls);
* ``ROCKET_TUNE_GEMMS=1``: also tune unlisted shapes at first use; results are written to
  ``ROCKET_TUNED_GEMMS_OUT`` (default ``./rocket_tunableop.csv``) at exit — merge them into the
  table to keep them;
* ``ROCKET_TUNED_GEMMS=0``: leave TunableOp alone.
"""

from __future__ import annotations

import os
import tempfile

import torch

TABLE = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tuning", "gemm_mi355x.csv")

_done = False


def use_tuned_gemms(table: str = TABLE) -> bool:
    """Enable TunableOp with the measured table (idempotent).  Returns whether it is active."""
    global _done
    if _done:
        return True
    if os.environ.get("ROCKET_TUNED_GEMMS", "1") == "0" or torch.version.hip is None or not torch.cuda.is_available():
        return False
    from torch.cuda import tunable

    tune = os.environ.get("ROCKET_TUNE_GEMMS", "0") == "1"
    tunable.enable(True)
    tunable.tuning_enable(tune)
    if tune:
        out = os.environ.get("ROCKET_TUNED_GEMMS_OUT", os.path.abspath("rocket_tunableop.csv"))
    else:  # anything TunableOp decides to write goes to scratch, never into the package
        out = os.path.join(tempfile.gettempdir(), f"rocket_tunableop_{os.getpid()}.csv")
    tunable.set_filename(out, insert_device_ordinal=False)
    if os.path.exists(table):
        tunable.read_file(table)
    _done = True
    return True
