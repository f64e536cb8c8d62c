"""Tuned hipBLASLt / rocBLAS solution choice for the dense (library) GEMMs.

The dense MLP GEMMs stay on the vendor libraries; their default heuristic picks
poor fp32 tiles for the tall-skinny shapes of the DIEN auxiliary net, the AUGRU/GRU input
projections and the MMOE experts (e.g. [811 008, 72] x [72, 80]). PyTorch's TunableOp measured
every candidate solution for every GEMM shape the benchmarked models run on MI355X
(tools/tune_all.sh); the winners are committed in tuned/tunableop_mi355x.csv and replayed here
with tuning OFF (no measurement at run time; a shape missing from the table takes the default
heuristic). DIEN cfg3: 6.63 -> 5.76 ms/step. The table is tied to the ROCm / hipBLASLt / PyTorch
versions in its Validator lines; on another stack TunableOp ignores it."""
from __future__ import annotations

import os

import torch

TUNED_TABLE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tuned",
                           "tunableop_mi355x.csv")
_active = False


def use_tuned_gemms(path: str | None = None) -> bool:
    """Enable TunableOp with the committed results (idempotent). Returns True when active."""
    global _active
    if _active:
        return True
    path = path or TUNED_TABLE
    if not (torch.cuda.is_available() and os.path.exists(path)):
        return False
    import torch.cuda.tunable as T

    T.enable(True)
    T.tuning_enable(False)
    T.record_untuned_enable(False)
    T.set_filename(os.path.join(os.environ.get("TMPDIR", "/tmp"), f"rs_tunableop_{os.getpid()}%d.csv"))
    _active = bool(T.read_file(path))
    return _active
