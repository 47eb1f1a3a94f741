"""rnnt_amd -- MI355X-native RNN-T inference hot path (host side).

The compute path is the HIP engine in ``librnnt_mi355x.so`` (built from ../csrc, C-ABI in
include/rnnt_mi355x.h); this package mirrors the reference's operator surface
(``torch.ops.intel_mlperf.*``, models/_C.py) and model driver (GreedyDecoder, SUT) on top.
"""
from .config import RNNTParam, LABELS, seq_to_sen  # noqa: F401
