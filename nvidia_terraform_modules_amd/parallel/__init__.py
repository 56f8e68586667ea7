"""RCCL-over-xGMI collectives: process-group bootstrap, C1 all-reduce sweep,
and the hand-written C2 peer-to-peer (xGMI mesh) all-reduce."""
from .collectives import (  # noqa: F401
    CollResult,
    all_reduce_sweep,
    bus_factor,
    format_table,
    peak_busbw,
    sweep_sizes,
)
from .dist import DistEnv, all_gather_obj, all_reduce_max, all_reduce_sum, barrier, init, shutdown  # noqa: F401
