"""Time-to-GPU-ready instrumentation (phase stamps, apply timeline, critical path)."""
from .phases import CLUSTER_PHASES, IN_NODE_PHASES, PhaseClock, process_start_time  # noqa: F401
