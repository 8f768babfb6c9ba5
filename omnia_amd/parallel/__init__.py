"""Intra-node parallelism: process groups (:mod:`.state`), the one-shot IPC
all-reduce for decode-size TP collectives (:mod:`.custom_allreduce`, K16), the
expert-parallel token all-to-all (:mod:`.expert`, K15) and the session-affine
DP replica router (:mod:`.router`)."""
from .state import ParallelState, get_state, init_distributed, set_state, tp_all_reduce

__all__ = ["ParallelState", "get_state", "init_distributed", "set_state", "tp_all_reduce"]
