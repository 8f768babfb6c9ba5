"""In-node inference engine (continuous batching, paged KV, hipGraph decode)."""
from .sampling_params import SamplingParams  # noqa: F401
