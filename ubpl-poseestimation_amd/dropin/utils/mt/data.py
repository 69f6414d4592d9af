"""utils/mt/data.py: TwoStreamBatchSampler."""
from ubpl_amd.sampler import TwoStreamBatchSampler  # noqa: F401
