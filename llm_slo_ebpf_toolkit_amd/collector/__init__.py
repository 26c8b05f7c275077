"""L1 collection: record formats, decoders, probe lifecycle and sample pipelines."""

from . import pipeline, probes, records  # noqa: F401
from .pipeline import (RawSample, SampleMeta, build_synthetic_sample,  # noqa: F401
                       generate_synthetic_samples, normalize_sample)
