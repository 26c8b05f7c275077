"""Signal catalogue, capability modes, synthetic generator and metadata enrichers."""

from . import catalog  # noqa: F401
