"""L2 contracts: typed events, compiled schema validation, semconv keys and config."""

from . import config, schemas, semconv, types, validator  # noqa: F401
